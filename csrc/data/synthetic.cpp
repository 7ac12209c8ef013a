// Host-side synthetic Criteo-shaped batch generator.
//
// Counter-based (splitmix64 of (seed, rank, batch, row, field)), so any batch
// can be produced independently, by any number of threads, reproducibly --
// the host twin of the on-device generator in tdfo_amd/data/synthetic.py
// (same teacher: label ~ Bernoulli(sigmoid((dense-3.6).w*2-1.1 + table
// biases of the first id per table)); its own random stream). Feeds CPU runs
// (DLRM-tiny, BASELINE config 1) and the GPU host data plane
// (tdfo_amd/data/prefetch.py), where it must outrun a ~0.6 ms training step:
//   * ids are produced table-major, i.e. in the order they are stored, so
//     every thread streams its rows of one table contiguously;
//   * uniform ids use the multiply-shift range reduction (no 64-bit modulo);
//   * a persistent worker pool (no thread creation per batch) splits the
//     batch rows; each worker owns its rows' label scores (no sharing).
// C ABI for ctypes.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

// uniform in [0, r): high 64 bits of a 64x64 product (Lemire's reduction)
inline int64_t below(uint64_t h, uint64_t r) {
  return (int64_t)(((unsigned __int128)h * r) >> 64);
}

// ln(x) for x >= 1 (dense features log1p(u * 100)): exponent + 2 atanh((m-1)/(m+1))
// series, |error| < 2e-5 -- glibc's log1pf costs ~25 ns, this ~2 ns
inline float fast_ln(float x) {
  uint32_t b;
  __builtin_memcpy(&b, &x, 4);
  const int e = (int)(b >> 23) - 127;
  b = (b & 0x007fffffu) | 0x3f800000u;
  float m;
  __builtin_memcpy(&m, &b, 4);                 // mantissa in [1, 2)
  const float z = (m - 1.f) / (m + 1.f), z2 = z * z;
  const float at = z * (1.f + z2 * (1.f / 3 + z2 * (1.f / 5 + z2 * (1.f / 7 + z2 * (1.f / 9)))));
  return (float)e * 0.69314718f + 2.f * at;
}

// Fixed pool of workers; run(n, fn) calls fn(i) for i in [0, n) and waits.
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size(); }
  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> one(call_);          // one batch at a time per pool
    std::unique_lock<std::mutex> g(m_);
    fn_ = &fn;
    n_ = n;
    next_.store(0);
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(g, [&] { return done_ == (int)th_.size(); });
    fn_ = nullptr;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      int n;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;
        n = n_;
      }
      for (int i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) (*fn)(i);
      {
        std::lock_guard<std::mutex> g(m_);
        ++done_;
      }
      done_cv_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex call_, m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  std::atomic<int> next_{0};
  bool stop_ = false;
};

Pool* pool_for(int nthreads) {
  static std::mutex m;
  static Pool* p = nullptr;
  std::lock_guard<std::mutex> g(m);
  if (p == nullptr || p->size() != nthreads) {
    delete p;
    p = new Pool(nthreads);
  }
  return p;
}

}  // namespace

extern "C" {

// ids are table-major: table t holds B * pooling[t] ids. dist: 0 uniform, 1 zipf.
// w_dense: [num_dense]; table_bias: [T, 64] (label model: per-table bias by id % 64).
void tdfo_synth_criteo(uint64_t seed, int rank, int64_t batch_index, int B, int num_dense, int T,
                       const int64_t* rows, const int* pooling, int dist, double alpha,
                       const float* w_dense, const float* table_bias, float* dense, int64_t* ids,
                       float* label, int nthreads) {
  std::vector<int64_t> base(T + 1, 0);
  for (int t = 0; t < T; ++t) base[t + 1] = base[t] + (int64_t)B * pooling[t];
  const uint64_t key = mix(seed * 0x100000001B3ull ^ mix((uint64_t)rank << 40 ^ (uint64_t)batch_index));
  const double bias_w = 3.0 / std::sqrt((double)T);
  // rows [b0, b1): dense features, ids of every table (table-major stores),
  // label -- all of it a pure function of (key, b)
  auto work = [&](int b0, int b1) {
    std::vector<double> score(b1 - b0, -1.1);
    std::vector<uint64_t> rks(b1 - b0);            // per-row keys, reused by every table
    for (int b = b0; b < b1; ++b) {
      const uint64_t rk = mix(key ^ (uint64_t)b * 0xD6E8FEB86659FD93ull);
      rks[b - b0] = rk;
      double sc = 0.0;
      for (int j = 0; j < num_dense; ++j) {
        const float x = fast_ln(1.f + (float)(u01(mix(rk + j)) * 100.0));
        dense[(int64_t)b * num_dense + j] = x;
        sc += (x - 3.6) * w_dense[j] * 2.0;
      }
      score[b - b0] += sc;
    }
    for (int t = 0; t < T; ++t) {
      const int L = pooling[t];
      const uint64_t r = (uint64_t)rows[t];
      const float* tb = table_bias + t * 64;
      int64_t* out = ids + base[t] + (int64_t)b0 * L;
      const uint64_t tk = (uint64_t)(t + 1) << 32;
      for (int b = b0; b < b1; ++b) {
        const uint64_t rk = rks[b - b0];
        for (int l = 0; l < L; ++l) {
          const uint64_t h = mix(rk ^ tk ^ (uint64_t)(l + 1000));
          int64_t id;
          if (dist == 1 && r > 1) {
            const double x = std::pow((std::pow((double)r, 1 - alpha) - 1) * u01(h) + 1,
                                      1 / (1 - alpha));
            id = std::min<int64_t>(std::max<int64_t>((int64_t)x - 1, 0), (int64_t)r - 1);
          } else {
            id = below(h, r);
          }
          *out++ = id;
          if (l == 0) score[b - b0] += tb[id & 63] * bias_w;
        }
      }
    }
    for (int b = b0; b < b1; ++b) {
      const double p = 1.0 / (1.0 + std::exp(-score[b - b0]));
      label[b] = u01(mix(rks[b - b0] ^ 0xABCDEFull)) < p ? 1.f : 0.f;
    }
  };
  const int nt = std::max(1, std::min(nthreads, B / 256 + 1));
  if (nt == 1) {
    work(0, B);
    return;
  }
  const int chunks = nt * 4;                        // a few rows ranges per worker
  const int per = (B + chunks - 1) / chunks;
  pool_for(nt)->run(chunks, [&](int i) {
    const int b0 = i * per, b1 = std::min(B, b0 + per);
    if (b0 < b1) work(b0, b1);
  });
}

}  // extern "C"
