// Host-side synthetic Criteo-shaped batch generator.
//
// Counter-based (splitmix64 of (seed, rank, batch, row, field)), so any batch
// can be produced independently, by any number of threads, reproducibly —
// the host twin of the on-device generator in tdfo_amd/data/synthetic.py
// (same teacher: label ~ Bernoulli(sigmoid((dense-3.6).w*2-1.1 + table
// biases of the first id per table)); its own random stream). Used for
// CPU runs (DLRM-tiny, BASELINE config 1) and host-pipeline benchmarks.
// C ABI for ctypes.
#include <algorithm>
#include <cmath>
#include <cstdint>
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
  auto work = [&](int b0, int b1) {
    for (int b = b0; b < b1; ++b) {
      const uint64_t rk = mix(key ^ (uint64_t)b * 0xD6E8FEB86659FD93ull);
      double score = -1.1;
      for (int j = 0; j < num_dense; ++j) {
        const float x = (float)std::log1p(u01(mix(rk + j)) * 100.0);
        dense[(int64_t)b * num_dense + j] = x;
        score += (x - 3.6) * w_dense[j] * 2.0;
      }
      for (int t = 0; t < T; ++t) {
        const int L = pooling[t];
        const int64_t r = rows[t];
        for (int l = 0; l < L; ++l) {
          const uint64_t h = mix(rk ^ ((uint64_t)(t + 1) << 32) ^ (uint64_t)(l + 1000));
          int64_t id;
          if (dist == 1 && r > 1) {
            const double x = std::pow((std::pow((double)r, 1 - alpha) - 1) * u01(h) + 1,
                                      1 / (1 - alpha));
            id = std::min<int64_t>(std::max<int64_t>((int64_t)x - 1, 0), r - 1);
          } else {
            id = (int64_t)(h % (uint64_t)r);
          }
          ids[base[t] + (int64_t)b * L + l] = id;
          if (l == 0) score += table_bias[t * 64 + (id % 64)] * (3.0 / std::sqrt((double)T));
        }
      }
      const double p = 1.0 / (1.0 + std::exp(-score));
      label[b] = u01(mix(rk ^ 0xABCDEFull)) < p ? 1.f : 0.f;
    }
  };
  const int nt = std::max(1, std::min(nthreads, B / 256 + 1));
  if (nt == 1) {
    work(0, B);
    return;
  }
  std::vector<std::thread> th;
  const int per = (B + nt - 1) / nt;
  for (int i = 0; i < nt; ++i) {
    const int b0 = i * per, b1 = std::min(B, b0 + per);
    if (b0 < b1) th.emplace_back(work, b0, b1);
  }
  for (auto& x : th) x.join();
}

}  // extern "C"
