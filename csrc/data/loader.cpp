// Host batch loader: shuffled, rank-sharded batch collation from columnar
// host arrays into a ring of (pinned) output slots, filled by worker threads
// ahead of the consumer. Replaces the reference's tf.data / HF-datasets
// shuffle+batch+prefetch runtimes (tensorflow2/data.py:171-210,
// jax-flax/train.py:52-87, torchrec/data.py:13-59) for data that lives in
// host memory; Python only sees ready batches (then issues one async H2D).
//
// Semantics:
//  * per-epoch permutation: Fisher-Yates driven by splitmix64(seed, epoch),
//    identical on every rank (deterministic, unlike reference quirk Q4);
//  * global batch g covers permutation[g*B*W, (g+1)*B*W); rank r takes the
//    contiguous sub-range [r*B, (r+1)*B) (jax `shard` / split_dataset_by_node);
//  * drop_last drops the trailing partial global batch; otherwise the final
//    batch is split evenly-as-possible across ranks (may be short / empty).
// C ABI for ctypes.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Loader {
  int ncols;
  std::vector<const uint8_t*> cols;
  std::vector<int> esize;
  int64_t nrows, batch;
  uint64_t seed;
  int shuffle, drop_last, rank, world, nslots;
  std::vector<std::vector<uint8_t*>> slots;  // [slot][col]
  std::vector<int64_t> perm;
  // epoch state
  int64_t nbatches = 0;
  std::atomic<int64_t> next_job{0};
  std::vector<int64_t> slot_batch;   // batch index held by slot (-1 free)
  std::vector<int64_t> slot_rows;
  std::vector<int> slot_ready;
  int64_t handed = 0;                // next batch index to hand out
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> workers;
  bool stop = false;
  int epoch_gen = 0;

  void rows_of(int64_t g, int64_t& start, int64_t& n) const {
    const int64_t gb = batch * world;
    const int64_t g0 = g * gb;
    const int64_t avail = std::min(gb, nrows - g0);
    if (avail == gb) {
      start = g0 + (int64_t)rank * batch;
      n = batch;
    } else {  // last partial global batch: split evenly across ranks
      const int64_t per = avail / world, rem = avail % world;
      start = g0 + rank * per + std::min<int64_t>(rank, rem);
      n = per + (rank < rem ? 1 : 0);
    }
  }

  void fill(int slot, int64_t g) {
    int64_t start, n;
    rows_of(g, start, n);
    for (int c = 0; c < ncols; ++c) {
      const int es = esize[c];
      const uint8_t* src = cols[c];
      uint8_t* dst = slots[slot][c];
      if (!shuffle) {
        memcpy(dst, src + start * es, (size_t)n * es);
        continue;
      }
      const int64_t* p = perm.data() + start;
      switch (es) {
        case 1: for (int64_t i = 0; i < n; ++i) dst[i] = src[p[i]]; break;
        case 2: for (int64_t i = 0; i < n; ++i) ((uint16_t*)dst)[i] = ((const uint16_t*)src)[p[i]]; break;
        case 4: for (int64_t i = 0; i < n; ++i) ((uint32_t*)dst)[i] = ((const uint32_t*)src)[p[i]]; break;
        case 8: for (int64_t i = 0; i < n; ++i) ((uint64_t*)dst)[i] = ((const uint64_t*)src)[p[i]]; break;
        default: for (int64_t i = 0; i < n; ++i) memcpy(dst + i * es, src + p[i] * es, es);
      }
    }
    std::lock_guard<std::mutex> lk(mu);
    slot_rows[slot] = n;
    slot_ready[slot] = 1;
    cv.notify_all();
  }

  void worker_loop() {
    int gen_seen = -1;
    while (true) {
      int slot = -1;
      int64_t g = -1;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] {
          if (stop) return true;
          if (next_job.load() >= nbatches) return false;
          // batch j goes to slot j % nslots once batch j - nslots was released
          const int64_t j = next_job.load();
          return slot_batch[j % nslots] == -1;
        });
        if (stop) return;
        g = next_job.fetch_add(1);
        slot = (int)(g % nslots);
        slot_batch[slot] = g;
        slot_ready[slot] = 0;
        gen_seen = epoch_gen;
      }
      (void)gen_seen;
      fill(slot, g);
    }
  }

  void start_epoch(int64_t epoch) {
    std::unique_lock<std::mutex> lk(mu);
    // wait for in-flight fills of the previous epoch to finish
    cv.wait(lk, [&] {
      for (int s = 0; s < nslots; ++s)
        if (slot_batch[s] != -1 && !slot_ready[s]) return false;
      return true;
    });
    if (shuffle) {
      uint64_t st = seed * 0x100000001B3ull + (uint64_t)epoch;
      for (int64_t i = 0; i < nrows; ++i) perm[i] = i;
      for (int64_t i = nrows - 1; i > 0; --i) {
        const int64_t j = (int64_t)(splitmix(st) % (uint64_t)(i + 1));
        std::swap(perm[i], perm[j]);
      }
    }
    const int64_t gb = batch * world;
    nbatches = drop_last ? nrows / gb : (nrows + gb - 1) / gb;
    handed = 0;
    for (int s = 0; s < nslots; ++s) { slot_batch[s] = -1; slot_ready[s] = 0; }
    next_job.store(0);
    ++epoch_gen;
    cv.notify_all();
  }

  // returns slot index (>=0) and rows, or -1 at the end of the epoch
  int next(int64_t* rows) {
    std::unique_lock<std::mutex> lk(mu);
    if (handed >= nbatches) return -1;
    const int slot = (int)(handed % nslots);
    const int64_t want = handed;
    cv.wait(lk, [&] { return slot_batch[slot] == want && slot_ready[slot]; });
    *rows = slot_rows[slot];
    ++handed;
    return slot;
  }

  void release(int slot) {
    std::lock_guard<std::mutex> lk(mu);
    slot_batch[slot] = -1;
    slot_ready[slot] = 0;
    cv.notify_all();
  }
};

}  // namespace

extern "C" {

void* tdfo_loader_create(int ncols, const void** cols, const int* esize, int64_t nrows,
                         int64_t batch, uint64_t seed, int shuffle, int drop_last, int rank,
                         int world, int nthreads, int nslots, void** slot_ptrs) {
  if (ncols <= 0 || batch <= 0 || world <= 0 || rank < 0 || rank >= world || nslots <= 0)
    return nullptr;
  auto* L = new Loader();
  L->ncols = ncols;
  for (int c = 0; c < ncols; ++c) {
    L->cols.push_back((const uint8_t*)cols[c]);
    L->esize.push_back(esize[c]);
  }
  L->nrows = nrows;
  L->batch = batch;
  L->seed = seed;
  L->shuffle = shuffle;
  L->drop_last = drop_last;
  L->rank = rank;
  L->world = world;
  L->nslots = nslots;
  L->slots.assign(nslots, std::vector<uint8_t*>(ncols));
  for (int s = 0; s < nslots; ++s)
    for (int c = 0; c < ncols; ++c) L->slots[s][c] = (uint8_t*)slot_ptrs[s * ncols + c];
  L->perm.resize(shuffle ? nrows : 0);
  L->slot_batch.assign(nslots, -1);
  L->slot_rows.assign(nslots, 0);
  L->slot_ready.assign(nslots, 0);
  L->nbatches = 0;
  const int nt = std::max(1, std::min(nthreads, nslots));
  for (int i = 0; i < nt; ++i) L->workers.emplace_back([L] { L->worker_loop(); });
  return L;
}

int64_t tdfo_loader_start_epoch(void* h, int64_t epoch) {
  auto* L = (Loader*)h;
  L->start_epoch(epoch);
  return L->nbatches;
}

int tdfo_loader_next(void* h, int64_t* rows) { return ((Loader*)h)->next(rows); }

void tdfo_loader_release(void* h, int slot) { ((Loader*)h)->release(slot); }

void tdfo_loader_destroy(void* h) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
    L->cv.notify_all();
  }
  for (auto& t : L->workers) t.join();
  delete L;
}

}  // extern "C"
