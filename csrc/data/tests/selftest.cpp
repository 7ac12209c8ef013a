// Host self-test of the C++ data library (loader threads, TFRecord codec,
// synthetic Criteo generator), built and run under AddressSanitizer +
// UndefinedBehaviorSanitizer and, separately, ThreadSanitizer by
// tests/test_host_sanitizers.py (host code only; GPU
// sanitizers are not available on this pool). Exit code 0 = all checks pass.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
void* tdfo_loader_create(int ncols, const void** cols, const int* esize, int64_t nrows,
                         int64_t batch, uint64_t seed, int shuffle, int drop_last, int rank,
                         int world, int nthreads, int nslots, void** slot_ptrs);
int64_t tdfo_loader_start_epoch(void* h, int64_t epoch);
int tdfo_loader_next(void* h, int64_t* rows);
void tdfo_loader_release(void* h, int slot);
void tdfo_loader_destroy(void* h);
int tdfo_tfrecord_write(const char* path, int gz, int ncols, const char** names, const int* types,
                        const void** cols, int64_t nrows);
int64_t tdfo_tfrecord_count(const char* path, int gz, int check_crc);
int64_t tdfo_tfrecord_read(const char* path, int gz, int ncols, const char** names,
                           const int* types, void** outs, int64_t max_rows, int check_crc);
void tdfo_synth_criteo(uint64_t seed, int rank, int64_t batch_index, int B, int num_dense, int T,
                       const int64_t* rows, const int* pooling, int dist, double alpha,
                       const float* w_dense, const float* table_bias, float* dense, int64_t* ids,
                       float* label, int nthreads);
}

#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

static int test_loader(int world, int shuffle) {
  const int64_t N = 10007, B = 64;
  std::vector<int64_t> a(N);
  std::vector<float> f(N);
  for (int64_t i = 0; i < N; ++i) { a[i] = i; f[i] = 0.5f * (float)i; }
  const void* cols[2] = {a.data(), f.data()};
  const int esize[2] = {8, 4};
  std::vector<int64_t> seen(N, 0);
  for (int rank = 0; rank < world; ++rank) {
    const int nslots = 3;
    std::vector<std::vector<uint8_t>> bufs(nslots * 2);
    std::vector<void*> ptrs(nslots * 2);
    for (int s = 0; s < nslots; ++s) {
      bufs[s * 2].resize(B * 8);
      bufs[s * 2 + 1].resize(B * 4);
      ptrs[s * 2] = bufs[s * 2].data();
      ptrs[s * 2 + 1] = bufs[s * 2 + 1].data();
    }
    void* h = tdfo_loader_create(2, cols, esize, N, B, 42, shuffle, 0, rank, world, 4, nslots,
                                 ptrs.data());
    CHECK(h != nullptr);
    for (int epoch = 0; epoch < 2; ++epoch) {
      const int64_t nb = tdfo_loader_start_epoch(h, epoch);
      CHECK(nb > 0);
      int64_t rows = 0;
      int slot;
      int64_t got = 0;
      while ((slot = tdfo_loader_next(h, &rows)) >= 0) {
        const int64_t* ia = (const int64_t*)ptrs[slot * 2];
        const float* fa = (const float*)ptrs[slot * 2 + 1];
        for (int64_t r = 0; r < rows; ++r) {
          CHECK(ia[r] >= 0 && ia[r] < N);
          CHECK(fa[r] == 0.5f * (float)ia[r]);
          if (epoch == 0) seen[ia[r]] += 1;
        }
        got += rows;
        tdfo_loader_release(h, slot);
      }
      CHECK(got > 0);
    }
    tdfo_loader_destroy(h);
  }
  for (int64_t i = 0; i < N; ++i) CHECK(seen[i] == 1);   // every row exactly once per epoch
  return 0;
}

static int test_tfrecord(const char* dir) {
  const int64_t N = 257;
  std::vector<int64_t> a(N);
  std::vector<float> f(N);
  for (int64_t i = 0; i < N; ++i) { a[i] = i * 7 - 100; f[i] = 0.25f * (float)i; }
  const char* names[2] = {"user_id", "avg_rating"};
  const int types[2] = {0, 1};
  const void* cols[2] = {a.data(), f.data()};
  for (int gz = 0; gz < 2; ++gz) {
    const std::string path = std::string(dir) + (gz ? "/t.tfrecord.gz" : "/t.tfrecord");
    CHECK(tdfo_tfrecord_write(path.c_str(), gz, 2, names, types, cols, N) == 0);
    CHECK(tdfo_tfrecord_count(path.c_str(), gz, 1) == N);
    std::vector<int64_t> ra(N);
    std::vector<float> rf(N);
    void* outs[2] = {ra.data(), rf.data()};
    CHECK(tdfo_tfrecord_read(path.c_str(), gz, 2, names, types, outs, N, 1) == N);
    CHECK(std::memcmp(ra.data(), a.data(), N * 8) == 0);
    CHECK(std::memcmp(rf.data(), f.data(), N * 4) == 0);
  }
  return 0;
}

static int test_synthetic() {
  const int B = 128, T = 4, ND = 13;
  const int64_t rows[T] = {10, 1000, 3, 100000};
  const int pooling[T] = {1, 3, 1, 2};
  int nnz = 0;
  for (int t = 0; t < T; ++t) nnz += B * pooling[t];
  std::vector<float> w(ND, 0.1f), tb(T * 64, 0.05f), dense(B * ND), label(B), dense2(B * ND),
      label2(B);   // table_bias is [T, 64]
  std::vector<int64_t> ids(nnz), ids2(nnz);
  for (int dist = 0; dist < 2; ++dist) {
    tdfo_synth_criteo(9, 1, 5, B, ND, T, rows, pooling, dist, 1.1, w.data(), tb.data(),
                      dense.data(), ids.data(), label.data(), 4);
    tdfo_synth_criteo(9, 1, 5, B, ND, T, rows, pooling, dist, 1.1, w.data(), tb.data(),
                      dense2.data(), ids2.data(), label2.data(), 1);
    CHECK(ids == ids2 && dense == dense2 && label == label2);   // thread-count independent
    int64_t p = 0;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < B * pooling[t]; ++i, ++p) CHECK(ids[p] >= 0 && ids[p] < rows[t]);
  }
  return 0;
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  if (test_loader(1, 1) || test_loader(3, 1) || test_loader(2, 0)) return 1;
  if (test_tfrecord(dir)) return 1;
  if (test_synthetic()) return 1;
  std::printf("selftest ok\n");
  return 0;
}
