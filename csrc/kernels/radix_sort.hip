// Deterministic LSD radix sort of (key, int32 value) pairs for gfx950.
//
// Used by the fused embedding backward to group duplicate row ids. Written
// in-house (instead of rocprim's onesweep, whose ordered-block-id path was
// observed to fault under hipGraph replay on gfx950) so the whole sort is a
// fixed, capture-safe sequence of 3 kernels per 8-bit digit:
//   hist    : one 1024-item tile per block, LDS digit histogram -> [tile][256]
//   scan    : 16 threads per digit scan digit d's column over tiles and emit
//             the digit totals (each scatter block scans those into bases)
//   scatter : per tile, 4 rounds of 256 items; the stable rank of an item
//             among equal digits is found with 8 wave ballots (lanes with the
//             same digit), per-wave digit counts in LDS and a running count
//             per digit, so the order of equal keys is the input order.
// Stable + fixed order => bitwise-reproducible downstream reductions.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 4;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;   // 1024 items per tile

template <typename K>
__global__ __launch_bounds__(256) void rs_hist_kernel(const K* __restrict__ keys, int64_t n,
                                                      int shift, int32_t* __restrict__ hist) {
  __shared__ int cnt[256];
  const int t = threadIdx.x;
  cnt[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t i = base + r * RS_THREADS + t;
    if (i < n) atomicAdd(&cnt[(int)((keys[i] >> shift) & 255)], 1);
  }
  __syncthreads();
  hist[(int64_t)blockIdx.x * 256 + t] = cnt[t];
}

// Column scan of the [tile][256] histogram: 4 blocks x 1024 threads; block b
// owns digits [64b, 64b+64), 16 threads per digit each scan a contiguous run
// of tiles, partial sums are combined in LDS, then every thread rewrites its
// run as exclusive prefixes. Digit totals go to `tot` (the scatter kernel
// turns them into digit bases).
__global__ __launch_bounds__(1024) void rs_scan_kernel(int32_t* __restrict__ hist, int ntiles,
                                                       int32_t* __restrict__ tot) {
  __shared__ int part[16][64];
  const int dl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int d = blockIdx.x * 64 + dl;
  const int per = (ntiles + 15) / 16;
  const int t0 = ph * per, t1 = min(ntiles, t0 + per);
  int s = 0;
  for (int t = t0; t < t1; ++t) s += hist[(int64_t)t * 256 + d];
  part[ph][dl] = s;
  __syncthreads();
  int run = 0;
  for (int q = 0; q < ph; ++q) run += part[q][dl];
  if (ph == 15) tot[d] = run + s;
  for (int t = t0; t < t1; ++t) {
    const int c = hist[(int64_t)t * 256 + d];
    hist[(int64_t)t * 256 + d] = run;
    run += c;
  }
}

template <typename K>
__global__ __launch_bounds__(256) void rs_scatter_kernel(const K* __restrict__ kin,
                                                         const int32_t* __restrict__ vin,
                                                         K* __restrict__ kout,
                                                         int32_t* __restrict__ vout, int64_t n,
                                                         int shift,
                                                         const int32_t* __restrict__ hist,
                                                         const int32_t* __restrict__ tot) {
  __shared__ int run[256];
  __shared__ int wcnt[4][256];
  __shared__ int start[256];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // digit bases: exclusive scan of the 256 digit totals (Hillis-Steele)
  const int mytot = tot[t];
  start[t] = mytot;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int v = t >= off ? start[t - off] : 0;
    __syncthreads();
    start[t] += v;
    __syncthreads();
  }
  start[t] = start[t] - mytot + hist[(int64_t)blockIdx.x * 256 + t];
  run[t] = 0;
  wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
  __syncthreads();
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tbase = (int64_t)blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t i = tbase + r * RS_THREADS + t;
    const bool valid = i < n;
    K k = 0;
    int32_t v = 0;
    int dg = 0;
    if (valid) {
      k = kin[i];
      v = vin[i];
      dg = (int)((k >> shift) & 255);
    }
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((dg >> b) & 1);
      m &= ((dg >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(m & lt_mask);
    if (valid && rank == 0) wcnt[w][dg] = __popcll(m);
    __syncthreads();
    if (valid) {
      int pos = start[dg] + run[dg] + rank;
      for (int q = 0; q < w; ++q) pos += wcnt[q][dg];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    run[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
    __syncthreads();
  }
}

template <typename K>
int sort_impl(K* ka, int32_t* va, K* kb, int32_t* vb, int64_t n, int key_bits, int32_t* hist,
              int32_t* base, hipStream_t s) {
  const int ntiles = (int)((n + RS_TILE - 1) / RS_TILE);
  const int passes = (key_bits + 7) / 8;
  K* kin = ka; int32_t* vin = va; K* kout = kb; int32_t* vout = vb;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    hipLaunchKernelGGL(rs_hist_kernel<K>, dim3(ntiles), dim3(256), 0, s, kin, n, shift, hist);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(4), dim3(1024), 0, s, hist, ntiles, base);
    hipLaunchKernelGGL(rs_scatter_kernel<K>, dim3(ntiles), dim3(256), 0, s, kin, vin, kout, vout,
                       n, shift, hist, base);
    TDFO_CHECK_HIP(hipGetLastError());
    K* tk = kin; kin = kout; kout = tk;
    int32_t* tv = vin; vin = vout; vout = tv;
  }
  return passes & 1;   // 1: result in (kb, vb)
}

}  // namespace

size_t radix_sort_workspace(int64_t n) {
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  return (size_t)(ntiles * 256 + 256) * sizeof(int32_t);
}

int radix_sort_pairs_u32(uint32_t* ka, int32_t* va, uint32_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  int32_t* hist = (int32_t*)ws;
  return sort_impl<uint32_t>(ka, va, kb, vb, n, key_bits, hist, hist + ntiles * 256, s);
}

int radix_sort_pairs_u64(uint64_t* ka, int32_t* va, uint64_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  int32_t* hist = (int32_t*)ws;
  return sort_impl<uint64_t>(ka, va, kb, vb, n, key_bits, hist, hist + ntiles * 256, s);
}

}  // namespace tdfo
