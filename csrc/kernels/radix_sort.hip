// Deterministic LSD radix sort of (key, int32 value) pairs for gfx950.
//
// Used by the fused embedding backward to group duplicate row ids. Written
// in-house (rocprim's onesweep, with its ordered-block-id counter, was
// observed to fault under hipGraph replay on gfx950) as a fixed,
// capture-safe kernel sequence. At DLRM sizes (~2e5 keys) launches dominate,
// so passes use up to 10-bit digits (28-bit keys: 10/9/9 = 3 passes) and the
// per-pass histogram is produced by the previous pass's scatter:
//   hist    : pass-0 digit histogram per 1024-item tile ([tile][bins])
//   scan    : column scan -> per-tile exclusive prefixes + digit totals
//   scatter : per tile, digit bases = scan(totals) + tile prefix; stable ranks
//             from one wave ballot per digit bit and per-wave digit counts in
//             LDS; scatter; and count the NEXT pass's digits of the written
//             items into the next histogram (int atomics: order-independent)
// Three histogram buffers rotate: pass p reads H[p%3], counts into H[(p+1)%3]
// (zeroed by pass p-1 or the hist kernel) and zeroes H[(p+2)%3].
// Stable + fixed order => bitwise-reproducible downstream reductions.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 4;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;   // 1024 items per tile
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_MAXB = 10;                       // digit bits per pass (<= 1024 bins)
constexpr int RS_MAXBINS = 1 << RS_MAXB;

template <typename K>
__global__ __launch_bounds__(256) void rs_hist_kernel(const K* __restrict__ keys, int64_t n,
                                                      int shift, int bits,
                                                      int32_t* __restrict__ hist,
                                                      int32_t* __restrict__ hzero) {
  __shared__ int cnt[RS_MAXBINS];
  const int t = threadIdx.x, nb = 1 << bits;
  for (int d = t; d < RS_MAXBINS; d += RS_THREADS) hzero[(int64_t)blockIdx.x * RS_MAXBINS + d] = 0;
  for (int d = t; d < nb; d += RS_THREADS) cnt[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t i = base + r * RS_THREADS + t;
    if (i < n) atomicAdd(&cnt[(int)((keys[i] >> shift) & (nb - 1))], 1);
  }
  __syncthreads();
  for (int d = t; d < nb; d += RS_THREADS) hist[(int64_t)blockIdx.x * nb + d] = cnt[d];
}

// Column scan of the [tile][nb] histogram: 1024-thread blocks, 16 digits per
// block, 64 threads per digit each own a contiguous run of tiles. Each thread
// loads its whole run (up to 32 tiles, i.e. inputs up to 2M keys) into
// registers with no dependency between the loads, so the scan costs ~two
// memory latencies instead of one per tile. Rewrites hist[tile][d] as the
// exclusive prefix over tiles; digit totals -> tot. Longer runs loop.
constexpr int SCAN_DPB = 16, SCAN_PH = 1024 / SCAN_DPB, SCAN_RUN = 32;

__global__ __launch_bounds__(1024) void rs_scan_kernel(int32_t* __restrict__ hist, int ntiles,
                                                       int nb, int32_t* __restrict__ tot) {
  __shared__ int part[SCAN_PH][SCAN_DPB];
  const int dl = threadIdx.x % SCAN_DPB, ph = threadIdx.x / SCAN_DPB;
  const int d = blockIdx.x * SCAN_DPB + dl;
  const int per = (ntiles + SCAN_PH - 1) / SCAN_PH;
  const int t0 = ph * per, t1 = d < nb ? min(ntiles, t0 + per) : t0;   // d >= nb: idle
  int s = 0;
  if (per <= SCAN_RUN) {
    // every load issued unconditionally at a clamped address and masked
    // after it lands: a "t0 + q < t1 ? load : 0" select makes hipcc branch
    // around each load and wait for it (one dependent round trip per tile:
    // 30-53 us per pass at 1712 tiles, profiles/dcnv2_1tb_b8192_timeline.txt)
    const int dc = d < nb ? d : nb - 1;
    const int tl = ntiles - 1;
    int c[SCAN_RUN];
#pragma unroll
    for (int q = 0; q < SCAN_RUN; ++q) c[q] = hist[(int64_t)min(t0 + q, tl) * nb + dc];
#pragma unroll
    for (int q = 0; q < SCAN_RUN; ++q) c[q] = (t0 + q < t1) ? c[q] : 0;
#pragma unroll
    for (int q = 0; q < SCAN_RUN; ++q) s += c[q];
    part[ph][dl] = s;
    __syncthreads();
    int run = 0;
    for (int q = 0; q < ph; ++q) run += part[q][dl];
    if (ph == SCAN_PH - 1 && d < nb) tot[d] = run + s;
#pragma unroll
    for (int q = 0; q < SCAN_RUN; ++q) {
      if (t0 + q < t1) hist[(int64_t)(t0 + q) * nb + d] = run;
      run += c[q];
    }
    return;
  }
  for (int t = t0; t < t1; ++t) s += hist[(int64_t)t * nb + d];
  part[ph][dl] = s;
  __syncthreads();
  int run = 0;
  for (int q = 0; q < ph; ++q) run += part[q][dl];
  if (ph == SCAN_PH - 1 && d < nb) tot[d] = run + s;
  for (int t = t0; t < t1; ++t) {
    const int c = hist[(int64_t)t * nb + d];
    hist[(int64_t)t * nb + d] = run;
    run += c;
  }
}

// Per tile: digit bases (exclusive scan of the digit totals + this tile's
// prefix), stable ranks from wave ballots (one per digit bit) and per-wave
// digit counts, scatter; and the next pass's digit counts into hnext.
template <typename K>
__global__ __launch_bounds__(256) void rs_scatter_kernel(
    const K* __restrict__ kin, const int32_t* __restrict__ vin, K* __restrict__ kout,
    int32_t* __restrict__ vout, int64_t n, int shift, int bits, int next_shift, int next_bits,
    const int32_t* __restrict__ hist, const int32_t* __restrict__ tot,
    int32_t* __restrict__ hnext, int32_t* __restrict__ hzero) {
  __shared__ int start[RS_MAXBINS];
  __shared__ int run[RS_MAXBINS];
  __shared__ int wcnt[RS_WAVES][RS_MAXBINS];
  __shared__ int wsum[RS_WAVES];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nb = 1 << bits, per_t = nb / RS_THREADS > 0 ? nb / RS_THREADS : 1;
  const int tile = blockIdx.x;
  const int nnb = next_shift >= 0 ? 1 << next_bits : 0;
  for (int d = t; d < RS_MAXBINS; d += RS_THREADS) hzero[(int64_t)tile * RS_MAXBINS + d] = 0;
  // exclusive scan of the digit totals: thread t owns digits [t*per_t, +per_t)
  int loc[RS_MAXBINS / RS_THREADS];
  int mysum = 0;
#pragma unroll
  for (int j = 0; j < RS_MAXBINS / RS_THREADS; ++j) {
    const int d = t * per_t + j;
    loc[j] = (j < per_t && d < nb) ? tot[d] : 0;
    mysum += loc[j];
  }
  int x = mysum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  for (int q = t; q < RS_WAVES * RS_MAXBINS; q += RS_THREADS) (&wcnt[0][0])[q] = 0;
  __syncthreads();
  int acc = x - mysum;
  for (int q = 0; q < w; ++q) acc += wsum[q];
#pragma unroll
  for (int j = 0; j < RS_MAXBINS / RS_THREADS; ++j) {
    const int d = t * per_t + j;
    if (j < per_t && d < nb) {
      start[d] = acc + hist[(int64_t)tile * nb + d];
      run[d] = 0;
      acc += loc[j];
    }
  }
  __syncthreads();
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tbase = (int64_t)tile * RS_TILE;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t i = tbase + r * RS_THREADS + t;
    const bool valid = i < n;
    K k = 0;
    int32_t v = 0;
    int dg = 0;
    if (valid) {
      k = kin[i];
      v = vin[i];
      dg = (int)((k >> shift) & (nb - 1));
    }
    uint64_t m = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      const uint64_t bb = __ballot((dg >> b) & 1);
      m &= ((dg >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(m & lt_mask);
    if (valid && rank == 0) wcnt[w][dg] = __popcll(m);
    __syncthreads();
    if (valid) {
      int64_t pos = start[dg] + run[dg] + rank;
      for (int q = 0; q < w; ++q) pos += wcnt[q][dg];
      kout[pos] = k;
      vout[pos] = v;
      if (nnb) atomicAdd(&hnext[(pos / RS_TILE) * nnb + (int)((k >> next_shift) & (nnb - 1))], 1);
    }
    __syncthreads();
    for (int d = t; d < nb; d += RS_THREADS) {
      int c = 0;
#pragma unroll
      for (int q = 0; q < RS_WAVES; ++q) { c += wcnt[q][d]; wcnt[q][d] = 0; }
      run[d] += c;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Tiled passes for large inputs (multi-hot DCN-v2: 1.75M keys). The
// 1024-item tiles above have ~1 item per 10-bit digit, so every scatter
// store is an isolated 4-B write (65 us per pass at 1.75M keys). Here a
// 512-thread block owns 4096 items and <= 8-bit digits (28-bit keys: 4
// passes of 7 bits, ~32 items per digit per tile): it ranks its items
// (stable: wave ballots per round + per-wave digit counters), sorts the
// tile by digit in LDS and writes each digit's run contiguously (128-B
// store runs). Per pass: hist (per-tile digit counts, LDS atomics), the
// column scan above, scatter.
constexpr int TS_THREADS = 512, TS_WAVES = 8, TS_ROUNDS = 8;
constexpr int TS_TILE = TS_THREADS * TS_ROUNDS;   // 4096 items
constexpr int TS_MAXB = 8, TS_MAXBINS = 1 << TS_MAXB;

template <typename K>
__global__ __launch_bounds__(512) void ts_hist_kernel(const K* __restrict__ keys, int64_t n,
                                                      int shift, int bits,
                                                      int32_t* __restrict__ hist) {
  __shared__ int cnt[TS_WAVES][TS_MAXBINS];
  const int t = threadIdx.x, w = t >> 6, nb = 1 << bits;
  for (int q = t; q < TS_WAVES * TS_MAXBINS; q += TS_THREADS) (&cnt[0][0])[q] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TS_TILE;
  K k[TS_ROUNDS];
#pragma unroll
  for (int r = 0; r < TS_ROUNDS; ++r) {
    const int64_t i = base + r * TS_THREADS + t;
    k[r] = keys[i < n ? i : n - 1];
  }
#pragma unroll
  for (int r = 0; r < TS_ROUNDS; ++r)
    if (base + r * TS_THREADS + t < n) atomicAdd(&cnt[w][(int)((k[r] >> shift) & (nb - 1))], 1);
  __syncthreads();
  for (int d = t; d < nb; d += TS_THREADS) {
    int c = 0;
#pragma unroll
    for (int q = 0; q < TS_WAVES; ++q) c += cnt[q][d];
    hist[(int64_t)blockIdx.x * nb + d] = c;
  }
}

// Exclusive block scan of one int per thread (TS_THREADS); returns the
// prefix, total in *total (LDS scratch ws[TS_WAVES]).
__device__ __forceinline__ int ts_block_scan(int x, int* ws, int* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int y = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(y, o, 64);
    if (lane >= o) y += u;
  }
  if (lane == 63) ws[w] = y;
  __syncthreads();
  int pre = y - x;
  int tot = 0;
#pragma unroll
  for (int q = 0; q < TS_WAVES; ++q) {
    if (q < w) pre += ws[q];
    tot += ws[q];
  }
  *total = tot;
  return pre;
}

// Column scan for the tiled passes: one 512-thread block per digit (<= 256
// digits -> <= 256 blocks), the digit's per-tile counts in registers (<= 8
// consecutive tiles per thread, loads unconditional at clamped addresses),
// one block-wide scan; rewrites hist[tile][d] as the exclusive prefix over
// tiles and writes the digit total. Replaces rs_scan_kernel there: its 8
// blocks walked 64-deep LDS prefix chains, 17.5 us per pass at 428 tiles
// (DCN-v2 multi-hot, profiles/r04/prof_dcn/summary.txt).
constexpr int SC2_R = 8;

__global__ __launch_bounds__(512) void ts_scan_col_kernel(int32_t* __restrict__ hist, int ntiles,
                                                          int nb, int32_t* __restrict__ tot) {
  __shared__ int ws[TS_WAVES];
  const int d = blockIdx.x, t = threadIdx.x;
  const int per = (ntiles + TS_THREADS - 1) / TS_THREADS;       // <= SC2_R (caller checks)
  const int t0 = t * per, tl = ntiles - 1;
  int c[SC2_R];
#pragma unroll
  for (int q = 0; q < SC2_R; ++q) c[q] = hist[(int64_t)min(t0 + q, tl) * nb + d];
#pragma unroll
  for (int q = 0; q < SC2_R; ++q) c[q] = (q < per && t0 + q < ntiles) ? c[q] : 0;
  int sum = 0;
#pragma unroll
  for (int q = 0; q < SC2_R; ++q) sum += c[q];
  int total;
  int run = ts_block_scan(sum, ws, &total);
  if (t == 0) tot[d] = total;
#pragma unroll
  for (int q = 0; q < SC2_R; ++q) {
    if (q < per && t0 + q < ntiles) hist[(int64_t)(t0 + q) * nb + d] = run;
    run += c[q];
  }
}

template <typename K>
__global__ __launch_bounds__(512) void ts_scatter_kernel(
    const K* __restrict__ kin, const int32_t* __restrict__ vin, K* __restrict__ kout,
    int32_t* __restrict__ vout, int64_t n, int shift, int bits,
    const int32_t* __restrict__ hist, const int32_t* __restrict__ tot) {
  __shared__ K sk[TS_TILE];
  __shared__ int32_t sv[TS_TILE];
  __shared__ int wcnt[TS_WAVES][TS_MAXBINS];   // per-wave counts -> per-wave prefixes
  __shared__ int dstart[TS_MAXBINS];           // tile-local digit start
  __shared__ int gofs[TS_MAXBINS];             // global position - local position, per digit
  __shared__ int scr[2][TS_WAVES];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nb = 1 << bits;
  const int64_t base = (int64_t)blockIdx.x * TS_TILE;
  const int cnt_tile = (int)min((int64_t)TS_TILE, n - base);
  for (int q = t; q < TS_WAVES * TS_MAXBINS; q += TS_THREADS) (&wcnt[0][0])[q] = 0;
  // wave w owns items [w*512, +512) of the tile; round r, lane l: item
  // w*512 + r*64 + l (round-major = position order: stable ranks)
  K k[TS_ROUNDS];
  int32_t v[TS_ROUNDS];
  int rk[TS_ROUNDS];
#pragma unroll
  for (int r = 0; r < TS_ROUNDS; ++r) {
    const int li = w * (TS_TILE / TS_WAVES) + r * 64 + lane;
    const int64_t i = base + (li < cnt_tile ? li : cnt_tile - 1);
    k[r] = kin[i];
    v[r] = vin[i];
  }
  __syncthreads();
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int r = 0; r < TS_ROUNDS; ++r) {
    const int li = w * (TS_TILE / TS_WAVES) + r * 64 + lane;
    const bool valid = li < cnt_tile;
    const int dg = (int)((k[r] >> shift) & (nb - 1));
    uint64_t m = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      const uint64_t bb = __ballot((dg >> b) & 1);
      m &= ((dg >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(m & lt_mask);
    const int c = wcnt[w][dg];                 // read by the whole wave, then the
    rk[r] = c + rank;                          // run's first lane advances it (LDS
    if (valid && rank == 0) wcnt[w][dg] = c + __popcll(m);   // ops of a wave stay in order)
  }
  __syncthreads();
  // per digit: per-wave exclusive prefixes, tile count; scans over digits of
  // the tile counts (local starts) and of the global totals (global starts)
  int dcount = 0, gtot = 0;
  if (t < nb) {
#pragma unroll
    for (int q = 0; q < TS_WAVES; ++q) {
      const int c = wcnt[q][t];
      wcnt[q][t] = dcount;
      dcount += c;
    }
    gtot = tot[t];
  }
  int tsum, gsum;
  const int lstart = ts_block_scan(dcount, scr[0], &tsum);
  const int gstart = ts_block_scan(gtot, scr[1], &gsum);
  if (t < nb) {
    dstart[t] = lstart;
    gofs[t] = gstart + hist[(int64_t)blockIdx.x * nb + t] - lstart;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < TS_ROUNDS; ++r) {
    const int li = w * (TS_TILE / TS_WAVES) + r * 64 + lane;
    if (li < cnt_tile) {
      const int dg = (int)((k[r] >> shift) & (nb - 1));
      const int lp = dstart[dg] + wcnt[w][dg] + rk[r];
      sk[lp] = k[r];
      sv[lp] = v[r];
    }
  }
  __syncthreads();
  for (int i = t; i < cnt_tile; i += TS_THREADS) {
    const K key = sk[i];
    const int64_t g = (int64_t)gofs[(int)((key >> shift) & (nb - 1))] + i;
    kout[g] = key;
    vout[g] = sv[i];
  }
}

// 0: 1024-item tiles, 10-bit digits; 1: 4096-item tiles from TS_MIN_N keys
// up; 2: always 4096-item tiles
int g_tiled = 1;
constexpr int64_t TS_MIN_N = 1 << 19;

bool use_tiled(int64_t n) { return g_tiled == 2 || (g_tiled == 1 && n >= TS_MIN_N); }

template <typename K>
int tiled_sort_impl(K* ka, int32_t* va, K* kb, int32_t* vb, int64_t n, int key_bits,
                    int32_t* ws, hipStream_t s) {
  const int ntiles = (int)((n + TS_TILE - 1) / TS_TILE);
  const int kbits = key_bits < 1 ? 1 : key_bits;
  const int passes = (kbits + TS_MAXB - 1) / TS_MAXB;
  int32_t* hist = ws;
  int32_t* tot = ws + (int64_t)ntiles * TS_MAXBINS;
  K* kin = ka; int32_t* vin = va; K* kout = kb; int32_t* vout = vb;
  for (int p = 0, sh = 0; p < passes; ++p) {     // e.g. 28 bits -> 7, 7, 7, 7
    const int bits = (kbits - sh + (passes - p) - 1) / (passes - p);
    const int nb = 1 << bits;
    hipLaunchKernelGGL(ts_hist_kernel<K>, dim3(ntiles), dim3(TS_THREADS), 0, s, kin, n, sh, bits,
                       hist);
    if (ntiles <= TS_THREADS * SC2_R)
      hipLaunchKernelGGL(ts_scan_col_kernel, dim3(nb), dim3(TS_THREADS), 0, s, hist, ntiles, nb,
                         tot);
    else
      hipLaunchKernelGGL(rs_scan_kernel, dim3((nb + SCAN_DPB - 1) / SCAN_DPB), dim3(1024), 0, s,
                         hist, ntiles, nb, tot);
    hipLaunchKernelGGL(ts_scatter_kernel<K>, dim3(ntiles), dim3(TS_THREADS), 0, s, kin, vin, kout,
                       vout, n, sh, bits, hist, tot);
    TDFO_CHECK_HIP(hipGetLastError());
    sh += bits;
    K* tk = kin; kin = kout; kout = tk;
    int32_t* tv = vin; vin = vout; vout = tv;
  }
  return passes & 1;
}

int g_max_bits = 10;  // digit bits per pass (<= RS_MAXB): 28-bit keys -> 10/9/9 (fastest measured)

// 1: each pass's histogram from its own coalesced hist kernel; 0: counted by
// the previous pass's scatter with global atomics (scattered addresses:
// slow at large n, see profiles/sort_digit_ab.jsonl)
int g_sep_hist = 1;

template <typename K>
int sort_impl(K* ka, int32_t* va, K* kb, int32_t* vb, int64_t n, int key_bits, int32_t* ws,
              hipStream_t s) {
  const int ntiles = (int)((n + RS_TILE - 1) / RS_TILE);
  const int kbits = key_bits < 1 ? 1 : key_bits;
  const int passes = (kbits + g_max_bits - 1) / g_max_bits;
  int pbits[8], pshift[8];
  for (int p = 0, sh = 0; p < passes; ++p) {   // e.g. 28 bits -> 10, 9, 9
    pbits[p] = (kbits - sh + (passes - p) - 1) / (passes - p);
    pshift[p] = sh;
    sh += pbits[p];
  }
  const int64_t hsz = (int64_t)ntiles * RS_MAXBINS;
  int32_t* H[3] = {ws, ws + hsz, ws + 2 * hsz};
  int32_t* tot = ws + 3 * hsz;
  hipLaunchKernelGGL(rs_hist_kernel<K>, dim3(ntiles), dim3(RS_THREADS), 0, s, ka, n, pshift[0],
                     pbits[0], H[0], H[1]);
  TDFO_CHECK_HIP(hipGetLastError());
  K* kin = ka; int32_t* vin = va; K* kout = kb; int32_t* vout = vb;
  for (int p = 0; p < passes; ++p) {
    const int nb = 1 << pbits[p];
    if (g_sep_hist && p > 0) {
      hipLaunchKernelGGL(rs_hist_kernel<K>, dim3(ntiles), dim3(RS_THREADS), 0, s, kin, n,
                         pshift[p], pbits[p], H[p % 3], H[(p + 1) % 3]);
    }
    hipLaunchKernelGGL(rs_scan_kernel, dim3((nb + SCAN_DPB - 1) / SCAN_DPB), dim3(1024), 0, s,
                       H[p % 3], ntiles, nb, tot);
    const bool last = p + 1 == passes || g_sep_hist;   // sep: next hist by its own kernel
    hipLaunchKernelGGL(rs_scatter_kernel<K>, dim3(ntiles), dim3(RS_THREADS), 0, s, kin, vin,
                       kout, vout, n, pshift[p], pbits[p], last ? -1 : pshift[p + 1],
                       last ? 0 : pbits[p + 1], H[p % 3], tot, H[(p + 1) % 3], H[(p + 2) % 3]);
    TDFO_CHECK_HIP(hipGetLastError());
    K* tk = kin; kin = kout; kout = tk;
    int32_t* tv = vin; vin = vout; vout = tv;
  }
  return passes & 1;   // 1: result in (kb, vb)
}

}  // namespace

int radix_sort_passes(int key_bits, int64_t n) {
  const int kbits = key_bits < 1 ? 1 : key_bits;
  if (use_tiled(n)) return (kbits + TS_MAXB - 1) / TS_MAXB;
  return (kbits + g_max_bits - 1) / g_max_bits;
}

int radix_sort_tiled(int v) {
  const int old = g_tiled;
  if (v >= 0 && v <= 2) g_tiled = v;
  return old;
}

int radix_sort_sep_hist(int v) {
  const int old = g_sep_hist;
  if (v >= 0) g_sep_hist = v ? 1 : 0;
  return old;
}

int radix_sort_max_bits(int b) {
  const int old = g_max_bits;
  if (b >= 4 && b <= RS_MAXB) g_max_bits = b;
  return old;
}

size_t radix_sort_workspace(int64_t n) {
  // sized for either variant (the 1024-item tiles' three histograms are larger)
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  return (size_t)(3 * ntiles * RS_MAXBINS + RS_MAXBINS) * sizeof(int32_t);
}

int radix_sort_pairs_u32(uint32_t* ka, int32_t* va, uint32_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s) {
  if (n <= 0) return 0;
  if (use_tiled(n)) return tiled_sort_impl<uint32_t>(ka, va, kb, vb, n, key_bits, (int32_t*)ws, s);
  return sort_impl<uint32_t>(ka, va, kb, vb, n, key_bits, (int32_t*)ws, s);
}

int radix_sort_pairs_u64(uint64_t* ka, int32_t* va, uint64_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s) {
  if (n <= 0) return 0;
  if (use_tiled(n)) return tiled_sort_impl<uint64_t>(ka, va, kb, vb, n, key_bits, (int32_t*)ws, s);
  return sort_impl<uint64_t>(ka, va, kb, vb, n, key_bits, (int32_t*)ws, s);
}

}  // namespace tdfo
