// Table-batched EmbeddingBag forward and fused backward+optimizer
// (N1/N2/K23/K27 in SURVEY.md; plays the role of fbgemm_gpu's TBE in the
// reference's torchrec/train.py:236-247, re-designed for CDNA4).
//
// Forward: every bag is served by D/4 lanes with 16-B (float4) row loads, so a
// wave gathers 64*16 B per instruction; D=128 puts two bags in one wave. Four
// rows per lane are kept in flight for multi-hot bags. The pooled row is
// written (bf16 or fp32) straight into the consumer's layout
// (out + b*out_stride + out_off[t]), e.g. the interaction input or the
// all-to-all send buffer, so no concat/permute pass follows.
//
// Backward + optimizer, with no float atomics (atomics run at ~1.3 TB/s on
// MI355X and are order-dependent) and load-balanced under skew
// (cdna_hip_programming.md Appendix B "Scatter / gather / embedding"):
//   keys   : key = row_offset[t] + id, val = position, bag_of[position]
//   sort   : in-house stable LSD radix sort (radix_sort.hip) on the key bits
//            actually used (32-bit keys whenever the shard has < 2^32 rows)
//   chunks : each wave reduces a fixed 32-entry chunk of the sorted list; runs
//            fully inside the chunk are finished (optimizer applied) in place,
//            runs crossing a chunk edge leave fp32 partials (head/tail slabs)
//   combine: the chunk where a crossing run starts adds the following chunks'
//            head partials in order and applies the optimizer once.
// Every unique row is updated exactly once per step, in a fixed order.
#include <cstdlib>
#include <type_traits>

#include "tdfo_common.h"
#include "tdfo_kernels.h"
#include "tdfo_reduce_adam.h"
#include "tdfo_two_tower_dev.h"

namespace tdfo {
namespace {

// ----------------------------------------------------------- forward ----
// One id per bag (offsets[j] == j): no offsets loads, and every lane group
// keeps two bags' row gathers in flight (index load -> row load is the whole
// dependency chain).
__device__ __forceinline__ void fwd_bumps(const EmbFwdArgs& a) {
  if (blockIdx.x == 0 && (int)threadIdx.x < a.bumps.n) {
    const int i = threadIdx.x;
    if (a.bumps.is_i64[i]) *(int64_t*)a.bumps.p[i] += 1;
    else                   *(float*)a.bumps.p[i] += 1.f;
  }
}

template <int D, bool OUT_BF16>
__global__ __launch_bounds__(256) void emb_fwd_onehot_kernel(EmbFwdArgs a) {
  fwd_bumps(a);
  constexpr int LPB = (D / 4) < 64 ? (D / 4) : 64;  // lanes per bag
  constexpr int BPW = 64 / LPB;                     // bags per wave
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPB, sl = lane - sub * LPB;
  const int64_t nbags = (int64_t)a.T * a.B;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t step = ((int64_t)gridDim.x * blockDim.x >> 6) * BPW;
  for (int64_t j0 = wave0 * BPW + sub; j0 < nbags; j0 += 2 * step) {
    const int64_t j1 = j0 + step;
    const bool has1 = j1 < nbags;
    const int t0 = (int)(j0 / a.B), t1 = has1 ? (int)(j1 / a.B) : t0;
    const int64_t id0 = a.indices[j0], id1 = has1 ? a.indices[j1] : id0;
    const float* r0 = a.W + (a.row_offset[t0] + id0) * D;
    const float* r1 = a.W + (a.row_offset[t1] + id1) * D;
    for (int c = sl * 4; c < D; c += LPB * 4) {
      const float4 v0 = *(const float4*)(r0 + c);
      const float4 v1 = *(const float4*)(r1 + c);
      const float w0 = a.psw ? a.psw[j0] : 1.f, w1 = a.psw ? a.psw[j1 < nbags ? j1 : j0] : 1.f;
      const float4 o0 = make_float4(v0.x * w0, v0.y * w0, v0.z * w0, v0.w * w0);
      const float4 o1 = make_float4(v1.x * w1, v1.y * w1, v1.z * w1, v1.w * w1);
      const int64_t b0 = j0 - (int64_t)t0 * a.B, b1 = j1 - (int64_t)t1 * a.B;
      const int64_t p0 = b0 * a.out_stride + a.out_off[t0] + c;
      const int64_t p1 = b1 * a.out_stride + a.out_off[t1] + c;
      if (OUT_BF16) {
        *(uint2*)((uint16_t*)a.out + p0) = make_uint2(pack2bf(o0.x, o0.y), pack2bf(o0.z, o0.w));
        if (has1)
          *(uint2*)((uint16_t*)a.out + p1) = make_uint2(pack2bf(o1.x, o1.y), pack2bf(o1.z, o1.w));
      } else {
        *(float4*)((float*)a.out + p0) = o0;
        if (has1) *(float4*)((float*)a.out + p1) = o1;
      }
    }
  }
}

// Multi-hot bags, LDS-staged index gather. A lane group of LPB lanes pools
// one bag (BPW bags per wave). The bag's ids are staged CH at a time into a
// per-wave LDS slice with one coalesced load per lane (plus the per-sample
// weights), then every lane of the group reads them back as broadcast LDS
// reads and keeps RIF row gathers in flight: the id -> row dependency no
// longer serialises each row load behind a global index load, and the next
// chunk's ids are loaded while this chunk's rows are in flight. Groups of a
// wave with different bag lengths run the wave-uniform maximum trip count,
// predicated per group.
__device__ __forceinline__ void emb_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D, bool OUT_BF16, int RIF>
__global__ __launch_bounds__(256) void emb_fwd_kernel(EmbFwdArgs a) {
  fwd_bumps(a);
  constexpr int LPB = (D / 4) < 64 ? (D / 4) : 64;  // lanes per bag
  constexpr int BPW = 64 / LPB;                     // bags per wave
  constexpr int NCP = D / (4 * LPB);                // float4 column passes per lane
  constexpr int CH = 64;                            // ids staged per bag per chunk
  constexpr int IPL = (CH + LPB - 1) / LPB;         // staging loads per lane
  // RIF: row gathers in flight per lane (a 100-id bag is ~100 / RIF dependent
  // round trips; TDFO_EMB_RIF picks 4 / 8 / 16 for A/B)
  __shared__ int64_t s_ids[4][BPW][CH];
  __shared__ float s_w[4][BPW][CH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane / LPB, sl = lane - sub * LPB;
  int64_t* ids = s_ids[w][sub];
  float* wts = s_w[w][sub];
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // work item k = (bag group, table) with the table fastest: a wave's BPW
  // bags share a table (same pooling), but consecutive waves -- and each
  // wave's successive items -- cycle through the tables, so a long-bag
  // table (DCN-v2's 100-id table: 47% of the rows) is spread over every
  // block instead of filling one contiguous run of blocks in one pass
  const int64_t groups = (a.B + BPW - 1) / BPW;
  const int64_t nitems = groups * a.T;
  const int64_t nw_iters = (nitems + nwaves - 1) / nwaves;
  for (int64_t it = 0; it < nw_iters; ++it) {
    const int64_t k = it * nwaves + wave0;
    const int tk = (int)(k % a.T);
    const int64_t bb = (k / a.T) * BPW + sub;
    const bool active = k < nitems && bb < a.B;
    const int t = active ? tk : 0;
    const int b = active ? (int)bb : 0;
    const int64_t j = (int64_t)t * a.B + b;
    const int64_t s = active ? a.offsets[j] : 0, e = active ? a.offsets[j + 1] : 0;
    const int len = (int)(e - s);
    // wave-uniform chunk count (max over the wave's bags)
    int nch = (len + CH - 1) / CH;
#pragma unroll
    for (int o = LPB; o < 64; o <<= 1) nch = max(nch, __shfl_xor(nch, o));
    const float* wbase = a.W + (active ? a.row_offset[t] : 0) * D;
    float4 acc[NCP];
#pragma unroll
    for (int cp = 0; cp < NCP; ++cp) acc[cp] = make_float4(0.f, 0.f, 0.f, 0.f);
    // ids of chunk 0 in registers
    int64_t nid[IPL];
    float nwt[IPL];
    auto fetch = [&](int c) {
#pragma unroll
      for (int k = 0; k < IPL; ++k) {
        const int u = sl + k * LPB;
        const int64_t p = s + (int64_t)c * CH + u;
        const bool ok = u < CH && p < e;
        nid[k] = ok ? a.indices[p] : 0;
        nwt[k] = ok ? (a.psw ? a.psw[p] : 1.f) : 0.f;
      }
    };
    fetch(0);
    for (int c = 0; c < nch; ++c) {
      emb_wave_sync();                       // previous chunk's LDS reads done
#pragma unroll
      for (int k = 0; k < IPL; ++k) {
        const int u = sl + k * LPB;
        if (u < CH) { ids[u] = nid[k]; wts[u] = nwt[k]; }
      }
      emb_wave_sync();
      if (c + 1 < nch) fetch(c + 1);         // next chunk's ids overlap this chunk's rows
      const int n = max(0, min(CH, len - c * CH));
      int nmax = n;
#pragma unroll
      for (int o = LPB; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o));
      for (int u0 = 0; u0 < nmax; u0 += RIF) {
        float4 r[RIF][NCP];
        float wt[RIF];
#pragma unroll
        for (int v = 0; v < RIF; ++v) {
          const bool ok = u0 + v < n;
          const int64_t row = ok ? ids[u0 + v] : 0;
          wt[v] = ok ? wts[u0 + v] : 0.f;
#pragma unroll
          for (int cp = 0; cp < NCP; ++cp)
            r[v][cp] = ok ? *(const float4*)(wbase + row * D + (cp * LPB + sl) * 4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int v = 0; v < RIF; ++v)
#pragma unroll
          for (int cp = 0; cp < NCP; ++cp) {
            acc[cp].x += wt[v] * r[v][cp].x; acc[cp].y += wt[v] * r[v][cp].y;
            acc[cp].z += wt[v] * r[v][cp].z; acc[cp].w += wt[v] * r[v][cp].w;
          }
      }
    }
    if (!active) continue;
    const float inv = (a.mean && len > 0) ? 1.f / (float)len : 1.f;
#pragma unroll
    for (int cp = 0; cp < NCP; ++cp) {
      const float4 v = make_float4(acc[cp].x * inv, acc[cp].y * inv, acc[cp].z * inv,
                                   acc[cp].w * inv);
      const int64_t o = (int64_t)b * a.out_stride + a.out_off[t] + (cp * LPB + sl) * 4;
      if (OUT_BF16) *(uint2*)((uint16_t*)a.out + o) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
      else          *(float4*)((float*)a.out + o) = v;
    }
  }
}

// ---------------------------------------------------------- backward ----
// entries per update wave for narrow rows (D <= 32; A/B builds:
// TDFO_HIPCC_EXTRA=-DTDFO_EMB_SMALL_CH=32). 16: twice the waves, half the
// serial per-row chain each -- TwoTower 0.0655 -> 0.0621 ms/step, Bert4Rec
// B=16 0.430 -> 0.426 (8: 0.0641 / 0.424; profiles/r06/notes.md)
#ifndef TDFO_EMB_SMALL_CH
#define TDFO_EMB_SMALL_CH 16
#endif
template <int D>
struct BwdCfg {
  static constexpr int EPL = D >= 64 ? D / 64 : 1;                  // elements per lane
  static constexpr int CH = D <= 32 ? TDFO_EMB_SMALL_CH
                                    : (EPL <= 2 ? 32 : (EPL == 4 ? 16 : 8));   // entries per wave
};

// keys[p] = row_offset[t] + id, vals[p] = p, goff[p] = offset of p's pooled
// gradient row, gscale[p] = per-id scale (psw, 1/len for mean) if needed.
// One thread per position, its bag by binary search over the bag offsets.
// (Measured alternatives for DCN-v2's 1.75M multi-hot ids: a thread per bag
// walking its bag 128 us, a wave per 512 positions sliding a 64-bag offset
// window 52-63 us, this one 51 us; with ~one id per bag the window variant
// slid ~8 times per wave and slowed TwoTower / Bert4Rec.)
constexpr int KEYS_REG_MAXT = 1024;           // fixed-length path: virtual tables in LDS

template <typename K>
__global__ __launch_bounds__(256) void emb_keys_kernel(const EmbBwdArgs a, K* __restrict__ keys,
                                        int32_t* __restrict__ vals, int64_t* __restrict__ goff,
                                        float* __restrict__ gscale, int32_t* __restrict__ tail_count) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // read by later kernels
    tail_count[0] = 0;
    tail_count[1] = 0;
  }
  const int64_t nbags = (int64_t)a.T * a.B;
  // fixed bag lengths: the virtual tables' first positions in LDS, a
  // position's table by a short search there, its bag by division
  __shared__ int64_t tstart[KEYS_REG_MAXT + 1];
  const bool reg = a.bag_len != nullptr;
  if (reg) {
    for (int v = threadIdx.x; v <= a.T; v += blockDim.x)
      tstart[v] = v < a.T ? a.offsets[(int64_t)v * a.B] : a.nnz;
    __syncthreads();
  }
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.nnz;
       p += (int64_t)gridDim.x * blockDim.x) {
    int64_t j;
    if (reg) {
      int lo = 0, hi = a.T;                     // last table v with tstart[v] <= p
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tstart[mid] <= p) lo = mid; else hi = mid;
      }
      j = (int64_t)lo * a.B + (p - tstart[lo]) / a.bag_len[lo];
    } else {
      int64_t lo = 0, hi = nbags;               // last bag j with offsets[j] <= p
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.offsets[mid] <= p) lo = mid; else hi = mid;
      }
      j = lo;
    }
    const int t = (int)(j / a.B);
    const int b = (int)(j - (int64_t)t * a.B);
    keys[p] = (K)(a.row_offset[t] + a.indices[p]);
    vals[p] = (int32_t)p;
    goff[p] = (int64_t)b * a.grad_stride + a.grad_off[t];
    if (gscale) {
      const int64_t s0 = a.offsets[j], s1 = a.offsets[j + 1];
      const float inv = (a.mean && s1 > s0) ? 1.f / (float)(s1 - s0) : 1.f;
      gscale[p] = (a.psw ? a.psw[p] : 1.f) * inv;
    }
  }
}

// ------------------------------------------- one-hot: per-table LDS sort ----
// When every bag holds exactly one id (nnz == T*B, Criteo one-hot) and
// B <= SEG_MAX, table t's ids are the contiguous positions [t*B, (t+1)*B),
// and sorting them by row inside the table is the whole job: the composite
// (row_offset[t] + id) order across tables is just table order. One
// 1024-thread block per table sorts its <= 8192 (row, position) pairs in LDS
// with a stable LSD radix sort (6-bit digits, only as many passes as the
// table's largest id needs) and also writes the keys kernel's per-position
// outputs -- replacing emb_keys_kernel + the device-wide sort (3 passes of
// hist/scan/scatter over all tables) with one launch.
//   per pass: digit ranks inside a wave by ballot matching (6 ballots per
//   element), per-(digit, slot, wave) counts, one block-wide exclusive scan
//   over them in (digit, slot, wave) order, scatter into LDS, re-read.
//   The counters sit at (slot, wave) * (BINS + 1) + digit: a wave's count
//   writes and offset reads (one digit per lane) hit distinct banks. In the
//   digit-major order they were 128 words apart, one bank for every digit of
//   an instruction (~40-way conflicts on random ids): 43 us per 26 x 8192
//   table sort (scripts/emb_iso.py, profiles/r06/).
constexpr int SEG_MAX = 8192;
constexpr int SEG_THREADS = 1024;
constexpr int SEG_K = SEG_MAX / SEG_THREADS;        // elements per thread
// 6-bit digits. 7-bit ones (4 passes for a 26-bit table instead of 5, 64 KiB
// of counters) measured slower: fused one-hot backward 123.6 vs 109.1 us at
// 26 x 8192 ids (scripts/bench_segsort.py), the bigger scans cost more than
// the saved pass.
#ifndef TDFO_SEG_BITS
#define TDFO_SEG_BITS 6
#endif
constexpr int SEG_BITS = TDFO_SEG_BITS;
constexpr int SEG_BINS = 1 << SEG_BITS;
constexpr int SEG_WAVES = SEG_THREADS / 64;
constexpr int SEG_CNT = SEG_BINS * SEG_K * SEG_WAVES;   // 8192 counters

// Stable LSD radix sort of the block's SK * 1024 (key, val) pairs held in
// registers (element i = k * 1024 + tid in slot k), over the low `bits` bits.
// Only slots k < skn hold entries (block-uniform); the others keep the
// all-ones sentinel and are skipped. Ends with the sorted pairs in registers.
template <int SK>
__device__ __forceinline__ void seg_lsd_sort(uint32_t (&key)[SK], uint32_t (&val)[SK], int bits,
                                             int skn, uint32_t* skey, uint32_t* sval,
                                             uint32_t* cnt, uint32_t* wsum) {
  constexpr int PER = SEG_BINS * SK * SEG_WAVES / SEG_THREADS;   // (= SK)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // only the skn used slots' counters are cleared and scanned: logical
  // order (digit, slot < skn, wave), skn entries per thread
  const int kwn = skn * SEG_WAVES;
  const int cpn = kwn * (SEG_BINS + 1);
  for (int shift = 0; shift < bits; shift += SEG_BITS) {
    for (int c = tid; c < cpn; c += SEG_THREADS) cnt[c] = 0;
    __syncthreads();
    uint32_t rank[SK];
    int dig[SK];
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      if (k >= skn) break;
      // invalid slots carry the all-ones key: digit 63 in every pass
      const int d = (int)((key[k] >> shift) & (SEG_BINS - 1));
      uint64_t peers = ~0ull;
#pragma unroll
      for (int b = 0; b < SEG_BITS; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1);
        peers &= ((d >> b) & 1) ? bal : ~bal;
      }
      rank[k] = (uint32_t)__popcll(peers & lt);
      dig[k] = d;
      if ((peers & lt) == 0) cnt[(k * SEG_WAVES + w) * (SEG_BINS + 1) + d] = (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // exclusive scan of cnt in (digit, slot, wave) order: skn logical
    // entries per thread, i = tid * skn + q -> digit i / kwn, pair i % kwn
    auto phys = [&](int i) { return (i % kwn) * (SEG_BINS + 1) + i / kwn; };
    uint32_t loc[PER];
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (q >= skn) break;
      loc[q] = run;
      run += cnt[phys(tid * skn + q)];
    }
    uint32_t incl = run;                             // wave inclusive scan of the totals
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t base = incl - run;
    for (int q = 0; q < w; ++q) base += wsum[q];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (q >= skn) break;
      cnt[phys(tid * skn + q)] = base + loc[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      if (k >= skn) break;
      const uint32_t dst = cnt[(k * SEG_WAVES + w) * (SEG_BINS + 1) + dig[k]] + rank[k];
      skey[dst] = key[k];
      sval[dst] = val[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      if (k >= skn) break;
      key[k] = skey[k * SEG_THREADS + tid];
      val[k] = sval[k * SEG_THREADS + tid];
    }
    __syncthreads();
  }
}

// SK: elements per thread (tables of <= SK * 1024 ids; 2 for small batches:
// a quarter of the counters to clear and scan per pass)
// Run metadata for the in-kernel combine (one-hot, one run per table, B a
// multiple of the update's chunk size CH): for every chunk c of the sorted
// list, meta[c].x = the chunk where the run holding c's FIRST entry starts
// (-1: it starts in c) and meta[c].y = the chunk where the run holding c's
// LAST entry ends (-1: it ends in c); rcnt[c] = 0 (arrival counters). Found
// by binary searches over the table's sorted keys in LDS.
__device__ __forceinline__ void seg_run_meta(const uint32_t* skey, int n, int64_t s0, int ch,
                                             int2* __restrict__ meta, int32_t* __restrict__ rcnt) {
  const int nch = n / ch;
  for (int lc = threadIdx.x; lc < nch; lc += blockDim.x) {
    const int f = lc * ch, e = f + ch - 1;
    const uint32_t kf = skey[f], ke = skey[e];
    int lo = 0, hi = f;                  // first index with key == kf (sorted: >= kf)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (skey[mid] < kf) lo = mid + 1; else hi = mid;
    }
    const int rs = lo;
    lo = e + 1; hi = n;                  // first index past e with key > ke
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (skey[mid] <= ke) lo = mid + 1; else hi = mid;
    }
    const int re = lo - 1;
    const int64_t c = s0 / ch + lc;
    meta[c] = make_int2(rs < f ? (int)((s0 + rs) / ch) : -1, re > e ? (int)((s0 + re) / ch) : -1);
    rcnt[c] = 0;
  }
}

// LDS of one per-table sort block
template <int SK>
struct SegSmem {
  uint32_t skey[SK * SEG_THREADS];
  uint32_t sval[SK * SEG_THREADS];
  uint32_t cnt[SK * SEG_WAVES * (SEG_BINS + 1)];
  uint32_t wsum[SEG_WAVES];
  uint32_t smax[SEG_WAVES];
};

// Sort of virtual table t by one 1024-thread block (the body of
// emb_segsort_kernel, also run by the sort blocks of the tower co-launch)
template <typename K, bool SORTED_G, int SK>
__device__ __forceinline__ void segsort_table(
    const EmbBwdArgs& a, int t, K* __restrict__ keys_out, int32_t* __restrict__ vals_out,
    int64_t* __restrict__ goff, float* __restrict__ gscale, int32_t* __restrict__ tail_count,
    int32_t* __restrict__ pos, int2* __restrict__ meta, int32_t* __restrict__ rcnt,
    int meta_ch, SegSmem<SK>& sm) {
  uint32_t* skey = sm.skey;
  uint32_t* sval = sm.sval;
  uint32_t* cnt = sm.cnt;
  uint32_t* wsum = sm.wsum;
  uint32_t* smax = sm.smax;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (t == 0 && tid == 0) {                         // read by later kernels
    tail_count[0] = 0;
    tail_count[1] = 0;
  }
  const int n = a.B;
  const int64_t s0 = (int64_t)t * a.B;
  uint32_t key[SK], val[SK];
  uint32_t kmax = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    if (i < n) {
      const int64_t p = s0 + i;
      key[k] = (uint32_t)a.indices[p];
      val[k] = (uint32_t)i;
      kmax = max(kmax, key[k]);
      if (!SORTED_G) {
        goff[p] = (int64_t)i * a.grad_stride + a.grad_off[t];
        if (gscale) gscale[p] = a.psw ? a.psw[p] : 1.f;
      }
    } else {
      key[k] = 0xffffffffu;                          // sorts after every real id
      val[k] = 0;
    }
  }
  // passes needed for this table's largest id
  for (int off = 32; off > 0; off >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, off));
  if (lane == 0) smax[w] = kmax;
  __syncthreads();
  uint32_t bmax = 0;
  for (int q = 0; q < SEG_WAVES; ++q) bmax = max(bmax, smax[q]);
  const int bits = bmax ? 32 - __clz(bmax) : 1;
  seg_lsd_sort<SK>(key, val, bits, SK, skey, sval, cnt, wsum);
  if (meta != nullptr) {                 // sorted keys back in LDS for the searches
#pragma unroll
    for (int k = 0; k < SK; ++k) skey[k * SEG_THREADS + tid] = key[k];
    __syncthreads();
    seg_run_meta(skey, n, s0, meta_ch, meta, rcnt);
  }
  const K kb = (K)a.row_offset[t];
  const int64_t go = a.grad_off[t];
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    if (i < n) {
      keys_out[s0 + i] = kb + (K)key[k];
      vals_out[s0 + i] = (int32_t)(s0 + val[k]);
      if (pos) pos[s0 + i] = i;            // its index in its own run (merge below)
      if (SORTED_G) {     // gradient-row offset (and scale) already in sorted order
        goff[s0 + i] = (int64_t)val[k] * a.grad_stride + go;
        if (gscale) gscale[s0 + i] = a.psw ? a.psw[s0 + val[k]] : 1.f;
      }
    }
  }
}

template <typename K, bool SORTED_G, int SK = SEG_K>
__global__ __launch_bounds__(SEG_THREADS) void emb_segsort_kernel(
    const EmbBwdArgs a, K* __restrict__ keys_out, int32_t* __restrict__ vals_out,
    int64_t* __restrict__ goff, float* __restrict__ gscale, int32_t* __restrict__ tail_count,
    int32_t* __restrict__ pos, int2* __restrict__ meta = nullptr,
    int32_t* __restrict__ rcnt = nullptr, int meta_ch = 0) {
  __shared__ SegSmem<SK> sm;
  const int t = blockIdx.x, tid = threadIdx.x;
  if (t >= a.T) {
    // side blocks (a.side_on): four 256-thread reduce_adam units each, in the
    // sort's LDS (units take 256 floats of skey each; the one AUC unit sval)
    static_assert(SK * SEG_THREADS >= 4 * RA_PH * RA_COLS &&
                  SK * SEG_THREADS >= 2 * REDUCE_ADAM_MAX_NB, "side-job LDS");
    const int slice = tid >> 8;
    reduce_adam_unit(a.side, (t - a.T) * (SEG_THREADS / 256) + slice, tid & 255,
                     (float(*)[RA_COLS])(sm.skey + slice * RA_PH * RA_COLS), sm.sval);
    return;
  }
  segsort_table<K, SORTED_G, SK>(a, t, keys_out, vals_out, goff, gscale, tail_count, pos, meta,
                                 rcnt, meta_ch, sm);
}

// TwoTower co-launch (a.tower_on): the per-table sorts of a one-hot batch of
// <= 2048 ids (blocks [0, T)) beside the fused tower step (blocks [T, ...):
// TT_CO_WAVES tower waves each, every wave writing its own partial row --
// the rows of the one-wave tower kernel, so the same bits). The sort needs
// only the ids, the towers nothing the sort writes: one launch instead of
// two dependent ones. The block's other waves pass the towers' barriers
// and leave.
constexpr int TT_CO_WAVES = 4;
template <typename K>
__global__ __launch_bounds__(SEG_THREADS) void emb_segsort_tower_kernel(
    const EmbBwdArgs a, K* __restrict__ keys_out, int32_t* __restrict__ vals_out,
    int64_t* __restrict__ goff, float* __restrict__ gscale, int32_t* __restrict__ tail_count,
    int2* __restrict__ meta, int32_t* __restrict__ rcnt, int meta_ch) {
  __shared__ SegSmem<2> sm;
  __shared__ tt::Smem<TT_CO_WAVES> tsm;
  static_assert(sizeof(SegSmem<2>) + sizeof(tt::Smem<TT_CO_WAVES>) <= 160 * 1024, "LDS");
  const int t = blockIdx.x;
  if (t < a.T) {
    segsort_table<K, true, 2>(a, t, keys_out, vals_out, goff, gscale, tail_count, nullptr, meta,
                              rcnt, meta_ch, sm);
    return;
  }
  if (threadIdx.x < 64 * TT_CO_WAVES) {
    tt::tower_block<true, false, TT_CO_WAVES, true>(a.tower, t - a.T, threadIdx.x, tsm);
  } else {
#pragma unroll
    for (int i = 0; i < tt::tower_barriers<true>(); ++i) __syncthreads();
  }
}

// One-hot, one run per table, split by value range over NB blocks per table
// (MSD split + LSD in LDS). The single-block sort above is latency-bound on
// T CUs: ballot ranking of 8 slots x 5 passes for a 26-bit table, 35 us for
// 26 x 8192 ids with the rest of the GPU idle. Here every block reads the
// table's B ids, takes the table's largest id, and keeps the ids of its value
// range (bucket = floor(id * NB / (max + 1)) in f32: monotone, so equal ids
// share a bucket and buckets are ordered), compacted in position order; the
// ids of lower buckets give its output offset. It LSD-sorts (id - its
// smallest id) over only the bits that span, touching only the slots that
// hold entries: a uniform table becomes NB sorts of ~B / NB ids (one slot,
// 4 passes) on NB CUs; a table of a few rows, a few buckets of one id each
// and no pass at all. Skewed ids degrade to one block holding most of the
// table, i.e. the single-block sort. Same stable order, so the same bits.
template <typename K, int NB>
__global__ __launch_bounds__(SEG_THREADS) void emb_segsort_split_kernel(
    const EmbBwdArgs a, K* __restrict__ keys_out, int32_t* __restrict__ vals_out,
    int64_t* __restrict__ goff, float* __restrict__ gscale, int32_t* __restrict__ tail_count) {
  constexpr int SK = SEG_K;
  constexpr int KW = SK * SEG_WAVES;
  __shared__ uint32_t skey[SK * SEG_THREADS];
  __shared__ uint32_t sval[SK * SEG_THREADS];
  __shared__ uint32_t cnt[KW * (SEG_BINS + 1)];
  __shared__ uint32_t wsum[SEG_WAVES];
  __shared__ uint32_t red[2][SEG_WAVES];
  __shared__ uint32_t moff[KW];                   // (slot, wave) compaction offsets
  const int t = blockIdx.x / NB, bk = blockIdx.x - t * NB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (blockIdx.x == 0 && tid == 0) {              // read by later kernels
    tail_count[0] = 0;
    tail_count[1] = 0;
  }
  const int n = a.B;
  const int64_t s0 = (int64_t)t * a.B;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t key[SK], val[SK];
  uint32_t kmax = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    key[k] = i < n ? (uint32_t)a.indices[s0 + i] : 0u;
    if (i < n) kmax = max(kmax, key[k]);
  }
  for (int off = 32; off > 0; off >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, off));
  if (lane == 0) red[0][w] = kmax;
  __syncthreads();
  uint32_t tmax = 0;
  for (int q = 0; q < SEG_WAVES; ++q) tmax = max(tmax, red[0][q]);
  const float scale = (float)NB / ((float)tmax + 1.f);
  // own bucket's entries: rank inside the wave, per-(slot, wave) counts, and
  // the count of lower buckets' entries (this block's output offset)
  bool mine[SK];
  uint32_t myrank[SK];
  uint32_t below = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    const int b = i < n ? min(NB - 1, (int)((float)key[k] * scale)) : NB;
    mine[k] = b == bk;
    const uint64_t m = __ballot(mine[k]);
    below += (uint32_t)__popcll(__ballot(b < bk));
    myrank[k] = (uint32_t)__popcll(m & lt);
    if (lane == 0) moff[k * SEG_WAVES + w] = (uint32_t)__popcll(m);
  }
  if (lane == 0) red[1][w] = below;
  __syncthreads();
  // exclusive scan of the KW = 128 (slot, wave) counts by waves 0 and 1
  uint32_t v = 0, incl = 0;
  if (tid < KW) {
    v = moff[tid];
    incl = v;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
  }
  uint32_t off = 0;
  for (int q = 0; q < SEG_WAVES; ++q) off += red[1][q];
  __syncthreads();
  const int nb = (int)(wsum[0] + wsum[1]);        // entries in this bucket
  if (tid < KW) moff[tid] = incl - v + (w == 1 ? wsum[0] : 0u);
  __syncthreads();
  if (nb == 0) return;                            // (block-uniform)
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    if (mine[k]) {
      const uint32_t d = moff[k * SEG_WAVES + w] + myrank[k];
      skey[d] = key[k];
      sval[d] = (uint32_t)(k * SEG_THREADS + tid);
    }
  }
  __syncthreads();
  const int skn = (nb + SEG_THREADS - 1) / SEG_THREADS;
  uint32_t lo = 0xffffffffu, hi = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    if (i < nb) {
      key[k] = skey[i];
      val[k] = sval[i];
      lo = min(lo, key[k]);
      hi = max(hi, key[k]);
    } else {
      key[k] = 0xffffffffu;
      val[k] = 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
  }
  if (lane == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
  }
  __syncthreads();
  uint32_t bmin = 0xffffffffu, bmax = 0;
  for (int q = 0; q < SEG_WAVES; ++q) {
    bmin = min(bmin, red[0][q]);
    bmax = max(bmax, red[1][q]);
  }
#pragma unroll
  for (int k = 0; k < SK; ++k)
    if (k * SEG_THREADS + tid < nb) key[k] -= bmin;
  const uint32_t span = bmax - bmin;
  const int bits = span ? 32 - __clz(span) : 0;   // one id only: already sorted
  seg_lsd_sort<SK>(key, val, bits, skn, skey, sval, cnt, wsum);
  const K kb = (K)a.row_offset[t] + (K)bmin;
  const int64_t go = a.grad_off[t];
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int i = k * SEG_THREADS + tid;
    if (i < nb) {
      const int64_t p = s0 + off + i;
      keys_out[p] = kb + (K)key[k];
      vals_out[p] = (int32_t)(s0 + val[k]);
      goff[p] = (int64_t)val[k] * a.grad_stride + go;
      if (gscale) gscale[p] = a.psw ? a.psw[s0 + val[k]] : 1.f;
    }
  }
}

// Multi-source one-hot (world > 1): a physical table's ids arrive as R runs
// (one per source rank, virtual table v = run * Tp + table), each sorted by
// emb_segsort_kernel. An element's final position in its table is its index
// in its own run plus, for every other run, the number of keys that sort
// before it there (ties: earlier runs first = the stable order of the
// positions). One block per (run, other run) pair -- Tp x R x (R-1) blocks,
// so the R-1 rank computations of a run run concurrently instead of one
// after another in one block (207 -> see profiles/embedding_bwd_segsort_vs_radix
// for the serial form at R = 8) -- loads the other run into LDS; each thread
// owns 8 consecutive keys, binary-searches the first, walks forward for the
// rest and adds its counts to pos[] (7 atomic adds per element at R = 8, on
// distinct addresses per block). emb_runscatter_kernel then places keys and
// values.
template <typename K>
__global__ __launch_bounds__(SEG_THREADS) void emb_runrank_kernel(
    int Tp, int R, int B, const K* __restrict__ kin, int32_t* __restrict__ pos) {
  __shared__ K other[SEG_MAX];
  const int pair = blockIdx.x, tid = threadIdx.x;
  const int v = pair / (R - 1), j = pair - v * (R - 1);
  const int run = v / Tp, p = v - run * Tp;
  const int r = j < run ? j : j + 1;
  const int64_t src = (int64_t)v * B;
  const int64_t o = (int64_t)(r * Tp + p) * B;
  for (int i = tid; i < B; i += SEG_THREADS) other[i] = kin[o + i];
  __syncthreads();
  const bool le = r < run;                 // earlier run: equal keys go first
  const int i0 = tid * SEG_K;
  if (i0 >= B) return;
  K key[SEG_K];
#pragma unroll
  for (int k = 0; k < SEG_K; ++k) key[k] = i0 + k < B ? kin[src + i0 + k] : key[0];
  int lo = 0, hi = B;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const bool before = le ? other[mid] <= key[0] : other[mid] < key[0];
    if (before) lo = mid + 1; else hi = mid;
  }
#pragma unroll
  for (int k = 0; k < SEG_K; ++k) {
    if (i0 + k >= B) break;
    while (lo < B && (le ? other[lo] <= key[k] : other[lo] < key[k])) ++lo;
    atomicAdd(&pos[src + i0 + k], lo);
  }
}

template <typename K>
__global__ __launch_bounds__(256) void emb_runscatter_kernel(
    int Tp, int R, int B, const K* __restrict__ kin, const int32_t* __restrict__ vin,
    const int32_t* __restrict__ pos, K* __restrict__ kout, int32_t* __restrict__ vout) {
  const int64_t n = (int64_t)Tp * R * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = e / B;
    const int p = (int)(v % Tp);
    const int64_t d = (int64_t)p * R * B + pos[e];
    kout[d] = kin[e];
    vout[d] = vin[e];
  }
}

template <int D>
__device__ __forceinline__ int elem0(int lane) {
  return D >= 64 ? lane * (D / 64) : lane;
}

template <typename K>
__device__ __forceinline__ K rdlane(K v, int l) {
  if constexpr (sizeof(K) == 4) {
    return (K)__builtin_amdgcn_readlane((uint32_t)v, l);
  } else {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), l);
    return (K)(((uint64_t)hi << 32) | lo);
  }
}

__device__ __forceinline__ float rdlanef(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// NT: the update's table-row reads and writes as non-temporal accesses --
// on multi-hot batches (random rows over a big table, each touched once per
// step): DCN-v2's update 503 -> 464 us isolated; on one-hot DLRM-1TB, whose
// short tables' rows are hot, 61.4 -> 65.3, so off there (profiles/r06/notes.md)
template <bool NT, typename T>
__device__ __forceinline__ T row_ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void row_st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int D, bool NT = false>
__device__ __forceinline__ void load_row(float (&wv)[BwdCfg<D>::EPL], const float* w) {
  constexpr int EPL = BwdCfg<D>::EPL;
  if constexpr (EPL == 2) {
    typedef __attribute__((ext_vector_type(2))) float f2v;
    const f2v v = row_ld<NT>((const f2v*)w); wv[0] = v.x; wv[1] = v.y;
  } else if constexpr (EPL == 4) {
    const float4 v = *(const float4*)w; wv[0] = v.x; wv[1] = v.y; wv[2] = v.z; wv[3] = v.w;
  } else if constexpr (EPL == 8) {
    const float4 v0 = *(const float4*)w, v1 = *(const float4*)(w + 4);
    wv[0] = v0.x; wv[1] = v0.y; wv[2] = v0.z; wv[3] = v0.w;
    wv[4] = v1.x; wv[5] = v1.y; wv[6] = v1.z; wv[7] = v1.w;
  } else {
    wv[0] = w[0];
  }
}

// raw gradient row slice (bf16 or fp32), branch-free
template <int D, bool GB>
struct GradRaw {
  using T = typename std::conditional<GB, uint16_t, float>::type;
  T v[BwdCfg<D>::EPL];
};

template <int D, bool GB>
__device__ __forceinline__ void load_grad_raw(GradRaw<D, GB>& r, const void* grad, int64_t off) {
  constexpr int EPL = BwdCfg<D>::EPL;
  if constexpr (GB) {
    const uint16_t* gp = (const uint16_t*)grad + off;
    if constexpr (EPL == 2) {
      const uint32_t v = *(const uint32_t*)gp;
      r.v[0] = (uint16_t)(v & 0xffff); r.v[1] = (uint16_t)(v >> 16);
    } else if constexpr (EPL == 4) {
      const uint2 v = *(const uint2*)gp;
      r.v[0] = (uint16_t)(v.x & 0xffff); r.v[1] = (uint16_t)(v.x >> 16);
      r.v[2] = (uint16_t)(v.y & 0xffff); r.v[3] = (uint16_t)(v.y >> 16);
    } else if constexpr (EPL == 8) {
      const uint4 v = *(const uint4*)gp;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        r.v[2 * q] = (uint16_t)(w[q] & 0xffff); r.v[2 * q + 1] = (uint16_t)(w[q] >> 16);
      }
    } else {
      r.v[0] = gp[0];
    }
  } else {
    const float* gp = (const float*)grad + off;
#pragma unroll
    for (int u = 0; u < EPL; ++u) r.v[u] = gp[u];
  }
}

template <int D, bool GB>
__device__ __forceinline__ float raw_f(const GradRaw<D, GB>& r, int u) {
  if constexpr (GB) return bf2f(r.v[u]);
  else return r.v[u];
}

struct OptScalars { float lr, bc1, bc2, gs; };

__device__ __forceinline__ OptScalars opt_scalars(const EmbBwdArgs& a) {
  OptScalars o;
  o.lr = a.hyper[0];
  const float step = a.hyper[1];
  o.bc1 = 1.f - powf(a.beta1, step);
  o.bc2 = 1.f - powf(a.beta2, step);
  o.gs = a.hyper_n > 2 ? a.hyper[2] : 1.f;         // loss-scale unscale factor
  return o;
}

// Dynamic loss scaling: a step whose gradients were not finite updates nothing.
__device__ __forceinline__ bool skip_step(const EmbBwdArgs& a) {
  return a.hyper_n > 3 && a.hyper[3] > 0.f;
}

// One optimizer update of one row; `wv` = current weights (prefetched).
// Adam with pre-loaded moments (mpre / vpre: this lane's elements of the
// row's m and v, issued with the chunk's other loads) or loading them here.
template <int D, int OPT, bool NT = false>
__device__ __forceinline__ void update_row(const EmbBwdArgs& a, const OptScalars& o,
                                           uint64_t row, const float (&acc_in)[BwdCfg<D>::EPL],
                                           float (&wv)[BwdCfg<D>::EPL], float st_row, int lane,
                                           const float* mpre = nullptr,
                                           const float* vpre = nullptr) {
#pragma clang fp contract(off)     // same bits wherever it is inlined
  constexpr int EPL = BwdCfg<D>::EPL;
  float acc[EPL];
#pragma unroll
  for (int u = 0; u < EPL; ++u) acc[u] = acc_in[u] * o.gs;
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  float* w = a.W + row * D + e0;
  if constexpr (OPT == EMB_DENSE_GRAD) {
    float* dg = a.dense_grad + row * D + e0;
#pragma unroll
    for (int u = 0; u < EPL; ++u) if (act) dg[u] += acc[u];
    return;
  } else {
    if constexpr (OPT == EMB_SGD) {
#pragma unroll
      for (int u = 0; u < EPL; ++u) wv[u] -= o.lr * (acc[u] + a.weight_decay * wv[u]);
    } else if constexpr (OPT == EMB_ROWWISE_ADAGRAD) {
      float g[EPL], sq = 0.f;
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        g[u] = acc[u] + a.weight_decay * wv[u];
        sq += act ? g[u] * g[u] : 0.f;
      }
      sq = wave_sum_dpp(sq) * (1.f / (float)D);
      const float stv = st_row + sq;
      if (lane == 0) a.state1[row] = stv;
      const float mult = o.lr / (sqrtf(stv) + a.eps);
#pragma unroll
      for (int u = 0; u < EPL; ++u) wv[u] -= mult * g[u];
    } else if constexpr (OPT == EMB_ADAGRAD) {
      float* stp = a.state1 + row * D + (act ? e0 : 0);
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        const float gg = acc[u] + a.weight_decay * wv[u];
        const float s2 = stp[u] + gg * gg;
        if (act) stp[u] = s2;
        wv[u] -= o.lr * gg / (sqrtf(s2) + a.eps);
      }
    } else {  // EMB_ADAM, decoupled weight decay, bias-corrected (fbgemm-style)
      float* m = a.state1 + row * D + (act ? e0 : 0);
      float* v = a.state2 + row * D + (act ? e0 : 0);
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        const float m0 = mpre ? mpre[u] : m[u], v0 = vpre ? vpre[u] : v[u];
        const float mm = a.beta1 * m0 + (1.f - a.beta1) * acc[u];
        const float vv = a.beta2 * v0 + (1.f - a.beta2) * acc[u] * acc[u];
        if (act) { m[u] = mm; v[u] = vv; }
        // (hardware sqrt / rcp and uniform bias-correction reciprocals, as
        // adam_elem: ~10 VALU ops instead of ~35 per element)
        const float den = __builtin_amdgcn_sqrtf(vv * (1.f / o.bc2)) + a.eps;
        wv[u] -= o.lr * ((mm * (1.f / o.bc1)) * __builtin_amdgcn_rcpf(den) +
                         a.weight_decay * wv[u]);
      }
    }
    if (act) {
      if constexpr (EPL == 2) {
        typedef __attribute__((ext_vector_type(2))) float f2v;
        row_st<NT>((f2v*)w, f2v{wv[0], wv[1]});
      } else if constexpr (EPL == 4) {
        row_st<NT>((f32x4_t*)w, f32x4_t{wv[0], wv[1], wv[2], wv[3]});
      } else {
#pragma unroll
        for (int u = 0; u < EPL; ++u) w[u] = wv[u];
      }
    }
  }
}

// Partials handed between waves of ONE launch (the in-kernel combine below):
// agent-scope (sc1) stores and loads; the producing wave's lane 0 signals
// with an agent-scope atomic add after the wave's vmcnt(0) wait, and the wave
// whose add comes last loads (MI355X_MICROARCH.md, inter-workgroup
// visibility, hand-off row 1). No wave ever waits for another. (Atomic
// read-modify-write hand-offs -- exchange / add 0 -- measured 18 us slower per
// DLRM-1TB step: a 3-row table's run walks 85 partials through them.)
template <int EPL>
__device__ __forceinline__ void part_store(float* p, const float (&v)[EPL]) {
  if constexpr (EPL % 2 == 0) {
#pragma unroll
    for (int u = 0; u < EPL; u += 2) {
      const uint64_t x = (uint64_t)__float_as_uint(v[u]) |
                         ((uint64_t)__float_as_uint(v[u + 1]) << 32);
      __hip_atomic_store((uint64_t*)(p + u), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    __hip_atomic_store((uint32_t*)p, __float_as_uint(v[0]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int EPL>
__device__ __forceinline__ void part_load(float (&v)[EPL], const float* p) {
  if constexpr (EPL % 2 == 0) {
#pragma unroll
    for (int u = 0; u < EPL; u += 2) {
      const uint64_t x =
          __hip_atomic_load((const uint64_t*)(p + u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[u] = __uint_as_float((uint32_t)x);
      v[u + 1] = __uint_as_float((uint32_t)(x >> 32));
    }
  } else {
    v[0] = __uint_as_float(
        __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
}

// A run crossing chunk edges, finished by the last of its chunks to arrive:
// the tail partial of its first chunk cs, then the head partials of chunks
// cs+1..ce in chunk order (HQ in flight) -- emb_combine_kernel's order, so the
// same bits -- and one optimizer update of `row`.
// emb_combine_kernel calls the same code, and FP contraction is off here and
// in update_row, so the in-kernel and the separate combine give identical
// bits (inlined into two kernels with contraction on, the update came out
// 1 ulp apart on 8 of 13 K rows; a non-inlined call cost the update kernel
// 224 B of scratch and 20 us).
template <int D, int OPT, int HQ_MAX = 32>
__device__ __forceinline__ void run_finish(const EmbBwdArgs& a, const OptScalars& o,
                                           int64_t cs, int64_t ce,
                           uint64_t row, float* head, float* tail, int lane) {
#pragma clang fp contract(off)
  constexpr int EPL = BwdCfg<D>::EPL;
  constexpr int HQ0 = EPL <= 2 ? 32 : (EPL <= 4 ? 16 : 8);
  constexpr int HQ = HQ0 < HQ_MAX ? HQ0 : HQ_MAX;     // (the sum order does not depend on it)
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  const int e0c = act ? e0 : 0;
  float acc[EPL];
  part_load<EPL>(acc, tail + cs * D + e0c);
#pragma unroll
  for (int u = 0; u < EPL; ++u) acc[u] = act ? acc[u] : 0.f;
  for (int64_t j0 = cs + 1; j0 <= ce; j0 += HQ) {
    float hv[HQ][EPL];
#pragma unroll
    for (int q = 0; q < HQ; ++q) part_load<EPL>(hv[q], head + min(j0 + q, ce) * D + e0c);
#pragma unroll
    for (int q = 0; q < HQ; ++q) {
      if (j0 + q <= ce && act) {
#pragma unroll
        for (int u = 0; u < EPL; ++u) acc[u] += hv[q][u];
      }
    }
  }
  float wv[EPL];
#pragma unroll
  for (int u = 0; u < EPL; ++u) wv[u] = 0.f;
  if constexpr (OPT != EMB_DENSE_GRAD) load_row<D>(wv, a.W + row * D + e0c);
  const float st = OPT == EMB_ROWWISE_ADAGRAD ? a.state1[row] : 0.f;
  update_row<D, OPT>(a, o, row, acc, wv, st, lane);
}

// One wave = one chunk of CH sorted entries. Every gradient row of the chunk
// and every weight row it may update are loaded up front with no control
// flow between the loads (hipcc keeps all of them in flight); runs are then
// reduced in registers in sorted order and each run that finishes inside the
// chunk gets exactly one optimizer update. Runs crossing chunk edges leave
// head / tail partials: with run metadata (``meta``, from the one-hot sort)
// the last of a run's chunks to arrive finishes it here; otherwise the
// chunk where it starts is listed for emb_combine_kernel.
template <int D, typename K, bool GB, int OPT, int CH, bool META = false, bool NT = false>
__global__ __launch_bounds__(256) void emb_chunk_kernel(
    EmbBwdArgs a, const K* __restrict__ keys, const int32_t* __restrict__ vals,
    const int64_t* __restrict__ goff, const float* __restrict__ gscale,
    float* __restrict__ head, float* __restrict__ tail, int32_t* __restrict__ tail_list,
    int32_t* __restrict__ tail_count, const int2* __restrict__ meta,
    int32_t* __restrict__ rcnt) {
  constexpr int EPL = BwdCfg<D>::EPL;
  constexpr bool NEED_W = OPT != EMB_DENSE_GRAD;
  const int lane = threadIdx.x & 63;
  int nblk = gridDim.x;
  if constexpr (META) {
    // side blocks (a.side_block0 > 0): one reduce_adam unit each
    if (a.side_block0 > 0) {
      if ((int)blockIdx.x >= a.side_block0) {
        __shared__ float sred[RA_PH][RA_COLS];
        __shared__ unsigned int slh[2 * REDUCE_ADAM_MAX_NB];
        reduce_adam_unit(a.side, blockIdx.x - a.side_block0, threadIdx.x, sred, slh);
        return;
      }
      nblk = a.side_block0;
    }
  }
  if (skip_step(a)) return;
  const OptScalars o = opt_scalars(a);
  const int64_t nch = (a.nnz + CH - 1) / CH;
  const int64_t nwv = ((int64_t)nblk * blockDim.x) >> 6;
  // one wave per chunk (grid-stride: any grid size walks every chunk)
  for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < nch; c += nwv) {
  const int64_t start = c * CH;
  const int64_t end = min(start + (int64_t)CH, a.nnz);
  const int len = (int)(end - start);
  const int li = lane < len ? lane : len - 1;     // lanes >= len duplicate the last entry
  const K mykey = keys[start + li];
  const int mypos = vals[start + li];
  const int64_t gi = a.goff_sorted ? start + li : mypos;   // sorted: no pos indirection
  const int64_t mygoff = goff[gi];
  const float mysc = gscale ? gscale[gi] : 1.f;
  const K prevk = start > 0 ? keys[start - 1] : (K)0;
  const K nextk = end < a.nnz ? keys[end] : (K)0;
  const int2 md = META ? meta[c] : make_int2(-1, -1);
  const K kup = __shfl_up(mykey, 1, 64);
  const K kdn = __shfl_down(mykey, 1, 64);
  const bool is_start = lane < len && (lane == 0 ? (start == 0 || prevk != mykey) : kup != mykey);
  const bool is_end = lane < len && (lane == len - 1 ? (end == a.nnz || nextk != mykey)
                                                     : kdn != mykey);
  const uint64_t smask = __ballot(is_start), emask = __ballot(is_end);
  const bool from_before = !(smask & 1ull);
  uint64_t fmask = emask;                                     // runs finishing here
  if (from_before && emask) fmask &= ~(emask & (~emask + 1));  // first run is not ours
  const float st_l = OPT == EMB_ROWWISE_ADAGRAD ? a.state1[(uint64_t)mykey] : 0.f;
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  const int e0c = act ? e0 : 0;

  GradRaw<D, GB> g[CH];
  float wr[CH][EPL];
  // Adam on narrow rows (one element per lane): the moments of every row of
  // the chunk are loaded up front too, not one dependent round trip per
  // finishing run (TwoTower / Bert4Rec, D = 16: a chunk's 32 updates waited
  // on 32 serial m / v loads)
  constexpr bool PRE_MV = OPT == EMB_ADAM && EPL == 1;
  float mr[PRE_MV ? CH : 1][EPL], vr[PRE_MV ? CH : 1][EPL];
#pragma unroll
  for (int p = 0; p < CH; ++p) {
    const int64_t go = (int64_t)rdlane((uint64_t)mygoff, p);
    load_grad_raw<D, GB>(g[p], a.grad, go + e0c);
    const uint64_t rowp = (uint64_t)rdlane(mykey, p);
    if constexpr (NEED_W) load_row<D, NT>(wr[p], a.W + rowp * D + e0c);
    if constexpr (PRE_MV) {
      mr[p][0] = a.state1[rowp * D + e0c];
      vr[p][0] = a.state2[rowp * D + e0c];
    }
  }
  float acc[EPL];
#pragma unroll
  for (int u = 0; u < EPL; ++u) acc[u] = 0.f;
#pragma unroll
  for (int p = 0; p < CH; ++p) {
    if (p < len) {
      const float sc = rdlanef(mysc, p);
#pragma unroll
      for (int u = 0; u < EPL; ++u) acc[u] += sc * raw_f<D, GB>(g[p], u);
      if ((emask >> p) & 1ull) {
        if ((fmask >> p) & 1ull) {
          float wv[EPL];
#pragma unroll
          for (int u = 0; u < EPL; ++u) wv[u] = NEED_W ? wr[p][u] : 0.f;
          if constexpr (PRE_MV)
            update_row<D, OPT, NT>(a, o, (uint64_t)rdlane(mykey, p), acc, wv, rdlanef(st_l, p),
                                   lane, mr[p], vr[p]);
          else
            update_row<D, OPT, NT>(a, o, (uint64_t)rdlane(mykey, p), acc, wv, rdlanef(st_l, p),
                                   lane);
        } else if (act) {
          part_store<EPL>(head + c * D + e0, acc);
        }
#pragma unroll
        for (int u = 0; u < EPL; ++u) acc[u] = 0.f;
      }
    }
  }
  const bool cont = !((emask >> (len - 1)) & 1ull);           // last run continues
  const bool started_here = smask != 0;
  if (cont) {
    if (act) part_store<EPL>((started_here ? tail : head) + c * D + e0, acc);
    if (!META && started_here && lane == 0) {
      const int slot = atomicAdd(tail_count, 1);
      if (slot < (int)((a.nnz + CH - 1) / CH)) tail_list[slot] = (int32_t)c;
    }
  }
  if constexpr (META) {
    // arrivals: a head partial of the run that came from before (it ends here,
    // or covers the whole chunk), a tail partial of the run that starts here
    // and continues; the run's counter sits at its first chunk
    const bool sig_h = from_before;
    const int64_t hcs = md.x, hce = emask ? c : (int64_t)md.y;
    const bool sig_t = cont && started_here;
    const int64_t tce = md.y;
    int last_h = 0, last_t = 0;
    if (sig_h || sig_t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's partials landed
      if (lane == 0) {
        if (sig_h) last_h = atomicAdd(&rcnt[hcs], 1) == (int)(hce - hcs);
        if (sig_t) last_t = atomicAdd(&rcnt[c], 1) == (int)(tce - c);
      }
      last_h = __builtin_amdgcn_readfirstlane(last_h);
      last_t = __builtin_amdgcn_readfirstlane(last_t);
      // the last arrival re-arms its counter (an apply replayed without a
      // new sort sees zeros again)
      if (lane == 0 && last_h) __hip_atomic_store(&rcnt[hcs], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0 && last_t) __hip_atomic_store(&rcnt[c], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (last_h)
      run_finish<D, OPT>(a, o, hcs, hce, (uint64_t)rdlane(mykey, 0), head, tail, lane);
    if (last_t)
      run_finish<D, OPT>(a, o, c, tce, (uint64_t)rdlane(mykey, len - 1), head, tail, lane);
  }
  }
}

// Runs crossing chunk edges: the chunk where a run starts adds the head
// partials of the chunks the run covers (found by binary search), in chunk
// order with 8 loads in flight, and applies the optimizer once.
// Runs longer than COMBINE_LONG chunks (hot rows of skewed ids: a Zipf-1.05
// DCN-v2 batch has runs of ~1.4 K chunks) are left to
// emb_combine_long_kernel, which splits the walk over a block's 16 waves: one
// wave walking them took 140 us of the DCN-v2 step. One-hot batches whose
// longest possible run (R sources x B ids) fits in COMBINE_LONG chunks never
// divert and skip that launch (DLRM-1TB at W=1: the 3-row tables' 85-chunk
// runs stay here; diverting runs over 64 chunks cost it 16 us per step).
constexpr int COMBINE_LONG = 256;
constexpr int LONG_WAVES = 16;

template <int D, typename K, int OPT, int CH>
__global__ __launch_bounds__(256) void emb_combine_kernel(
    EmbBwdArgs a, const K* __restrict__ keys, float* __restrict__ head,
    float* __restrict__ tail, const int32_t* __restrict__ tail_list,
    int32_t* __restrict__ tail_count, int64_t* __restrict__ long_list, int allow_long) {
  const int lane = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  if (skip_step(a)) return;
  const int n = min(*tail_count, (int)((a.nnz + CH - 1) / CH));
  const OptScalars o = opt_scalars(a);
  for (int i = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6); i < n; i += nw) {
    const int64_t c = tail_list[i];
    const int64_t endc = min((c + 1) * CH, a.nnz);
    const K last = keys[endc - 1];
    // Last chunk of the run: the chunks it covers are exactly the ones after
    // c whose FIRST key is `last` (sorted keys: a prefix of c+1, c+2, ...), so
    // each lane probes one chunk's first key and a ballot counts the prefix --
    // one dependent load per 64 chunks instead of a ~18-step binary search
    // over every key after the chunk (that chain was most of this kernel's
    // 16 us in the DLRM-1TB step).
    const int64_t nch = (a.nnz + CH - 1) / CH;
    int64_t jlast = c;
    for (int64_t jb = c + 1; jb < nch; jb += 64) {
      const int64_t j = jb + lane;
      const K kj = keys[min(j, nch - 1) * CH];
      const int cnt = __popcll(__ballot(j < nch && kj == last));
      jlast += cnt;
      if (cnt < 64) break;
    }
    if (allow_long && jlast - c > COMBINE_LONG) {
      if (lane == 0) {
        const int slot = atomicAdd(tail_count + 1, 1);
        long_list[2 * slot] = c;
        long_list[2 * slot + 1] = jlast;
      }
      continue;
    }
    run_finish<D, OPT>(a, o, c, jlast, (uint64_t)last, head, tail, lane);
  }
}

// One block of LONG_WAVES waves per long run (block-stride over the list):
// wave w sums the head partials of a contiguous 1/LONG_WAVES of the run's
// chunks in chunk order (HQ loads in flight), and wave 0 adds the run's tail
// partial and the waves' sums in wave order, then applies the optimizer once.
// Fixed order throughout: bitwise reproducible.
template <int D, typename K, int OPT, int CH>
__global__ __launch_bounds__(64 * LONG_WAVES) void emb_combine_long_kernel(
    EmbBwdArgs a, const K* __restrict__ keys, const float* __restrict__ head,
    const float* __restrict__ tail, const int32_t* __restrict__ tail_count,
    const int64_t* __restrict__ long_list) {
  constexpr int EPL = BwdCfg<D>::EPL;
  __shared__ float part[LONG_WAVES][64 * EPL];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (skip_step(a)) return;
  const int n = tail_count[1];
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  const int e0c = act ? e0 : 0;
  const OptScalars o = opt_scalars(a);
  constexpr int HQ = EPL <= 2 ? 32 : (EPL <= 4 ? 16 : 8);
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t c = long_list[2 * i], jlast = long_list[2 * i + 1];
    const int64_t len = jlast - c;                     // chunks c+1 .. jlast
    const int64_t j_lo = c + 1 + len * w / LONG_WAVES;
    const int64_t j_hi = c + 1 + len * (w + 1) / LONG_WAVES;   // exclusive
    float acc[EPL];
#pragma unroll
    for (int u = 0; u < EPL; ++u) acc[u] = 0.f;
    for (int64_t j0 = j_lo; j0 < j_hi; j0 += HQ) {
      float hv[HQ][EPL];
#pragma unroll
      for (int q = 0; q < HQ; ++q) {
        const int64_t j = min(j0 + q, j_hi - 1);
#pragma unroll
        for (int u = 0; u < EPL; ++u) hv[q][u] = head[j * D + e0c + u];
      }
#pragma unroll
      for (int q = 0; q < HQ; ++q) {
        if (j0 + q < j_hi) {
#pragma unroll
          for (int u = 0; u < EPL; ++u) acc[u] += hv[q][u];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < EPL; ++u) part[w][lane * EPL + u] = acc[u];
    __syncthreads();
    if (w == 0) {
      float t[EPL];
#pragma unroll
      for (int u = 0; u < EPL; ++u) t[u] = act ? tail[c * D + e0 + u] : 0.f;
      for (int q = 0; q < LONG_WAVES; ++q) {
#pragma unroll
        for (int u = 0; u < EPL; ++u) t[u] += part[q][lane * EPL + u];
      }
      const int64_t endc = min((c + 1) * CH, a.nnz);
      const K last = keys[endc - 1];
      float wv[EPL];
#pragma unroll
      for (int u = 0; u < EPL; ++u) wv[u] = 0.f;
      if constexpr (OPT != EMB_DENSE_GRAD) load_row<D>(wv, a.W + (uint64_t)last * D + e0c);
      const float st = OPT == EMB_ROWWISE_ADAGRAD ? a.state1[(uint64_t)last] : 0.f;
      update_row<D, OPT>(a, o, (uint64_t)last, t, wv, st, lane);
    }
    __syncthreads();                                   // part[] is reused
  }
}

// Row-wise owner backward: entry (r, i) of the received [W][cap+1] exchange
// buffer (rowwise.hip) -> key = owner-local row, val = position, gradient
// row offset in the all-gathered [W][B][grad_ld] pooled gradients. Slots past
// a segment's count point at the store's scratch row (their gradient row is
// row 0: harmless, the scratch row is never read by a forward).
template <typename K>
__global__ void emb_rw_keys_kernel(const EmbBwdArgs a, const int64_t* __restrict__ recv,
                                   const int64_t* __restrict__ meta, int nrw, int W,
                                   int64_t cap, int64_t grad_ld, int64_t dummy_row, int rows,
                                   K* __restrict__ keys, int32_t* __restrict__ vals,
                                   int64_t* __restrict__ goff, float* __restrict__ gscale,
                                   int32_t* __restrict__ tail_count) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    tail_count[0] = 0;
    tail_count[1] = 0;
  }
  const int64_t* L = meta + nrw;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.nnz;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(p / cap);
    const int64_t i = p - (int64_t)r * cap;
    const int64_t* seg = recv + (int64_t)r * (cap + 1);
    const int64_t cnt = seg[cap];
    K key = (K)dummy_row;
    int64_t go = 0;
    float sc = 1.f;
    if (i < cnt) {
      const uint64_t v = (uint64_t)seg[i];
      const int64_t bk = (int64_t)(v >> 32);
      const int j = (int)(bk / a.B);
      const int64_t b = bk - (int64_t)j * a.B;
      key = (K)(v & 0xffffffffull);
      go = rows ? ((int64_t)r * (cap + 1) + i) * grad_ld
                : ((int64_t)r * a.B + b) * grad_ld + (int64_t)j * a.D;
      if (a.mean) sc = 1.f / (float)L[j];
    }
    keys[p] = key;
    vals[p] = (int32_t)p;
    goff[p] = go;
    if (gscale) gscale[p] = sc;
  }
}

// Dense update of every row of a (replicated) table batch from a dense fp32
// gradient [rows, D] -- the data-parallel tables' step after their gradient
// all-reduce. One wave per row; rows with an all-zero gradient are left
// untouched for SGD / row-wise Adagrad / Adagrad without weight decay, so the
// result equals the sparse update of the touched rows. ``gclr`` (== g or
// null): zero each gradient row once read, so the next step's backward
// accumulates into a clean buffer without a separate fill pass (also on a
// skipped step).
template <int D>
__device__ __forceinline__ void zero_row(float* w) {
  constexpr int EPL = BwdCfg<D>::EPL;
  if constexpr (EPL == 2) {
    *(float2*)w = make_float2(0.f, 0.f);
  } else if constexpr (EPL == 4) {
    *(float4*)w = make_float4(0.f, 0.f, 0.f, 0.f);
  } else if constexpr (EPL == 8) {
    *(float4*)w = make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(w + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    w[0] = 0.f;
  }
}

template <int D, int OPT>
__global__ __launch_bounds__(256) void emb_dense_update_kernel(EmbBwdArgs a, int64_t rows,
                                                              const float* __restrict__ g,
                                                              float* gclr) {
  constexpr int EPL = BwdCfg<D>::EPL;
  const int lane = threadIdx.x & 63;
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  const int e0c = act ? e0 : 0;
  const OptScalars o = opt_scalars(a);
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (skip_step(a)) {
    if (gclr && act)
      for (int64_t row = row0; row < rows; row += nw) zero_row<D>(gclr + row * D + e0);
    return;
  }
  for (int64_t row = row0; row < rows; row += nw) {
    float acc[EPL], wv[EPL];
    load_row<D>(acc, g + row * D + e0c);
    if (gclr && act) zero_row<D>(gclr + row * D + e0);
    load_row<D>(wv, a.W + row * D + e0c);
    if (!act) {
#pragma unroll
      for (int u = 0; u < EPL; ++u) acc[u] = 0.f;
    }
    const float st = OPT == EMB_ROWWISE_ADAGRAD ? a.state1[row] : 0.f;
    update_row<D, OPT>(a, o, (uint64_t)row, acc, wv, st, lane);
  }
}

template <int D>
void dense_update_dispatch(const EmbBwdArgs& a, int64_t rows, const float* g, float* gclr,
                           hipStream_t s) {
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  if (blocks < 1) return;
#define TDFO_DU(OPT) hipLaunchKernelGGL((emb_dense_update_kernel<D, OPT>), dim3(blocks), dim3(256), \
                                        0, s, a, rows, g, gclr)
  switch (a.opt) {
    case EMB_SGD: TDFO_DU(EMB_SGD); break;
    case EMB_ROWWISE_ADAGRAD: TDFO_DU(EMB_ROWWISE_ADAGRAD); break;
    case EMB_ADAM: TDFO_DU(EMB_ADAM); break;
    case EMB_ADAGRAD: TDFO_DU(EMB_ADAGRAD); break;
    default: throw std::runtime_error("embedding_dense_update: unsupported optimizer");
  }
#undef TDFO_DU
  TDFO_CHECK_HIP(hipGetLastError());
}

int g_emb_segsort = 1;   // one-hot batches: per-table LDS sort (0: device-wide radix sort)
// one-hot, one run, B > 2048: the value-range split sort (TDFO_SEG_SPLIT=1).
// Off by default: isolated it sorts 26 x 8192 ids in 17.7-20 us against
// 35 us for one block per table, but it keeps 8x the CUs busy (208 CU x
// ~28 us in the step against 26 x ~56), and the sort runs beside the top-MLP
// forward GEMMs, off the critical path: DLRM-1TB 0.433-0.436 vs 0.421-0.422
// ms/step (same box, profiles/r06/). What the step pays for a background
// kernel is its CU-time and bytes, not its latency.
constexpr int SEG_SPLIT = 8;
const int g_emb_seg_split = [] {
  const char* e = getenv("TDFO_SEG_SPLIT");
  return e ? atoi(e) : 0;
}();

// (Rejected, round 4: capping the fused update's grid so GEMM blocks get CUs
// beside it, with the full or a half-chunk 94-VGPR update kernel that fits
// next to a 256x128 GEMM block: DCN-v2 2.62-2.99 vs 2.37 ms/step, DLRM-1TB
// 0.465-0.496 vs 0.453-0.458; half chunks alone 2.40-2.42 / 0.454-0.457,
// profiles/r04/notes.md)

struct WsLayout {
  size_t keys_in, keys_out, vals_in, vals_out, goff, gscale, head, tail, tlist, tcount, sortws,
      pos, llist, meta, rcnt;
  size_t total;
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

int ch_for(int D) { return D <= 32 ? TDFO_EMB_SMALL_CH : (D <= 128 ? 32 : (D == 256 ? 16 : 8)); }

WsLayout ws_layout(int64_t nnz, int D) {
  WsLayout L;
  const int64_t nch = (nnz + ch_for(D) - 1) / ch_for(D);
  size_t o = 0;
  L.keys_in = o;  o += al(nnz * 8);
  L.keys_out = o; o += al(nnz * 8);
  L.vals_in = o;  o += al(nnz * 4);
  L.vals_out = o; o += al(nnz * 4);
  L.goff = o;     o += al(nnz * 8);
  L.gscale = o;   o += al(nnz * 4);
  L.head = o;     o += al((size_t)nch * D * 4);
  L.tail = o;     o += al((size_t)nch * D * 4);
  L.tlist = o;    o += al((size_t)nch * 4);
  L.tcount = o;   o += al(16);
  L.sortws = o;   o += al(radix_sort_workspace(nnz));
  L.pos = o;      o += al(nnz * 4);
  L.llist = o;    o += al((size_t)(nch / COMBINE_LONG + 1) * 16);   // (c, jlast) per long run
  L.meta = o;     o += al((size_t)nch * 8);                          // run metadata per chunk
  L.rcnt = o;     o += al((size_t)nch * 4);                          // arrival counters
  L.total = o;
  return L;
}

// prepare's choice of path (apply must read the layout prepare wrote): a pure
// function of the call's arguments -- the caller resolves the global A/B
// toggle into a.segsort once and passes the same value to both halves
bool onehot_path(const EmbBwdArgs& a) {
  const int R = a.segsort;
  return R > 0 && a.T % R == 0 && a.nnz == (int64_t)a.T * a.B &&
         a.B <= SEG_MAX && !a.mean;
}

// one run per table, chunks never straddling tables, single-block sort: the
// sort writes run metadata and the update finishes crossing runs in-kernel
// (no emb_combine_kernel launch; TDFO_EMB_INKERNEL_COMBINE=1). Off by
// default: isolated it takes the DLRM-1TB update from 57.5 to 43.2 us, but
// the step runs 0.430-0.434 vs 0.412-0.414 ms with the separate combine
// (same box, 300 steps; profiles/r06/notes.md): the last-arriving chunk's
// walk over a tiny table's ~85 partials becomes the update kernel's tail,
// which the next lookup waits behind.
// TDFO_EMB_INKERNEL_COMBINE: 1 always, 0 never, unset: batches of at most
// IKC_AUTO_MAX ids. Small batches (TwoTower 7 x 2048, Bert4Rec 320 ids) gain
// from dropping the combine launch (TwoTower 0.0762 -> 0.0735 ms/step,
// Bert4Rec B=16 0.436 -> 0.433); on DLRM-1TB (213 K ids) the last arrival's
// walk over a short table's ~85 partials became the update's tail: 0.430 vs
// 0.413 (profiles/r06/notes.md).
constexpr int64_t IKC_AUTO_MAX = 65536;
const bool g_emb_nt = [] {            // TDFO_EMB_NT=0: plain row accesses everywhere
  const char* e = getenv("TDFO_EMB_NT");
  return !(e && atoi(e) == 0);
}();
const int g_emb_inkernel_combine = [] {
  const char* e = getenv("TDFO_EMB_INKERNEL_COMBINE");
  return e ? atoi(e) : -1;
}();

bool meta_path(const EmbBwdArgs& a) {
  const bool on = g_emb_inkernel_combine > 0 ||
                  (g_emb_inkernel_combine < 0 && (int64_t)a.T * a.B <= IKC_AUTO_MAX);
  return on && onehot_path(a) && a.segsort == 1 &&
         a.B % ch_for(a.D) == 0 && !(g_emb_seg_split && a.B > 2 * SEG_THREADS);
}

// What a prepare did with the optional co-launched work: the towers are
// always done by its end; the side job (reduce_adam) is done unless the
// towers rode in the sort launch (it reads their partials: then the update
// launch takes it).
struct PrepDone { bool side = false; };

template <typename K>
PrepDone prep_impl(const EmbBwdArgs& a, const WsLayout& L, hipStream_t s) {
  char* ws = (char*)a.workspace;
  K* keys_in = (K*)(ws + L.keys_in);
  K* keys_out = (K*)(ws + L.keys_out);
  int32_t* vals_in = (int32_t*)(ws + L.vals_in);
  int32_t* vals_out = (int32_t*)(ws + L.vals_out);
  int64_t* goff = (int64_t*)(ws + L.goff);
  float* gscale = (a.psw || a.mean) ? (float*)(ws + L.gscale) : nullptr;
  int32_t* tcount = (int32_t*)(ws + L.tcount);
  const int R = a.segsort;                 // runs per physical table (0: off)
  bool side_done = false;
  const bool co_tower = a.tower_on && a.tower.B > 0 && onehot_path(a) && R == 1 &&
                        a.B <= 2 * SEG_THREADS;
  if (a.tower_on && !co_tower) two_tower(a.tower, 1, s);   // first: the backward needs dX
  if (co_tower) {
    int2* meta = meta_path(a) ? (int2*)(ws + L.meta) : nullptr;
    int32_t* rcnt = (int32_t*)(ws + L.rcnt);
    const int tblocks = (two_tower_parts(a.tower.B) + TT_CO_WAVES - 1) / TT_CO_WAVES;
    hipLaunchKernelGGL((emb_segsort_tower_kernel<K>), dim3(a.T + tblocks), dim3(SEG_THREADS), 0,
                       s, a, keys_out, vals_out, goff, gscale, tcount, meta, rcnt, ch_for(a.D));
    TDFO_CHECK_HIP(hipGetLastError());
    return PrepDone{false};
  }
  if (onehot_path(a)) {
    if (R == 1) {
      int2* meta = meta_path(a) ? (int2*)(ws + L.meta) : nullptr;
      int32_t* rcnt = (int32_t*)(ws + L.rcnt);
      const int ch = ch_for(a.D);
      // side job: its units ride in extra blocks of the sort (4 per block)
      const int side_blocks =
          a.side_on ? (reduce_adam_units(a.side) + SEG_THREADS / 256 - 1) / (SEG_THREADS / 256) : 0;
      if (a.B <= 2 * SEG_THREADS) {
        hipLaunchKernelGGL((emb_segsort_kernel<K, true, 2>), dim3(a.T + side_blocks),
                           dim3(SEG_THREADS), 0, s, a, keys_out, vals_out, goff, gscale, tcount,
                           (int32_t*)nullptr, meta, rcnt, ch);
        side_done = true;
      } else if (g_emb_seg_split) {
        hipLaunchKernelGGL((emb_segsort_split_kernel<K, SEG_SPLIT>), dim3(a.T * SEG_SPLIT),
                           dim3(SEG_THREADS), 0, s, a, keys_out, vals_out, goff, gscale, tcount);
      } else {
        hipLaunchKernelGGL((emb_segsort_kernel<K, true>), dim3(a.T + side_blocks),
                           dim3(SEG_THREADS), 0, s, a, keys_out, vals_out, goff, gscale, tcount,
                           (int32_t*)nullptr, meta, rcnt, ch);
        side_done = true;
      }
    } else {
      int32_t* pos = (int32_t*)(ws + L.pos);
      hipLaunchKernelGGL((emb_segsort_kernel<K, false>), dim3(a.T), dim3(SEG_THREADS), 0, s, a, keys_in,
                         vals_in, goff, gscale, tcount, pos, (int2*)nullptr, (int32_t*)nullptr, 0);
      TDFO_CHECK_HIP(hipGetLastError());
      const int Tp = a.T / R;
      hipLaunchKernelGGL(emb_runrank_kernel<K>, dim3(a.T * (R - 1)), dim3(SEG_THREADS), 0, s, Tp,
                         R, a.B, keys_in, pos);
      TDFO_CHECK_HIP(hipGetLastError());
      int64_t sb = (a.nnz + 255) / 256;
      if (sb > 4096) sb = 4096;
      hipLaunchKernelGGL(emb_runscatter_kernel<K>, dim3(sb), dim3(256), 0, s, Tp, R, a.B,
                         keys_in, vals_in, pos, keys_out, vals_out);
    }
  } else {
    // generate where an even/odd number of passes leaves the result in *_out
    const bool odd = radix_sort_passes(a.key_bits, a.nnz) & 1;
    K* k0 = odd ? keys_in : keys_out;
    K* k1 = odd ? keys_out : keys_in;
    int32_t* v0 = odd ? vals_in : vals_out;
    int32_t* v1 = odd ? vals_out : vals_in;
    int64_t kb = (a.nnz + 255) / 256;
    if (kb > 8192) kb = 8192;
    EmbBwdArgs ak = a;
    if (ak.T > KEYS_REG_MAXT) ak.bag_len = nullptr;   // (LDS table of starts too small)
    hipLaunchKernelGGL(emb_keys_kernel<K>, dim3(kb), dim3(256), 0, s, ak, k0, v0, goff, gscale,
                       tcount);
    TDFO_CHECK_HIP(hipGetLastError());
    if constexpr (sizeof(K) == 4)
      radix_sort_pairs_u32(k0, v0, k1, v1, a.nnz, a.key_bits, ws + L.sortws, s);
    else
      radix_sort_pairs_u64(k0, v0, k1, v1, a.nnz, a.key_bits, ws + L.sortws, s);
  }
  TDFO_CHECK_HIP(hipGetLastError());
  if (a.side_on && !side_done) reduce_adam(a.side, s);     // no sort launch to ride in
  return PrepDone{true};
}

template <int D, typename K, int OPT>
void apply_impl(const EmbBwdArgs& a0, const WsLayout& L, hipStream_t s) {
  EmbBwdArgs a = a0;
  a.goff_sorted = onehot_path(a0) && a0.segsort == 1;
  char* ws = (char*)a.workspace;
  K* keys_out = (K*)(ws + L.keys_out);
  int32_t* vals_out = (int32_t*)(ws + L.vals_out);
  int64_t* goff = (int64_t*)(ws + L.goff);
  float* gscale = (a.psw || a.mean) ? (float*)(ws + L.gscale) : nullptr;
  float* head = (float*)(ws + L.head);
  float* tail = (float*)(ws + L.tail);
  int32_t* tlist = (int32_t*)(ws + L.tlist);
  int32_t* tcount = (int32_t*)(ws + L.tcount);
  const int2* meta = meta_path(a0) ? (const int2*)(ws + L.meta) : nullptr;
  int32_t* rcnt = (int32_t*)(ws + L.rcnt);
  auto run = [&](auto ch_c) {
    constexpr int CH = decltype(ch_c)::value;
    const int64_t nch = (a.nnz + CH - 1) / CH;
    int64_t blocks = (nch + 3) / 4;
    // side job (reduce_adam) left by the prepare: extra blocks of the
    // in-kernel-combine update launch, one 256-thread unit each
    const bool side_here = a.side_on && meta != nullptr;
    if (side_here) {
      a.side_block0 = (int)blocks;
      blocks += reduce_adam_units(a.side);
    } else {
      a.side_block0 = 0;
    }
#define TDFO_CK(GBV, MV, NTV)                                                              \
    hipLaunchKernelGGL((emb_chunk_kernel<D, K, GBV, OPT, CH, MV, NTV>), dim3(blocks), dim3(256), 0, \
                       s, a, keys_out, vals_out, goff, gscale, head, tail, tlist, tcount, meta, rcnt)
    // non-temporal row accesses on multi-hot batches (see row_ld)
    const bool nt = g_emb_nt && !onehot_path(a0);
    if (meta != nullptr) {
      if (a.grad_bf16) TDFO_CK(true, true, false); else TDFO_CK(false, true, false);
    } else if (nt) {
      if (a.grad_bf16) TDFO_CK(true, false, true); else TDFO_CK(false, false, true);
    } else {
      if (a.grad_bf16) TDFO_CK(true, false, false); else TDFO_CK(false, false, false);
    }
#undef TDFO_CK
    TDFO_CHECK_HIP(hipGetLastError());
    if (a.side_on && !side_here) reduce_adam(a.side, s);
    if (meta != nullptr) return;        // crossing runs finished inside the update
    int64_t cblocks = (nch + 3) / 4;
    if (cblocks > 1024) cblocks = 1024;
    int64_t* llist = (int64_t*)(ws + L.llist);
    // one id per bag (segsort = R sources): no run is longer than R x B ids
    const bool may_long =
        !(a.segsort > 0 && (int64_t)a.segsort * a.B <= (int64_t)COMBINE_LONG * CH);
    hipLaunchKernelGGL((emb_combine_kernel<D, K, OPT, CH>), dim3(cblocks), dim3(256), 0, s, a,
                       keys_out, head, tail, tlist, tcount, llist, (int)may_long);
    TDFO_CHECK_HIP(hipGetLastError());
    if (may_long) {
      // long runs: at most nch / COMBINE_LONG of them
      int64_t lblocks = nch / COMBINE_LONG + 1;
      if (lblocks > 256) lblocks = 256;
      hipLaunchKernelGGL((emb_combine_long_kernel<D, K, OPT, CH>), dim3(lblocks),
                         dim3(64 * LONG_WAVES), 0, s, a, keys_out, head, tail, tcount, llist);
      TDFO_CHECK_HIP(hipGetLastError());
    }
  };
  run(std::integral_constant<int, BwdCfg<D>::CH>{});
}

template <int D, typename K>
void bwd_opt(const EmbBwdArgs& a, const WsLayout& L, hipStream_t s) {
  switch (a.opt) {
    case EMB_SGD: apply_impl<D, K, EMB_SGD>(a, L, s); break;
    case EMB_ROWWISE_ADAGRAD: apply_impl<D, K, EMB_ROWWISE_ADAGRAD>(a, L, s); break;
    case EMB_ADAM: apply_impl<D, K, EMB_ADAM>(a, L, s); break;
    case EMB_ADAGRAD: apply_impl<D, K, EMB_ADAGRAD>(a, L, s); break;
    case EMB_DENSE_GRAD: apply_impl<D, K, EMB_DENSE_GRAD>(a, L, s); break;
    default: throw std::runtime_error("unknown embedding optimizer");
  }
}

template <int D>
void bwd_dispatch(const EmbBwdArgs& a, const WsLayout& L, hipStream_t s) {
  if (a.key_bits <= 32) bwd_opt<D, uint32_t>(a, L, s);
  else bwd_opt<D, uint64_t>(a, L, s);
}

}  // namespace

int emb_rif() {
  static const int v = [] {
    const char* e = getenv("TDFO_EMB_RIF");
    return e ? atoi(e) : 4;
  }();
  return v;
}

void embedding_bag_fwd(const EmbFwdArgs& a, hipStream_t s) {
  const int64_t nbags = (int64_t)a.T * a.B;
  if (nbags == 0) {
    bump(a.bumps, s);                 // (the counters still advance)
    return;
  }
  const int rif = emb_rif();
  const int lpb = a.D / 4 < 64 ? a.D / 4 : 64;
  const int64_t waves = (nbags * lpb + 63) / 64;
  int64_t blocks = (waves + 3) / 4;
  if (blocks > 8192) blocks = 8192;
#define TDFO_EF(DD)                                                            \
  if (a.onehot && !a.mean) {                                                   \
    if (a.out_bf16) hipLaunchKernelGGL((emb_fwd_onehot_kernel<DD, true>),      \
                                       dim3(blocks), dim3(256), 0, s, a);      \
    else hipLaunchKernelGGL((emb_fwd_onehot_kernel<DD, false>), dim3(blocks),  \
                            dim3(256), 0, s, a);                               \
  } else if (rif == 8) {                                                       \
    if (a.out_bf16) hipLaunchKernelGGL((emb_fwd_kernel<DD, true, 8>), dim3(blocks), \
                                       dim3(256), 0, s, a);                    \
    else hipLaunchKernelGGL((emb_fwd_kernel<DD, false, 8>), dim3(blocks),      \
                            dim3(256), 0, s, a);                               \
  } else if (rif == 16) {                                                      \
    if (a.out_bf16) hipLaunchKernelGGL((emb_fwd_kernel<DD, true, 16>), dim3(blocks), \
                                       dim3(256), 0, s, a);                    \
    else hipLaunchKernelGGL((emb_fwd_kernel<DD, false, 16>), dim3(blocks),     \
                            dim3(256), 0, s, a);                               \
  } else if (a.out_bf16) hipLaunchKernelGGL((emb_fwd_kernel<DD, true, 4>),     \
                                            dim3(blocks), dim3(256), 0, s, a); \
  else hipLaunchKernelGGL((emb_fwd_kernel<DD, false, 4>), dim3(blocks),        \
                          dim3(256), 0, s, a)
  switch (a.D) {
    case 16: TDFO_EF(16); break;
    case 32: TDFO_EF(32); break;
    case 64: TDFO_EF(64); break;
    case 128: TDFO_EF(128); break;
    case 256: TDFO_EF(256); break;
    case 512: TDFO_EF(512); break;
  }
#undef TDFO_EF
  TDFO_CHECK_HIP(hipGetLastError());
}

int embedding_segsort(int v) {
  const int old = g_emb_segsort;
  if (v >= 0) g_emb_segsort = v ? 1 : 0;
  return old;
}

size_t embedding_bwd_workspace(int64_t nnz, int D) {
  return ws_layout(nnz < 1 ? 1 : nnz, D).total;
}

namespace {
PrepDone prepare_any(const EmbBwdArgs& a, hipStream_t s) {
  if (a.nnz <= 0) {
    if (a.tower_on) two_tower(a.tower, 1, s);
    if (a.side_on) reduce_adam(a.side, s);
    return PrepDone{true};
  }
  const WsLayout L = ws_layout(a.nnz, a.D);
  if (a.key_bits <= 32) return prep_impl<uint32_t>(a, L, s);
  return prep_impl<uint64_t>(a, L, s);
}
}  // namespace

void embedding_bwd_fused(const EmbBwdArgs& a, hipStream_t s) {
  const PrepDone d = prepare_any(a, s);
  EmbBwdArgs b = a;
  b.tower_on = 0;
  if (d.side) b.side_on = 0;         // else the update launch takes it
  embedding_bwd_apply(b, s);
}

void embedding_bwd_prepare(const EmbBwdArgs& a, hipStream_t s) {
  const PrepDone d = prepare_any(a, s);
  if (!d.side && a.side_on) reduce_adam(a.side, s);   // (split API: nothing carried over)
}

template <typename K>
void prep_rw_impl(const EmbBwdArgs& a, const WsLayout& L, const int64_t* recv,
                  const int64_t* meta, int nrw, int W, int64_t cap, int64_t grad_ld,
                  int64_t dummy_row, int rows, hipStream_t s) {
  char* ws = (char*)a.workspace;
  K* keys_in = (K*)(ws + L.keys_in);
  K* keys_out = (K*)(ws + L.keys_out);
  int32_t* vals_in = (int32_t*)(ws + L.vals_in);
  int32_t* vals_out = (int32_t*)(ws + L.vals_out);
  int64_t* goff = (int64_t*)(ws + L.goff);
  float* gscale = a.mean ? (float*)(ws + L.gscale) : nullptr;
  int32_t* tcount = (int32_t*)(ws + L.tcount);
  const bool odd = radix_sort_passes(a.key_bits, a.nnz) & 1;
  K* k0 = odd ? keys_in : keys_out;
  K* k1 = odd ? keys_out : keys_in;
  int32_t* v0 = odd ? vals_in : vals_out;
  int32_t* v1 = odd ? vals_out : vals_in;
  int64_t kb = (a.nnz + 255) / 256;
  if (kb > 8192) kb = 8192;
  hipLaunchKernelGGL(emb_rw_keys_kernel<K>, dim3(kb), dim3(256), 0, s, a, recv, meta, nrw, W,
                     cap, grad_ld, dummy_row, rows, k0, v0, goff, gscale, tcount);
  TDFO_CHECK_HIP(hipGetLastError());
  if constexpr (sizeof(K) == 4)
    radix_sort_pairs_u32(k0, v0, k1, v1, a.nnz, a.key_bits, ws + L.sortws, s);
  else
    radix_sort_pairs_u64(k0, v0, k1, v1, a.nnz, a.key_bits, ws + L.sortws, s);
  TDFO_CHECK_HIP(hipGetLastError());
}

void embedding_bwd_prepare_rw(const EmbBwdArgs& a, const int64_t* recv, const int64_t* meta,
                              int nrw, int W, int64_t cap, int64_t grad_ld, int64_t dummy_row,
                              int rows, hipStream_t s) {
  if (a.nnz <= 0) return;
  const WsLayout L = ws_layout(a.nnz, a.D);
  if (a.key_bits <= 32)
    prep_rw_impl<uint32_t>(a, L, recv, meta, nrw, W, cap, grad_ld, dummy_row, rows, s);
  else
    prep_rw_impl<uint64_t>(a, L, recv, meta, nrw, W, cap, grad_ld, dummy_row, rows, s);
}

void embedding_dense_update(const EmbBwdArgs& a, int64_t rows, const float* grad, float* clear,
                            hipStream_t s) {
  switch (a.D) {
    case 16: dense_update_dispatch<16>(a, rows, grad, clear, s); break;
    case 32: dense_update_dispatch<32>(a, rows, grad, clear, s); break;
    case 64: dense_update_dispatch<64>(a, rows, grad, clear, s); break;
    case 128: dense_update_dispatch<128>(a, rows, grad, clear, s); break;
    case 256: dense_update_dispatch<256>(a, rows, grad, clear, s); break;
    case 512: dense_update_dispatch<512>(a, rows, grad, clear, s); break;
  }
}

void embedding_bwd_apply(const EmbBwdArgs& a, hipStream_t s) {
  if (a.nnz <= 0) {
    if (a.side_on) reduce_adam(a.side, s);
    return;
  }
  const WsLayout L = ws_layout(a.nnz, a.D);
  switch (a.D) {
    case 16: bwd_dispatch<16>(a, L, s); break;
    case 32: bwd_dispatch<32>(a, L, s); break;
    case 64: bwd_dispatch<64>(a, L, s); break;
    case 128: bwd_dispatch<128>(a, L, s); break;
    case 256: bwd_dispatch<256>(a, L, s); break;
    case 512: bwd_dispatch<512>(a, L, s); break;
  }
}

}  // namespace tdfo
