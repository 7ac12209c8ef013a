// Fused Bert4Rec transformer block, forward and backward (reference
// torchrec/models.py:11-28 MultiHeadedAttention, :75-92 PositionwiseFeedForward,
// :95-106 SublayerConnection, :109-127 TransformerBlock).
//
// At the reference shapes (T = max_len = 20, E = 16, 2 heads, FFN 4E) one
// block is ~20 dependent tensor ops on [T, E]-sized tensors per sequence;
// run as library ops each is a launch of a few microseconds doing almost no
// work. Here one 256-thread workgroup owns one sequence for the whole block,
// with every intermediate in LDS:
//
//   h1 = LN1(x)            qkv = h1 Wqkv^T + bqkv
//   ctx = MHA(qkv; key-padding mask from ids, softmax, dropout on P)
//   x1 = x + drop_a(ctx Wo^T + bo)
//   h2 = LN2(x1)           f = relu(h2 W1^T + b1)
//   x2 = x1 + drop_g(drop_f(f) W2^T + b2)        y = drop_blk(x2)
//
// Dropout masks come from the same counter hash as attention.hip (attention
// probabilities use exactly its (seed, step, b, h, i, j) stream, so the
// attention reference matches); the four sublayer sites mix a site constant
// into the seed. Nothing random is stored: the backward regenerates masks.
// The forward saves qkv, ctx, x1 and f (post-ReLU, pre-dropout); LN outputs
// are recomputed. The backward writes dx and one row of parameter-gradient
// partials per sequence ([B][P], fixed layout below); enc_reduce sums the B
// rows in order (no atomics: deterministic).
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

// threads per sequence workgroup. E = 16 (the Bert4Rec config): 1024 each
// way (backward 95 VGPRs, forward 62 with dotw unrolled 16 at a time) -- the
// phases' element loops run in one or two passes instead of four or five
// (measured vs 256 / 512: profiles/r06/notes.md); wider E keeps 256.
#ifndef TDFO_ENC_FWD_THREADS
#define TDFO_ENC_FWD_THREADS 1024
#endif
#ifndef TDFO_ENC_BWD_THREADS
#define TDFO_ENC_BWD_THREADS 1024
#endif
__host__ __device__ constexpr int enc_fwd_threads(int E) { return E == 16 ? TDFO_ENC_FWD_THREADS : 256; }
__host__ __device__ constexpr int enc_bwd_threads(int E) { return E == 16 ? TDFO_ENC_BWD_THREADS : 256; }

__device__ __forceinline__ uint32_t ehash3(uint32_t a, uint32_t b, uint32_t c) {
  // identical to attention.hip's hash3
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// dropout multiplier (0 or 1/(1-rate)) of sublayer site s at (b, t, n)
__device__ __forceinline__ float site_mul(const EncArgs& a, uint32_t sd, int site, int b, int t,
                                          int n) {
  if (a.rate <= 0.f) return 1.f;
  const uint32_t r = ehash3(sd ^ ((uint32_t)site * 0x27D4EB2Fu), (uint32_t)(b * 64 + t),
                            (uint32_t)n);
  return (float)(r >> 8) * (1.0f / 16777216.0f) >= a.rate ? 1.f / (1.f - a.rate) : 0.f;
}

// attention-probability dropout multiplier, same stream as attention.hip
__device__ __forceinline__ float prob_mul(const EncArgs& a, uint32_t sd, int b, int h, int i,
                                          int j) {
  if (a.rate <= 0.f) return 1.f;
  const uint32_t r = ehash3(sd, (uint32_t)((b * a.H + h) * 64 + i), (uint32_t)j);
  return (float)(r >> 8) * (1.0f / 16777216.0f) >= a.rate ? 1.f / (1.f - a.rate) : 0.f;
}

enum { SITE_A = 1, SITE_F = 2, SITE_G = 3, SITE_BLK = 4 };

struct POff {                    // parameter-gradient partial layout
  int wqkv, bqkv, wo, bo, g1, be1, g2, be2, w1, b1, w2, b2, P;
};
__host__ __device__ constexpr inline POff poff(int E, int FF) {
  POff o{};
  o.wqkv = 0;
  o.bqkv = o.wqkv + 3 * E * E;
  o.wo = o.bqkv + 3 * E;
  o.bo = o.wo + E * E;
  o.g1 = o.bo + E;
  o.be1 = o.g1 + E;
  o.g2 = o.be1 + E;
  o.be2 = o.g2 + E;
  o.w1 = o.be2 + E;
  o.b1 = o.w1 + FF * E;
  o.w2 = o.b1 + FF;
  o.b2 = o.w2 + E * FF;
  o.P = o.b2 + E;
  return o;
}

// Stage every block parameter into LDS in the POff layout (one coalesced
// pass): the dot-product loops then read LDS, not dependent global loads.
struct WPtr {
  const float *wqkv, *bqkv, *wo, *bo, *g1, *be1, *g2, *be2, *w1, *b1, *w2, *b2;
};
// Global -> LDS copies of several arrays with every thread's loads (K per
// array) issued before any is waited for: one memory round trip per
// K * NT elements of the longest array, not one per array / per
// loop iteration.
struct Seg {
  const float* src;
  float* dst;
  int n;
};
template <int NT, int NS, int K>
__device__ __forceinline__ void stage_multi(const Seg (&sg)[NS], int tid) {
  int nmax = 0;
#pragma unroll
  for (int q = 0; q < NS; ++q) nmax = max(nmax, sg[q].n);
  auto batch = [&](int base) {
    float v[NS][K];
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int i = base + tid + k * NT;
        v[q][k] = i < sg[q].n ? sg[q].src[i] : 0.f;
      }
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int i = base + tid + k * NT;
        if (i < sg[q].n) sg[q].dst[i] = v[q][k];
      }
  };
  // (straight-line when one batch covers everything: a loop here made the
  // compiler wait for the caller's outstanding loads at its entry)
  if (nmax <= K * NT) {
    batch(0);
  } else {
    for (int base = 0; base < nmax; base += K * NT) batch(base);
  }
}

// mid() runs between the weight loads and their LDS stores: the caller's own
// global -> LDS staging shares the same memory round trip.
template <int NT, int EC, class Mid>
__device__ __forceinline__ WPtr stage_weights(const EncArgs& a, const POff& po, float* w,
                                              int tid, Mid&& mid) {
  // Q / K / V projections from three separate tensors (a.wk != null: the
  // module's own parameters, no concatenated copy per step) or one [3E, E]
  const int E = a.E, EE = E * E;
  const bool sep = a.wk != nullptr;
  const float* src[16] = {a.wqkv, sep ? a.wk : a.wqkv + EE, sep ? a.wv : a.wqkv + 2 * EE,
                          a.bqkv, sep ? a.bk : a.bqkv + E, sep ? a.bv : a.bqkv + 2 * E,
                          a.wo, a.bo, a.g1, a.be1, a.g2, a.be2, a.w1, a.b1, a.w2, a.b2};
  const int off[17] = {po.wqkv, po.wqkv + EE, po.wqkv + 2 * EE, po.bqkv, po.bqkv + E,
                       po.bqkv + 2 * E, po.wo, po.bo, po.g1, po.be1, po.g2,
                       po.be2, po.w1, po.b1, po.w2, po.b2, po.P};
  // One flat pass over the whole layout: every thread's loads are issued
  // before the first is waited for (16 loops of their own were 16 dependent
  // memory round trips per launch).
  constexpr int NPER = (poff(EC, 4 * EC).P + NT - 1) / NT;
  float v[NPER];
#pragma unroll
  for (int k = 0; k < NPER; ++k) {
    const int i = tid + k * NT;
    v[k] = 0.f;
    if (i < po.P) {
      const float* p = src[0] + i;
#pragma unroll
      for (int q = 1; q < 16; ++q)
        if (i >= off[q]) p = src[q] + (i - off[q]);
      v[k] = *p;
    }
  }
  mid();
#pragma unroll
  for (int k = 0; k < NPER; ++k) {
    const int i = tid + k * NT;
    if (i < po.P) w[i] = v[k];
  }
  return {w + po.wqkv, w + po.bqkv, w + po.wo, w + po.bo, w + po.g1, w + po.be1,
          w + po.g2, w + po.be2, w + po.w1, w + po.b1, w + po.w2, w + po.b2};
}

// y[t][:] = LN(x[t][:]) for t < T (one thread per row); optional xhat/rstd out
template <int NT, int E>
__device__ __forceinline__ void ln_rows(const float* x, float* y, float* xhat, float* rstd_out,
                                        const float* g, const float* be, int T, float eps,
                                        int tid) {
  for (int t = tid; t < T; t += NT) {
    const float* xr = x + t * E;
    float m = 0.f;
    for (int k = 0; k < E; ++k) m += xr[k];
    m /= (float)E;
    float v = 0.f;
    for (int k = 0; k < E; ++k) {
      const float d = xr[k] - m;
      v += d * d;
    }
    const float rs = rsqrtf(v / (float)E + eps);
    for (int k = 0; k < E; ++k) {
      const float xh = (xr[k] - m) * rs;
      if (xhat) xhat[t * E + k] = xh;
      if (y) y[t * E + k] = xh * g[k] + be[k];
    }
    if (rstd_out) rstd_out[t] = rs;
  }
}

// out[t][n] = sum_k in[t][k] W[n][k] (+ bias[n]) for t < T, n < N
template <int K>
__device__ __forceinline__ float dotw(const float* in, const float* w) {
  float s[4] = {0.f, 0.f, 0.f, 0.f};          // 4 chains: LDS loads issue back to back
  // (16 at a time: a fully unrolled K = 64 product held 128 operands in
  // registers; the chain order, hence the sum, is the same either way)
#pragma unroll 16
  for (int k = 0; k < K; ++k) s[k & 3] = fmaf(in[k], w[k], s[k & 3]);
  return (s[0] + s[1]) + (s[2] + s[3]);
}

template <int E, int DK>
__global__ __launch_bounds__(enc_fwd_threads(E)) void enc_fwd_kernel(EncArgs a) {
  constexpr int ENC_FWD_THREADS = enc_fwd_threads(E);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, tid = threadIdx.x;
  constexpr int FF = 4 * E, H = E / DK, dk = DK, E3 = 3 * E;
  const int T = a.T;
  float* xs = sm;                 // [T][E]   layer input
  float* hs = xs + T * E;         // [T][E]   LN outputs
  float* qs = hs + T * E;         // [T][3E]
  float* cs = qs + T * E3;        // [T][E]   attention context
  float* x1s = cs + T * E;        // [T][E]
  float* fs = x1s + T * E;        // [T][FF]
  float* ps = fs + T * FF;        // [H][T][T] scores -> P~
  int* kv = (int*)(ps + H * T * T);  // [T]   key valid
  const POff po = poff(E, FF);
  const int64_t bo_te = (int64_t)b * T * E;
  const uint32_t step = a.step ? (uint32_t)a.step[0] : 0u;
  const WPtr W = stage_weights<ENC_FWD_THREADS, E>(a, po, (float*)(kv + T), tid, [&] {
    const int64_t id = tid < T ? a.ids[(int64_t)b * T + tid] : 0;   // (T <= 64)
    const Seg sg[1] = {{a.x + bo_te, xs, T * E}};
    stage_multi<ENC_FWD_THREADS, 1, 2048 / ENC_FWD_THREADS>(sg, tid);
    if (tid < T) kv[tid] = id != a.pad_id;
  });
  const uint32_t sd = (uint32_t)a.seed ^ (step * 0x632BE5ABu);
  __syncthreads();
  ln_rows<ENC_FWD_THREADS, E>(xs, hs, nullptr, nullptr, W.g1, W.be1, T, a.eps, tid);
  __syncthreads();
  for (int o = tid; o < T * E3; o += ENC_FWD_THREADS) {
    const int t = o / E3, n = o - t * E3;
    const float v = W.bqkv[n] + dotw<E>(hs + t * E, W.wqkv + n * E);
    qs[o] = v;
    a.qkv[(int64_t)b * T * E3 + o] = v;
  }
  __syncthreads();
  // attention, element-parallel: scores [H][T][T] -> row softmax with the
  // dropout multiplier folded in (P~) -> ctx = P~ V
  const float scale = rsqrtf((float)dk);
  for (int e = tid; e < H * T * T; e += ENC_FWD_THREADS) {
    const int h = e / (T * T), r = e - h * T * T, i = r / T, j = r - i * T;
    ps[e] = kv[j] ? dotw<DK>(qs + i * E3 + h * dk, qs + j * E3 + E + h * dk) * scale : -1e9f;
  }
  __syncthreads();
  for (int u = tid; u < H * T; u += ENC_FWD_THREADS) {
    float* row = ps + u * T;
    float mx = -3.0e38f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) mx = fmaxf(mx, row[j]);
    float sum = 0.f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) {
      const float ev = __expf(row[j] - mx);
      row[j] = ev;
      sum += ev;
    }
    const float inv = 1.f / sum;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) row[j] *= inv;
  }
  __syncthreads();
  for (int e = tid; e < H * T * T; e += ENC_FWD_THREADS) {
    const int h = e / (T * T), r = e - h * T * T, i = r / T, j = r - i * T;
    ps[e] *= prob_mul(a, sd, b, h, i, j);
  }
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_FWD_THREADS) {
    const int i = o / E, c = o - i * E, h = c / dk;
    const float* prow = ps + (h * T + i) * T;
    float acc = 0.f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) acc = fmaf(prow[j], qs[j * E3 + 2 * E + c], acc);
    cs[o] = acc;
  }
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_FWD_THREADS) {
    a.ctx[bo_te + o] = cs[o];
    const int t = o / E, n = o - t * E;
    const float v = W.bo[n] + dotw<E>(cs + t * E, W.wo + n * E);
    const float x1 = xs[o] + v * site_mul(a, sd, SITE_A, b, t, n);
    x1s[o] = x1;
    a.x1[bo_te + o] = x1;
  }
  __syncthreads();
  ln_rows<ENC_FWD_THREADS, E>(x1s, hs, nullptr, nullptr, W.g2, W.be2, T, a.eps, tid);
  __syncthreads();
  for (int o = tid; o < T * FF; o += ENC_FWD_THREADS) {
    const int t = o / FF, n = o - t * FF;
    const float v = fmaxf(W.b1[n] + dotw<E>(hs + t * E, W.w1 + n * E), 0.f);
    a.f[(int64_t)b * T * FF + o] = v;
    fs[o] = v * site_mul(a, sd, SITE_F, b, t, n);
  }
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_FWD_THREADS) {
    const int t = o / E, n = o - t * E;
    const float g = W.b2[n] + dotw<FF>(fs + t * FF, W.w2 + n * FF);
    const float x2 = x1s[o] + g * site_mul(a, sd, SITE_G, b, t, n);
    a.y[bo_te + o] = x2 * site_mul(a, sd, SITE_BLK, b, t, n);
  }
}

// LN backward for T rows: dx (+)= LN'(dh); per-column dgamma/dbeta partials
template <int NT, int E>
__device__ __forceinline__ void ln_bwd_rows(const float* xhat, const float* rstd, const float* dh,
                                            const float* g, float* dx, int T, int tid) {
  for (int t = tid; t < T; t += NT) {
    float m1 = 0.f, m2 = 0.f;
    for (int k = 0; k < E; ++k) {
      const float dxh = dh[t * E + k] * g[k];
      m1 += dxh;
      m2 += dxh * xhat[t * E + k];
    }
    m1 /= (float)E;
    m2 /= (float)E;
    for (int k = 0; k < E; ++k) {
      const float dxh = dh[t * E + k] * g[k];
      dx[t * E + k] += rstd[t] * (dxh - m1 - xhat[t * E + k] * m2);
    }
  }
}

template <int E, int DK>
__global__ __launch_bounds__(enc_bwd_threads(E)) void enc_bwd_kernel(EncArgs a) {
  constexpr int ENC_BWD_THREADS = enc_bwd_threads(E);
  if ((int)blockIdx.x >= a.B) {        // a parked reduction's extra blocks (no barrier)
    enc_red_col(a.red, ((int)blockIdx.x - a.B) * ENC_BWD_THREADS + (int)threadIdx.x);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, tid = threadIdx.x;
  constexpr int FF = 4 * E, H = E / DK, dk = DK, E3 = 3 * E;
  const int T = a.T;
  const POff po = poff(E, FF);
  float* part = a.part + (int64_t)b * po.P;
  float* dxs = sm;                // [T][E]   running dx (dx1, then dx0)
  float* ts = dxs + T * E;        // [T][E]   temp (dg, then da)
  float* hs = ts + T * E;         // [T][E]   LN output (h2, then h1)
  float* xh = hs + T * E;         // [T][E]   LN xhat
  float* dh = xh + T * E;         // [T][E]   grad wrt LN output
  float* cs = dh + T * E;         // [T][E]   ctx, then dctx
  float* rs = cs + T * E;         // [T]      LN rstd
  float* fs = rs + T;             // [T][FF]  dropped f
  float* dfs = fs + T * FF;       // [T][FF]  df
  float* qs = dfs + T * FF;       // [T][3E]
  float* dq = qs + T * E3;        // [T][3E]
  float* pt = dq + T * E3;        // [H][T][T] dropped probabilities P~
  float* ds = pt + H * T * T;     // [H][T][T] dS
  float* rdot = ds + H * T * T;   // [H][T]  sum_j P dP
  float* x0s = rdot + H * T;      // [T][E]  layer input x0
  int* kv = (int*)(x0s + T * E);
  const int64_t bo_te = (int64_t)b * T * E;
  const uint32_t step = a.step ? (uint32_t)a.step[0] : 0u;
  // the weights and every saved activation the block reads, staged in one
  // round trip: dy (-> dxs), f (-> fs), x1 (LN2 input, -> hs), ctx (-> cs),
  // qkv (-> qs), x0 (LN1 input, -> x0s), ids (-> key-valid flags)
  const WPtr W = stage_weights<ENC_BWD_THREADS, E>(a, po, (float*)(kv + T), tid, [&] {
    const int64_t id = tid < T ? a.ids[(int64_t)b * T + tid] : 0;   // (T <= 64)
    const Seg sg[6] = {{a.dy + bo_te, dxs, T * E},
                       {a.f + (int64_t)b * T * FF, fs, T * FF},
                       {a.x1 + bo_te, hs, T * E},
                       {a.ctx + bo_te, cs, T * E},
                       {a.qkv + (int64_t)b * T * E3, qs, T * E3},
                       {a.x + bo_te, x0s, T * E}};
    stage_multi<ENC_BWD_THREADS, 6, 2048 / ENC_BWD_THREADS>(sg, tid);
    if (tid < T) kv[tid] = id != a.pad_id;
  });
  const uint32_t sd = (uint32_t)a.seed ^ (step * 0x632BE5ABu);
  __syncthreads();
  // block dropout, then the FFN residual: dx1 = dx2, dg = drop_g'(dx2)
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int t = o / E, n = o - t * E;
    const float d2 = dxs[o] * site_mul(a, sd, SITE_BLK, b, t, n);
    dxs[o] = d2;
    ts[o] = d2 * site_mul(a, sd, SITE_G, b, t, n);
  }
  for (int o = tid; o < T * FF; o += ENC_BWD_THREADS) {
    const int t = o / FF, n = o - t * FF;
    fs[o] *= site_mul(a, sd, SITE_F, b, t, n);
  }
  __syncthreads();
  // W2 grads; dfd = dg W2 -> df (dropout f, ReLU mask); LN2 recompute
  for (int o = tid; o < E * FF; o += ENC_BWD_THREADS) {
    const int n = o / FF, k = o - n * FF;
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s = fmaf(ts[t * E + n], fs[t * FF + k], s);
    part[po.w2 + o] = s;
  }
  for (int n = tid; n < E; n += ENC_BWD_THREADS) {
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s += ts[t * E + n];
    part[po.b2 + n] = s;
  }
  for (int o = tid; o < T * FF; o += ENC_BWD_THREADS) {
    const int t = o / FF, k = o - t * FF;
    float s = 0.f;
    for (int n = 0; n < E; ++n) s = fmaf(ts[t * E + n], W.w2[n * FF + k], s);
    // ReLU mask from the dropped f: f >= 0, and where the dropout multiplier
    // is 0 (fs = 0 although f > 0) the product below is 0 anyway
    dfs[o] = fs[o] > 0.f ? s * site_mul(a, sd, SITE_F, b, t, k) : 0.f;
  }
  ln_rows<ENC_BWD_THREADS, E>(hs, nullptr, xh, rs, W.g2, W.be2, T, a.eps, tid);     // xhat2, rstd2
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int k = o % E;
    hs[o] = xh[o] * W.g2[k] + W.be2[k];                             // h2
  }
  __syncthreads();
  // W1 grads; dh2 = df W1
  for (int o = tid; o < FF * E; o += ENC_BWD_THREADS) {
    const int n = o / E, k = o - n * E;
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s = fmaf(dfs[t * FF + n], hs[t * E + k], s);
    part[po.w1 + o] = s;
  }
  for (int n = tid; n < FF; n += ENC_BWD_THREADS) {
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s += dfs[t * FF + n];
    part[po.b1 + n] = s;
  }
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int t = o / E, k = o - t * E;
    float s = 0.f;
    for (int n = 0; n < FF; ++n) s = fmaf(dfs[t * FF + n], W.w1[n * E + k], s);
    dh[o] = s;
  }
  __syncthreads();
  for (int k = tid; k < E; k += ENC_BWD_THREADS) {
    float sg = 0.f, sb = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) {
      sg = fmaf(dh[t * E + k], xh[t * E + k], sg);
      sb += dh[t * E + k];
    }
    part[po.g2 + k] = sg;
    part[po.be2 + k] = sb;
  }
  ln_bwd_rows<ENC_BWD_THREADS, E>(xh, rs, dh, W.g2, dxs, T, tid);                    // dx1 += LN2'(dh2)
  __syncthreads();
  // attention-out dropout; Wo grads; dctx = da Wo
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int t = o / E, n = o - t * E;
    ts[o] = dxs[o] * site_mul(a, sd, SITE_A, b, t, n);
  }
  __syncthreads();
  for (int o = tid; o < E * E; o += ENC_BWD_THREADS) {
    const int n = o / E, k = o - n * E;
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s = fmaf(ts[t * E + n], cs[t * E + k], s);
    part[po.wo + o] = s;
  }
  for (int n = tid; n < E; n += ENC_BWD_THREADS) {
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s += ts[t * E + n];
    part[po.bo + n] = s;
  }
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int t = o / E, k = o - t * E;
    float s = 0.f;
    for (int n = 0; n < E; ++n) s = fmaf(ts[t * E + n], W.wo[n * E + k], s);
    cs[o] = s;                                                      // dctx
  }
  __syncthreads();
  // attention backward, element-parallel over [H][T][T] and [T][E]
  const float scale = rsqrtf((float)dk);
  for (int e = tid; e < H * T * T; e += ENC_BWD_THREADS) {
    const int h = e / (T * T), r = e - h * T * T, i = r / T, j = r - i * T;
    pt[e] = kv[j] ? dotw<DK>(qs + i * E3 + h * dk, qs + j * E3 + E + h * dk) * scale : -1e9f;
    ds[e] = prob_mul(a, sd, b, h, i, j) *
            dotw<DK>(cs + i * E + h * dk, qs + j * E3 + 2 * E + h * dk);          // dP
  }
  __syncthreads();
  for (int u = tid; u < H * T; u += ENC_BWD_THREADS) {       // P rows, rowdot = sum_j P dP
    float* prow = pt + u * T;
    const float* drow = ds + u * T;
    float mx = -3.0e38f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) mx = fmaxf(mx, prow[j]);
    float sum = 0.f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) {
      const float ev = __expf(prow[j] - mx);
      prow[j] = ev;
      sum += ev;
    }
    const float inv = 1.f / sum;
    float dot = 0.f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) {
      prow[j] *= inv;
      dot = fmaf(prow[j], drow[j], dot);
    }
    rdot[u] = dot;
  }
  __syncthreads();
  for (int e = tid; e < H * T * T; e += ENC_BWD_THREADS) {   // dS; P -> P~
    const int h = e / (T * T), r = e - h * T * T, i = r / T, j = r - i * T;
    const float p = pt[e];
    // masked keys hold a constant score (masked_fill): no gradient through them
    ds[e] = kv[j] ? p * (ds[e] - rdot[h * T + i]) * scale : 0.f;
    pt[e] = p * prob_mul(a, sd, b, h, i, j);
  }
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {       // dq, dk, dv
    const int i = o / E, c = o - i * E, h = c / dk;
    float aq = 0.f, ak = 0.f, av = 0.f;
    #pragma unroll 4
    for (int j = 0; j < T; ++j) {
      aq = fmaf(ds[(h * T + i) * T + j], qs[j * E3 + E + c], aq);
      ak = fmaf(ds[(h * T + j) * T + i], qs[j * E3 + c], ak);
      av = fmaf(pt[(h * T + j) * T + i], cs[j * E + c], av);
    }
    dq[i * E3 + c] = aq;
    dq[i * E3 + E + c] = ak;
    dq[i * E3 + 2 * E + c] = av;
  }
  // LN1 recompute from x0
  __syncthreads();
  ln_rows<ENC_BWD_THREADS, E>(x0s, nullptr, xh, rs, W.g1, W.be1, T, a.eps, tid);
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int k = o % E;
    hs[o] = xh[o] * W.g1[k] + W.be1[k];                             // h1
  }
  __syncthreads();
  // Wqkv grads; dh1 = dqkv Wqkv
  for (int o = tid; o < E3 * E; o += ENC_BWD_THREADS) {
    const int n = o / E, k = o - n * E;
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s = fmaf(dq[t * E3 + n], hs[t * E + k], s);
    part[po.wqkv + o] = s;
  }
  for (int n = tid; n < E3; n += ENC_BWD_THREADS) {
    float s = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) s += dq[t * E3 + n];
    part[po.bqkv + n] = s;
  }
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) {
    const int t = o / E, k = o - t * E;
    float s = 0.f;
    for (int n = 0; n < E3; ++n) s = fmaf(dq[t * E3 + n], W.wqkv[n * E + k], s);
    dh[o] = s;
  }
  __syncthreads();
  for (int k = tid; k < E; k += ENC_BWD_THREADS) {
    float sg = 0.f, sb = 0.f;
    #pragma unroll 4
    for (int t = 0; t < T; ++t) {
      sg = fmaf(dh[t * E + k], xh[t * E + k], sg);
      sb += dh[t * E + k];
    }
    part[po.g1 + k] = sg;
    part[po.be1 + k] = sb;
  }
  ln_bwd_rows<ENC_BWD_THREADS, E>(xh, rs, dh, W.g1, dxs, T, tid);                    // dx0 = dx1 + LN1'(dh1)
  __syncthreads();
  for (int o = tid; o < T * E; o += ENC_BWD_THREADS) a.dx[bo_te + o] = dxs[o];
}

// grad[c] = sum_b part[b][c], fixed order (loads in flight together)
__global__ __launch_bounds__(256) void enc_reduce_kernel(EncRedJob j) {
  enc_red_col(j, (int)(blockIdx.x * 256 + threadIdx.x));
}

thread_local EncRedJob g_red{};
thread_local bool g_red_on = false;

size_t fwd_smem(const EncArgs& a) {
  const int T = a.T, E = a.E, FF = a.FF;
  return (size_t)(T * E * 4 + T * 3 * E + T * FF + a.H * T * T + T + poff(E, FF).P) * 4;
}

size_t bwd_smem(const EncArgs& a) {
  const int T = a.T, E = a.E, FF = a.FF, H = a.H;
  return (size_t)(T * E * 7 + T + 2 * T * FF + 2 * T * 3 * E + 2 * H * T * T + H * T + T +
                  poff(E, FF).P) * 4;
}

bool shape_ok(int E, int H) {
  if (H < 1 || E % H != 0) return false;
  const int dk = E / H;
  return (E == 16 || E == 32 || E == 64) && (dk == 4 || dk == 8 || dk == 16 || dk == 32);
}

void check(const EncArgs& a) {
  if (a.T < 1 || a.T > 64 || !shape_ok(a.E, a.H) || a.FF != 4 * a.E ||
      bwd_smem(a) > 160 * 1024 || fwd_smem(a) > 160 * 1024)
    throw std::runtime_error(
        "encoder_layer: unsupported shape (E in {16,32,64}, d_k in {4..32}, FF = 4E, T <= 64)");
}

template <bool BWD>
void launch(const EncArgs& a, size_t sm, hipStream_t s) {
  const int dk = a.E / a.H;
#define TDFO_ENC(EE, DD)                                                                   \
  if (a.E == EE && dk == DD) {                                                             \
    const void* fn = BWD ? (const void*)enc_bwd_kernel<EE, DD> : (const void*)enc_fwd_kernel<EE, DD>; \
    static bool attr = false;                                                              \
    if (!attr) {                                                                           \
      TDFO_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                         160 * 1024));                                     \
      attr = true;                                                                         \
    }                                                                                      \
    if (BWD) hipLaunchKernelGGL((enc_bwd_kernel<EE, DD>),                                   \
                                dim3(a.B + (a.red_on ? (a.red.P + enc_bwd_threads(EE) - 1) /     \
                                                           enc_bwd_threads(EE) : 0)),            \
                                dim3(enc_bwd_threads(EE)), sm, s, a);                            \
    else hipLaunchKernelGGL((enc_fwd_kernel<EE, DD>), dim3(a.B), dim3(enc_fwd_threads(EE)), sm, s, a);     \
    return;                                                                                \
  }
  TDFO_ENC(16, 4) TDFO_ENC(16, 8) TDFO_ENC(16, 16)
  TDFO_ENC(32, 4) TDFO_ENC(32, 8) TDFO_ENC(32, 16) TDFO_ENC(32, 32)
  TDFO_ENC(64, 4) TDFO_ENC(64, 8) TDFO_ENC(64, 16) TDFO_ENC(64, 32)
#undef TDFO_ENC
  throw std::runtime_error("encoder_layer: no kernel for this shape");
}

}  // namespace

int encoder_param_count(int E, int FF) { return poff(E, FF).P; }

bool encoder_layer_supported(int T, int E, int H, int FF) {
  EncArgs a{};
  a.T = T; a.E = E; a.H = H; a.FF = FF;
  try {
    check(a);
  } catch (const std::exception&) {
    return false;
  }
  return true;
}

void encoder_layer_fwd(const EncArgs& a, hipStream_t s) {
  check(a);
  if (a.B <= 0) return;
  launch<false>(a, fwd_smem(a), s);
  TDFO_CHECK_HIP(hipGetLastError());
}

bool encoder_reduce_take(EncRedJob* j) {
  if (!g_red_on) return false;
  *j = g_red;
  g_red_on = false;
  return true;
}

void encoder_reduce_flush(hipStream_t s) {
  EncRedJob j;
  if (!encoder_reduce_take(&j)) return;
  hipLaunchKernelGGL(enc_reduce_kernel, dim3((j.P + 255) / 256), dim3(256), 0, s, j);
  TDFO_CHECK_HIP(hipGetLastError());
}

void encoder_layer_bwd(const EncArgs& a, float* grad, hipStream_t s, const int64_t* gidx,
                       bool defer) {
  check(a);
  if (a.B <= 0) return;
  EncArgs b = a;
  b.red_on = encoder_reduce_take(&b.red) ? 1 : 0;     // the previous layer's reduction
  launch<true>(b, bwd_smem(b), s);
  TDFO_CHECK_HIP(hipGetLastError());
  const EncRedJob mine{a.part, a.B, poff(a.E, a.FF).P, grad, gidx};
  if (defer) {
    g_red = mine;
    g_red_on = true;
    return;
  }
  hipLaunchKernelGGL(enc_reduce_kernel, dim3((mine.P + 255) / 256), dim3(256), 0, s, mine);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
