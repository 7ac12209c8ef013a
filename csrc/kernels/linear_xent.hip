// Fused output projection + label-smoothed cross-entropy (fwd AND bwd)
// without materialising the [tokens, V] logits (gfx950).
//
// Reference: Bert4Rec `self.out = nn.Linear(E, V)` (torchrec/models.py:206,
// 223) followed by CrossEntropyLoss(ignore_index=0, label_smoothing=0.1)
// (torchrec/train.py:93,99-101). With V = n_items + 2 (millions of books)
// the reference writes and re-reads a [B*T, V] fp32 logits tensor; here:
//
//   compact : valid tokens (label != ignore) -> idx[], n_valid (device)
//   pass1   : grid (vocab split s, 128-token block); one wave per block runs
//             a flash-attention-style pass on the f32-input MFMA
//             (v_mfma_f32_16x16x4_f32, exact f32): per 16-row W tile and
//             16-token group, X = W H^T (bias as the C input), a per-token
//             running max (shared by the 4 lane rows), P = e^{X-m}, and
//             O^T += W^T P^T with P taken straight from the accumulator
//             registers -> part[token][s] = (m, sum, O); block-row 0 also
//             emits sum_v W_v, sum_v b_v
//   merge   : one 256-thread block per token merges the splits: lse, loss,
//             dH = scale * (E_p[W] - (1-eps) W_y - eps/V sum_v W_v)
//   wgrad   : one wave per run of 16-row tiles: X^T = H W^T on the MFMA,
//             dz = scale * (e^{z-lse} - eps/V - (1-eps)[v==y]) in registers,
//             dW^T += H^T dz^T on the MFMA, db_v = sum_n dz (no atomics)
//   (impl 0 keeps the earlier VALU pass1/wgrad: lane = token / lane = row,
//    W or H rows through scalar loads — an A/B point for the MFMA path.)
//
// loss_n = lse - (1-eps) z_y - eps * mean_v z_v, mean_v z_v = (H.sumW + sumb)/V;
// scale = 1 / n_valid (mean over non-ignored tokens, torch semantics).
#include "tdfo_common.h"
#include "tdfo_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace tdfo {
namespace {

constexpr int XE = 16;          // hidden width (embed_dim)
constexpr int XP = 20;          // partial record: m, s, acc[16], pad

__global__ __launch_bounds__(1024) void xent_compact_kernel(const int64_t* __restrict__ labels,
                                                            int N, int ignore,
                                                            int32_t* __restrict__ idx,
                                                            int32_t* __restrict__ count,
                                                            float* __restrict__ dH,
                                                            float* __restrict__ lossv) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) base = 0;
  __syncthreads();
  for (int s0 = 0; s0 < N; s0 += 1024) {
    const int j = s0 + t;
    const bool v = j < N && labels[j] != ignore;
    if (j < N && !v) {
      lossv[j] = 0.f;
#pragma unroll
      for (int k = 0; k < XE; k += 4) *(float4*)(dH + (int64_t)j * XE + k) = make_float4(0, 0, 0, 0);
    }
    const uint64_t bal = __ballot(v);
    const int pre = __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int q = 0; q < w; ++q) off += wsum[q];
    if (v) idx[off + pre] = j;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int q = 0; q < 16; ++q) tot += wsum[q];
      base += tot;
    }
    __syncthreads();
  }
  if (t == 0) *count = base;
}

// One wave per block: lane = token. W rows are wave-uniform, so they come
// through scalar loads (s_load_dwordx16, SGPR operands of the FMAs) — no LDS
// broadcast, which would cost 4 ds_read_b128 (32 LDS clocks) per row.
__global__ __launch_bounds__(64) void xent_pass1_kernel(const float* __restrict__ H,
                                                        const float* __restrict__ W,
                                                        const float* __restrict__ bias, int64_t V,
                                                        int64_t VS, int S,
                                                        const int32_t* __restrict__ idx,
                                                        const int32_t* __restrict__ count,
                                                        float* __restrict__ part,
                                                        float* __restrict__ wpart) {
  const int s = blockIdx.x, chunk = blockIdx.y, t = threadIdx.x;
  const int nv = *count;
  const int64_t v0 = (int64_t)s * VS, v1 = min(V, v0 + VS);
  if (chunk == 0 && t <= XE) {      // column sums of [W | b] over this split
    float a = 0.f;
    if (t < XE)
      for (int64_t r = v0; r < v1; ++r) a += W[r * XE + t];
    else
      for (int64_t r = v0; r < v1; ++r) a += bias[r];
    wpart[(int64_t)s * (XE + 1) + t] = a;
  }
  if (chunk * 64 >= nv) return;
  const int j = chunk * 64 + t;
  const bool valid = j < nv;
  float h[XE];
  const float* hr = H + (int64_t)idx[valid ? j : 0] * XE;
#pragma unroll
  for (int k = 0; k < XE; k += 4) {
    const float4 q = *(const float4*)(hr + k);
    h[k] = q.x; h[k + 1] = q.y; h[k + 2] = q.z; h[k + 3] = q.w;
  }
  float m = -INFINITY, sum = 0.f, acc[XE];
#pragma unroll
  for (int k = 0; k < XE; ++k) acc[k] = 0.f;
  // 4 rows per iteration: 4 scalar row loads in flight, one rescale check
  int64_t r = v0;
  for (; r + 4 <= v1; r += 4) {
    float z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* wr = W + (r + q) * XE;     // uniform -> scalar loads
      float a = bias[r + q];
#pragma unroll
      for (int k = 0; k < XE; ++k) a = fmaf(wr[k], h[k], a);
      z[q] = a;
    }
    const float zm = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
    if (zm > m) {
      const float c = __expf(m - zm);
      sum *= c;
#pragma unroll
      for (int k = 0; k < XE; ++k) acc[k] *= c;
      m = zm;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* wr = W + (r + q) * XE;
      const float e = __expf(z[q] - m);
      sum += e;
#pragma unroll
      for (int k = 0; k < XE; ++k) acc[k] = fmaf(e, wr[k], acc[k]);
    }
  }
  for (; r < v1; ++r) {
    const float* wr = W + r * XE;
    float z = bias[r];
#pragma unroll
    for (int k = 0; k < XE; ++k) z = fmaf(wr[k], h[k], z);
    if (z > m) {
      const float c = __expf(m - z);
      sum *= c;
#pragma unroll
      for (int k = 0; k < XE; ++k) acc[k] *= c;
      m = z;
    }
    const float e = __expf(z - m);
    sum += e;
#pragma unroll
    for (int k = 0; k < XE; ++k) acc[k] = fmaf(e, wr[k], acc[k]);
  }
  if (valid) {
    float* p = part + ((int64_t)j * S + s) * XP;
    p[0] = m;
    p[1] = sum;
#pragma unroll
    for (int k = 0; k < XE; ++k) p[2 + k] = acc[k];
  }
}

// One 256-thread block per valid token: threads stride over the splits,
// then a wave shuffle + LDS combine of the online-softmax states.
__device__ __forceinline__ void sm_combine(float& m, float& s, float* acc, float om, float os,
                                           const float* oacc) {
  const float nm = fmaxf(m, om);
  const float c0 = (m == -INFINITY) ? 0.f : __expf(m - nm);
  const float c1 = (om == -INFINITY) ? 0.f : __expf(om - nm);
  s = s * c0 + os * c1;
#pragma unroll
  for (int k = 0; k < XE; ++k) acc[k] = acc[k] * c0 + oacc[k] * c1;
  m = nm;
}

__global__ __launch_bounds__(256) void xent_merge_kernel(const float* __restrict__ H,
                                                         const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const int64_t* __restrict__ labels,
                                                         int64_t V, int S, float eps,
                                                         const int32_t* __restrict__ idx,
                                                         const int32_t* __restrict__ count,
                                                         const float* __restrict__ part,
                                                         const float* __restrict__ wpart,
                                                         float* __restrict__ lse_out,
                                                         float* __restrict__ dH,
                                                         float* __restrict__ lossv,
                                                         float* __restrict__ htok,
                                                         int32_t* __restrict__ ytok) {
  __shared__ float red[4][XP + XE + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = blockIdx.x;
  const int nv = *count;
  if (j >= nv) return;
  const float scale = 1.f / (float)max(1, nv);
  float m = -INFINITY, sum = 0.f, acc[XE], ws[XE + 1];
#pragma unroll
  for (int k = 0; k < XE; ++k) acc[k] = 0.f;
#pragma unroll
  for (int k = 0; k <= XE; ++k) ws[k] = 0.f;
  const float* p0 = part + (int64_t)j * S * XP;
  // XMU splits' loads issued together, then combined in split order (one
  // memory round trip per XMU splits instead of per split)
  constexpr int XMU = 4;
  for (int s0 = tid; s0 < S; s0 += XMU * 256) {
    float r[XMU][XP], wv[XMU][XE + 1];
#pragma unroll
    for (int u = 0; u < XMU; ++u) {
      const int s = s0 + u * 256;
      if (s < S) {
        const f32x4_t* p = (const f32x4_t*)(p0 + (int64_t)s * XP);
#pragma unroll
        for (int q = 0; q < XP / 4; ++q) {
          const f32x4_t v = p[q];
          r[u][4 * q] = v[0]; r[u][4 * q + 1] = v[1]; r[u][4 * q + 2] = v[2];
          r[u][4 * q + 3] = v[3];
        }
        const float* wp = wpart + (int64_t)s * (XE + 1);
#pragma unroll
        for (int k = 0; k <= XE; ++k) wv[u][k] = wp[k];
      } else {
        r[u][0] = -INFINITY;
#pragma unroll
        for (int k = 0; k <= XE; ++k) wv[u][k] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < XMU; ++u) {
      if (r[u][0] != -INFINITY) sm_combine(m, sum, acc, r[u][0], r[u][1], r[u] + 2);
#pragma unroll
      for (int k = 0; k <= XE; ++k) ws[k] += wv[u][k];
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    float o[XE];
#pragma unroll
    for (int k = 0; k < XE; ++k) o[k] = __shfl_xor(acc[k], off);
    sm_combine(m, sum, acc, __shfl_xor(m, off), __shfl_xor(sum, off), o);
  }
#pragma unroll
  for (int k = 0; k <= XE; ++k) ws[k] = wave_sum(ws[k]);
  if (lane == 0) {
    red[w][0] = m;
    red[w][1] = sum;
#pragma unroll
    for (int k = 0; k < XE; ++k) red[w][2 + k] = acc[k];
#pragma unroll
    for (int k = 0; k <= XE; ++k) red[w][XP + k] = ws[k];
  }
  __syncthreads();
  if (tid != 0) return;
  for (int q = 1; q < 4; ++q) {
    sm_combine(m, sum, acc, red[q][0], red[q][1], &red[q][2]);
#pragma unroll
    for (int k = 0; k <= XE; ++k) ws[k] += red[q][XP + k];
  }
  const int n = idx[j];
  const float* hr = H + (int64_t)n * XE;
  int64_t y = labels[n];
  if (y < 0 || y >= V) y = 0;   // host validates; never read out of bounds
  ytok[j] = (int32_t)y;
#pragma unroll
  for (int k = 0; k < XE; k += 4) *(f32x4_t*)(htok + (int64_t)j * XE + k) = *(const f32x4_t*)(hr + k);
  const float* wy = W + y * XE;
  float zy = bias[y], zmean = ws[XE];
#pragma unroll
  for (int k = 0; k < XE; ++k) {
    zy = fmaf(wy[k], hr[k], zy);
    zmean = fmaf(ws[k], hr[k], zmean);
  }
  zmean /= (float)V;
  const float lse = m + __logf(sum);
  lse_out[j] = lse;
  lossv[n] = lse - (1.f - eps) * zy - eps * zmean;
  const float inv = 1.f / sum;
#pragma unroll
  for (int k = 0; k < XE; k += 4) {
    float d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      d[e] = scale * (acc[k + e] * inv - (1.f - eps) * wy[k + e] - eps * ws[k + e] / (float)V);
    *(float4*)(dH + (int64_t)n * XE + k) = make_float4(d[0], d[1], d[2], d[3]);
  }
}

// One thread per vocab row; the tokens are wave-uniform (scalar loads of
// idx, H row, lse and label), so the loop body is pure VALU.
__global__ __launch_bounds__(256) void xent_wgrad_kernel(const float* __restrict__ H,
                                                         const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const int64_t* __restrict__ labels,
                                                         int64_t V, float eps,
                                                         const int32_t* __restrict__ idx,
                                                         const int32_t* __restrict__ count,
                                                         const float* __restrict__ lse,
                                                         float* __restrict__ dW,
                                                         float* __restrict__ db) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = v < V;
  const int64_t vr = valid ? v : V - 1;
  const int nv = *count;
  const float scale = 1.f / (float)max(1, nv);
  const float off = eps / (float)V, hit = 1.f - eps;
  float w[XE], g[XE], gb = 0.f;
#pragma unroll
  for (int k = 0; k < XE; k += 4) {
    const float4 q = *(const float4*)(W + vr * XE + k);
    w[k] = q.x; w[k + 1] = q.y; w[k + 2] = q.z; w[k + 3] = q.w;
  }
  const float b = bias[vr];
#pragma unroll
  for (int k = 0; k < XE; ++k) g[k] = 0.f;
#pragma unroll 2
  for (int j = 0; j < nv; ++j) {
    const int n = idx[j];
    const float* hr = H + (int64_t)n * XE;     // uniform -> scalar loads
    const float l = lse[j];
    const int64_t y = labels[n];
    float z = b;
#pragma unroll
    for (int k = 0; k < XE; ++k) z = fmaf(w[k], hr[k], z);
    float dz = __expf(z - l) - off;
    if (y == v) dz -= hit;
    dz *= scale;
    gb += dz;
#pragma unroll
    for (int k = 0; k < XE; ++k) g[k] = fmaf(dz, hr[k], g[k]);
  }
  if (valid) {
#pragma unroll
    for (int k = 0; k < XE; k += 4)
      *(float4*)(dW + v * XE + k) = make_float4(g[k], g[k + 1], g[k + 2], g[k + 3]);
    db[v] = gb;
  }
}


// ------------------------------------------------------------ MFMA path --
// v_mfma_f32_16x16x4_f32 lane maps (16x16 tiles, lane l: t = l&15, g = l>>4):
// A[i=t][k=g], B[k=g][j=t], C/D[row 4g+r][col t]. The hidden dim (16) is the
// contraction of the first product; it is walked as k-step s <-> dim 4g+s, so
// every W/H operand of it is one float4 per lane.
constexpr int XG = 8;           // 16-token groups per wave (128 tokens)
// Logits are produced in log2 units (H and b pre-scaled by log2 e), so every
// softmax term is one v_sub + v_exp_f32.
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float max4rows(float v) {     // max over lanes t, t+16, t+32, t+48
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

__device__ __forceinline__ float sum4rows(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

struct XentTile {               // one 16-row W tile in both operand layouts
  f32x4_t wa;                   // W[r0+t][4g..4g+3]
  float wb[4];                  // W[r0+4g+r][t]
  float bb[4];                  // bias[r0+4g+r]
};

__device__ __forceinline__ void xent_load_tile(XentTile& T, const float* __restrict__ W,
                                               const float* __restrict__ bias, int64_t r0,
                                               int64_t v1, int t, int g) {
  const int64_t ra = min(r0 + t, v1 - 1);
  T.wa = *(const f32x4_t*)(W + ra * XE + 4 * g);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t rb = min(r0 + 4 * g + r, v1 - 1);
    T.wb[r] = W[rb * XE + t];
    T.bb[r] = bias[rb];
  }
}

// Lazy rescaling: the running max m (log2 units) only moves when a logit
// exceeds it by more than XTH (2^12 headroom keeps p and the sums far from
// overflow); the (m, sum, O) triple is consistent for any m, so the merge is
// unaffected.
constexpr float XTH = 12.f;

// One 16-row tile of the online softmax for NG token groups: X = W H^T (bias
// as C input), lazy max update, P = 2^{X-m}, O^T += W^T P^T.
template <int NG>
__device__ __forceinline__ void xent_pass1_tile(const XentTile& T, const f32x4_t* hb,
                                                const float* bb, f32x4_t* o, float* m,
                                                float* sum) {
  f32x4_t x[NG];
  bool up = false;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    x[q] = (f32x4_t){bb[0], bb[1], bb[2], bb[3]};
    x[q] = mfma4(T.wa[0], hb[q][0], x[q]);
    x[q] = mfma4(T.wa[1], hb[q][1], x[q]);
    x[q] = mfma4(T.wa[2], hb[q][2], x[q]);
    x[q] = mfma4(T.wa[3], hb[q][3], x[q]);
    up |= fmaxf(fmaxf(x[q][0], x[q][1]), fmaxf(x[q][2], x[q][3])) > m[q] + XTH;
  }
  if (__any(up)) {                         // wave-uniform; first tile and rare after
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const float mx = max4rows(fmaxf(fmaxf(x[q][0], x[q][1]), fmaxf(x[q][2], x[q][3])));
      const float nm = fmaxf(m[q], mx);     // finite: row r0 of a tile is always valid
      const float c = exp2_fast(m[q] - nm);
      sum[q] *= c;
      o[q] *= c;
      m[q] = nm;
    }
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    float p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = exp2_fast(x[q][r] - m[q]);
    sum[q] += (p[0] + p[1]) + (p[2] + p[3]);
    o[q] = mfma4(T.wb[0], p[0], o[q]);
    o[q] = mfma4(T.wb[1], p[1], o[q]);
    o[q] = mfma4(T.wb[2], p[2], o[q]);
    o[q] = mfma4(T.wb[3], p[3], o[q]);
  }
}

// Full tiles: a wave-uniform tile pointer plus constant per-lane offsets
// (no clamps, no masks), two tiles per iteration from a 2-slot register ring.
__device__ __forceinline__ void xent_load_full(XentTile& T, const float* __restrict__ Wt,
                                               const float* __restrict__ bt, int la, int t, int g) {
  T.wa = *(const f32x4_t*)(Wt + la);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    T.wb[r] = Wt[(4 * g + r) * XE + t];
    T.bb[r] = bt[4 * g + r];
  }
}

// Column sums of [W | b] over one vocabulary split (the label-smoothing term's
// sum of logits is h . colsum(W) + sum(b)).
__device__ __forceinline__ void xent_colsums(const float* __restrict__ W,
                                             const float* __restrict__ bias, int64_t v0,
                                             int64_t v1, float* __restrict__ wp, int t, int g,
                                             int l) {
  f32x4_t cs = {0.f, 0.f, 0.f, 0.f};
  float bs = 0.f;
  // (unrolled: 8 row loads in flight per lane, not one memory round trip
  // per row; the sums keep their sequential order)
#pragma unroll 8
  for (int64_t r = v0 + t; r < v1; r += 16) cs += *(const f32x4_t*)(W + r * XE + 4 * g);
#pragma unroll 8
  for (int64_t r = v0 + l; r < v1; r += 64) bs += bias[r];
#pragma unroll
  for (int off = 1; off < 16; off <<= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[e] += __shfl_xor(cs[e], off);
  bs = wave_sum(bs);
  if (t == 0) *(f32x4_t*)(wp + 4 * g) = cs;
  if (l == 0) wp[XE] = bs;
}

template <int NG>
__device__ __forceinline__ void xent_pass1_body(const float* __restrict__ H,
                                                const float* __restrict__ W,
                                                const float* __restrict__ bias, int64_t v0,
                                                int64_t v1, int S, int s,
                                                const int32_t* __restrict__ idx, int nv,
                                                int tok0, float* __restrict__ part, int t, int g) {
  f32x4_t hb[NG], o[NG];
  float m[NG], sum[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int j = tok0 + 16 * q + t;
    hb[q] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    if (j < nv) hb[q] = *(const f32x4_t*)(H + (int64_t)idx[j] * XE + 4 * g) * LOG2E;
    o[q] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    m[q] = -INFINITY;
    sum[q] = 0.f;
  }
  const int la = t * XE + 4 * g;
  const int nfull = (int)((v1 - v0) / 16);
  const float* Wt = W + v0 * XE;
  const float* bt = bias + v0;
  XentTile ta, tb;
  if (nfull > 0) xent_load_full(ta, Wt, bt, la, t, g);
  if (nfull > 1) xent_load_full(tb, Wt + 16 * XE, bt + 16, la, t, g);
  for (int i = 0; i < nfull; i += 2) {
    {
      const XentTile cur = ta;
      if (i + 2 < nfull) xent_load_full(ta, Wt + (i + 2) * 16 * XE, bt + (i + 2) * 16, la, t, g);
      float bb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bb[r] = cur.bb[r] * LOG2E;
      xent_pass1_tile<NG>(cur, hb, bb, o, m, sum);
    }
    if (i + 1 < nfull) {
      const XentTile cur = tb;
      if (i + 3 < nfull) xent_load_full(tb, Wt + (i + 3) * 16 * XE, bt + (i + 3) * 16, la, t, g);
      float bb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bb[r] = cur.bb[r] * LOG2E;
      xent_pass1_tile<NG>(cur, hb, bb, o, m, sum);
    }
  }
  const int64_t r0 = v0 + 16 * (int64_t)nfull;
  if (r0 < v1) {                           // ragged last tile of the vocabulary
    XentTile cur;
    xent_load_tile(cur, W, bias, r0, v1, t, g);
    float bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bb[r] = r0 + 4 * g + r < v1 ? cur.bb[r] * LOG2E : -INFINITY;
    xent_pass1_tile<NG>(cur, hb, bb, o, m, sum);
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const float tot = sum4rows(sum[q]);
    const int j = tok0 + 16 * q + t;
    if (j < nv) {
      float* p = part + ((int64_t)j * S + s) * XP;
      *(f32x4_t*)(p + 2 + 4 * g) = o[q];     // O^T[4g+r][t] = O[t][4g+r]
      if (g == 0) {
        p[0] = m[q] * LN2;
        p[1] = tot;
      }
    }
  }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void xent_pass1_mfma_kernel(const float* __restrict__ H,
                                                             const float* __restrict__ W,
                                                             const float* __restrict__ bias,
                                                             int64_t V, int64_t VS, int S,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ count,
                                                             float* __restrict__ part,
                                                             float* __restrict__ wpart) {
  const int s = blockIdx.x, l = threadIdx.x, t = l & 15, g = l >> 4;
  const int nv = *count;
  const int tok0 = blockIdx.y * 16 * XG;
  const int ng = min(XG, max(0, (nv - tok0 + 15) / 16));
  const int64_t v0 = (int64_t)s * VS, v1 = min(V, v0 + VS);
  if (blockIdx.y == 0) xent_colsums(W, bias, v0, v1, wpart + (int64_t)s * (XE + 1), t, g, l);
  switch (ng) {
#define XCASE(n) \
    case n: xent_pass1_body<n>(H, W, bias, v0, v1, S, s, idx, nv, tok0, part, t, g); break;
    XCASE(1) XCASE(2) XCASE(3) XCASE(4) XCASE(5) XCASE(6) XCASE(7) XCASE(8)
#undef XCASE
    default: break;
  }
}

// ------------------------------------------------- 3-pass bf16 MFMA path --
// Both products of the online softmax on v_mfma_f32_16x16x32_bf16 with every
// fp32 operand split as x = hi + lo (hi = bf16(x), lo = bf16(x - hi)) and
// a*b ~= ah*bh + al*bh + ah*bl: relative error ~2^-16 per product (fp32
// accumulation), at 16 cycles per K=32 instruction instead of 32 per K=4 f32
// one. The K=32 slots of a lane (8g..8g+7) are chosen so that no operand
// crosses lanes: the contraction index of each slot only has to agree between
// A and B.
//   X = W H^T over a tile: slots {hi(e=4g+r), lo(e=4g+r)} of W row t against
//     {hi(h), hi(h)} of token t, then {hi(e)} against {lo(h)}: 2 instructions.
//   O^T += W^T P^T over a PAIR of tiles (a, b): slots {a: v=4g+r, b: v=4g+r}
//     -- exactly the rows the lane's C fragments of X hold -- so P feeds the
//     B operand straight from the X accumulators: 3 instructions (hh, lh, hl).
__device__ __forceinline__ f32x4_t mfma32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void bf_split(float x, __bf16& h, __bf16& l) {
  h = (__bf16)x;
  l = (__bf16)(x - (float)h);
}

struct XHop {                   // B operands of X for one 16-token group
  bf16x8_t hh;                  // {hi(h[4g..4g+3]), hi(h[4g..4g+3])}
  bf16x8_t lo;                  // {lo(h[4g..4g+3]), 0}
};

__device__ __forceinline__ XHop xhop_of(f32x4_t h) {
  XHop o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    __bf16 hi, lo;
    bf_split(h[r], hi, lo);
    o.hh[r] = hi;
    o.hh[4 + r] = hi;
    o.lo[r] = lo;
    o.lo[4 + r] = (__bf16)0.f;
  }
  return o;
}

__device__ __forceinline__ bf16x8_t wsplit_a(f32x4_t w) {     // {hi(w), lo(w)}
  bf16x8_t a;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    __bf16 hi, lo;
    bf_split(w[r], hi, lo);
    a[r] = hi;
    a[4 + r] = lo;
  }
  return a;
}

// X for one tile and NG groups (bias as C input, log2 units)
template <int NG>
__device__ __forceinline__ void xent_x3_logits(bf16x8_t a, const float* bb, const XHop* hb,
                                               f32x4_t* x) {
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    x[q] = (f32x4_t){bb[0], bb[1], bb[2], bb[3]};
    x[q] = mfma32(a, hb[q].hh, x[q]);
    x[q] = mfma32(a, hb[q].lo, x[q]);
  }
}

// One PAIR of 16-row tiles of the online softmax (b may be a null tile:
// W = 0, bias = -inf, so P = 0 there).
template <int NG>
__device__ __forceinline__ void xent_pass1_pair(const XentTile& A, const XentTile& B,
                                                const float* bba, const float* bbb,
                                                const XHop* hb, f32x4_t* o, float* m,
                                                float* sum) {
  f32x4_t xa[NG], xb[NG];
  xent_x3_logits<NG>(wsplit_a(A.wa), bba, hb, xa);
  xent_x3_logits<NG>(wsplit_a(B.wa), bbb, hb, xb);
  bool up = false;
  float mxl[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    mxl[q] = fmaxf(fmaxf(fmaxf(xa[q][0], xa[q][1]), fmaxf(xa[q][2], xa[q][3])),
                   fmaxf(fmaxf(xb[q][0], xb[q][1]), fmaxf(xb[q][2], xb[q][3])));
    up |= mxl[q] > m[q] + XTH;
  }
  if (__any(up)) {                         // wave-uniform; first pair and rare after
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const float mx = max4rows(mxl[q]);
      const float nm = fmaxf(m[q], mx);     // finite: row r0 of tile a is always valid
      const float c = exp2_fast(m[q] - nm);
      sum[q] *= c;
      o[q] *= c;
      m[q] = nm;
    }
  }
  // A operands of O^T: W^T rows e = t over the pair's 8 vocab slots
  bf16x8_t wh, wl;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    __bf16 h, l;
    bf_split(A.wb[r], h, l);
    wh[r] = h;
    wl[r] = l;
    bf_split(B.wb[r], h, l);
    wh[4 + r] = h;
    wl[4 + r] = l;
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    bf16x8_t ph, pl;
    float pa[4], pb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[r] = exp2_fast(xa[q][r] - m[q]);
      pb[r] = exp2_fast(xb[q][r] - m[q]);
      __bf16 h, l;
      bf_split(pa[r], h, l);
      ph[r] = h;
      pl[r] = l;
      bf_split(pb[r], h, l);
      ph[4 + r] = h;
      pl[4 + r] = l;
    }
    sum[q] += ((pa[0] + pa[1]) + (pa[2] + pa[3])) + ((pb[0] + pb[1]) + (pb[2] + pb[3]));
    o[q] = mfma32(wh, ph, o[q]);
    o[q] = mfma32(wl, ph, o[q]);
    o[q] = mfma32(wh, pl, o[q]);
  }
}

__device__ __forceinline__ XentTile xent_null_tile() {
  XentTile z;
  z.wa = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    z.wb[r] = 0.f;
    z.bb[r] = -INFINITY;
  }
  return z;
}

template <int NG>
__device__ __forceinline__ void xent_pass1_x3_body(const float* __restrict__ H,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ bias, int64_t v0,
                                                   int64_t v1, int S, int s,
                                                   const int32_t* __restrict__ idx, int nv,
                                                   int tok0, float* __restrict__ part, int t,
                                                   int g) {
  XHop hb[NG];
  f32x4_t o[NG];
  float m[NG], sum[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int j = tok0 + 16 * q + t;
    f32x4_t h = {0.f, 0.f, 0.f, 0.f};
    if (j < nv) h = *(const f32x4_t*)(H + (int64_t)idx[j] * XE + 4 * g) * LOG2E;
    hb[q] = xhop_of(h);
    o[q] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    m[q] = -INFINITY;
    sum[q] = 0.f;
  }
  const int la = t * XE + 4 * g;
  const int nfull = (int)((v1 - v0) / 16);
  const float* Wt = W + v0 * XE;
  const float* bt = bias + v0;
  const XentTile null_tile = xent_null_tile();
  // 4-tile register ring: the loads of pair i+2 are in flight for two pairs'
  // work (one pair's was shorter than a loaded HBM round trip)
  // (NG > 6: a 2-tile ring, the 4-tile one would spill)
  constexpr int RD = NG <= 6 ? 4 : 2;
  XentTile ta = null_tile, tb = null_tile, tc = null_tile, td = null_tile;
  if (nfull > 0) xent_load_full(ta, Wt, bt, la, t, g);
  if (nfull > 1) xent_load_full(tb, Wt + 16 * XE, bt + 16, la, t, g);
  if constexpr (RD == 4) {
    if (nfull > 2) xent_load_full(tc, Wt + 32 * XE, bt + 32, la, t, g);
    if (nfull > 3) xent_load_full(td, Wt + 48 * XE, bt + 48, la, t, g);
  }
  for (int i = 0; i < nfull; i += 2) {
    const XentTile ca = ta;
    const XentTile cb = i + 1 < nfull ? tb : null_tile;
    if constexpr (RD == 4) {
      ta = tc;
      tb = td;
    }
    if (i + RD < nfull)
      xent_load_full(RD == 4 ? tc : ta, Wt + (i + RD) * 16 * XE, bt + (i + RD) * 16, la, t, g);
    if (i + RD + 1 < nfull)
      xent_load_full(RD == 4 ? td : tb, Wt + (i + RD + 1) * 16 * XE, bt + (i + RD + 1) * 16, la,
                     t, g);
    float ba[4], bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ba[r] = ca.bb[r] * LOG2E;
      bb[r] = cb.bb[r] * LOG2E;            // (-inf stays -inf)
    }
    xent_pass1_pair<NG>(ca, cb, ba, bb, hb, o, m, sum);
  }
  const int64_t r0 = v0 + 16 * (int64_t)nfull;
  if (r0 < v1) {                           // ragged last tile of the vocabulary
    XentTile cur;
    xent_load_tile(cur, W, bias, r0, v1, t, g);
    float ba[4], bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ba[r] = r0 + 4 * g + r < v1 ? cur.bb[r] * LOG2E : -INFINITY;
      bb[r] = -INFINITY;
    }
    xent_pass1_pair<NG>(cur, null_tile, ba, bb, hb, o, m, sum);
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const float tot = sum4rows(sum[q]);
    const int j = tok0 + 16 * q + t;
    if (j < nv) {
      float* p = part + ((int64_t)j * S + s) * XP;
      *(f32x4_t*)(p + 2 + 4 * g) = o[q];
      if (g == 0) {
        p[0] = m[q] * LN2;
        p[1] = tot;
      }
    }
  }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void xent_pass1_x3_kernel(
    const float* __restrict__ H, const float* __restrict__ W, const float* __restrict__ bias,
    int64_t V, int64_t VS, int S, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ count, float* __restrict__ part, float* __restrict__ wpart) {
  const int s = blockIdx.x, l = threadIdx.x, t = l & 15, g = l >> 4;
  const int nv = *count;
  const int tok0 = blockIdx.y * 16 * XG;
  const int ng = min(XG, max(0, (nv - tok0 + 15) / 16));
  const int64_t v0 = (int64_t)s * VS, v1 = min(V, v0 + VS);
  if (blockIdx.y == 0) xent_colsums(W, bias, v0, v1, wpart + (int64_t)s * (XE + 1), t, g, l);
  switch (ng) {
#define XCASE(n) \
    case n: xent_pass1_x3_body<n>(H, W, bias, v0, v1, S, s, idx, nv, tok0, part, t, g); break;
    XCASE(1) XCASE(2) XCASE(3) XCASE(4) XCASE(5) XCASE(6) XCASE(7) XCASE(8)
#undef XCASE
    default: break;
  }
}

// wgrad token operands, staged by the merge kernel as htok[j][16] (H rows in
// valid-token order) and ytok[j] (int32 labels): no idx indirection here.
// Padding tokens get hb = 0 (no dW contribution), lse = +inf (e = 0) and
// y = -1; their constant -eps/V terms in db are removed once per run.
struct XentTok {
  f32x4_t ha;                   // H[tok t][4g..4g+3] * log2 e  (A of X^T = H W^T)
  float hb[4];                  // H[tok 4g+r][t] * scale       (A of dW^T = H^T dz^T)
  float lse[4];                 // per C row 4g+r, log2 units
  int y[4];
};

__device__ __forceinline__ void xent_load_tok(XentTok& K, const float* __restrict__ htok,
                                              const int32_t* __restrict__ ytok,
                                              const float* __restrict__ lse, int j0, int nv,
                                              float scale, int t, int g) {
  const int ja = j0 + t;
  K.ha = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  if (ja < nv) K.ha = *(const f32x4_t*)(htok + (int64_t)ja * XE + 4 * g) * LOG2E;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int jb = j0 + 4 * g + r;
    const bool ok = jb < nv;
    K.hb[r] = ok ? htok[(int64_t)jb * XE + t] * scale : 0.f;
    K.lse[r] = ok ? lse[jb] * LOG2E : INFINITY;
    K.y[r] = ok ? ytok[jb] : -1;
  }
}

// Fused output-layer optimizer step (LinearXentArgs.okind >= 0): the rows'
// final gradient updates W / bias in place (adam_elem, the flat optimizer's
// own element update) instead of being written to dW / db and re-read by the
// flat optimizer: one fewer 17 M-element gradient round trip per Bert4Rec
// step. Only the launch that holds the complete gradient does it (the wgrad
// kernel when every valid token fits one 128-token block, else the slab sum).
struct XOpt {
  float* W; float* bias; float* mW; float* vW; float* mb; float* vb;
  float lr, bc1, bc2, b1, b2, eps, wd, gs;
  bool adamw, on;
};

__device__ __forceinline__ XOpt xopt_of(const LinearXentArgs& a) {
  XOpt o{};
  o.on = a.okind >= 0;
  if (!o.on) return o;
  o.W = (float*)a.W; o.bias = (float*)a.bias;
  o.mW = a.mW; o.vW = a.vW; o.mb = a.mb; o.vb = a.vb;
  o.lr = a.ohyper[0];
  const float step = a.ohyper[1];
  o.gs = a.ohyper[2];
  o.bc1 = 1.f - powf(a.beta1, step);
  o.bc2 = 1.f - powf(a.beta2, step);
  o.b1 = a.beta1; o.b2 = a.beta2; o.eps = a.oeps; o.wd = a.owd;
  o.adamw = a.okind == OPT_ADAMW;
  return o;
}

// W[v][c0..c0+3] (p = those weights, already in registers) and, if wb, bias[v]
// The row's Adam moments, loaded ahead (XMom: a tile's, prefetched with its
// W fragment two tiles before use)
struct XMom {
  f32x4_t m, v;
  float mb, vb;
};

__device__ __forceinline__ XMom xopt_load(const XOpt& o, int64_t v, int c0, bool wb) {
  XMom r;
  const int64_t i = v * XE + c0;
  r.m = *(const f32x4_t*)(o.mW + i);
  r.v = *(const f32x4_t*)(o.vW + i);
  r.mb = wb ? o.mb[v] : 0.f;
  r.vb = wb ? o.vb[v] : 0.f;
  return r;
}

__device__ __forceinline__ void xopt_row_pre(const XOpt& o, int64_t v, int c0, f32x4_t p,
                                             f32x4_t g, bool wb, float gb, const XMom& mo) {
  const int64_t i = v * XE + c0;
  const f32x4_t m4 = mo.m, w4 = mo.v;
  float pp[4], mm[4], ww[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    pp[r] = p[r]; mm[r] = m4[r]; ww[r] = w4[r];
    adam_elem(pp[r], g[r] * o.gs, mm[r], ww[r], o.lr, o.bc1, o.bc2, o.b1, o.b2, o.eps, o.wd,
              o.adamw);
  }
  *(f32x4_t*)(o.W + i) = (f32x4_t){pp[0], pp[1], pp[2], pp[3]};
  *(f32x4_t*)(o.mW + i) = (f32x4_t){mm[0], mm[1], mm[2], mm[3]};
  *(f32x4_t*)(o.vW + i) = (f32x4_t){ww[0], ww[1], ww[2], ww[3]};
  if (wb) {
    float pb = o.bias[v], mbv = mo.mb, vbv = mo.vb;
    adam_elem(pb, gb * o.gs, mbv, vbv, o.lr, o.bc1, o.bc2, o.b1, o.b2, o.eps, o.wd, o.adamw);
    o.bias[v] = pb;
    o.mb[v] = mbv;
    o.vb[v] = vbv;
  }
}

__device__ __forceinline__ void xopt_row(const XOpt& o, int64_t v, int c0, f32x4_t p, f32x4_t g,
                                         bool wb, float gb) {
  const int64_t i = v * XE + c0;
  const f32x4_t m4 = *(const f32x4_t*)(o.mW + i), w4 = *(const f32x4_t*)(o.vW + i);
  float pp[4], mm[4], ww[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    pp[r] = p[r]; mm[r] = m4[r]; ww[r] = w4[r];
    adam_elem(pp[r], g[r] * o.gs, mm[r], ww[r], o.lr, o.bc1, o.bc2, o.b1, o.b2, o.eps, o.wd,
              o.adamw);
  }
  *(f32x4_t*)(o.W + i) = (f32x4_t){pp[0], pp[1], pp[2], pp[3]};
  *(f32x4_t*)(o.mW + i) = (f32x4_t){mm[0], mm[1], mm[2], mm[3]};
  *(f32x4_t*)(o.vW + i) = (f32x4_t){ww[0], ww[1], ww[2], ww[3]};
  if (wb) {
    float pb = o.bias[v], mbv = o.mb[v], vbv = o.vb[v];
    adam_elem(pb, gb * o.gs, mbv, vbv, o.lr, o.bc1, o.bc2, o.b1, o.b2, o.eps, o.wd, o.adamw);
    o.bias[v] = pb;
    o.mb[v] = mbv;
    o.vb[v] = vbv;
  }
}

// One 16-row tile for NG token groups: X^T = H W^T (bias as C input), dz in
// registers, dW^T = H^T dz^T; writes dW rows (float4 per lane) and db.
template <int NG>
__device__ __forceinline__ void xent_wgrad_tile(const XentTok* K, f32x4_t wa, float b, int v,
                                                int64_t V, float off, float hit, float pad_off,
                                                float scale, float* __restrict__ dW,
                                                float* __restrict__ db, int g, const XOpt& xo,
                                                const XMom* mo = nullptr) {
  f32x4_t dw[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float dbs = 0.f;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    f32x4_t x = {b, b, b, b};
    x = mfma4(K[q].ha[0], wa[0], x);
    x = mfma4(K[q].ha[1], wa[1], x);
    x = mfma4(K[q].ha[2], wa[2], x);
    x = mfma4(K[q].ha[3], wa[3], x);
    float dz[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float d = exp2_fast(x[r] - K[q].lse[r]) - off;
      if (K[q].y[r] == v) d -= hit;
      dz[r] = d;
    }
    dbs += (dz[0] + dz[1]) + (dz[2] + dz[3]);
    f32x4_t& acc = dw[q & 1];
    acc = mfma4(K[q].hb[0], dz[0], acc);
    acc = mfma4(K[q].hb[1], dz[1], acc);
    acc = mfma4(K[q].hb[2], dz[2], acc);
    acc = mfma4(K[q].hb[3], dz[3], acc);
  }
  dbs = (sum4rows(dbs) + pad_off) * scale;
  if (v < V) {
    if (xo.on) {                           // the complete gradient: step in place
      if (mo != nullptr) xopt_row_pre(xo, v, 4 * g, wa, dw[0] + dw[1], g == 0, dbs, *mo);
      else xopt_row(xo, v, 4 * g, wa, dw[0] + dw[1], g == 0, dbs);
      return;
    }
    *(f32x4_t*)(dW + (int64_t)v * XE + 4 * g) = dw[0] + dw[1];    // dW^T[4g+r][v]
    if (g == 0) db[v] = dbs;
  }
}

// 3-pass bf16 operands of the wgrad tile (see the pass1 x3 notes): X^T's A
// is {hi, lo} of the token's H row; dW^T's A covers a PAIR of token groups,
// slots {q: tok 4g+r, q+1: tok 4g+r} -- the rows the lane's dz fragments of
// the two groups hold, so dz feeds the B operand from its own registers.
template <int NG>
struct XTok3 {
  static constexpr int NP = (NG + 1) / 2;
  bf16x8_t ha[NG];
  bf16x8_t hbh[NP], hbl[NP];
  float lse[NG][4];
  int y[NG][4];
};

template <int NG>
__device__ __forceinline__ void xtok3_of(XTok3<NG>& T, const XentTok* K) {
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    T.ha[q] = wsplit_a(K[q].ha);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      T.lse[q][r] = K[q].lse[r];
      T.y[q][r] = K[q].y[r];
    }
  }
#pragma unroll
  for (int p = 0; p < XTok3<NG>::NP; ++p) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int q = 2 * p + hh;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __bf16 h = (__bf16)0.f, l = (__bf16)0.f;
        if (q < NG) bf_split(K[q].hb[r], h, l);
        T.hbh[p][4 * hh + r] = h;
        T.hbl[p][4 * hh + r] = l;
      }
    }
  }
}

template <int NG>
__device__ __forceinline__ void xent_wgrad_tile3(const XTok3<NG>& K, f32x4_t wa, float b, int v,
                                                 int64_t V, float off, float hit, float pad_off,
                                                 float scale, float* __restrict__ dW,
                                                 float* __restrict__ db, int g, const XOpt& xo,
                                                 const XMom* mo = nullptr) {
  bf16x8_t wh, wl;                         // B of X^T: {hi(w), hi(w)}, {lo(w), 0}
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    __bf16 h, l;
    bf_split(wa[r], h, l);
    wh[r] = h;
    wh[4 + r] = h;
    wl[r] = l;
    wl[4 + r] = (__bf16)0.f;
  }
  f32x4_t dw[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float dbs = 0.f;
#pragma unroll
  for (int p = 0; p < XTok3<NG>::NP; ++p) {
    float dz[8];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int q = 2 * p + hh;
      if (q < NG) {
        f32x4_t x = {b, b, b, b};
        x = mfma32(K.ha[q], wh, x);
        x = mfma32(K.ha[q], wl, x);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float d = exp2_fast(x[r] - K.lse[q][r]) - off;
          if (K.y[q][r] == v) d -= hit;
          dz[4 * hh + r] = d;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) dz[4 * hh + r] = 0.f;
      }
    }
    dbs += ((dz[0] + dz[1]) + (dz[2] + dz[3])) + ((dz[4] + dz[5]) + (dz[6] + dz[7]));
    bf16x8_t zh, zl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 h, l;
      bf_split(dz[e], h, l);
      zh[e] = h;
      zl[e] = l;
    }
    f32x4_t& acc = dw[p & 1];
    acc = mfma32(K.hbh[p], zh, acc);
    acc = mfma32(K.hbl[p], zh, acc);
    acc = mfma32(K.hbh[p], zl, acc);
  }
  dbs = (sum4rows(dbs) + pad_off) * scale;
  if (v < V) {
    if (xo.on) {                           // the complete gradient: step in place
      if (mo != nullptr) xopt_row_pre(xo, v, 4 * g, wa, dw[0] + dw[1], g == 0, dbs, *mo);
      else xopt_row(xo, v, 4 * g, wa, dw[0] + dw[1], g == 0, dbs);
      return;
    }
    *(f32x4_t*)(dW + (int64_t)v * XE + 4 * g) = dw[0] + dw[1];
    if (g == 0) db[v] = dbs;
  }
}

// Full tiles read through a wave-uniform tile pointer + constant lane
// offsets from a 2-slot register ring (two tiles per iteration).
template <int NG, bool X3>
__device__ __forceinline__ void xent_wgrad_body(const float* __restrict__ W,
                                                const float* __restrict__ bias, int64_t V,
                                                float eps, int64_t tile0, int tpw,
                                                const float* __restrict__ htok,
                                                const int32_t* __restrict__ ytok,
                                                const float* __restrict__ lse, int nv, int tok0,
                                                float* __restrict__ dW, float* __restrict__ db,
                                                int t, int g, const XOpt& xo) {
  const float scale = 1.f / (float)max(1, nv);
  const float off = eps / (float)V, hit = 1.f - eps;
  XentTok K[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) xent_load_tok(K[q], htok, ytok, lse, tok0 + 16 * q, nv, scale, t, g);
  XTok3<NG> K3;
  if constexpr (X3) xtok3_of<NG>(K3, K);
  const float pad_off = (float)(16 * NG - min(nv - tok0, 16 * NG)) * off;
  auto tile = [&](f32x4_t wa, float b, int v, const XMom* mo) {
    if constexpr (X3)
      xent_wgrad_tile3<NG>(K3, wa, b, v, V, off, hit, pad_off, scale, dW, db,
                           g, xo, mo);
    else
      xent_wgrad_tile<NG>(K, wa, b, v, V, off, hit, pad_off, scale, dW, db, g,
                          xo, mo);
  };
  const int64_t tile1 = min(tile0 + tpw, V / 16);        // full tiles
  const int nfull = (int)max<int64_t>(0, tile1 - tile0);
  const int la = t * XE + 4 * g;
  const float* Wt = W + tile0 * 16 * XE;
  const float* bt = bias + tile0 * 16;
  const int vb = (int)(tile0 * 16) + t;
  f32x4_t wa0, wa1;
  float b0, b1;
  // fused step: the rows' Adam moments ride in the same 2-tile prefetch ring
  // as W (without it each tile waited a full memory round trip for them);
  // not for NG > 6, where the ring's 20 registers would spill
  XMom mo0{}, mo1{};
  const bool pre = NG <= 6 && xo.on;
  if (nfull > 0) {
    wa0 = *(const f32x4_t*)(Wt + la); b0 = bt[t];
    if (pre) mo0 = xopt_load(xo, vb, 4 * g, g == 0);
  }
  if (nfull > 1) {
    wa1 = *(const f32x4_t*)(Wt + 16 * XE + la); b1 = bt[16 + t];
    if (pre) mo1 = xopt_load(xo, vb + 16, 4 * g, g == 0);
  }
  for (int i = 0; i < nfull; i += 2) {
    {
      const f32x4_t wa = wa0;
      const float b = b0 * LOG2E;
      const XMom mo = mo0;
      if (i + 2 < nfull) {
        wa0 = *(const f32x4_t*)(Wt + (i + 2) * 16 * XE + la);
        b0 = bt[(i + 2) * 16 + t];
        if (pre) mo0 = xopt_load(xo, vb + 16 * (i + 2), 4 * g, g == 0);
      }
      tile(wa, b, vb + 16 * i, pre ? &mo : nullptr);
    }
    if (i + 1 < nfull) {
      const f32x4_t wa = wa1;
      const float b = b1 * LOG2E;
      const XMom mo = mo1;
      if (i + 3 < nfull) {
        wa1 = *(const f32x4_t*)(Wt + (i + 3) * 16 * XE + la);
        b1 = bt[(i + 3) * 16 + t];
        if (pre) mo1 = xopt_load(xo, vb + 16 * (i + 3), 4 * g, g == 0);
      }
      tile(wa, b, vb + 16 * (i + 1), pre ? &mo : nullptr);
    }
  }
  const int64_t rt = V / 16;                             // ragged last tile
  if (V % 16 != 0 && rt >= tile0 && rt < tile0 + tpw) {
    const int64_t vr = min(rt * 16 + t, V - 1);
    const f32x4_t wa = *(const f32x4_t*)(W + vr * XE + 4 * g);
    tile(wa, bias[vr] * LOG2E, (int)(rt * 16) + t, nullptr);
  }
}

// grid (runs of `tpw` 16-row tiles, 128-token blocks). Block-row 0 writes
// dW/db; block-row k > 0 writes slab k-1 ([V][16] + [V]), summed by
// xent_slab_reduce_kernel — no atomics, fixed order.
template <bool X3>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void xent_wgrad_mfma_kernel(const float* __restrict__ W,
                                                             const float* __restrict__ bias,
                                                             int64_t V, float eps, int tpw,
                                                             const float* __restrict__ htok,
                                                             const int32_t* __restrict__ ytok,
                                                             const int32_t* __restrict__ count,
                                                             const float* __restrict__ lse,
                                                             float* __restrict__ dW,
                                                             float* __restrict__ db,
                                                             float* __restrict__ slab,
                                                             LinearXentArgs xa) {
  const int l = threadIdx.x, t = l & 15, g = l >> 4;
  const int nv = *count;
  const int tb = blockIdx.y, tok0 = tb * 16 * XG;
  const int ng = min(XG, max(0, (nv - tok0 + 15) / 16));
  if (tb > 0 && ng == 0) return;
  // fused optimizer only when this launch holds the whole gradient (one
  // 128-token block); else xent_slab_reduce_kernel steps after the sum
  XOpt xo = xopt_of(xa);
  xo.on = xo.on && nv <= 16 * XG;
  float* dWo = dW;
  float* dbo = db;
  if (tb > 0) {
    dWo = slab + (int64_t)(tb - 1) * V * (XE + 1);
    dbo = dWo + V * XE;
  }
  const int64_t tile0 = (int64_t)blockIdx.x * tpw;
  switch (ng) {
#define XCASE(n)                                                                            \
    case n:                                                                                 \
      xent_wgrad_body<n, X3>(W, bias, V, eps, tile0, tpw, htok, ytok, lse, nv, tok0, dWo, dbo, \
                         t, g, xo);                                                         \
      break;
    XCASE(1) XCASE(2) XCASE(3) XCASE(4) XCASE(5) XCASE(6) XCASE(7) XCASE(8)
#undef XCASE
    default: {                    // no valid token: dW = db = 0 for this run
      const int64_t r1 = min((tile0 + tpw) * 16, V);
      for (int64_t v = tile0 * 16 + t; v < r1; v += 16) {
        if (xo.on) {                 // (a zero-gradient step still moves W)
          xopt_row(xo, v, 4 * g, *(const f32x4_t*)(W + v * XE + 4 * g),
                   (f32x4_t){0.f, 0.f, 0.f, 0.f}, g == 0, 0.f);
          continue;
        }
        *(f32x4_t*)(dWo + v * XE + 4 * g) = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        if (g == 0) dbo[v] = 0.f;
      }
    }
  }
}

// dW/db += the active slabs (token blocks 1..nblk-1), fixed order.
// (thread g of G in all: element i = g, g + G, ...; the sums do not depend
// on how the threads are grouped into blocks)
__device__ __forceinline__ void xent_slab_reduce_body(int64_t V, const int32_t* __restrict__ count,
                                                      const float* __restrict__ slab,
                                                      float* __restrict__ dW,
                                                      float* __restrict__ db,
                                                      const LinearXentArgs& xa, int64_t g,
                                                      int64_t G) {
  const int nblk = (*count + 16 * XG - 1) / (16 * XG);
  if (nblk <= 1) return;           // (the wgrad kernel holds the whole gradient)
  const XOpt xo = xopt_of(xa);
  const int64_t n4 = V * XE / 4;
  for (int64_t i = g; i < n4 + V; i += G) {
    if (i < n4) {
      f32x4_t a = ((f32x4_t*)dW)[i];
      for (int k = 1; k < nblk; ++k)
        a += ((const f32x4_t*)(slab + (int64_t)(k - 1) * V * (XE + 1)))[i];
      if (xo.on) {
        const int64_t v = i / (XE / 4);
        const int c0 = (int)(i - v * (XE / 4)) * 4;
        xopt_row(xo, v, c0, *(const f32x4_t*)(xo.W + v * XE + c0), a, false, 0.f);
      } else {
        ((f32x4_t*)dW)[i] = a;
      }
    } else {
      const int64_t v = i - n4;
      float a = db[v];
      for (int k = 1; k < nblk; ++k) a += slab[(int64_t)(k - 1) * V * (XE + 1) + V * XE + v];
      if (xo.on) {
        float pb = xo.bias[v], mbv = xo.mb[v], vbv = xo.vb[v];
        adam_elem(pb, a * xo.gs, mbv, vbv, xo.lr, xo.bc1, xo.bc2, xo.b1, xo.b2, xo.eps, xo.wd,
                  xo.adamw);
        xo.bias[v] = pb;
        xo.mb[v] = mbv;
        xo.vb[v] = vbv;
      } else {
        db[v] = a;
      }
    }
  }
}

__global__ __launch_bounds__(256) void xent_slab_reduce_kernel(int64_t V,
                                                               const int32_t* __restrict__ count,
                                                               const float* __restrict__ slab,
                                                               float* __restrict__ dW,
                                                               float* __restrict__ db,
                                                               LinearXentArgs xa) {
  xent_slab_reduce_body(V, count, slab, dW, db, xa, (int64_t)blockIdx.x * 256 + threadIdx.x,
                        (int64_t)gridDim.x * 256);
}

}  // namespace

// 2: 3-pass bf16 MFMA (default), 1: f32 MFMA, 0: VALU kernels; TDFO_XENT_IMPL
// picks another at load (A/B runs)
static int xent_impl_env() {
  const char* e = getenv("TDFO_XENT_IMPL");
  if (e == nullptr || *e == 0) return 2;
  const int v = atoi(e);
  return v < 0 ? 0 : (v > 2 ? 2 : v);
}
int g_xent_impl = xent_impl_env();

// VALU pass1: ~8 waves per SIMD (one wave per (split, 64-token chunk)).
// MFMA pass1: ~2048 splits of whole 16-row tiles per 128-token block. The
// number of valid tokens is device-side, so size for the capacity N.
void linear_xent_splits(int N, int64_t V, int64_t* VS, int* S) {
  int64_t vs;
  if (g_xent_impl >= 1) {
    const int blocks = std::max(1, (N + 16 * XG - 1) / (16 * XG));
    const int64_t want = std::max(64, std::min(2048, 8192 / blocks));
    vs = std::max<int64_t>(16, (V + want - 1) / want);
    vs = (vs + 15) / 16 * 16;
  } else {
    const int chunks = std::max(1, (N + 63) / 64);
    int64_t want = std::min<int64_t>(8192, std::max<int64_t>(64, 16384 / chunks));
    vs = std::max<int64_t>(64, (V + want - 1) / want);
  }
  *VS = vs;
  *S = (int)((V + vs - 1) / vs);
}

int linear_xent_impl(int impl) {
  const int old = g_xent_impl;
  if (impl >= 0) g_xent_impl = impl > 2 ? 2 : impl;
  return old;
}

static int xent_blocks(int N) { return std::max(1, (N + 16 * XG - 1) / (16 * XG)); }

size_t linear_xent_workspace(int N, int64_t V) {
  int64_t VS;
  int S;
  linear_xent_splits(N, V, &VS, &S);
  // idx[N] + count + lse[N] + ytok[N] (ints/floats) + htok[N][16] + part[N][S][XP]
  // + wpart[S][17] + wgrad slabs[(blocks-1)][V][17]
  return (size_t)(3 * N + 16) * 4 + (size_t)N * XE * 4 + (size_t)N * S * XP * 4 +
         (size_t)S * (XE + 1) * 4 + (size_t)(xent_blocks(N) - 1) * V * (XE + 1) * 4 + 512;
}

// Mean loss over the valid tokens in fixed order (one block, fixed reduction
// tree: deterministic), optionally accumulated into a device fp64 running sum
// -- replaces the count / sum / clamp / divide / accumulate library ops.
__device__ __forceinline__ void xent_loss_body(const float* __restrict__ lossv, int N,
                                               const int32_t* __restrict__ count,
                                               float* __restrict__ loss, double* __restrict__ acc,
                                               float* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float v = 0.f;
  for (int i = tid; i < N; i += 1024) v += lossv[i];
  v = wave_sum(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  if (w == 0) {
    float t = lane < 16 ? red[lane] : 0.f;
    t = wave_sum(t);
    if (lane == 0) {
      const float L = t / (float)max(1, *count);
      loss[0] = L;
      if (acc) acc[0] += (double)L;
    }
  }
}

__global__ __launch_bounds__(1024) void xent_loss_kernel(const float* __restrict__ lossv, int N,
                                                         const int32_t* __restrict__ count,
                                                         float* __restrict__ loss,
                                                         double* __restrict__ acc) {
  __shared__ float red[16];
  xent_loss_body(lossv, N, count, loss, acc, red);
}

// The step's tail in one launch: the wgrad slab sum (+ fused Adam) over the
// first XT_SLAB_BLOCKS 1024-thread blocks -- the same 524,288 threads, so the
// same per-element sums as xent_slab_reduce_kernel's 2048 x 256 -- and the
// mean loss in the last block (xent_loss_kernel's 1024-thread tree). With at
// most 128 valid tokens the slab part exits at once: the launch it would
// have cost (Bert4Rec B=16: 4.6 us per step) is gone.
constexpr int XT_SLAB_BLOCKS = 512;
__global__ __launch_bounds__(1024) void xent_tail_kernel(int64_t V,
                                                         const int32_t* __restrict__ count,
                                                         const float* __restrict__ slab,
                                                         float* __restrict__ dW,
                                                         float* __restrict__ db,
                                                         LinearXentArgs xa) {
  __shared__ float red[16];
  if (blockIdx.x == XT_SLAB_BLOCKS) {
    xent_loss_body(xa.lossv, xa.N, count, xa.loss, xa.loss_acc, red);
    return;
  }
  xent_slab_reduce_body(V, count, slab, dW, db, xa, (int64_t)blockIdx.x * 1024 + threadIdx.x,
                        (int64_t)XT_SLAB_BLOCKS * 1024);
}

void linear_xent(const LinearXentArgs& a, hipStream_t s) {
  if (a.N <= 0) return;
  if (a.V <= 0 || a.V >= (int64_t(1) << 31))
    throw std::runtime_error("linear_xent: vocab must be in [1, 2^31)");
  int64_t VS;
  int S;
  linear_xent_splits(a.N, a.V, &VS, &S);
  char* ws = (char*)a.workspace;
  int32_t* idx = (int32_t*)ws;
  int32_t* count = idx + a.N;
  float* lse = (float*)(count + 16);
  float* part = lse + a.N;
  part = (float*)(((uintptr_t)part + 15) & ~(uintptr_t)15);
  float* wpart = part + (int64_t)a.N * S * XP;
  int32_t* ytok = (int32_t*)(wpart + (int64_t)S * (XE + 1));
  float* htok = (float*)(((uintptr_t)(ytok + a.N) + 15) & ~(uintptr_t)15);
  float* slab = htok + (int64_t)a.N * XE;
  hipLaunchKernelGGL(xent_compact_kernel, dim3(1), dim3(1024), 0, s, a.labels, a.N, a.ignore, idx,
                     count, a.dH, a.lossv);
  const int blocks = xent_blocks(a.N);
  if (g_xent_impl == 2) {
    hipLaunchKernelGGL(xent_pass1_x3_kernel, dim3(S, blocks), dim3(64), 0, s, a.H, a.W, a.bias,
                       a.V, VS, S, idx, count, part, wpart);
  } else if (g_xent_impl == 1) {
    hipLaunchKernelGGL(xent_pass1_mfma_kernel, dim3(S, blocks), dim3(64), 0, s, a.H, a.W, a.bias,
                       a.V, VS, S, idx, count, part, wpart);
  } else {
    const int chunks = (a.N + 63) / 64;
    hipLaunchKernelGGL(xent_pass1_kernel, dim3(S, chunks), dim3(64), 0, s, a.H, a.W, a.bias, a.V,
                       VS, S, idx, count, part, wpart);
  }
  hipLaunchKernelGGL(xent_merge_kernel, dim3(a.N), dim3(256), 0, s, a.H, a.W, a.bias, a.labels,
                     a.V, S, a.eps, idx, count, part, wpart, lse, a.dH, a.lossv, htok, ytok);
  if (a.dW) {
    if (g_xent_impl >= 1) {
      const int64_t tiles = (a.V + 15) / 16;
      const int tpw = (int)std::max<int64_t>(1, (tiles + 4095) / 4096);
      const dim3 grid((unsigned)((tiles + tpw - 1) / tpw), blocks);
      if (g_xent_impl == 2)
        hipLaunchKernelGGL(xent_wgrad_mfma_kernel<true>, grid, dim3(64), 0, s, a.W, a.bias, a.V,
                           a.eps, tpw, htok, ytok, count, lse, a.dW, a.db, slab, a);
      else
        hipLaunchKernelGGL(xent_wgrad_mfma_kernel<false>, grid, dim3(64), 0, s, a.W, a.bias, a.V,
                           a.eps, tpw, htok, ytok, count, lse, a.dW, a.db, slab, a);
      if (blocks > 1 && a.loss) {
        hipLaunchKernelGGL(xent_tail_kernel, dim3(XT_SLAB_BLOCKS + 1), dim3(1024), 0, s, a.V,
                           count, slab, a.dW, a.db, a);
        TDFO_CHECK_HIP(hipGetLastError());
        return;                     // (the loss is done too)
      }
      if (blocks > 1)
        hipLaunchKernelGGL(xent_slab_reduce_kernel, dim3(2048), dim3(256), 0, s, a.V, count,
                           slab, a.dW, a.db, a);
    } else {
      hipLaunchKernelGGL(xent_wgrad_kernel, dim3((unsigned)((a.V + 255) / 256)), dim3(256), 0, s,
                         a.H, a.W, a.bias, a.labels, a.V, a.eps, idx, count, lse, a.dW, a.db);
      if (a.okind >= 0) {           // VALU path: the flat optimizer's kernel on W, bias
        for (int part = 0; part < 2; ++part) {
          DenseOptArgs o{};
          o.p = part ? (float*)a.bias : (float*)a.W;
          o.g = part ? a.db : a.dW;
          o.m = part ? a.mb : a.mW;
          o.v = part ? a.vb : a.vW;
          o.n = part ? (a.V + 3) / 4 * 4 : a.V * XE;    // (flat buffers are padded)
          o.opt = a.okind; o.hyper = a.ohyper;
          o.beta1 = a.beta1; o.beta2 = a.beta2; o.eps = a.oeps; o.weight_decay = a.owd;
          dense_optimizer(o, s);
        }
      }
    }
  }
  if (a.loss)
    hipLaunchKernelGGL(xent_loss_kernel, dim3(1), dim3(1024), 0, s, a.lossv, a.N, count, a.loss,
                       a.loss_acc);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
