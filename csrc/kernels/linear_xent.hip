// Fused output projection + label-smoothed cross-entropy (fwd AND bwd)
// without materialising the [tokens, V] logits (gfx950).
//
// Reference: Bert4Rec `self.out = nn.Linear(E, V)` (torchrec/models.py:206,
// 223) followed by CrossEntropyLoss(ignore_index=0, label_smoothing=0.1)
// (torchrec/train.py:93,99-101). With V = n_items + 2 (millions of books)
// the reference writes and re-reads a [B*T, V] fp32 logits tensor; here:
//
//   compact : valid tokens (label != ignore) -> idx[], n_valid (device)
//   pass1   : grid (vocab split s, token chunk); each thread owns one token,
//             streams its split's W rows through LDS (broadcast reads) and
//             keeps an online-softmax state (m, s, acc = sum_v e^{z_v-m} W_v)
//             -> part[token][s]; chunk-0 blocks also emit sum_v W_v, sum_v b_v
//   merge   : one wave per token merges the splits: lse, loss, and
//             dH = scale * (E_p[W] - (1-eps) W_y - eps/V sum_v W_v)
//   wgrad   : one thread per vocab row v, tokens staged in LDS:
//             dz = scale * (e^{z-lse} - eps/V - (1-eps)[v==y]);
//             dW_v = sum_n dz H_n, db_v = sum_n dz   (no atomics)
//
// loss_n = lse - (1-eps) z_y - eps * mean_v z_v, mean_v z_v = (H.sumW + sumb)/V;
// scale = 1 / n_valid (mean over non-ignored tokens, torch semantics).
#include "tdfo_common.h"
#include "tdfo_kernels.h"

#include <algorithm>

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

// one wave per valid token
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
                                                         float* __restrict__ lossv) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nv = *count;
  if (j >= nv) return;
  const float scale = 1.f / (float)max(1, nv);
  // merge online-softmax states over splits
  float m = -INFINITY, sum = 0.f, acc[XE];
#pragma unroll
  for (int k = 0; k < XE; ++k) acc[k] = 0.f;
  const float* p0 = part + (int64_t)j * S * XP;
  for (int s = lane; s < S; s += 64) {
    const float* p = p0 + (int64_t)s * XP;
    const float pm = p[0];
    if (pm == -INFINITY) continue;
    const float nm = fmaxf(m, pm);
    const float c0 = __expf(m - nm), c1 = __expf(pm - nm);
    sum = sum * c0 + p[1] * c1;
#pragma unroll
    for (int k = 0; k < XE; ++k) acc[k] = acc[k] * c0 + p[2 + k] * c1;
    m = nm;
  }
  // wave reduction of (m, sum, acc)
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off);
    const float os = __shfl_xor(sum, off);
    const float nm = fmaxf(m, om);
    const float c0 = (m == -INFINITY) ? 0.f : __expf(m - nm);
    const float c1 = (om == -INFINITY) ? 0.f : __expf(om - nm);
    sum = sum * c0 + os * c1;
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const float oa = __shfl_xor(acc[k], off);
      acc[k] = acc[k] * c0 + oa * c1;
    }
    m = nm;
  }
  // sum_v [W_v | b_v]
  float ws[XE + 1];
#pragma unroll
  for (int k = 0; k <= XE; ++k) ws[k] = 0.f;
  for (int s = lane; s < S; s += 64) {
#pragma unroll
    for (int k = 0; k <= XE; ++k) ws[k] += wpart[(int64_t)s * (XE + 1) + k];
  }
#pragma unroll
  for (int k = 0; k <= XE; ++k) ws[k] = wave_sum(ws[k]);
  if (lane != 0) return;
  const int n = idx[j];
  const float* hr = H + (int64_t)n * XE;
  int64_t y = labels[n];
  if (y < 0 || y >= V) y = 0;   // host validates; never read out of bounds
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
  for (int k = 0; k < XE; ++k)
    dH[(int64_t)n * XE + k] = scale * (acc[k] * inv - (1.f - eps) * wy[k] - eps * ws[k] / (float)V);
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

}  // namespace

// ~8 waves per SIMD for pass1 (one wave per (split, 64-token chunk)); the
// number of valid tokens is device-side, so size for the capacity N.
void linear_xent_splits(int N, int64_t V, int64_t* VS, int* S) {
  const int chunks = std::max(1, (N + 63) / 64);
  int64_t want = std::min<int64_t>(8192, std::max<int64_t>(64, 16384 / chunks));
  int64_t vs = std::max<int64_t>(64, (V + want - 1) / want);
  *VS = vs;
  *S = (int)((V + vs - 1) / vs);
}

size_t linear_xent_workspace(int N, int64_t V) {
  int64_t VS;
  int S;
  linear_xent_splits(N, V, &VS, &S);
  // idx[N] + count + lse[N] (ints/floats) + part[N][S][XP] + wpart[S][17]
  return (size_t)(2 * N + 16) * 4 + (size_t)N * S * XP * 4 + (size_t)S * (XE + 1) * 4 + 256;
}

void linear_xent(const LinearXentArgs& a, hipStream_t s) {
  if (a.N <= 0) return;
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
  hipLaunchKernelGGL(xent_compact_kernel, dim3(1), dim3(1024), 0, s, a.labels, a.N, a.ignore, idx,
                     count, a.dH, a.lossv);
  const int chunks = (a.N + 63) / 64;
  hipLaunchKernelGGL(xent_pass1_kernel, dim3(S, chunks), dim3(64), 0, s, a.H, a.W, a.bias, a.V, VS,
                     S, idx, count, part, wpart);
  hipLaunchKernelGGL(xent_merge_kernel, dim3((a.N + 3) / 4), dim3(256), 0, s, a.H, a.W, a.bias,
                     a.labels, a.V, S, a.eps, idx, count, part, wpart, lse, a.dH, a.lossv);
  if (a.dW)
    hipLaunchKernelGGL(xent_wgrad_kernel, dim3((unsigned)((a.V + 255) / 256)), dim3(256), 0, s,
                       a.H, a.W, a.bias, a.labels, a.V, a.eps, idx, count, lse, a.dW, a.db);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
