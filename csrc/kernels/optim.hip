// Fused dense optimizers over one flat fp32 parameter buffer (N11/K21 in
// SURVEY.md): all dense parameters of a model live in a single buffer, so one
// launch updates every tensor (no per-tensor launches, no multi-tensor apply
// lists). The same pass refreshes the bf16 shadow copy the MFMA GEMMs read,
// so no separate cast kernel runs per step. Hyper-parameters that change
// over training (lr, step, grad scale) are read from device memory so the
// launch can be captured once in a hipGraph and replayed.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

// One float4 of parameters per thread. Every load the element needs is issued
// before the first wait: p / m / v, and the split-K slabs of its layer 8 at a
// time at clamped addresses (a predicated load makes hipcc branch around it and
// wait for each one); the segment is picked with wave-uniform selects over the
// kernel-argument table (dynamically indexing that table compiles to dependent
// global loads). Slabs are summed in slab order, as before.
__global__ __launch_bounds__(256) void dense_opt_kernel(DenseOptArgs a) {
  if (a.found_inf && a.found_inf[0] > 0.f) return;
  const float lr = a.hyper[0], step = a.hyper[1], gs = a.hyper[2];
  const float bc1 = 1.f - powf(a.beta1, step), bc2 = 1.f - powf(a.beta2, step);
  const bool adam = a.opt == OPT_ADAMW || a.opt == OPT_ADAM;
  const bool has_m = adam || a.opt != OPT_SGD || a.momentum != 0.f;
  const int64_t n4 = a.n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    const float4 p = ((const float4*)a.p)[i];
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f), v = m;
    if (has_m) m = ((const float4*)a.m)[i];
    if (adam) v = ((const float4*)a.v)[i];
    const int64_t e = 4 * i;
    const float* sp = a.g + e;
    int64_t L = 0;
    int S = 0;
    for (int k = 0; k < a.nseg; ++k) {
      const int64_t st = a.seg_start[k], ln = a.seg_len[k];
      const bool in = e >= st && e < st + ln;
      sp = in ? a.seg_ptr[k] + (e - st) : sp;
      L = in ? ln : L;
      S = in ? a.seg_splits[k] : S;
    }
    float4 g;
    if (S == 0) {
      g = *(const float4*)sp;
    } else {
      // split-K weight-grad slabs of one layer, summed in fixed order here
      // instead of by a separate reduce launch
      g = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = 0; q < S; q += 8) {
        float4 t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = *(const float4*)(sp + min(q + u, S - 1) * L);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (q + u < S) { g.x += t[u].x; g.y += t[u].y; g.z += t[u].z; g.w += t[u].w; }
      }
    }
    float pv[4] = {p.x, p.y, p.z, p.w};
    float gv[4] = {g.x * gs, g.y * gs, g.z * gs, g.w * gs};
    float mv[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
    if (adam) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        adam_elem(pv[u], gv[u], mv[u], vv[u], lr, bc1, bc2, a.beta1, a.beta2, a.eps,
                  a.weight_decay, a.opt == OPT_ADAMW);
      ((float4*)a.m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      ((float4*)a.v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    } else if (a.opt == OPT_SGD) {
      if (a.momentum != 0.f) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float gg = gv[u] + a.weight_decay * pv[u];
          mv[u] = step > 1.f ? a.momentum * mv[u] + gg : gg;
          pv[u] -= lr * mv[u];
        }
        ((float4*)a.m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) pv[u] -= lr * (gv[u] + a.weight_decay * pv[u]);
      }
    } else {  // adagrad
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float gg = gv[u] + a.weight_decay * pv[u];
        mv[u] += gg * gg;
        pv[u] -= lr * gg / (sqrtf(mv[u]) + a.eps);
      }
      ((float4*)a.m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
    }
    ((float4*)a.p)[i] = make_float4(pv[0], pv[1], pv[2], pv[3]);
    if (a.p_bf16) {
      ((uint2*)a.p_bf16)[i] = make_uint2(pack2bf(pv[0], pv[1]), pack2bf(pv[2], pv[3]));
    }
  }
}

__global__ void finite_kernel(const float* __restrict__ g, int64_t n,
                              float* found) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) found[0] = 1.f;
}

__global__ void cast_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                            int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

int blocks_for(int64_t n, int per_thread) {
  int64_t b = (n / per_thread + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b > 4096 ? 4096 : b);
}

}  // namespace

void dense_optimizer(const DenseOptArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(dense_opt_kernel, dim3(blocks_for(a.n, 4)), dim3(256), 0, s, a);
}

void check_finite(const float* g, int64_t n, float* found_inf, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(finite_kernel, dim3(blocks_for(n, 4)), dim3(256), 0, s, g,
                     n, found_inf);
}

void cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cast_kernel, dim3(blocks_for(n, 4)), dim3(256), 0, s, x, y, n);
}

}  // namespace tdfo
