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
//   sort   : hipcub radix sort on the key bits actually used
//   chunks : each wave reduces a fixed 32-entry chunk of the sorted list; runs
//            fully inside the chunk are finished (optimizer applied) in place,
//            runs crossing a chunk edge leave fp32 partials (head/tail slabs)
//   combine: the chunk where a crossing run starts adds the following chunks'
//            head partials in order and applies the optimizer once.
// Every unique row is updated exactly once per step, in a fixed order.
#include <hipcub/hipcub.hpp>

#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

// ----------------------------------------------------------- forward ----
template <int D, bool OUT_BF16>
__global__ __launch_bounds__(256) void emb_fwd_kernel(EmbFwdArgs a) {
  constexpr int LPB = (D / 4) < 64 ? (D / 4) : 64;  // lanes per bag
  constexpr int BPW = 64 / LPB;                     // bags per wave
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPB, sl = lane - sub * LPB;
  const int64_t nbags = (int64_t)a.T * a.B;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t j = wave0 * BPW + sub; j < nbags; j += nwaves * BPW) {
    const int t = (int)(j / a.B);
    const int b = (int)(j - (int64_t)t * a.B);
    const int64_t s = a.offsets[j], e = a.offsets[j + 1];
    const float* wbase = a.W + a.row_offset[t] * D;
    for (int c = sl * 4; c < D; c += LPB * 4) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int64_t p = s;
      for (; p + 4 <= e; p += 4) {
        float4 r[4];
        float wt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u] = *(const float4*)(wbase + a.indices[p + u] * D + c);
          wt[u] = a.psw ? a.psw[p + u] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc.x += wt[u] * r[u].x; acc.y += wt[u] * r[u].y;
          acc.z += wt[u] * r[u].z; acc.w += wt[u] * r[u].w;
        }
      }
      for (; p < e; ++p) {
        const float4 r = *(const float4*)(wbase + a.indices[p] * D + c);
        const float wt = a.psw ? a.psw[p] : 1.f;
        acc.x += wt * r.x; acc.y += wt * r.y; acc.z += wt * r.z; acc.w += wt * r.w;
      }
      if (a.mean && e > s) {
        const float inv = 1.f / (float)(e - s);
        acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
      }
      const int64_t o = (int64_t)b * a.out_stride + a.out_off[t] + c;
      if (OUT_BF16) {
        uint2 v = make_uint2(pack2bf(acc.x, acc.y), pack2bf(acc.z, acc.w));
        *(uint2*)((uint16_t*)a.out + o) = v;
      } else {
        *(float4*)((float*)a.out + o) = acc;
      }
    }
  }
}

// ---------------------------------------------------------- backward ----
constexpr int CH = 32;  // sorted entries per chunk (one wave)

__global__ void emb_keys_kernel(const int64_t* __restrict__ row_offset,
                                const int64_t* __restrict__ indices,
                                const int64_t* __restrict__ offsets, int T,
                                int B, uint64_t* __restrict__ keys,
                                int32_t* __restrict__ vals,
                                int32_t* __restrict__ bag_of) {
  const int64_t nbags = (int64_t)T * B;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nbags;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(j / B);
    const int64_t ro = row_offset[t];
    for (int64_t p = offsets[j]; p < offsets[j + 1]; ++p) {
      keys[p] = (uint64_t)(ro + indices[p]);
      vals[p] = (int32_t)p;
      bag_of[p] = (int32_t)j;
    }
  }
}

template <int D>
struct RowAcc {
  static constexpr int EPL = D >= 64 ? D / 64 : 1;  // elements per lane
  float v[EPL];
};

template <int D>
__device__ __forceinline__ int elem0(int lane) {
  return D >= 64 ? lane * (D / 64) : lane;
}

template <int D>
__device__ __forceinline__ void acc_grad(RowAcc<D>& acc, const EmbBwdArgs& a,
                                         int bag, float scale, int lane) {
  const int t = bag / a.B, b = bag - t * a.B;
  const int64_t o = (int64_t)b * a.grad_stride + a.grad_off[t];
  const int e0 = elem0<D>(lane);
  if (D < 64 && e0 >= D) return;
  if (a.grad_bf16) {
    const uint16_t* g = (const uint16_t*)a.grad + o + e0;
    if constexpr (RowAcc<D>::EPL == 2) {
      const uint32_t u = *(const uint32_t*)g;
      acc.v[0] += scale * bf2f((uint16_t)(u & 0xffff));
      acc.v[1] += scale * bf2f((uint16_t)(u >> 16));
    } else {
#pragma unroll
      for (int u = 0; u < RowAcc<D>::EPL; ++u) acc.v[u] += scale * bf2f(g[u]);
    }
  } else {
    const float* g = (const float*)a.grad + o + e0;
#pragma unroll
    for (int u = 0; u < RowAcc<D>::EPL; ++u) acc.v[u] += scale * g[u];
  }
}

template <int D>
__device__ __forceinline__ void apply_update(const EmbBwdArgs& a, uint64_t row,
                                             const RowAcc<D>& acc, int lane) {
  constexpr int EPL = RowAcc<D>::EPL;
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  const float lr = a.hyper[0];
  float* w = a.W + row * D + e0;
  float g[EPL], wv[EPL];
#pragma unroll
  for (int u = 0; u < EPL; ++u) {
    wv[u] = act ? w[u] : 0.f;
    g[u] = acc.v[u];
  }
  switch (a.opt) {
    case EMB_SGD:
#pragma unroll
      for (int u = 0; u < EPL; ++u) wv[u] -= lr * (g[u] + a.weight_decay * wv[u]);
      break;
    case EMB_ROWWISE_ADAGRAD: {
      float sq = 0.f;
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        g[u] += a.weight_decay * wv[u];
        sq += act ? g[u] * g[u] : 0.f;
      }
      sq = wave_sum(sq) / (float)D;
      const float st = a.state1[row] + sq;
      if (lane == 0) a.state1[row] = st;
      const float mult = lr / (sqrtf(st) + a.eps);
#pragma unroll
      for (int u = 0; u < EPL; ++u) wv[u] -= mult * g[u];
      break;
    }
    case EMB_ADAGRAD: {
      float* st = a.state1 + row * D + e0;
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        if (!act) break;
        const float gg = g[u] + a.weight_decay * wv[u];
        const float s2 = st[u] + gg * gg;
        st[u] = s2;
        wv[u] -= lr * gg / (sqrtf(s2) + a.eps);
      }
      break;
    }
    case EMB_ADAM: {
      // decoupled weight decay, bias-corrected (fbgemm-style fused Adam)
      const float step = a.hyper[1];
      const float bc1 = 1.f - powf(a.beta1, step), bc2 = 1.f - powf(a.beta2, step);
      float* m = a.state1 + row * D + e0;
      float* v = a.state2 + row * D + e0;
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        if (!act) break;
        const float mm = a.beta1 * m[u] + (1.f - a.beta1) * g[u];
        const float vv = a.beta2 * v[u] + (1.f - a.beta2) * g[u] * g[u];
        m[u] = mm; v[u] = vv;
        wv[u] -= lr * ((mm / bc1) / (sqrtf(vv / bc2) + a.eps) + a.weight_decay * wv[u]);
      }
      break;
    }
    case EMB_DENSE_GRAD: {
      float* dg = a.dense_grad + row * D + e0;
#pragma unroll
      for (int u = 0; u < EPL; ++u) if (act) dg[u] += g[u];
      return;
    }
  }
#pragma unroll
  for (int u = 0; u < EPL; ++u) if (act) w[u] = wv[u];
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

template <int D>
__global__ __launch_bounds__(256) void emb_chunk_kernel(
    EmbBwdArgs a, const uint64_t* __restrict__ keys,
    const int32_t* __restrict__ vals, const int32_t* __restrict__ bag_of,
    float* __restrict__ head, float* __restrict__ tail) {
  constexpr int EPL = RowAcc<D>::EPL;
  const int lane = threadIdx.x & 63;
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t start = c * CH;
  if (start >= a.nnz) return;
  const int64_t end = min(start + (int64_t)CH, a.nnz);
  const int len = (int)(end - start);
  uint64_t mykey = 0; int mypos = 0;
  if (lane < len) { mykey = keys[start + lane]; mypos = vals[start + lane]; }
  const uint64_t first = readlane64(mykey, 0);
  const bool from_before = start > 0 && keys[start - 1] == first;
  const bool continues = end < a.nnz && keys[end] == readlane64(mykey, len - 1);

  RowAcc<D> acc;
#pragma unroll
  for (int u = 0; u < EPL; ++u) acc.v[u] = 0.f;
  uint64_t cur = first;
  bool started_here = !from_before;
  const int e0 = elem0<D>(lane);
  for (int p = 0; p < len; ++p) {
    const uint64_t k = readlane64(mykey, p);
    if (k != cur) {
      if (started_here) {
        apply_update<D>(a, cur, acc, lane);
      } else if (D >= 64 || e0 < D) {
#pragma unroll
        for (int u = 0; u < EPL; ++u) head[c * D + e0 + u] = acc.v[u];
      }
#pragma unroll
      for (int u = 0; u < EPL; ++u) acc.v[u] = 0.f;
      cur = k;
      started_here = true;
    }
    const int pos = __builtin_amdgcn_readlane(mypos, p);
    const int bag = bag_of[pos];
    float scale = a.psw ? a.psw[pos] : 1.f;
    if (a.mean) scale /= (float)(a.offsets[bag + 1] - a.offsets[bag]);
    acc_grad<D>(acc, a, bag, scale, lane);
  }
  float* dst = nullptr;
  if (!continues) {
    if (started_here) apply_update<D>(a, cur, acc, lane);
    else dst = head + c * D;
  } else {
    dst = (started_here ? tail : head) + c * D;
  }
  if (dst && (D >= 64 || e0 < D)) {
#pragma unroll
    for (int u = 0; u < EPL; ++u) dst[e0 + u] = acc.v[u];
  }
}

template <int D>
__global__ __launch_bounds__(256) void emb_combine_kernel(
    EmbBwdArgs a, const uint64_t* __restrict__ keys,
    const float* __restrict__ head, const float* __restrict__ tail) {
  constexpr int EPL = RowAcc<D>::EPL;
  const int lane = threadIdx.x & 63;
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t start = c * CH;
  if (start >= a.nnz) return;
  const int64_t end = min(start + (int64_t)CH, a.nnz);
  if (end >= a.nnz) return;
  const uint64_t last = keys[end - 1];
  if (keys[end] != last) return;                    // no run leaves this chunk
  // keys are sorted: keys[start-1] == last means the whole chunk is a middle
  // piece of a run owned by an earlier chunk
  if (start > 0 && keys[start - 1] == last) return;
  const int e0 = elem0<D>(lane);
  const bool act = D >= 64 || e0 < D;
  RowAcc<D> acc;
#pragma unroll
  for (int u = 0; u < EPL; ++u) acc.v[u] = act ? tail[c * D + e0 + u] : 0.f;
  int64_t j = c + 1;
  while (true) {
#pragma unroll
    for (int u = 0; u < EPL; ++u) if (act) acc.v[u] += head[j * D + e0 + u];
    const int64_t ej = min((j + 1) * CH, a.nnz);
    if (ej < a.nnz && keys[ej] == last) ++j;
    else break;
  }
  apply_update<D>(a, last, acc, lane);
}

struct WsLayout {
  size_t keys_in, keys_out, vals_in, vals_out, bag_of, head, tail, cub, total;
  size_t cub_bytes;
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

WsLayout ws_layout(int64_t nnz, int D) {
  WsLayout L;
  const int64_t nch = (nnz + CH - 1) / CH;
  size_t cub_bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (uint64_t*)nullptr,
                                     (uint64_t*)nullptr, (int32_t*)nullptr,
                                     (int32_t*)nullptr, (int)nnz, 0, 64);
  size_t o = 0;
  L.keys_in = o;  o += al(nnz * 8);
  L.keys_out = o; o += al(nnz * 8);
  L.vals_in = o;  o += al(nnz * 4);
  L.vals_out = o; o += al(nnz * 4);
  L.bag_of = o;   o += al(nnz * 4);
  L.head = o;     o += al((size_t)nch * D * 4);
  L.tail = o;     o += al((size_t)nch * D * 4);
  L.cub = o;      o += al(cub_bytes);
  L.cub_bytes = cub_bytes;
  L.total = o;
  return L;
}

}  // namespace

void embedding_bag_fwd(const EmbFwdArgs& a, hipStream_t s) {
  const int64_t nbags = (int64_t)a.T * a.B;
  if (nbags == 0) return;
  const int lpb = a.D / 4 < 64 ? a.D / 4 : 64;
  const int64_t waves = (nbags * lpb + 63) / 64;
  int64_t blocks = (waves + 3) / 4;
  if (blocks > 8192) blocks = 8192;
#define TDFO_EF(DD)                                                            \
  if (a.out_bf16) hipLaunchKernelGGL((emb_fwd_kernel<DD, true>), dim3(blocks), \
                                     dim3(256), 0, s, a);                     \
  else hipLaunchKernelGGL((emb_fwd_kernel<DD, false>), dim3(blocks),           \
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
}

size_t embedding_bwd_workspace(int64_t nnz, int D) {
  return ws_layout(nnz < 1 ? 1 : nnz, D).total;
}

void embedding_bwd_fused(const EmbBwdArgs& a, hipStream_t s) {
  if (a.nnz <= 0) return;
  const WsLayout L = ws_layout(a.nnz, a.D);
  char* ws = (char*)a.workspace;
  uint64_t* keys_in = (uint64_t*)(ws + L.keys_in);
  uint64_t* keys_out = (uint64_t*)(ws + L.keys_out);
  int32_t* vals_in = (int32_t*)(ws + L.vals_in);
  int32_t* vals_out = (int32_t*)(ws + L.vals_out);
  int32_t* bag_of = (int32_t*)(ws + L.bag_of);
  float* head = (float*)(ws + L.head);
  float* tail = (float*)(ws + L.tail);

  const int64_t nbags = (int64_t)a.T * a.B;
  int64_t kb = (nbags + 255) / 256;
  if (kb > 4096) kb = 4096;
  hipLaunchKernelGGL(emb_keys_kernel, dim3(kb), dim3(256), 0, s, a.row_offset,
                     a.indices, a.offsets, a.T, a.B, keys_in, vals_in, bag_of);
  size_t cub_bytes = L.cub_bytes;
  hipcub::DeviceRadixSort::SortPairs(ws + L.cub, cub_bytes, keys_in, keys_out,
                                     vals_in, vals_out, (int)a.nnz, 0,
                                     a.key_bits, s);
  const int64_t nch = (a.nnz + CH - 1) / CH;
  const int64_t blocks = (nch + 3) / 4;
#define TDFO_EB(DD)                                                            \
  hipLaunchKernelGGL(emb_chunk_kernel<DD>, dim3(blocks), dim3(256), 0, s, a,   \
                     keys_out, vals_out, bag_of, head, tail);                  \
  hipLaunchKernelGGL(emb_combine_kernel<DD>, dim3(blocks), dim3(256), 0, s, a, \
                     keys_out, head, tail)
  switch (a.D) {
    case 16: TDFO_EB(16); break;
    case 32: TDFO_EB(32); break;
    case 64: TDFO_EB(64); break;
    case 128: TDFO_EB(128); break;
    case 256: TDFO_EB(256); break;
    case 512: TDFO_EB(512); break;
  }
#undef TDFO_EB
}

}  // namespace tdfo
