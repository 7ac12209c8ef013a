// Fused small-T multi-head self-attention core for Bert4Rec (K14/K15 in
// SURVEY.md §2.3; reference torchrec/models.py:11-28,49-71).
//
// The reference materialises scores [B,H,T,T], a repeated key-padding mask
// [B,1,T,T] (models.py:214-219), softmax, dropout and P.V as separate ops.
// At T = max_len = 20 and d_k = 8 a whole (sample, head) fits one wave:
//   forward : lane i = query row i; q_i in registers, K/V rows of the head
//             staged in LDS; scores q_i.k_j / sqrt(d_k) with the key mask
//             computed from the ids (never materialised), masked_fill(-1e9),
//             softmax in registers, dropout from a counter-based hash of
//             (seed, step, b, h, i, j) -- regenerated, not stored, by the
//             backward -- then P.V.
//   backward: recompute P row i (lane = i), dP = dO.V^T, dS = P*(dP - rowsum);
//             dQ on the query lanes; then lane = key j for dK = dS^T Q and
//             dV = P~^T dO from the LDS copies of P~ and dS.
// qkv: [B, T, 3E] fp32 = the fused QKV Linear output (q | k | v, each
// H x d_k), out/dout: [B, T, E]; dqkv: [B, T, 3E]. T <= 64, d_k <= 64.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int AT_MAXT = 64;
constexpr int AT_MAXDK = 64;

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // murmur3-style finaliser over a mixed triple (counter-based, stateless)
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// keep-mask of dropout for element (b, h, i, j) at this step
__device__ __forceinline__ bool keep(const AttnArgs& a, int b, int h, int i, int j,
                                     uint32_t step) {
  if (a.rate <= 0.f) return true;
  const uint32_t r = hash3((uint32_t)a.seed ^ (step * 0x632BE5ABu),
                           (uint32_t)((b * a.H + h) * AT_MAXT + i), (uint32_t)j);
  return (float)(r >> 8) * (1.0f / 16777216.0f) >= a.rate;
}

// Fill LDS with this (b, h)'s K and V rows: [T][dk] each.
__device__ __forceinline__ void stage_kv(const AttnArgs& a, int b, int h, float* ks, float* vs,
                                         int lane) {
  const int E = a.H * a.dk, T = a.T, dk = a.dk;
  const float* base = a.qkv + (int64_t)b * T * 3 * E;
  for (int e = lane; e < T * dk; e += 64) {
    const int j = e / dk, d = e - j * dk;
    ks[e] = base[(int64_t)j * 3 * E + E + h * dk + d];
    vs[e] = base[(int64_t)j * 3 * E + 2 * E + h * dk + d];
  }
}

template <int DK>
__global__ __launch_bounds__(64) void attn_fwd_kernel(AttnArgs a) {
  __shared__ float ks[AT_MAXT * AT_MAXDK], vs[AT_MAXT * AT_MAXDK];
  __shared__ int kvalid[AT_MAXT];
  const int lane = threadIdx.x;
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int T = a.T, E = a.H * DK;
  constexpr int dk = DK;
  const uint32_t step = a.step ? (uint32_t)a.step[0] : 0u;
  stage_kv(a, b, h, ks, vs, lane);
  if (lane < T) kvalid[lane] = a.ids[(int64_t)b * T + lane] != a.pad_id;
  __syncthreads();
  if (lane >= T) return;
  const int i = lane;
  float q[DK];
  const float* qp = a.qkv + ((int64_t)b * T + i) * 3 * E + h * dk;
  _Pragma("unroll") for (int d = 0; d < dk; ++d) q[d] = qp[d] * a.scale;
  float mx = -3.0e38f;
  for (int j = 0; j < T; ++j) {
    float s = 0.f;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) s += q[d] * ks[j * dk + d];
    s = kvalid[j] ? s : -1e9f;
    mx = fmaxf(mx, s);
  }
  float sum = 0.f;
  for (int j = 0; j < T; ++j) {
    float s = 0.f;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) s += q[d] * ks[j * dk + d];
    s = kvalid[j] ? s : -1e9f;
    sum += __expf(s - mx);
  }
  const float inv = 1.f / sum, kscale = 1.f / (1.f - a.rate);
  float o[DK];
  _Pragma("unroll") for (int d = 0; d < dk; ++d) o[d] = 0.f;
  for (int j = 0; j < T; ++j) {
    float s = 0.f;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) s += q[d] * ks[j * dk + d];
    s = kvalid[j] ? s : -1e9f;
    float p = __expf(s - mx) * inv;
    p = keep(a, b, h, i, j, step) ? p * kscale : 0.f;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) o[d] += p * vs[j * dk + d];
  }
  float* op = a.out + ((int64_t)b * T + i) * E + h * dk;
  _Pragma("unroll") for (int d = 0; d < dk; ++d) op[d] = o[d];
}

template <int DK>
__global__ __launch_bounds__(64) void attn_bwd_kernel(AttnArgs a) {
  __shared__ float ks[AT_MAXT * AT_MAXDK], vs[AT_MAXT * AT_MAXDK];
  __shared__ float qs[AT_MAXT * AT_MAXDK], dos[AT_MAXT * AT_MAXDK];
  __shared__ float pt[AT_MAXT * AT_MAXT], dsm[AT_MAXT * AT_MAXT];   // [i][j]
  __shared__ int kvalid[AT_MAXT];
  const int lane = threadIdx.x;
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int T = a.T, E = a.H * DK;
  constexpr int dk = DK;
  const uint32_t step = a.step ? (uint32_t)a.step[0] : 0u;
  stage_kv(a, b, h, ks, vs, lane);
  for (int e = lane; e < T * dk; e += 64) {
    const int i = e / dk, d = e - i * dk;
    qs[e] = a.qkv[((int64_t)b * T + i) * 3 * E + h * dk + d] * a.scale;
    dos[e] = a.dout[((int64_t)b * T + i) * E + h * dk + d];
  }
  if (lane < T) kvalid[lane] = a.ids[(int64_t)b * T + lane] != a.pad_id;
  __syncthreads();
  const float kscale = 1.f / (1.f - a.rate);
  if (lane < T) {
    const int i = lane;
    float mx = -3.0e38f;
    for (int j = 0; j < T; ++j) {
      float s = 0.f;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) s += qs[i * dk + d] * ks[j * dk + d];
      s = kvalid[j] ? s : -1e9f;
      mx = fmaxf(mx, s);
    }
    float sum = 0.f;
    for (int j = 0; j < T; ++j) {
      float s = 0.f;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) s += qs[i * dk + d] * ks[j * dk + d];
      s = kvalid[j] ? s : -1e9f;
      sum += __expf(s - mx);
    }
    const float inv = 1.f / sum;
    // P row, dP (through the dropout mask), rowsum(P * dP)
    float rs = 0.f;
    for (int j = 0; j < T; ++j) {
      float s = 0.f;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) s += qs[i * dk + d] * ks[j * dk + d];
      s = kvalid[j] ? s : -1e9f;
      const float p = __expf(s - mx) * inv;
      const float m = keep(a, b, h, i, j, step) ? kscale : 0.f;
      float dpt = 0.f;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) dpt += dos[i * dk + d] * vs[j * dk + d];
      const float dp = dpt * m;
      pt[i * AT_MAXT + j] = p * m;          // P~ (post-dropout)
      dsm[i * AT_MAXT + j] = dp;            // dP for now
      rs += p * dp;
    }
    // dS = P * (dP - rs); masked keys get no gradient (masked_fill)
    float dq[DK];
    _Pragma("unroll") for (int d = 0; d < dk; ++d) dq[d] = 0.f;
    for (int j = 0; j < T; ++j) {
      float s = 0.f;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) s += qs[i * dk + d] * ks[j * dk + d];
      s = kvalid[j] ? s : -1e9f;
      const float pp = __expf(s - mx) * inv;
      const float ds = kvalid[j] ? pp * (dsm[i * AT_MAXT + j] - rs) : 0.f;
      dsm[i * AT_MAXT + j] = ds;
      _Pragma("unroll") for (int d = 0; d < dk; ++d) dq[d] += ds * ks[j * dk + d];
    }
    float* dqp = a.dqkv + ((int64_t)b * T + i) * 3 * E + h * dk;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) dqp[d] = dq[d] * a.scale;
  }
  __syncthreads();
  if (lane < T) {
    const int j = lane;
    float dkk[DK], dv[DK];
    _Pragma("unroll") for (int d = 0; d < dk; ++d) { dkk[d] = 0.f; dv[d] = 0.f; }
    for (int i = 0; i < T; ++i) {
      const float ds = dsm[i * AT_MAXT + j], p = pt[i * AT_MAXT + j];
      _Pragma("unroll") for (int d = 0; d < dk; ++d) {
        dkk[d] += ds * qs[i * dk + d];     // qs already carries 1/sqrt(dk)
        dv[d] += p * dos[i * dk + d];
      }
    }
    float* base = a.dqkv + ((int64_t)b * T + j) * 3 * E + h * dk;
    _Pragma("unroll") for (int d = 0; d < dk; ++d) {
      base[E + d] = dkk[d];
      base[2 * E + d] = dv[d];
    }
  }
}

}  // namespace

#define TDFO_ATTN_DISPATCH(KERNEL)                                               \
  switch (a.dk) {                                                                \
    case 4: hipLaunchKernelGGL(KERNEL<4>, dim3(a.B * a.H), dim3(64), 0, s, a); break;   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, dim3(a.B * a.H), dim3(64), 0, s, a); break;   \
    case 16: hipLaunchKernelGGL(KERNEL<16>, dim3(a.B * a.H), dim3(64), 0, s, a); break; \
    case 32: hipLaunchKernelGGL(KERNEL<32>, dim3(a.B * a.H), dim3(64), 0, s, a); break; \
    case 64: hipLaunchKernelGGL(KERNEL<64>, dim3(a.B * a.H), dim3(64), 0, s, a); break; \
    default: throw std::runtime_error("attention: d_k must be 4/8/16/32/64");          \
  }

void attention_fwd(const AttnArgs& a, hipStream_t s) {
  if (a.B <= 0) return;
  if (a.T > AT_MAXT) throw std::runtime_error("attention: T > 64");
  TDFO_ATTN_DISPATCH(attn_fwd_kernel);
  TDFO_CHECK_HIP(hipGetLastError());
}

void attention_bwd(const AttnArgs& a, hipStream_t s) {
  if (a.B <= 0) return;
  if (a.T > AT_MAXT) throw std::runtime_error("attention: T > 64");
  TDFO_ATTN_DISPATCH(attn_bwd_kernel);
  TDFO_CHECK_HIP(hipGetLastError());
}
#undef TDFO_ATTN_DISPATCH

}  // namespace tdfo
