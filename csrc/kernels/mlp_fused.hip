// Fused three-layer MLP forward for the DLRM / DCN-v2 bottom MLP
// (13 -> 512 -> 256 -> 128, each layer bias + ReLU), one launch instead of
// three GEMMs: a block owns 32 batch rows and carries them through all three
// layers with the activations in LDS; each layer's output is also written to
// global memory (the backward reads it: ReLU masks and weight-grad inputs).
//
// Why: the three bottom GEMMs are ~0.3-2 GFLOP each, so every launch is mostly
// ramp and drain (26.8 us in the DLRM-1TB step for 2.7 GFLOP,
// profiles/r04/final/prof_dlrm/step_lanes.txt), and they sit on the MLP
// stream's critical path right before the interaction forward.
//
// Layout per layer (K in, N out, 4 waves): wave w owns output columns
// [w N/4, (w+1) N/4) for all 32 rows (2 x N/64 fragments of
// v_mfma_f32_16x16x32_bf16). The A operand (activations, row-major, K
// contiguous) comes from LDS with one ds_read_b128 per fragment (rows padded
// by 16 B: conflict-free); the B operand (weights [N][K] row-major, L2
// resident, every block reads all of them) comes straight from global memory
// into registers -- the loop is fully unrolled so the loads issue ahead of
// the MFMAs. As in the GEMM kernels the weight fragment is the MFMA's first
// operand, so lane l / register r of accumulator (i, j) holds
// C[16 i + (l & 15)][16 j + 4 (l >> 4) + r]; k is accumulated in the same
// order as the tiled GEMMs (32-deep steps), so the result equals the
// three-GEMM path.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int MR = 32;        // batch rows per block
constexpr int PADE = 8;       // LDS row padding (elements)

template <int K, int N, bool TO_LDS>
__device__ __forceinline__ void mlp_layer(const uint16_t* lds_in, const uint16_t* __restrict__ W,
                                          int64_t ldw, const float* __restrict__ bias,
                                          int64_t bstride, uint16_t* __restrict__ gout,
                                          int64_t ldo, uint16_t* lds_out, int row0, int w,
                                          int lane) {
  static_assert(K % 32 == 0 && N % 64 == 0, "mlp_layer: K % 32, N % 64");
  constexpr int NT = N / 64;             // 16-column fragments per wave
  constexpr int KS = K / 32;
  const int n0 = w * (N / 4);
  const int r = lane & 15, g = lane >> 4;
  f32x4_t acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8_t bfr[NT], af[2];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      bfr[j] = *(const bf16x8_t*)(W + (int64_t)(n0 + 16 * j + r) * ldw + ks * 32 + 8 * g);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *(const bf16x8_t*)(lds_in + (16 * i + r) * (K + PADE) + ks * 32 + 8 * g);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
  // bias + ReLU; 4 consecutive columns of one row per fragment and lane
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + 16 * j + 4 * g;
    float b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) b[q] = bias ? bias[(int64_t)(n + q) * bstride] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = 16 * i + r;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fmaxf(acc[i][j][q] + b[q], 0.f);
      const uint2 pk = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      *(uint2*)(gout + (int64_t)(row0 + m) * ldo + n) = pk;
      if constexpr (TO_LDS) *(uint2*)(lds_out + m * (N + PADE) + n) = pk;
    }
  }
}

template <int K0, int N0, int N1, int N2>
__global__ __launch_bounds__(256) void mlp3_fwd_kernel(Mlp3Args a) {
  __shared__ __attribute__((aligned(16))) uint16_t s_x[MR * (K0 + PADE)];
  __shared__ __attribute__((aligned(16))) uint16_t s_h1[MR * (N0 + PADE)];
  __shared__ __attribute__((aligned(16))) uint16_t s_h2[MR * (N1 + PADE)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row0 = blockIdx.x * MR;
  // input rows: 16 B per thread per pass
  constexpr int CPR = K0 / 8;            // 16-B chunks per row
#pragma unroll
  for (int c = tid; c < MR * CPR; c += 256) {
    const int m = c / CPR, q = c - (c / CPR) * CPR;
    *(uint4*)(s_x + m * (K0 + PADE) + q * 8) = *(const uint4*)(a.x + (int64_t)(row0 + m) * a.ldx + q * 8);
  }
  __syncthreads();
  mlp_layer<K0, N0, true>(s_x, a.W[0], a.ldw[0], a.bias[0], a.bstride[0], a.out[0], a.ldo[0], s_h1,
                          row0, w, lane);
  __syncthreads();
  mlp_layer<N0, N1, true>(s_h1, a.W[1], a.ldw[1], a.bias[1], a.bstride[1], a.out[1], a.ldo[1], s_h2,
                          row0, w, lane);
  __syncthreads();
  mlp_layer<N1, N2, false>(s_h2, a.W[2], a.ldw[2], a.bias[2], a.bstride[2], a.out[2], a.ldo[2],
                           nullptr, row0, w, lane);
}

}  // namespace

bool mlp3_fwd_supported(int K0, int N0, int N1, int N2, int B) {
  return K0 == 64 && N0 == 512 && N1 == 256 && N2 == 128 && B % MR == 0;
}

void mlp3_fwd(const Mlp3Args& a, int K0, int N0, int N1, int N2, hipStream_t s) {
  if (!mlp3_fwd_supported(K0, N0, N1, N2, a.B))
    throw std::runtime_error("mlp3_fwd: unsupported shape");
  hipLaunchKernelGGL((mlp3_fwd_kernel<64, 512, 256, 128>), dim3(a.B / MR), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
