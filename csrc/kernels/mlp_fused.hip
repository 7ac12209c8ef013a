// Fused three-layer MLP forward for the DLRM / DCN-v2 bottom MLP
// (13 dense features + bias column, K0 = 64 -> 512 -> 256 -> 128, ReLU after
// every layer; reference call sites jax-flax/models.py:59-70 Dense stacks,
// torchrec/models.py:82-88).
//
// The three GEMMs of this MLP are tiny (8192 x 512 x 64, 8192 x 256 x 512,
// 8192 x 128 x 256: 2.6 GFLOP together) and, launched one by one, each pays a
// launch, a pipeline fill and a drain (6-12 us apiece on MI355X, ~28 us for
// the three). Here one 512-thread block owns 32 samples and runs all three
// layers on-chip: the input rows and every intermediate activation stay in
// LDS, each layer's 32-feature output tiles are computed by one wave with
// v_mfma_f32_32x32x16_bf16, and the weights (384 KB, L2-resident: every block
// reads the same ones) are loaded straight into MFMA operand registers, issued
// ahead of the layers that use them.
//
// Operands are swapped (C^T = W X^T): A = weight rows (lane l: row n0 +
// (l & 31), k = 16 ks + 8 (l >> 5) + j), B = activation rows from LDS (lane
// l: sample l & 31, same k), so each lane's 16 accumulators are 4 runs of 4
// consecutive features of ONE sample -> 8-B LDS writes into the next layer's
// input image. Activation LDS rows are padded by 16 B: the 16 lanes of a
// ds_read_b128 group read 16 rows at the same column from 16 distinct
// 16-B bank slots.
//
// Every layer's activations are also stored to HBM (row-major, 16-B stores of
// whole LDS rows) because the backward reads them; the store of layer l
// overlaps layer l+1's MFMAs.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int MR = 32;          // samples per block
constexpr int MT = 512;         // threads (8 waves, 2 per SIMD)
constexpr int MW = MT / 64;

template <int K>
struct Img {
  static constexpr int P = K + 8;           // row pitch (elements)
  static constexpr int SZ = MR * P;         // elements
};

// A-operand fragments of one 32-feature weight tile: lane l holds
// W[n0 + (l & 31)][16 ks + 8 (l >> 5) .. +8].
template <int K>
__device__ __forceinline__ void load_wtile(bf16x8_t (&wf)[K / 16], const uint16_t* __restrict__ W,
                                           int64_t ldw, int n0, int lane) {
  const uint16_t* wrow = W + (int64_t)(n0 + (lane & 31)) * ldw + 8 * (lane >> 5);
#pragma unroll
  for (int ks = 0; ks < K / 16; ++ks) wf[ks] = *(const bf16x8_t*)(wrow + 16 * ks);
}

// The 16 bias values of a tile in accumulator order (bv[4g + q] = bias of
// feature n0 + 8g + 4h + q), zeros without a bias; one wave-uniform branch
// around all 16 loads (a select per load makes hipcc wait for each one)
__device__ __forceinline__ void load_bias(float (&bv)[16], const float* __restrict__ bias,
                                          int64_t bstride, int n0, int lane) {
  const int h = lane >> 5;
  if (bias) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      bv[r] = bias[(int64_t)(n0 + 8 * (r >> 2) + 4 * h + (r & 3)) * bstride];
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = 0.f;
  }
}

// out[s][n0 + f] = relu(sum_k W[n0 + f][k] in[s][k] + bias) for one tile
// (C^T = W X^T: acc[4g + q] = C^T[n0 + 8g + 4h + q][sample l & 31]).
template <int K, int N>
__device__ __forceinline__ void tile_fwd(const bf16x8_t (&wf)[K / 16], const float (&bv)[16],
                                         const uint16_t* ins, uint16_t* outs, int n0, int lane) {
  const int r = lane & 31, h = lane >> 5;
  f32x16_t acc = {};
  const uint16_t* xrow = ins + r * Img<K>::P + 8 * h;
#pragma unroll
  for (int ks = 0; ks < K / 16; ++ks) {
    const bf16x8_t xf = *(const bf16x8_t*)(xrow + 16 * ks);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], xf, acc, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int f = n0 + 8 * g + 4 * h;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = fmaxf(acc[4 * g + q] + bv[4 * g + q], 0.f);
    *(uint2*)(outs + r * Img<N>::P + f) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
  }
}

// Block barrier for the LDS images only: __syncthreads would also drain every
// outstanding global load and store (vmcnt(0)), i.e. wait for the prefetched
// weights and the activation stores of the previous layer.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Store an [MR][N] LDS image to rows m0.. of a row-major [B][ld] tensor.
template <int N>
__device__ __forceinline__ void store_rows(const uint16_t* img, uint16_t* __restrict__ y,
                                           int64_t ld, int m0, int rows, int tid) {
  constexpr int CPR = N / 8;                 // 16-B chunks per row
  for (int c = tid; c < MR * CPR; c += MT) {
    const int rr = c / CPR, ch = c - rr * CPR;
    if (rr < rows)
      *(uint4*)(y + (int64_t)(m0 + rr) * ld + ch * 8) = *(const uint4*)(img + rr * Img<N>::P + ch * 8);
  }
}

// Wave w: layer-0 tiles w and w + 8, layer-1 tile w, layer-2 tile w (w < 4).
// Every weight fragment a wave needs for layers 0 and 1 is requested before
// the first MFMA, layer 2's right after layer 1's MFMAs are issued: the
// weight loads (L2 hits) overlap the input staging and the earlier layers
// instead of stalling each tile (one-tile-at-a-time loading measured 45 us
// for this kernel in the DLRM step).
template <int K0, int N0, int N1, int N2>
__global__ __launch_bounds__(MT) void mlp3_fwd_kernel(Mlp3Args a) {
  static_assert(N0 == 32 * 2 * MW && N1 == 32 * MW && N2 == 32 * (MW / 2), "tile split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[Img<K0>::SZ + Img<N0>::SZ +
                                                        Img<N1>::SZ + Img<N2>::SZ];
  uint16_t* x0s = smem;
  uint16_t* h1s = x0s + Img<K0>::SZ;
  uint16_t* h2s = h1s + Img<N0>::SZ;
  uint16_t* h3s = h2s + Img<N1>::SZ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * MR;
  const int rows = min(MR, a.B - m0);
  // input rows first (the weight loads queue behind them), clamped: rows past
  // B repeat the last one and are never stored
  constexpr int CPR0 = K0 / 8;
  static_assert(MR * CPR0 <= MT, "one input chunk per thread");
  const bool xin = tid < MR * CPR0;
  const int xr = tid / CPR0, xc = tid - xr * CPR0;
  uint4 xv = make_uint4(0, 0, 0, 0);
  if (xin) xv = *(const uint4*)(a.x + (int64_t)(m0 + min(xr, rows - 1)) * a.ldx + xc * 8);
  // issue order = use order (vmcnt retires loads in order)
  bf16x8_t w0a[K0 / 16], w0b[K0 / 16], w1f[N0 / 16];
  float b0a[16], b0b[16], b1[16];
  load_wtile<K0>(w0a, a.w[0], a.ldw[0], 32 * w, lane);
  load_bias(b0a, a.bias[0], a.bstride[0], 32 * w, lane);
  load_wtile<K0>(w0b, a.w[0], a.ldw[0], 32 * (w + MW), lane);
  load_bias(b0b, a.bias[0], a.bstride[0], 32 * (w + MW), lane);
  load_wtile<N0>(w1f, a.w[1], a.ldw[1], 32 * w, lane);
  load_bias(b1, a.bias[1], a.bstride[1], 32 * w, lane);
  if (xin) *(uint4*)(x0s + xr * Img<K0>::P + xc * 8) = xv;
  lds_barrier();
  tile_fwd<K0, N0>(w0a, b0a, x0s, h1s, 32 * w, lane);
  tile_fwd<K0, N0>(w0b, b0b, x0s, h1s, 32 * (w + MW), lane);
  lds_barrier();
  store_rows<N0>(h1s, a.y[0], a.ldy[0], m0, rows, tid);
  tile_fwd<N0, N1>(w1f, b1, h1s, h2s, 32 * w, lane);
  bf16x8_t w2f[N1 / 16];
  float b2[16];
  const bool l2 = w < MW / 2;
  if (l2) {
    load_wtile<N1>(w2f, a.w[2], a.ldw[2], 32 * w, lane);
    load_bias(b2, a.bias[2], a.bstride[2], 32 * w, lane);
  }
  lds_barrier();
  store_rows<N1>(h2s, a.y[1], a.ldy[1], m0, rows, tid);
  if (l2) tile_fwd<N1, N2>(w2f, b2, h2s, h3s, 32 * w, lane);
  lds_barrier();
  store_rows<N2>(h3s, a.y[2], a.ldy[2], m0, rows, tid);
}

}  // namespace

bool mlp3_fwd_supported(int k0, int n0, int n1, int n2) {
  return k0 == 64 && n0 == 512 && n1 == 256 && n2 == 128;
}

void mlp3_fwd(const Mlp3Args& a, hipStream_t s) {
  if (a.B <= 0) return;
  if (!mlp3_fwd_supported(a.k[0], a.k[1], a.k[2], a.k[3]))
    throw std::runtime_error("mlp3_fwd: unsupported widths");
  const int blocks = (a.B + MR - 1) / MR;
  hipLaunchKernelGGL((mlp3_fwd_kernel<64, 512, 256, 128>), dim3(blocks), dim3(MT), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
