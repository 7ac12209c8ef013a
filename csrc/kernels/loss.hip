// Loss head, deterministic reductions and the device-side AUC histogram.
//
// head_bce fuses the final K->1 layer, sigmoid BCE-with-logits (K5), its
// gradient, the ReLU mask of the layer below and the partial sums of dW/db:
// one pass over H produces everything the backward needs (the reference runs
// these as separate XLA / torch ops: jax-flax/train.py:35, torchrec-style
// BCE). Cross-sample sums go to per-block fp32 partial rows that
// reduce_rows() adds in a fixed order, so gradients are bitwise reproducible.
// auc_hist replaces the host-side tf.keras AUC of jax-flax/train_dp.py:215
// (a per-step device->host sync) with on-device counts.
#include "tdfo_common.h"
#include "tdfo_kernels.h"
#include "tdfo_reduce_adam.h"

namespace tdfo {
namespace {

constexpr int HEAD_SPB = 16;  // samples per block (4 per wave)
static_assert(HEAD_SPB % 4 == 0, "head: samples split over the 4 waves");

template <int K>
__global__ __launch_bounds__(256) void head_bce_kernel(
    const uint16_t* __restrict__ H, int64_t ldh, int B,
    const float* __restrict__ w, const float* __restrict__ bptr,
    const float* __restrict__ label, float inv_n, int relu_mask,
    float* __restrict__ logits, uint16_t* __restrict__ dH, int64_t lddh,
    float* __restrict__ part) {
  constexpr int EPL = K >= 64 ? K / 64 : 1;   // K < 64: lanes >= K idle
  __shared__ float red[4][K + 2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e0 = lane * EPL;
  const bool act = e0 < K;
  float wr[EPL], dw[EPL];
#pragma unroll
  for (int u = 0; u < EPL; ++u) { wr[u] = act ? w[e0 + u] : 0.f; dw[u] = 0.f; }
  const float bias = bptr[0];
  float db = 0.f, lsum = 0.f;
  const int s0 = blockIdx.x * HEAD_SPB;
  // the wave's HEAD_SPB / 4 samples: every H row and label loaded before the
  // first use (clamped rows; the loop below stops at B), so the wave pays one
  // memory round trip instead of one per sample (same per-sample math and
  // accumulation order as a sample-at-a-time loop)
  constexpr int SPW = HEAD_SPB / 4;
  float hv[SPW][EPL], yv[SPW];
#pragma unroll
  for (int q = 0; q < SPW; ++q) {
    const int s = min(s0 + wv + 4 * q, B - 1);
    const uint16_t* hp = H + (int64_t)s * ldh + e0;
#pragma unroll
    for (int u = 0; u < EPL; ++u) hv[q][u] = act ? bf2f(hp[u]) : 0.f;
    yv[q] = label[s];
  }
#pragma unroll
  for (int q = 0; q < SPW; ++q) {
    const int s = s0 + wv + 4 * q;
    if (s >= B) break;
    float d = 0.f;
#pragma unroll
    for (int u = 0; u < EPL; ++u) d += hv[q][u] * wr[u];
    const float x = wave_sum(d) + bias;
    const float y = yv[q];
    const float sig = 1.f / (1.f + __expf(-x));
    const float g = (sig - y) * inv_n;
    if (lane == 0) {
      logits[s] = x;
      lsum += fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
      db += g;
    }
    uint16_t* dp = dH + (int64_t)s * lddh + e0;
    if (act) {
#pragma unroll
      for (int u = 0; u < EPL; ++u) {
        float gh = g * wr[u];
        if (relu_mask && !(hv[q][u] > 0.f)) gh = 0.f;
        dp[u] = f2bf(gh);
        dw[u] += g * hv[q][u];
      }
    }
  }
  if (act) {
#pragma unroll
    for (int u = 0; u < EPL; ++u) red[wv][e0 + u] = dw[u];
  }
  if (lane == 0) { red[wv][K] = db; red[wv][K + 1] = lsum; }
  __syncthreads();
  for (int j = threadIdx.x; j < K + 2; j += 256)
    part[(int64_t)blockIdx.x * (K + 2) + j] =
        red[0][j] + red[1][j] + red[2][j] + red[3][j];
}

// out[j] = sum_r in[r*ld + j]: COLS columns x (256/COLS) row phases per
// block, fixed-order LDS combine (bitwise reproducible).
template <int COLS>
__global__ __launch_bounds__(256) void reduce_rows_kernel(
    const float* __restrict__ in, int rows, int64_t n, int64_t ld,
    float* __restrict__ out, int accumulate, float scale, const int64_t* __restrict__ idx) {
  constexpr int PH = 256 / COLS;
  __shared__ float red[PH][COLS];
  const int c = threadIdx.x % COLS, ph = threadIdx.x / COLS;
  for (int64_t j0 = (int64_t)blockIdx.x * COLS; j0 < n; j0 += (int64_t)gridDim.x * COLS) {
    const int64_t j = j0 + c;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (j < n) {
      int r = ph;
      for (; r + 3 * PH < rows; r += 4 * PH) {
        s0 += in[(int64_t)r * ld + j];
        s1 += in[(int64_t)(r + PH) * ld + j];
        s2 += in[(int64_t)(r + 2 * PH) * ld + j];
        s3 += in[(int64_t)(r + 3 * PH) * ld + j];
      }
      for (; r < rows; r += PH) s0 += in[(int64_t)r * ld + j];
    }
    red[ph][c] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (ph == 0 && j < n) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < PH; ++q) t += red[q][c];
      t *= scale;
      const int64_t o = idx ? idx[j] : j;
      out[o] = accumulate ? out[o] + t : t;
    }
    __syncthreads();
  }
}

// Head epilogue in one launch: grad[j] = sum_r part[r][j] (j <= K) and
// loss_acc[0] += sum_r part[r][K+1] with reduce_rows' fixed-order structure
// (16 columns x 16 row phases per block), plus the step counters
// bump[i][1] += 1 of the optimizers that run later in the step (saves two
// reduce launches and two counter-increment launches).
__global__ __launch_bounds__(256) void head_reduce_kernel(const float* __restrict__ part,
                                                          int nparts, int K,
                                                          float* __restrict__ grad,
                                                          float* __restrict__ loss_acc,
                                                          HeadBumps bumps) {
  constexpr int COLS = 16, PH = 256 / COLS;
  __shared__ float red[PH][COLS];
  const int ld = K + 2;
  const int c = threadIdx.x % COLS, ph = threadIdx.x / COLS;
  const int j = blockIdx.x * COLS + c;
  red[ph][c] = (j < ld && nparts > 0) ? col_phase_sum<PH>(part, nparts, ld, j, ph) : 0.f;
  __syncthreads();
  if (ph == 0 && j < ld) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < PH; ++q) t += red[q][c];
    if (j <= K) grad[j] = t;
    else loss_acc[0] += t;
  }
  if (blockIdx.x == 0 && threadIdx.x < bumps.n) bumps.p[threadIdx.x][1] += 1.f;
}

// reduce_rows + the flat Adam / AdamW + the loss accumulation (+ the AUC
// binning) of a small model's step in one launch (TwoTower: 2,400 parameters
// from 128 block partials; four dependent ~4.5-us launches before,
// profiles/r05/two_tower). Same column sums as reduce_rows_kernel<16>, same
// adam_elem as dense_opt_kernel: bit-identical to the separate launches.
__global__ __launch_bounds__(256) void reduce_adam_kernel(ReduceAdamArgs a) {
  __shared__ float red[RA_PH][RA_COLS];
  __shared__ unsigned int lh[2 * REDUCE_ADAM_MAX_NB];
  reduce_adam_unit(a, blockIdx.x, threadIdx.x, red, lh);
}

constexpr int COLSUM_CHUNKS = 16;

// Column sums of a bf16 [M, N] matrix: block = 64 columns (8 x 16-B groups)
// x 32 row phases over one of COLSUM_CHUNKS row chunks.
__global__ __launch_bounds__(256) void colsum_kernel(const uint16_t* __restrict__ x,
                                                     int M, int N, int64_t ldx,
                                                     float* __restrict__ part) {
  __shared__ float red[32][65];
  const int cg = threadIdx.x & 7, ph = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cg * 8;
  const int rows_per = (M + COLSUM_CHUNKS - 1) / COLSUM_CHUNKS;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(M, r0 + rows_per);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < N) {
    for (int r = r0 + ph; r < r1; r += 32) {
      const uint4 v = *(const uint4*)(x + (int64_t)r * ldx + c0);
      const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += bf2f((uint16_t)(u[q] & 0xffff));
        acc[2 * q + 1] += bf2f((uint16_t)(u[q] >> 16));
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[ph][cg * 8 + q] = acc[q];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int col = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
    for (int q = 0; q < 32; ++q) t += red[q][threadIdx.x];
    if (col < N) part[(int64_t)blockIdx.y * N + col] = t;
  }
}

__global__ __launch_bounds__(256) void auc_hist_kernel(
    const float* __restrict__ logits, const float* __restrict__ labels, int n,
    int nb, unsigned long long* __restrict__ hist) {
  extern __shared__ unsigned int lh[];
  for (int i = threadIdx.x; i < 2 * nb; i += 256) lh[i] = 0;
  __syncthreads();
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float p = 1.f / (1.f + __expf(-logits[i]));
    int bkt = (int)(p * nb);
    bkt = bkt < 0 ? 0 : (bkt >= nb ? nb - 1 : bkt);
    atomicAdd(&lh[(labels[i] > 0.5f ? nb : 0) + bkt], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * nb; i += 256)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

}  // namespace

int head_bce_parts(int B) { return (B + HEAD_SPB - 1) / HEAD_SPB; }

void head_bce(const uint16_t* H, int64_t ldh, int B, int K, const float* w,
              const float* b, const float* label, float inv_n, int relu_mask,
              float* logits, uint16_t* dH, int64_t lddh, float* part,
              int nparts, hipStream_t s) {
  if (B <= 0) return;
  dim3 grid(nparts);
#define TDFO_HB(KK)                                                            \
  hipLaunchKernelGGL(head_bce_kernel<KK>, grid, dim3(256), 0, s, H, ldh, B, w, \
                     b, label, inv_n, relu_mask, logits, dH, lddh, part)
  switch (K) {
    case 16: TDFO_HB(16); break;
    case 32: TDFO_HB(32); break;
    case 64: TDFO_HB(64); break;
    case 128: TDFO_HB(128); break;
    case 256: TDFO_HB(256); break;
    case 512: TDFO_HB(512); break;
    case 1024: TDFO_HB(1024); break;
  }
#undef TDFO_HB
}

void reduce_rows(const float* in, int rows, int64_t n, int64_t ld, float* out,
                 int accumulate, float scale, hipStream_t s, const int64_t* idx) {
  if (n <= 0) return;
  if (n >= 16384) {
    int64_t blocks = (n + 63) / 64;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(reduce_rows_kernel<64>, dim3(blocks), dim3(256), 0, s, in,
                       rows, n, ld, out, accumulate, scale, idx);
  } else {
    int64_t blocks = (n + 15) / 16;
    hipLaunchKernelGGL(reduce_rows_kernel<16>, dim3(blocks), dim3(256), 0, s, in,
                       rows, n, ld, out, accumulate, scale, idx);
  }
}

// Split-K weight-grad slabs of several layers summed in ONE launch (the
// multi-rank step's per-bucket reduce before the dense all-reduce; one
// reduce_rows launch per layer cost ~6.7 us each, profiles/r03/mstreams):
// out[j] = sum_{r = 0..S-1} in[r * n + j] in split order (deterministic),
// 16 B per thread, grid-stride over the segments' concatenated float4 work.
__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabReduceArgs a) {
  const int64_t total = a.start[a.nseg];
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    // the segment by wave-uniform-ish selects over the kernel-argument table
    // (a dynamically indexed table compiles to dependent loads)
    const float* in = a.seg[0].in;
    float* out = a.seg[0].out;
    int64_t n = a.seg[0].n, s0 = 0;
    int S = a.seg[0].S;
#pragma unroll
    for (int k = 1; k < SLAB_MAX_SEGS; ++k) {
      const bool here = k < a.nseg && q >= a.start[k];
      in = here ? a.seg[k].in : in;
      out = here ? a.seg[k].out : out;
      n = here ? a.seg[k].n : n;
      S = here ? a.seg[k].S : S;
      s0 = here ? a.start[k] : s0;
    }
    const int64_t j = (q - s0) * 4;
    float4 acc = *(const float4*)(in + j);
    // slabs 1.. in order, 8 loads in flight (clamped addresses: no branch
    // around a load), so an S-way split is not S dependent round trips
    for (int r0 = 1; r0 < S; r0 += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *(const float4*)(in + (int64_t)min(r0 + u, S - 1) * n + j);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r0 + u < S) { acc.x += t[u].x; acc.y += t[u].y; acc.z += t[u].z; acc.w += t[u].w; }
    }
    *(float4*)(out + j) = acc;
  }
}

void slab_reduce(const SlabReduceArgs& a, hipStream_t s) {
  const int64_t total = a.start[a.nseg];
  if (total <= 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(blocks), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

int colsum_parts(int M) { return COLSUM_CHUNKS; }

void reduce_adam(const ReduceAdamArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(reduce_adam_kernel, dim3(reduce_adam_units(a)), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

namespace {
thread_local bool g_hr_pending = false;
thread_local HeadReduceJob g_hr{};
}  // namespace

void head_reduce_park(const HeadReduceJob& j) {
  if (g_hr_pending) throw std::runtime_error("head_reduce: a parked job is still waiting");
  g_hr = j;
  g_hr_pending = true;
}

bool head_reduce_take(HeadReduceJob* j) {
  if (!g_hr_pending) return false;
  *j = g_hr;
  g_hr_pending = false;
  return true;
}

void head_reduce_flush(hipStream_t s) {
  HeadReduceJob j;
  if (head_reduce_take(&j)) head_reduce(j.part, j.nparts, j.K, j.grad, j.loss_acc, j.bumps, s);
}

void head_reduce(const float* part, int nparts, int K, float* grad, float* loss_acc,
                 const HeadBumps& bumps, hipStream_t s) {
  hipLaunchKernelGGL(head_reduce_kernel, dim3((K + 2 + 15) / 16), dim3(256), 0, s, part, nparts,
                     K, grad, loss_acc, bumps);
  TDFO_CHECK_HIP(hipGetLastError());
}

void colsum_bf16(const uint16_t* x, int M, int N, int64_t ldx, float* part,
                 int nparts, float* out, int accumulate, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  dim3 grid((N + 63) / 64, COLSUM_CHUNKS);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, s, x, M, N, ldx, part);
  reduce_rows(part, nparts, N, N, out, accumulate, 1.f, s);
}

void auc_hist(const float* logits, const float* labels, int n, int nb,
              unsigned long long* hist, hipStream_t s) {
  if (n <= 0) return;
  int blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(auc_hist_kernel, dim3(blocks), dim3(256),
                     (size_t)2 * nb * sizeof(unsigned int), s, logits, labels,
                     n, nb, hist);
}

}  // namespace tdfo
