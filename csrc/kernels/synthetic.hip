// On-device twin of the C++ synthetic Criteo generator (csrc/data/synthetic.cpp;
// SURVEY.md §2.7 NS1): one launch writes a whole fresh batch -- dense
// features, table-major ids (uniform or Zipf), labels from the fixed logistic
// teacher -- so the benchmark can draw a new batch every step on a side
// stream instead of cycling a pool of pre-generated batches.
//
// Counter-based like the host generator: every value is a splitmix64 hash of
// (seed, rank, batch index, sample, field), with the same hash chain, so a
// uniform-id batch is bit-identical to the host's (ids are pure integer
// arithmetic; dense features use the same float ln series with FMA
// contraction off). Labels sum the teacher score in another order (per-table
// groups), which can only flip a label whose uniform draw lies within
// ~1e-16 of its probability.
//
// Block = 64 samples x 4 table groups (256 threads): lane b of group g draws
// the ids of tables t = g, g + 4, ... for sample b (64 consecutive samples ->
// coalesced id stores per table) and its teacher-score part; the four parts
// are summed through LDS in a fixed order.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

#pragma clang fp contract(off)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double u01(uint64_t h) {
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

// ln(x), x >= 1: exponent + 2 atanh((m-1)/(m+1)) series (host fast_ln)
__device__ __forceinline__ float fast_ln(float x) {
  uint32_t b = __float_as_uint(x);
  const int e = (int)(b >> 23) - 127;
  b = (b & 0x007fffffu) | 0x3f800000u;
  const float m = __uint_as_float(b);
  const float z = (m - 1.f) / (m + 1.f), z2 = z * z;
  const float at = z * (1.f + z2 * (1.f / 3 + z2 * (1.f / 5 + z2 * (1.f / 7 + z2 * (1.f / 9)))));
  return (float)e * 0.69314718f + 2.f * at;
}

constexpr int SB = 64;   // samples per block
constexpr int TG = 4;    // table groups per block

__global__ __launch_bounds__(256) void synth_criteo_kernel(SynthArgs a) {
  __shared__ double part[TG][SB];
  const int bl = threadIdx.x & (SB - 1), g = threadIdx.x / SB;
  const int b = blockIdx.x * SB + bl;
  const bool live = b < a.B;
  const uint64_t key =
      mix64(a.seed * 0x100000001B3ull ^ mix64((uint64_t)a.rank << 40 ^ (uint64_t)a.batch_index));
  const uint64_t rk = mix64(key ^ (uint64_t)b * 0xD6E8FEB86659FD93ull);
  const double bias_w = 3.0 / sqrt((double)a.T);
  double sc = 0.0;
  if (live && g == 0) {
    for (int j = 0; j < a.num_dense; ++j) {
      const float x = fast_ln(1.f + (float)(u01(mix64(rk + j)) * 100.0));
      a.dense[(int64_t)b * a.num_dense + j] = x;
      sc += (x - 3.6) * a.w_dense[j] * 2.0;
    }
  }
  if (live) {
    for (int t = g; t < a.T; t += TG) {
      const int L = a.pooling[t];
      const uint64_t r = (uint64_t)a.rows[t];
      const uint64_t tk = (uint64_t)(t + 1) << 32;
      int64_t* out = a.ids + a.base[t] + (int64_t)b * L;
      for (int l = 0; l < L; ++l) {
        const uint64_t h = mix64(rk ^ tk ^ (uint64_t)(l + 1000));
        int64_t id;
        if (a.dist == 1 && r > 1) {
          const double x = pow((pow((double)r, 1 - a.alpha) - 1) * u01(h) + 1, 1 / (1 - a.alpha));
          id = (int64_t)x - 1;
          id = id < 0 ? 0 : (id > (int64_t)r - 1 ? (int64_t)r - 1 : id);
        } else {
          id = (int64_t)__umul64hi(h, r);
        }
        out[l] = id;
        if (l == 0) sc += a.table_bias[t * 64 + (id & 63)] * bias_w;
      }
    }
  }
  part[g][bl] = sc;
  __syncthreads();
  if (live && g == 0) {
    double s = -1.1;
    for (int q = 0; q < TG; ++q) s += part[q][bl];
    const double p = 1.0 / (1.0 + exp(-s));
    a.label[b] = u01(mix64(rk ^ 0xABCDEFull)) < p ? 1.f : 0.f;
  }
}

__device__ __forceinline__ int64_t batch_of(const SynthArgs& a) {
  return a.index_ptr ? a.batch_index + (int64_t)a.index_ptr[0] : a.batch_index;
}

__device__ __forceinline__ uint64_t sample_key(const SynthArgs& a, int64_t bi, int b) {
  const uint64_t key = mix64(a.seed * 0x100000001B3ull ^ mix64((uint64_t)a.rank << 40 ^ (uint64_t)bi));
  return mix64(key ^ (uint64_t)b * 0xD6E8FEB86659FD93ull);
}

// id l of table t for the sample with key rk (synth_criteo's formula)
__device__ __forceinline__ int64_t draw_id(const SynthArgs& a, uint64_t rk, int t, int l) {
  const uint64_t r = (uint64_t)a.rows[t];
  const uint64_t tk = (uint64_t)(t + 1) << 32;
  const uint64_t h = mix64(rk ^ tk ^ (uint64_t)(l + 1000));
  if (a.dist == 1 && r > 1) {
    const double x = pow((pow((double)r, 1 - a.alpha) - 1) * u01(h) + 1, 1 / (1 - a.alpha));
    int64_t id = (int64_t)x - 1;
    return id < 0 ? 0 : (id > (int64_t)r - 1 ? (int64_t)r - 1 : id);
  }
  return (int64_t)__umul64hi(h, r);
}

// ids only: thread (t, b) writes sample b's L_t ids of table t -- the same
// values synth_criteo writes, with 26x its parallelism (it runs on the
// embedding stream right before the lookup, on the step's critical chain)
__global__ __launch_bounds__(256) void synth_ids_kernel(SynthArgs a) {
  const int64_t bi = batch_of(a);
  const int64_t n = (int64_t)a.T * a.B;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(q / a.B), b = (int)(q - (int64_t)t * a.B);
    const uint64_t rk = sample_key(a, bi, b);
    const int L = a.pooling[t];
    int64_t* out = a.ids + a.base[t] + (int64_t)b * L;
    for (int l = 0; l < L; ++l) out[l] = draw_id(a, rk, t, l);
  }
}

// dense features (bf16 into x0) and labels: one thread per sample; the
// teacher score is summed in synth_criteo's order (dense part, then table
// groups g = 0..3 over t = g, g + 4, ...) so the labels are identical
__global__ __launch_bounds__(256) void synth_dense_kernel(SynthArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int64_t bi = batch_of(a);
  const uint64_t rk = sample_key(a, bi, b);
  const double bias_w = 3.0 / sqrt((double)a.T);
  double part[TG];
  double sc = 0.0;
  for (int j = 0; j < a.num_dense; ++j) {
    const float x = fast_ln(1.f + (float)(u01(mix64(rk + j)) * 100.0));
    a.x0[(int64_t)b * a.ldx + j] = f2bf(x);
    sc += (x - 3.6) * a.w_dense[j] * 2.0;
  }
  for (int g = 0; g < TG; ++g) {
    double pg = g == 0 ? sc : 0.0;
    for (int t = g; t < a.T; t += TG) {
      const int64_t id = draw_id(a, rk, t, 0);
      pg += a.table_bias[t * 64 + (id & 63)] * bias_w;
    }
    part[g] = pg;
  }
  double s = -1.1;
  for (int q = 0; q < TG; ++q) s += part[q];
  const double p = 1.0 / (1.0 + exp(-s));
  a.label[b] = u01(mix64(rk ^ 0xABCDEFull)) < p ? 1.f : 0.f;
}

}  // namespace

void synth_ids(const SynthArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.T * a.B;
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(synth_ids_kernel, dim3(blocks), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

void synth_dense(const SynthArgs& a, hipStream_t s) {
  if (a.B <= 0) return;
  hipLaunchKernelGGL(synth_dense_kernel, dim3((a.B + 255) / 256), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

void synth_criteo(const SynthArgs& a, hipStream_t s) {
  if (a.B <= 0) return;
  hipLaunchKernelGGL(synth_criteo_kernel, dim3((a.B + SB - 1) / SB), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
