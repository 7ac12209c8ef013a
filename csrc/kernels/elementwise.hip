// Memory-bound glue of the DCN-v2 path: feature concat / split (reading and
// writing the pooled embeddings in place in the all-to-all buffers through a
// SlotMap) and the cross-layer backward. All accesses are 16-B vectors
// (cdna_hip_programming.md Guideline 13); one 8-element group per thread.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

__global__ __launch_bounds__(256) void concat_kernel(const uint16_t* __restrict__ dense,
                                                     int64_t ld_dense,
                                                     const uint16_t* __restrict__ emb,
                                                     SlotMap sm, int F, int D, int B,
                                                     uint16_t* __restrict__ out) {
  const int gpr = D / 8;                       // 8-element groups per feature row
  const int64_t total = (int64_t)B * F * gpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % gpr);
    const int64_t bf = i / gpr;
    const int f = (int)(bf % F);
    const int64_t b = bf / F;
    const uint16_t* src = f == 0 ? dense + b * ld_dense : emb + sm.off[f] + b * sm.stride[f];
    *(uint4*)(out + (b * F + f) * D + g * 8) = *(const uint4*)(src + g * 8);
  }
}

__global__ __launch_bounds__(256) void split_kernel(const uint16_t* __restrict__ dx,
                                                    int64_t ld_dx, int F, int D, int B,
                                                    const uint16_t* __restrict__ dense,
                                                    int64_t ld_dense,
                                                    uint16_t* __restrict__ d_dense,
                                                    int64_t ld_ddense,
                                                    uint16_t* __restrict__ d_emb, SlotMap sm,
                                                    int relu_mask) {
  const int gpr = D / 8;
  const int64_t total = (int64_t)B * F * gpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % gpr);
    const int64_t bf = i / gpr;
    const int f = (int)(bf % F);
    const int64_t b = bf / F;
    uint4 v = *(const uint4*)(dx + b * ld_dx + f * D + g * 8);
    if (f == 0) {
      if (relu_mask) {
        const uint4 h = *(const uint4*)(dense + b * ld_dense + g * 8);
        uint32_t vv[4] = {v.x, v.y, v.z, v.w};
        const uint32_t hh[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t lo = vv[q] & 0xffff, hi = vv[q] >> 16;
          if (!(bf2f((uint16_t)(hh[q] & 0xffff)) > 0.f)) lo = 0;
          if (!(bf2f((uint16_t)(hh[q] >> 16)) > 0.f)) hi = 0;
          vv[q] = lo | (hi << 16);
        }
        v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
      }
      *(uint4*)(d_dense + b * ld_ddense + g * 8) = v;
    } else {
      *(uint4*)(d_emb + sm.off[f] + b * sm.stride[f] + g * 8) = v;
    }
  }
}

__global__ __launch_bounds__(256) void cross_bwd_kernel(const uint16_t* __restrict__ dout,
                                                        const uint16_t* __restrict__ x0,
                                                        const uint16_t* __restrict__ y,
                                                        int64_t n8, uint16_t* __restrict__ dy,
                                                        uint16_t* __restrict__ dx0,
                                                        int accumulate, int add_dout) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 a = ((const uint4*)dout)[i], b = ((const uint4*)x0)[i], c = ((const uint4*)y)[i];
    uint4 d0 = accumulate ? ((const uint4*)dx0)[i] : make_uint4(0, 0, 0, 0);
    const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w},
                   cv[4] = {c.x, c.y, c.z, c.w};
    uint32_t dv[4] = {d0.x, d0.y, d0.z, d0.w};
    uint32_t ov[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a0 = bf2f((uint16_t)(av[q] & 0xffff)), a1 = bf2f((uint16_t)(av[q] >> 16));
      const float b0 = bf2f((uint16_t)(bv[q] & 0xffff)), b1 = bf2f((uint16_t)(bv[q] >> 16));
      const float c0 = bf2f((uint16_t)(cv[q] & 0xffff)), c1 = bf2f((uint16_t)(cv[q] >> 16));
      const float e0 = bf2f((uint16_t)(dv[q] & 0xffff)), e1 = bf2f((uint16_t)(dv[q] >> 16));
      ov[q] = pack2bf(a0 * b0, a1 * b1);
      const float r0 = add_dout ? a0 : 0.f, r1 = add_dout ? a1 : 0.f;
      dv[q] = pack2bf(e0 + a0 * c0 + r0, e1 + a1 * c1 + r1);
    }
    ((uint4*)dy)[i] = make_uint4(ov[0], ov[1], ov[2], ov[3]);
    ((uint4*)dx0)[i] = make_uint4(dv[0], dv[1], dv[2], dv[3]);
  }
}

int grid_of(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

void concat_features(const uint16_t* dense, int64_t ld_dense, const uint16_t* emb,
                     const SlotMap& slots, int F, int D, int B, uint16_t* out, hipStream_t s) {
  const int64_t n = (int64_t)B * F * (D / 8);
  hipLaunchKernelGGL(concat_kernel, dim3(grid_of(n)), dim3(256), 0, s, dense, ld_dense, emb,
                     slots, F, D, B, out);
  TDFO_CHECK_HIP(hipGetLastError());
}

void split_features(const uint16_t* dx, int64_t ld_dx, int F, int D, int B,
                    const uint16_t* dense, int64_t ld_dense, uint16_t* d_dense,
                    int64_t ld_ddense, uint16_t* d_emb, const SlotMap& dslots, int relu_mask,
                    hipStream_t s) {
  const int64_t n = (int64_t)B * F * (D / 8);
  hipLaunchKernelGGL(split_kernel, dim3(grid_of(n)), dim3(256), 0, s, dx, ld_dx, F, D, B, dense,
                     ld_dense, d_dense, ld_ddense, d_emb, dslots, relu_mask);
  TDFO_CHECK_HIP(hipGetLastError());
}

void cross_bwd(const uint16_t* dout, const uint16_t* x0, const uint16_t* y, int64_t n,
               uint16_t* dy, uint16_t* dx0, int accumulate, int add_dout, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(cross_bwd_kernel, dim3(grid_of(n8)), dim3(256), 0, s, dout, x0, y, n8, dy,
                     dx0, accumulate, add_dout);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo

// ------------------------------------------------------------------------
// Batch assembly from HBM-resident columns (tdfo_amd/data/columnar.py): one
// launch gathers row idx[i] (or row0 + i) of every column, converts it
// (int8/16/32/64 or fp32 -> int64 or fp32) and stores it at
// out_c + i * out_stride_c. Replaces one index_select + one copy per column
// per step (22 launches for TwoTower) with a single kernel.
namespace tdfo {
namespace {

template <typename T>
__device__ __forceinline__ double load_as(const void* p, int64_t r) {
  return (double)((const T*)p)[r];
}

__global__ __launch_bounds__(256) void gather_columns_kernel(GatherColsArgs a) {
  const int64_t total = a.n * a.ncols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e / a.n);
    const int64_t i = e - (int64_t)c * a.n;
    const int64_t r = a.idx ? a.idx[i] : a.row0 + i;
    const void* src = a.src[c];
    double v;
    switch (a.src_dtype[c]) {
      case 0: v = load_as<int8_t>(src, r); break;
      case 1: v = load_as<int16_t>(src, r); break;
      case 2: v = load_as<int32_t>(src, r); break;
      case 3: v = load_as<int64_t>(src, r); break;
      default: v = load_as<float>(src, r); break;
    }
    if (a.dst_int[c]) {
      ((int64_t*)a.dst[c])[i * a.dst_stride[c]] =
          a.src_dtype[c] == 3 ? ((const int64_t*)src)[r] : (int64_t)v;
    } else {
      ((float*)a.dst[c])[i * a.dst_stride[c]] = (float)v;
    }
  }
}


// One launch for a training batch's host-visible inputs: the int64 ids, the
// fp32 labels and the fp32 dense features cast into the bf16 bottom-MLP input
// (row stride ldx, first nd columns). Replaces three copies and a cast kernel
// per step (each small launch costs ~5 us of device time).
__global__ __launch_bounds__(256) void batch_load_kernel(
    const float* __restrict__ dense, int nd, int64_t ld_dense, uint16_t* __restrict__ x0,
    int64_t ldx, const int64_t* __restrict__ ids, int64_t* __restrict__ ids_dst, int64_t n,
    const float* __restrict__ label, float* __restrict__ label_dst, int B) {
  const int64_t n2 = n / 2, nden = (int64_t)B * nd;
  const int64_t total = n2 + (n & 1) + nden + B;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n2) {
      ((longlong2*)ids_dst)[i] = ((const longlong2*)ids)[i];
    } else if (i < n2 + (n & 1)) {
      ids_dst[n - 1] = ids[n - 1];
    } else if (i < n2 + (n & 1) + nden) {
      const int64_t e = i - n2 - (n & 1);
      const int64_t b = e / nd;
      const int c = (int)(e - b * nd);
      x0[b * ldx + c] = f2bf(dense[b * ld_dense + c]);
    } else {
      const int64_t b = i - n2 - (n & 1) - nden;
      label_dst[b] = label[b];
    }
  }
}
}  // namespace

void gather_columns(const GatherColsArgs& a, hipStream_t s) {
  const int64_t total = a.n * a.ncols;
  if (total <= 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gather_columns_kernel, dim3(blocks), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

// One wave that occupies its stream for `ticks` of the 100 MHz constant
// clock, sleeping between reads (modelled link time of an emulated
// collective, parallel/comm.py LoopbackComm). Every wave exits once the
// clock has advanced by `ticks`.
// Device warm-up load (bench --preheat-ms): every wave issues MFMAs back to
// back until `ticks` of the 100 MHz wall clock have passed since it started,
// so the chip is at its sustained clock when a timed window begins. The
// result is stored only under a condition that never holds (keeps the loop).
__device__ float g_burn_sink[256];

__global__ __launch_bounds__(256) void burn_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  const bf16x8_t one = __builtin_bit_cast(
      bf16x8_t, (s16x8_t){0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  while (wall_clock64() - t0 < ticks) {
#pragma unroll
    for (int i = 0; i < 32; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(one, one, acc, 0, 0, 0);
  }
  if (acc[0] < -1.f) g_burn_sink[threadIdx.x] = acc[1];
}

__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// In-graph timestamps for schedule probes (labs/probes/mr_sched_probe.py): the
// k-th run of segment `seg` writes the 100 MHz wall clock to
// buf[(k * nseg + seg) * 2 + which]; its end stamp (which = 1) advances k.
// One lane, vector stores; a segment's runs are ordered on its stream.
__global__ void stamp_kernel(uint64_t* buf, int64_t* cnt, int seg, int nseg, int which,
                             int64_t cap) {
  if (threadIdx.x != 0) return;
  const int64_t k = cnt[seg];
  const int64_t i = (k * nseg + seg) * 2 + which;
  if (i < cap) buf[i] = (uint64_t)wall_clock64();
  if (which == 1) cnt[seg] = k + 1;
}

void stamp(uint64_t* buf, int64_t* cnt, int seg, int nseg, int which, int64_t cap,
           hipStream_t s) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, buf, cnt, seg, nseg, which, cap);
  TDFO_CHECK_HIP(hipGetLastError());
}

// Static segment permutation of an int64 buffer (the sharded engine's id
// layouts: table-wise / column-wise send order, replicated tables' ids, the
// all-gathered ids rank-major -> table-major): block b copies chunk b,
// chunks[b] = (src_off, dst_off, len <= SEG_CHUNK), built once on the host.
// Replaces a torch index_select (and its int64 index array read).
__global__ __launch_bounds__(256) void seg_copy_kernel(const int64_t* __restrict__ src,
                                                       int64_t* __restrict__ dst,
                                                       const int64_t* __restrict__ chunks) {
  const int64_t so = chunks[3 * blockIdx.x], d0 = chunks[3 * blockIdx.x + 1];
  const int64_t len = chunks[3 * blockIdx.x + 2];
  for (int64_t i = threadIdx.x; i < len; i += 256) dst[d0 + i] = src[so + i];
}

// Column-wise shards' row assembly: piece p moves a B x w bf16 block between
// two strided views of one buffer (dst row b = buf + dst_off + b * dst_ld,
// src likewise), 16 B per thread; every piece in one launch.
__global__ __launch_bounds__(256) void piece_copy_kernel(uint16_t* buf, const int64_t* pieces,
                                                         int npieces, int B, int w) {
  const int g8 = w / 8;
  const int64_t total = (int64_t)npieces * B * g8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % g8);
    const int64_t pb = i / g8;
    const int p = (int)(pb / B);
    const int64_t b = pb - (int64_t)p * B;
    const int64_t* q = pieces + 4 * p;            // src_off, src_ld, dst_off, dst_ld
    *(uint4*)(buf + q[2] + b * q[3] + g * 8) = *(const uint4*)(buf + q[0] + b * q[1] + g * 8);
  }
}

void piece_copy_bf16(uint16_t* buf, const int64_t* pieces, int npieces, int B, int w,
                     hipStream_t s) {
  const int64_t total = (int64_t)npieces * B * (w / 8);
  if (total <= 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(piece_copy_kernel, dim3(blocks), dim3(256), 0, s, buf, pieces, npieces, B,
                     w);
  TDFO_CHECK_HIP(hipGetLastError());
}

void seg_copy(const int64_t* src, int64_t* dst, const int64_t* chunks, int nchunks,
              hipStream_t s) {
  if (nchunks <= 0) return;
  hipLaunchKernelGGL(seg_copy_kernel, dim3(nchunks), dim3(256), 0, s, src, dst, chunks);
  TDFO_CHECK_HIP(hipGetLastError());
}

// Host mailbox (parallel/mailbox.py): one lane bumps the slot's device
// sequence number and stores (seq << 32 | value) into host-mapped coherent
// memory with ONE 64-bit system-scope vector store -- no fence, no L2
// writeback (a system-scope event release idles every queue ~24 us). The host
// polls the word until the sequence number it expects appears, so a late or
// reordered store can only delay it, never hand it a stale value.
__global__ void host_publish_kernel(const int32_t* value, int32_t* seq, uint64_t* host_word) {
  if (threadIdx.x != 0) return;
  const uint32_t s = (uint32_t)seq[0] + 1u;
  seq[0] = (int32_t)s;
  const uint64_t w = ((uint64_t)s << 32) | (uint64_t)(uint32_t)value[0];
  __hip_atomic_store(host_word, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void host_publish(const int32_t* value, int32_t* seq, uint64_t* host_word, hipStream_t s) {
  hipLaunchKernelGGL(host_publish_kernel, dim3(1), dim3(64), 0, s, value, seq, host_word);
  TDFO_CHECK_HIP(hipGetLastError());
}

// Step counters (optimizer step numbers, dropout RNG step) bumped by one
// launch instead of one library add kernel each.
__global__ void bump_kernel(BumpArgs a) {
  const int i = threadIdx.x;
  if (i >= a.n) return;
  if (a.is_i64[i]) *(int64_t*)a.p[i] += 1;
  else             *(float*)a.p[i] += 1.f;
}

void bump(const BumpArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(64), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

void burn_ticks(uint64_t ticks, int blocks, hipStream_t s) {
  if (ticks == 0 || blocks <= 0) return;
  hipLaunchKernelGGL(burn_kernel, dim3(blocks), dim3(256), 0, s, ticks);
  TDFO_CHECK_HIP(hipGetLastError());
}

void spin_ticks(uint64_t ticks, hipStream_t s) {
  if (ticks == 0) return;
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks);
  TDFO_CHECK_HIP(hipGetLastError());
}

void batch_load(const float* dense, int nd, int64_t ld_dense, uint16_t* x0, int64_t ldx,
                const int64_t* ids, int64_t* ids_dst, int64_t n, const float* label,
                float* label_dst, int B, hipStream_t s) {
  const int64_t total = n / 2 + (n & 1) + (int64_t)B * nd + B;
  if (total <= 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(batch_load_kernel, dim3(blocks), dim3(256), 0, s, dense, nd, ld_dense, x0,
                     ldx, ids, ids_dst, n, label, label_dst, B);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
