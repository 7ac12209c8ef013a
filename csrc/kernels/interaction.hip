// DLRM pairwise-dot feature interaction on MFMA (K24 in SURVEY.md §2.3).
//
// Forward, one wave per sample: the sample's F<=32 feature rows X [F, D] are
// loaded straight into registers in the operand layout of
// v_mfma_f32_32x32x16_bf16 (lane l: row l&31, k = 8*(l>>5)+j). Because
// Z = X X^T uses X as both A and B, the same registers feed both operands:
// D/16 MFMAs produce the 32x32 Gram matrix with no LDS traffic. The strict
// lower triangle is packed through a per-wave LDS row so the output row
// [dense | tril | 0-pad] leaves with one 16-B store per lane.
//
// Backward, one wave per sample: dX = S X with S the symmetric matrix built
// from dZ. S comes from an LDS copy of the dZ row; X is staged in LDS and
// read as the MFMA B operand with ds_read_b64_tr_b16 (k = feature index).
// All column tiles' MFMAs issue back to back before their epilogue, which
// reads nothing from LDS. The concat passthrough (dZ[:, :D]) and the
// bottom-MLP ReLU mask are fused into the dense-slot store (by the lanes that
// hold those dZ / X chunks), and embedding-slot gradients are written
// directly in the layout the embedding backward / all-to-all consumes.
//
// Feature rows are addressed through a SlotMap so the kernels read the
// pooled embeddings in place from the all-to-all receive buffer (no permute).
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int WAVES = 4;
constexpr int SLOT_BYTES = 128 * 8;  // backward: both SlotMaps' copies at the LDS base

__device__ __forceinline__ const uint16_t* feat_row(const uint16_t* dense,
                                                    int64_t ld_dense,
                                                    const uint16_t* emb,
                                                    const SlotMap& sm, int i,
                                                    int F, int b) {
  if (i >= F) return nullptr;
  if (i == 0) return dense + (int64_t)b * ld_dense;
  return emb + sm.off[i] + (int64_t)b * sm.stride[i];
}

// Each wave owns its LDS region and its samples, and LDS executes a wave's
// instructions in order, so a wave-local fence (no block barrier) orders its
// cross-lane LDS writes and reads; the waves of a block never wait for each
// other, so one wave's global loads overlap another's MFMAs and stores.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D>
__global__ __launch_bounds__(256) void inter_fwd_kernel(
    const uint16_t* __restrict__ dense, int64_t ld_dense,
    const uint16_t* __restrict__ emb, SlotMap sm, int F, int B,
    uint16_t* __restrict__ out, int64_t ldo, int ones_col) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* row = (uint16_t*)smem_raw + w * ldo;
  constexpr int KS = D / 16;
  const int P = F * (F - 1) / 2;
  // pad tail written once (zeros, plus the constant-1 column that carries the
  // next layer's bias through its GEMM); never overwritten afterwards
  for (int e = D + P + lane; e < ldo; e += 64) row[e] = e == ones_col ? (uint16_t)0x3f80 : 0;

  const int i = lane & 31, h = lane >> 5;
  constexpr int PC = (D / 8 + 63) / 64;
  // each wave walks several samples; sample n+1's feature rows are loaded
  // into a second register set while sample n's MFMAs, LDS packing and
  // stores run, so the HBM round trip overlaps the previous sample's work
  // loads unconditional at clamped addresses, masked after (a predicated load
  // makes hipcc branch around it and wait for it: no prefetch overlap)
  auto load = [&](int b, bf16x8_t (&fr)[KS], s16x8_t (&pv)[PC]) {
    const uint16_t* rp = feat_row(dense, ld_dense, emb, sm, i < F ? i : F - 1, F, b);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const s16x8_t v = *(const s16x8_t*)(rp + 16 * s + 8 * h);
      const s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      fr[s] = __builtin_bit_cast(bf16x8_t, i < F ? v : z);
    }
    // dense passthrough chunk, loaded with the feature rows
    const uint16_t* dp = dense + (int64_t)b * ld_dense;
#pragma unroll
    for (int k = 0; k < PC; ++k)
      pv[k] = *(const s16x8_t*)(dp + min(lane + 64 * k, D / 8 - 1) * 8);
  };
  const int iters = (B + gridDim.x * WAVES - 1) / (gridDim.x * WAVES);
  bf16x8_t fr[KS], frn[KS];
  s16x8_t pv[PC], pvn[PC];
  int b = blockIdx.x * WAVES + w;
  if (b < B) load(b, fr, pv);
  for (int it = 0; it < iters; ++it) {
    const bool valid = b < B;
    const int bn = b + gridDim.x * WAVES;
    if (it + 1 < iters && bn < B) load(bn, frn, pvn);
    if (valid) {
      f32x16_t acc = {};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[s], fr[s], acc, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < PC; ++k)
        if (lane + 64 * k < D / 8) *(s16x8_t*)(row + (lane + 64 * k) * 8) = pv[k];
      const int col = lane & 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (rr < F && col < rr) row[D + rr * (rr - 1) / 2 + col] = f2bf(acc[r]);
      }
    }
    wave_sync();
    if (valid) {
      uint16_t* op = out + (int64_t)b * ldo;
      for (int c = lane; c < ldo / 8; c += 64)
        *(uint4*)(op + c * 8) = *(const uint4*)(row + c * 8);
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < KS; ++s) fr[s] = frn[s];
#pragma unroll
    for (int k = 0; k < PC; ++k) pv[k] = pvn[k];
    b = bn;
  }
}

// swizzle (16-B chunk xor) of the X image rows for conflict-free tr reads
template <int D>
__device__ __forceinline__ int xswz(int j) {
  return (D >= 128) ? ((j & 3) << 2) : 0;
}

// swizzle of the dX image: the epilogue writes one 8-B piece of each of the
// 32 rows per instruction, all at the same column; rows 256 B apart share
// banks, so X's 4-way swizzle left those writes 8-way bank-conflicted (PMC:
// conflicts = 53 % of LDS-active cycles). XOR-ing the chunk with the row
// spreads the 32 rows over every chunk position. Only where all column
// tiles' MFMAs (hence every X tr read) precede the epilogue (<= 4 tiles):
// with more, dX tile nt overwrites X columns a later tile still reads, which
// is safe only when both images share one layout.
template <int D>
__device__ __forceinline__ int yswz(int j) {
  return (D >= 64 && D <= 128) ? (j & (D / 8 - 1)) : xswz<D>(j);
}

template <int D>
__global__ __launch_bounds__(256) void inter_bwd_kernel(
    const uint16_t* __restrict__ dz, int64_t ldz,
    const uint16_t* __restrict__ dense, int64_t ld_dense,
    const uint16_t* __restrict__ emb, SlotMap sm, int F, int B,
    uint16_t* __restrict__ d_dense, int64_t ld_ddense,
    uint16_t* __restrict__ d_emb, SlotMap dsm, int relu_mask) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int XB = 32 * D * 2;  // X image bytes per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ldz_al = (int)((ldz + 7) & ~7LL);
  // slot offsets / strides in LDS: the unrolled chunk loads below index them
  // per lane, which on the kernel-argument struct would go through scratch
  // (and the gradient slots' too: read per lane in the store loop, the
  // kernel-argument copy costs a vector load + vmcnt(0) per row, which also
  // drained the next sample's prefetch every iteration)
  int64_t* slot = (int64_t*)smem_raw;   // [0, 32): off, [32, 64): stride
  int64_t* dslot = slot + 64;           // the same for the gradient slots
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      slot[q] = sm.off[q]; slot[32 + q] = sm.stride[q];
      dslot[q] = dsm.off[q]; dslot[32 + q] = dsm.stride[q];
    }
  }
  __syncthreads();
  char* base = smem_raw + SLOT_BYTES + w * (XB + ldz_al * 2 + 16 + D * 4);
  char* xs = base;
  // dX image [32][D] aliases the X image (same chunk swizzle): column tile nt
  // is written only after its MFMAs consumed X's same columns, and the
  // ReLU-mask read of X row 0, column d happens in the lane that then
  // overwrites it
  uint16_t* ys = (uint16_t*)base;
  uint16_t* zrow = (uint16_t*)(base + XB);
  // fp32 dX row 0 (the dense slot): its passthrough and ReLU mask are
  // applied in the store loop by the CPR lanes that hold that row's dZ / X
  // chunks in registers, instead of by every lane of every epilogue step
  float* drow = (float*)(base + XB + ldz_al * 2 + 16);
  constexpr int CPR = D / 8;  // 16-B chunks per X row
  constexpr int XC = (32 * CPR + 63) / 64;  // X chunks per lane (F <= 32)
  const int h = lane >> 5;

  // rows >= F of the image stay zero for every sample
  for (int c = lane; c < 32 * CPR; c += 64) {
    const int j = c / CPR;
    if (j >= F) *(uint4*)(xs + c * 16) = make_uint4(0, 0, 0, 0);
  }

  // each wave walks several samples: sample n+1's X rows and dZ row are
  // loaded into registers right after sample n's went to LDS, so the HBM
  // round trip overlaps sample n's MFMAs and gradient stores
  const int nzc = (D + F * (F - 1) / 2 + 7) / 8;   // dZ chunks read (<= 94 <= 2 x 64)
  // this lane's 16 S entries (row i = lane & 31, k = 16 ks + 8 h + jj) as
  // dZ-row offsets of the strict lower triangle, and which of them exist
  const int i = lane & 31;
  // (entries outside the triangle read a zero kept past the dZ row: no
  // per-entry select when S is assembled)
  if (lane == 0) *(uint4*)(zrow + ldz_al) = make_uint4(0, 0, 0, 0);
  int soff[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int k = 16 * (e >> 3) + 8 * h + (e & 7);
    const bool ok = i < F && k < F && i != k;
    const int hi = i > k ? i : k, lo = i > k ? k : i;
    soff[e] = ok ? D + hi * (hi - 1) / 2 + lo : ldz_al;
  }
  // Every load is issued unconditionally at a clamped address (chunks past
  // the row re-read its last chunk and are never written to LDS): a
  // predicated load made hipcc branch around it, wait for it and park the
  // dZ chunks in scratch -- no prefetch overlap at all.
  s16x8_t xv[XC];
  uint4 zv0, zv1;
  auto load = [&](int b) {
#pragma unroll
    for (int k = 0; k < XC; ++k) {
      const int c = min(lane + 64 * k, F * CPR - 1);
      const int j = c / CPR, ch = c - j * CPR;
      const uint16_t* rp = j == 0 ? dense + (int64_t)b * ld_dense
                                  : emb + slot[j] + (int64_t)b * slot[32 + j];
      xv[k] = *(const s16x8_t*)(rp + ch * 8);
    }
    const uint16_t* zp = dz + (int64_t)b * ldz;
    zv0 = *(const uint4*)(zp + min(lane, nzc - 1) * 8);
    zv1 = *(const uint4*)(zp + min(lane + 64, nzc - 1) * 8);
  };
  const int iters = (B + gridDim.x * WAVES - 1) / (gridDim.x * WAVES);
  int b = blockIdx.x * WAVES + w;
  if (b < B) load(b);
  for (int it = 0; it < iters; ++it) {
    const bool valid = b < B;
    const int bn = b + gridDim.x * WAVES;
    if (valid) {
      if (lane < nzc) *(uint4*)(zrow + lane * 8) = zv0;
      if (lane + 64 < nzc) *(uint4*)(zrow + (lane + 64) * 8) = zv1;
#pragma unroll
      for (int k = 0; k < XC; ++k) {
        const int c = lane + 64 * k;
        if (c < F * CPR) {
          const int j = c / CPR, ch = c - j * CPR;
          *(s16x8_t*)(xs + j * D * 2 + ((ch ^ xswz<D>(j)) << 4)) = xv[k];
        }
      }
    }
    // this sample's dZ chunk and X chunk 0 (lanes < D / 8: the dense slot)
    // outlive the prefetch below: the epilogue's passthrough / ReLU mask
    const uint4 zv0s = zv0;
    const uint4 xv0s = __builtin_bit_cast(uint4, xv[0]);
    // unconditional (clamped) prefetch: a conditional one makes hipcc copy
    // the loaded registers at the join and wait for them right away
    load(bn < B ? bn : B - 1);
    wave_sync();
    if (valid) {
      // S operand: S[i][k], i = lane&31, k = 16ks + 8h + jj, read from the
      // dZ row at the per-lane offsets computed once per kernel
      bf16x8_t sa[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s16x8_t t;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          t[jj] = (short)zrow[soff[8 * ks + jj]];
        }
        sa[ks] = __builtin_bit_cast(bf16x8_t, t);
      }
      const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
      // D = 16: one 32-wide column tile whose upper half reads past the row
      // (finite LDS data, never stored)
      constexpr int NT = D >= 32 ? D / 32 : 1;
      // column tiles in batches of up to 4: every batch's MFMAs issue back to
      // back (their transposing reads ahead of them), then its epilogue --
      // no MFMA result is read right after its own MFMA and no LDS round
      // trip sits between them (the dense slot's passthrough and ReLU mask
      // come from registers: lane c of zv0s / xv0s holds chunk c of the dZ
      // row / of X row 0, broadcast with readlane)
      constexpr int NB = NT < 4 ? NT : 4;
#pragma unroll
      for (int nb = 0; nb < NT; nb += NB) {
        f32x16_t acc[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const int nt = nb + t;
          acc[t] = f32x16_t{};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            s16x4_t v[2];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              const int j = 16 * ks + 8 * (g >> 1) + 4 * hf + q;
              const int d = 32 * nt + 16 * (g & 1) + 4 * pp;
              const int off = j * D * 2 + (((d >> 3) ^ xswz<D>(j)) << 4) + ((d & 7) << 1);
              v[hf] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((TDFO_LDS s16x4_t*)(
                  (TDFO_LDS char*)xs + off));
            }
            s16x8_t bb = {v[0][0], v[0][1], v[0][2], v[0][3],
                          v[1][0], v[1][1], v[1][2], v[1][3]};
            // dX^T = X^T S (S symmetric): the X fragment as A, S as B, so each
            // lane's accumulators are 4 runs of 4 consecutive d of ONE feature
            // row i = lane & 31 (8-B LDS writes below instead of 16 scalar ones)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf16x8_t, bb), sa[ks], acc[t], 0, 0, 0);
          }
        }
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const int nt = nb + t;
          // dX rows -> per-wave bf16 image ys [32][D]; row 0 (the dense
          // slot) -> fp32 drow, finished in the store loop
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const int d0 = 32 * nt + 8 * gq + 4 * h;
            if (D < 32 && d0 >= D) continue;
            float v[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) v[q4] = acc[t][4 * gq + q4];
            if (i == 0) {
              *(float4*)(drow + d0) = make_float4(v[0], v[1], v[2], v[3]);
            } else if (i < F) {
              *(uint2*)((char*)ys + i * D * 2 + (((d0 >> 3) ^ yswz<D>(i)) << 4) + ((d0 & 7) << 1)) =
                  make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
            }
          }
        }
      }
      // coalesced 16-B stores of the F gradient rows into their slots (the
      // wave's own LDS image: in-wave LDS order, no barrier needed)
      // (a fixed, unrolled count of predicated stores: hipcc can then count
      // them and wait for the next sample's prefetched rows at the loop top
      // with vmcnt(stores) instead of draining the stores with vmcnt(0))
#pragma unroll
      for (int k = 0; k < XC; ++k) {
        const int c = lane + 64 * k;
        if (c < F * CPR) {
          const int j = c / CPR, ch = c - j * CPR;
          uint4 v;
          if (k == 0 && c < CPR) {
            // dense slot chunk ch = lane: dX (fp32) + the concat passthrough
            // dZ[:, :D], times the bottom-MLP ReLU mask -- this lane holds
            // chunk ch of the dZ row (zv0s) and of X row 0 (xv0s)
            const float4 f0 = *(const float4*)(drow + 8 * ch);
            const float4 f1 = *(const float4*)(drow + 8 * ch + 4);
            float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            const uint32_t zw[4] = {zv0s.x, zv0s.y, zv0s.z, zv0s.w};
            const uint32_t xw[4] = {xv0s.x, xv0s.y, xv0s.z, xv0s.w};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const uint16_t zq = (uint16_t)(zw[q >> 1] >> (16 * (q & 1)));
              const uint16_t xq = (uint16_t)(xw[q >> 1] >> (16 * (q & 1)));
              f[q] += bf2f(zq);
              if (relu_mask && !(bf2f(xq) > 0.f)) f[q] = 0.f;
            }
            v = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]),
                           pack2bf(f[6], f[7]));
          } else {
            v = *(const uint4*)((const char*)ys + j * D * 2 + ((ch ^ yswz<D>(j)) << 4));
          }
          uint16_t* dst = j == 0 ? d_dense + (int64_t)b * ld_ddense
                                 : d_emb + dslot[j] + (int64_t)b * dslot[32 + j];
          *(uint4*)(dst + ch * 8) = v;
        }
      }
    }
    wave_sync();
    b = bn;
  }
}

// Samples per wave of the software-pipelined walk. Measured on MI355X
// (B = 8192, F = 27, D = 128; labs/inter_ab.sh): fwd 15.4 / 15.1 / 16.3 us
// and bwd 43.3 / 37.8 / 34.4 us at 1 / 2 / 4 samples per wave (round 1's
// one-sample-per-wave kernels: 20 / 42 us in the step). TDFO_INTER_SPW
// overrides both.
int grid_for(int B, int spw_default) {
  static const int env = [] {
    const char* e = getenv("TDFO_INTER_SPW");
    return e ? atoi(e) : 0;
  }();
  const int spw = env >= 1 ? env : spw_default;
  const int waves = (B + WAVES * spw - 1) / (WAVES * spw);
  return waves > 0 ? waves : 1;
}

}  // namespace

void interaction_fwd(const uint16_t* dense, int64_t ld_dense,
                     const uint16_t* emb, const SlotMap& slots, int F, int D,
                     int B, uint16_t* out, int64_t ldo, int ones_col, hipStream_t s) {
  if (B <= 0) return;
  const size_t smem = (size_t)WAVES * ldo * 2;
  dim3 grid(grid_for(B, 2));
#define TDFO_IFWD(DD)                                                          \
  hipLaunchKernelGGL(inter_fwd_kernel<DD>, grid, dim3(256), smem, s, dense,    \
                     ld_dense, emb, slots, F, B, out, ldo, ones_col)
  switch (D) {
    case 16: TDFO_IFWD(16); break;
    case 32: TDFO_IFWD(32); break;
    case 64: TDFO_IFWD(64); break;
    case 128: TDFO_IFWD(128); break;
    case 256: TDFO_IFWD(256); break;
  }
  TDFO_CHECK_HIP(hipGetLastError());
#undef TDFO_IFWD
}

void interaction_bwd(const uint16_t* dz, int64_t ldz, const uint16_t* dense,
                     int64_t ld_dense, const uint16_t* emb,
                     const SlotMap& slots, int F, int D, int B,
                     uint16_t* d_dense, int64_t ld_ddense, uint16_t* d_emb,
                     const SlotMap& dslots, int relu_mask, hipStream_t s) {
  if (B <= 0) return;
  const int ldz_al = (int)((ldz + 7) & ~7LL);
  const size_t smem = SLOT_BYTES + (size_t)WAVES * (32 * D * 2 + ldz_al * 2 + 16 + D * 4);
  dim3 grid(grid_for(B, 4));
#define TDFO_IBWD(DD)                                                          \
  if (smem > 65536)                                                            \
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)inter_bwd_kernel<DD>,      \
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));               \
  hipLaunchKernelGGL(inter_bwd_kernel<DD>, grid, dim3(256), smem, s, dz, ldz,  \
                     dense, ld_dense, emb, slots, F, B, d_dense, ld_ddense,    \
                     d_emb, dslots, relu_mask)
  switch (D) {
    case 16: TDFO_IBWD(16); break;
    case 32: TDFO_IBWD(32); break;
    case 64: TDFO_IBWD(64); break;
    case 128: TDFO_IBWD(128); break;
    case 256: TDFO_IBWD(256); break;
  }
  TDFO_CHECK_HIP(hipGetLastError());
#undef TDFO_IBWD
}

}  // namespace tdfo
