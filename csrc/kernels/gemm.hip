// bf16 MFMA GEMM with fused epilogue for the DLRM / DCN-v2 / tower MLPs.
//
// One kernel template covers the three products of a Linear layer without
// ever materialising a transposed copy:
//   forward  y  = x  W^T   A=[M][K] (a_col=0)  B=W [N][K]   (b_col=0)
//   dgrad    dx = dy W     A=[M][K] (a_col=0)  B=W as [K][N] (b_col=1)
//   wgrad    dW = dy^T x   A=dy as [K][M] (a_col=1) B=x as [K][N] (b_col=1)
// "col" operands are staged row-linear into LDS and read as MFMA fragments
// with the gfx950 transposing LDS read ds_read_b64_tr_b16
// (cdna_hip_programming.md §5.5 T10); "row" operands are read with
// ds_read_b128. Both LDS images are XOR-swizzled on the *global source*
// address (glds writes lane-linear, rule 21) so every fragment read is
// bank-conflict free (swizzles checked against the lane groups of
// MI355X_MICROARCH.md §LDS).
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4
// v_mfma_f32_16x16x32_bf16 tiles. Operands are staged with
// global_load_lds_dwordx4 into a 2-deep LDS ring (64 KiB) so the next
// K-tile's loads overlap this tile's MFMAs. Block ids are XCD-remapped.
// Split-K (gridDim.z) writes fp32 slabs reduced by reduce_rows().
#include <cstdlib>

#include "tdfo_common.h"
#include "tdfo_kernels.h"
#include "tdfo_reduce_adam.h"

namespace tdfo {
namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;            // 16 KiB per operand
constexpr int STAGE_BYTES = 2 * TILE_BYTES;        // A + B
constexpr int SMEM_BYTES = 2 * STAGE_BYTES;        // double buffered

typedef __attribute__((address_space(1))) const void* gptr_t;

__device__ __forceinline__ void glds16(const void* src, TDFO_LDS char* dst) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (TDFO_LDS void*)dst, 16, 0, 0);
}

// swizzle of the 16-B chunk index for [k][128] (256-B row) images, chosen so
// the tr-read pattern below touches 32 distinct 8-B slots per half-wave.
__device__ __forceinline__ int swz_col(int k) {
  return ((k & 3) | (((k >> 3) & 1) << 2)) << 1;
}

// One 1-KiB global_load_lds piece (index ii in 0..15) of a [128 rows][64 k]
// image of a row operand (K contiguous): 8 rows x 128 B per piece.
__device__ __forceinline__ void glds_row(const uint16_t* g, int64_t ld, int row0, int rows,
                                         int k0, TDFO_LDS char* tile, int ii, int lane) {
  const int r = ii * 8 + (lane >> 3);
  const int c = (lane & 7) ^ (r & 7);
  int gr = row0 + r;
  gr = gr < rows ? gr : rows - 1;
  glds16(g + (int64_t)gr * ld + k0 + c * 8, tile + ii * 1024);
}

// One piece (ii in 0..15) of a [64 k][128 cols] image of a col operand
// (M/N contiguous): 4 k-rows x 256 B per piece.
__device__ __forceinline__ void glds_col(const uint16_t* g, int64_t ld, int col0, int cols,
                                         int k0, TDFO_LDS char* tile, int ii, int lane) {
  const int kr = ii * 4 + (lane >> 4);
  const int c = (lane & 15) ^ swz_col(kr);
  int gc = col0 + c * 8;
  gc = gc <= cols - 8 ? gc : cols - 8;
  glds16(g + (int64_t)(k0 + kr) * ld + gc, tile + ii * 1024);
}

// The same pieces issued through inline asm (M0 = wave-uniform LDS base). The
// compiler does not see these as LDS DMA, so it does not put a vmcnt(0)
// before every ds_read that might alias an in-flight DMA (it cannot tell the
// ring slots apart inside one LDS array); the big kernel orders its reads
// itself with counted vmcnt + s_barrier. The kernel issues no other vector
// memory ops in its main loop, so those counts are exact.
__device__ __forceinline__ void glds16_asm(const void* src, TDFO_LDS char* dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(src), "s"(lds) : "memory", "m0");
}

template <bool COL>
__device__ __forceinline__ void glds_piece_asm(const uint16_t* g, int64_t ld, int x0, int xs,
                                               int k0, TDFO_LDS char* tile, int ii, int lane) {
  if (COL) {
    const int kr = ii * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_col(kr);
    int gc = x0 + c * 8;
    gc = gc <= xs - 8 ? gc : xs - 8;
    glds16_asm(g + (int64_t)(k0 + kr) * ld + gc, tile + ii * 1024);
  } else {
    const int r = ii * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int gr = x0 + r;
    gr = gr < xs ? gr : xs - 1;
    glds16_asm(g + (int64_t)gr * ld + k0 + c * 8, tile + ii * 1024);
  }
}

template <bool COL>
__device__ __forceinline__ void glds_piece(const uint16_t* g, int64_t ld, int x0, int xs, int k0,
                                           TDFO_LDS char* tile, int ii, int lane) {
  if (COL) glds_col(g, ld, x0, xs, k0, tile, ii, lane);
  else     glds_row(g, ld, x0, xs, k0, tile, ii, lane);
}

// Stage a whole 16-KiB image with the 4 waves of a 256-thread block.
__device__ __forceinline__ void stage_row(const uint16_t* g, int64_t ld,
                                          int row0, int rows, int k0,
                                          TDFO_LDS char* tile, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) glds_row(g, ld, row0, rows, k0, tile, w * 4 + i, lane);
}

__device__ __forceinline__ void stage_col(const uint16_t* g, int64_t ld,
                                          int col0, int cols, int k0,
                                          TDFO_LDS char* tile, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) glds_col(g, ld, col0, cols, k0, tile, w * 4 + i, lane);
}

// MFMA operand fragment (16 rows x 32 k) of a row image: lane l holds
// row r0 + (l&15), k = 32*ks + 8*(l>>4) + j.
__device__ __forceinline__ bf16x8_t frag_row(const TDFO_LDS char* tile, int r0,
                                             int ks, int lane) {
  const int r = r0 + (lane & 15);
  const int c = (ks * 4 + (lane >> 4)) ^ (r & 7);
  return *(const TDFO_LDS bf16x8_t*)(tile + r * 128 + c * 16);
}

// Same fragment from a [k][128] col image via two transposing reads: the
// 16-lane group g = l>>4 reads rows k0..k0+3 (k0 = 32ks + 8g + 4h) x 16 cols;
// lane 4q+p supplies row q, cols 4p..4p+3 and receives column (l&15).
__device__ __forceinline__ bf16x8_t frag_col(const TDFO_LDS char* tile, int c0,
                                             int ks, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int m = c0 + 4 * p;
  s16x4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = ks * 32 + 8 * g + 4 * h + q;
    const int off = k * 256 + (((m >> 3) ^ swz_col(k)) << 4) + ((m & 7) << 1);
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (TDFO_LDS s16x4_t*)(tile + off));
  }
  s16x8_t r = {v[0][0], v[0][1], v[0][2], v[0][3],
               v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

// Output tile and K-split of this block. The grid is 1-D over tiles x splits
// and remapped so that each XCD receives a contiguous run of that space: with
// split-K, one XCD then works on one K-range (its own slices of A and B), so
// the operands a split re-reads across its tiles stay in that XCD's L2.
// (Row-major tile order within a split. M-fastest order, or per shape the
// order with fewer unique operand bytes per XCD, measured the same on every
// DLRM / DCN-v2 GEMM and step: profiles/r04/notes.md.)
struct TileIdx {
  int tm, tn, split;
};
__device__ __forceinline__ TileIdx tile_of(int tiles_m, int tiles_n, int splits,
                                           int bid = -1) {
  const int tiles = tiles_m * tiles_n;
  const int w = xcd_remap(bid < 0 ? (int)blockIdx.x : bid, tiles * splits);
  const int split = w / tiles, t = w - split * tiles;
  return {t / tiles_n, t - (t / tiles_n) * tiles_n, split};
}

// Epilogue shared by both tile shapes: bias + ReLU in registers, then the
// ROWS x 128 fp32 tile is staged through the (now idle) LDS ring so global
// traffic leaves as coalesced 16-B accesses (mask loads, bf16 stores, fp32
// stores, DCN Hadamard/residual second output).
// The MFMAs run with the B (output-column) fragment as the A operand, so the
// accumulator holds C transposed: lane l, register r of fragment (i, j) is
// C[row 16i + (l&15)][col 16j + 4(l>>4) + r] -- four consecutive columns of
// one row, staged with one 16-B LDS write per fragment (16 per lane instead
// of 64 scalar writes).
// Register-direct epilogue preconditions: whole tile in range, every touched
// operand row 16-B aligned (8 bf16 / 4 fp32 columns).
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

__device__ __forceinline__ bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }
__device__ __forceinline__ bool direct_ok(const GemmArgs& p, int m0, int n0, int rows) {
  // operand reads (ReLU mask, DCN mul/add) in this layout are 32-B row runs;
  // the LDS path reads them as 256-B rows (measured: DCN-v2 3.16 vs 3.05 ms)
  if (p.mul || p.add) return false;
  if (p.mask) return false;
  if (m0 + rows > p.M || n0 + 128 > p.N) return false;
  if (p.C && ((p.ldc & 7) || !al16(p.C))) return false;
  if (p.mask && ((p.ldm & 7) || !al16(p.mask))) return false;
  if (p.C2 && ((p.ldc2 & 7) || !al16(p.C2))) return false;
  if (p.mul && ((p.ldmul & 7) || !al16(p.mul))) return false;
  if (p.add && ((p.ldadd & 7) || !al16(p.add))) return false;
  if (p.C32 && ((p.ldc32 & 3) || !al16(p.C32))) return false;
  return true;
}

template <int ROWS, int NT, int MI = 4>
__device__ __forceinline__ void epilogue(const GemmArgs& p, const f32x4_t (&acc)[MI][4],
                                         char* smem_raw, int m0, int n0, int wr, int wc,
                                         int lane, int tid, int split) {
  // Plain fp32 output (split-K weight-grad slabs): each lane already holds 4
  // consecutive columns (16 B) of a row per fragment, so store straight from
  // the accumulators -- no LDS round trip, no barrier; 64-B row runs per
  // 4-lane group.
  if (p.C32 && !p.C && !p.C2 && !p.bias && !p.relu && !p.mask && (p.ldc32 & 3) == 0 &&
      (p.N & 3) == 0) {
    float* c32 = p.C32 + (int64_t)split * p.M * p.ldc32;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wr * (MI * 16) + i * 16 + (lane & 15);
        if (m < p.M) *(f32x4_t*)(c32 + (int64_t)m * p.ldc32 + n) = acc[i][j];
      }
    }
    return;
  }
  // Full tiles with 16-B aligned operands: no LDS round trip either. Row
  // fragments (i, i+1) are paired and v_permlane16_swap exchanges 4-column
  // groups between lane rows g and g^1, after which every lane holds 8
  // consecutive columns (16 B of bf16) of ONE row: lanes of even g row i,
  // odd g row i+1 (guide T21 with the 16-lane swap). Same store count as the
  // LDS path, no staging writes/reads and no barrier.
  if (direct_ok(p, m0, n0, ROWS)) {
    const int rho = lane & 15, g = lane >> 4;
    float* c32 = p.C32 ? p.C32 + (int64_t)split * p.M * p.ldc32 : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = wc * 64 + j * 16 + 4 * g;
      float bias[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bias[r] = p.bias ? p.bias[(int64_t)(n0 + cl + r) * p.bias_stride] : 0.f;
      const int n = n0 + wc * 64 + j * 16 + 8 * (g >> 1);
#pragma unroll
      for (int i = 0; i < MI; i += 2) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a = acc[i][j][r] + bias[r], b = acc[i + 1][j][r] + bias[r];
          if (p.relu) {
            a = fmaxf(a, 0.f);
            b = fmaxf(b, 0.f);
          }
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b),
                                                           false, false);
          v[r] = __uint_as_float(sw[0]);
          v[4 + r] = __uint_as_float(sw[1]);
        }
        const int m = m0 + wr * (MI * 16) + (i + (g & 1)) * 16 + rho;
        if (p.mask) {
          const uint4 mk = *(const uint4*)(p.mask + (int64_t)m * p.ldm + n);
          const uint32_t mu[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!(bf2f((uint16_t)(mu[q] & 0xffff)) > 0.f)) v[2 * q] = 0.f;
            if (!(bf2f((uint16_t)(mu[q] >> 16)) > 0.f)) v[2 * q + 1] = 0.f;
          }
        }
        if (p.C)
          *(uint4*)(p.C + (int64_t)m * p.ldc + n) =
              make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]),
                         pack2bf(v[6], v[7]));
        if (p.C2) {
          float w2[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) w2[q] = v[q];
          if (p.mul) {
            const uint4 mv = *(const uint4*)(p.mul + (int64_t)m * p.ldmul + n);
            const uint32_t mu[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              w2[2 * q] *= bf2f((uint16_t)(mu[q] & 0xffff));
              w2[2 * q + 1] *= bf2f((uint16_t)(mu[q] >> 16));
            }
          }
          if (p.add) {
            const uint4 av = *(const uint4*)(p.add + (int64_t)m * p.ldadd + n);
            const uint32_t au[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              w2[2 * q] += bf2f((uint16_t)(au[q] & 0xffff));
              w2[2 * q + 1] += bf2f((uint16_t)(au[q] >> 16));
            }
          }
          *(uint4*)(p.C2 + (int64_t)m * p.ldc2 + n) =
              make_uint4(pack2bf(w2[0], w2[1]), pack2bf(w2[2], w2[3]), pack2bf(w2[4], w2[5]),
                         pack2bf(w2[6], w2[7]));
        }
        if (c32) {
          float* o = c32 + (int64_t)m * p.ldc32 + n;
          *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
          *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    return;
  }
  float* ctile = (float*)smem_raw;   // [ROWS][128] fp32, 16-B chunks XOR-swizzled
  // Epilogue operands (ReLU mask, DCN Hadamard / residual inputs) of the
  // whole tile are loaded into registers here, before the accumulator LDS
  // round trip: one memory round trip per block, hidden behind the staging,
  // instead of one per unrolled pair of store-loop iterations (those loads
  // were issued two at a time and waited on before each store). Addresses
  // are clamped into the operand, so the loads are unconditional (no
  // branch-around-load per element); the store loop drops out-of-range rows.
  constexpr int IT = ROWS * 16 / NT;
  // bias first: its loads must not queue behind the prefetch (vmcnt retires
  // in issue order)
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wc * 64 + j * 16 + 4 * (lane >> 4) + r;
      bv[j][r] = (p.bias && n < p.N) ? p.bias[(int64_t)n * p.bias_stride] : 0.f;
    }
  const bool pf = (p.N & 7) == 0 &&
                  (p.mask || (p.C2 && (p.mul || p.add)));
  uint4 pk[IT], pm[IT], pa[IT];
  if (pf) {
    auto pf_load = [&](const uint16_t* base, int64_t ld, uint4 (&dst)[IT]) {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int c = it * NT + tid;
        const int m = min(m0 + (c >> 4), p.M - 1);
        const int n = min(n0 + (c & 15) * 8, p.N - 8);
        dst[it] = *(const uint4*)(base + (int64_t)m * ld + n);
      }
    };
    if (p.mask) pf_load(p.mask, p.ldm, pk);
    if (p.C2 && p.mul) pf_load(p.mul, p.ldmul, pm);
    if (p.C2 && p.add) pf_load(p.add, p.ldadd, pa);
  }
  // with loads in flight, barriers that wait only for LDS traffic
  // (__syncthreads would drain vmcnt first)
  auto lds_barrier = [&]() {
    if (pf) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  lds_barrier();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wc * 64 + j * 16 + 4 * (lane >> 4);       // first of 4 columns
    const float* bias = bv[j];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int rl = wr * (MI * 16) + i * 16 + (lane & 15);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bias[r];
        if (p.relu) v[r] = fmaxf(v[r], 0.f);
      }
      const int chunk = (cl >> 2) ^ (rl & 31);
      *(float4*)(ctile + rl * 128 + chunk * 4) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  lds_barrier();
  float* c32 = p.C32 ? p.C32 + (int64_t)split * p.M * p.ldc32 : nullptr;
  const bool nfull = (n0 + BN <= p.N) && ((p.N & 7) == 0);
  auto store_loop = [&](auto pf_on) {
  constexpr bool PF = decltype(pf_on)::value;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * NT + tid;           // 8-column group id in the tile
    const int rl = c >> 4, cg = (c & 15) * 8;
    const int m = m0 + rl;
    if (m >= p.M) continue;
    const float4 lo = *(const float4*)(ctile + rl * 128 + (((cg >> 2) ^ (rl & 31)) << 2));
    const float4 hi = *(const float4*)(ctile + rl * 128 + ((((cg >> 2) + 1) ^ (rl & 31)) << 2));
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const int n = n0 + cg;
    if (nfull || n + 8 <= p.N) {
      if (p.mask) {
        const uint4 mk = PF ? pk[it] : *(const uint4*)(p.mask + (int64_t)m * p.ldm + n);
        const uint32_t mu[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (!(bf2f((uint16_t)(mu[q] & 0xffff)) > 0.f)) v[2 * q] = 0.f;
          if (!(bf2f((uint16_t)(mu[q] >> 16)) > 0.f)) v[2 * q + 1] = 0.f;
        }
      }
      if (p.C) {
        *(uint4*)(p.C + (int64_t)m * p.ldc + n) =
            make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]),
                       pack2bf(v[6], v[7]));
      }
      if (p.C2) {
        float w2[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w2[q] = v[q];
        if (p.mul) {
          const uint4 mv = PF ? pm[it] : *(const uint4*)(p.mul + (int64_t)m * p.ldmul + n);
          const uint32_t mu[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w2[2 * q] *= bf2f((uint16_t)(mu[q] & 0xffff));
            w2[2 * q + 1] *= bf2f((uint16_t)(mu[q] >> 16));
          }
        }
        if (p.add) {
          const uint4 av = PF ? pa[it] : *(const uint4*)(p.add + (int64_t)m * p.ldadd + n);
          const uint32_t au[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w2[2 * q] += bf2f((uint16_t)(au[q] & 0xffff));
            w2[2 * q + 1] += bf2f((uint16_t)(au[q] >> 16));
          }
        }
        *(uint4*)(p.C2 + (int64_t)m * p.ldc2 + n) =
            make_uint4(pack2bf(w2[0], w2[1]), pack2bf(w2[2], w2[3]), pack2bf(w2[4], w2[5]),
                       pack2bf(w2[6], w2[7]));
      }
      if (c32) {
        float* o = c32 + (int64_t)m * p.ldc32 + n;
        *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else {
      for (int q = 0; q < 8 && n + q < p.N; ++q) {
        float x = v[q];
        if (p.mask && !(bf2f(p.mask[(int64_t)m * p.ldm + n + q]) > 0.f)) x = 0.f;
        if (p.C) p.C[(int64_t)m * p.ldc + n + q] = f2bf(x);
        if (c32) c32[(int64_t)m * p.ldc32 + n + q] = x;
        if (p.C2) {
          float x2 = x;
          if (p.mul) x2 *= bf2f(p.mul[(int64_t)m * p.ldmul + n + q]);
          if (p.add) x2 += bf2f(p.add[(int64_t)m * p.ldadd + n + q]);
          p.C2[(int64_t)m * p.ldc2 + n + q] = f2bf(x2);
        }
      }
    }
  }
  };
  if (pf) store_loop(BoolC<true>{});
  else    store_loop(BoolC<false>{});
}

// 16 MFMAs of one 64-deep K step for a wave's 64x64 sub-tile (two 32-deep
// halves). ta/tb: 16-KiB images holding the wave's A rows / B cols at
// a_r0 / b_c0.
// CS (col-layout A only): running column sums of A, as one extra MFMA per
// fragment pair against an all-ones B fragment -- the sum over the
// fragment's 32 k of row 16 i + (l & 15) lands in every register of the
// lane. The two waves of a row pair (cs_par = wc) take alternate fragments,
// picked with a select so the MFMA stream has no branches. VALU sums of the
// unpacked bf16 cost ~4x the MFMA time of the waves that carry them
// (measured: bot/top3 wgrads 13 vs 10 us).
template <bool A_COL, bool B_COL, int MI = 4, bool CS = false>
__device__ __forceinline__ void mfma_k64(f32x4_t (&acc)[MI][4], const TDFO_LDS char* ta,
                                         int a_r0, const TDFO_LDS char* tb, int b_c0, int lane,
                                         f32x4_t* cs = nullptr, int cs_par = 0) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    bf16x8_t af[MI], bfr[4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      af[i] = A_COL ? frag_col(ta, a_r0 + i * 16, ks, lane) : frag_row(ta, a_r0 + i * 16, ks, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = B_COL ? frag_col(tb, b_c0 + j * 16, ks, lane) : frag_row(tb, b_c0 + j * 16, ks, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if constexpr (A_COL && CS) {
      const bf16x8_t ones = __builtin_bit_cast(
          bf16x8_t, (s16x8_t){0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});
#pragma unroll
      for (int h = 0; h < MI / 2; ++h) {
        const bf16x8_t a = cs_par ? af[2 * h + 1] : af[2 * h];
        cs[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, a, cs[h], 0, 0, 0);
      }
    }
  }
}

// Store this wave's column sums (fragments 2 h + cs_par) into this split's
// fp32 slab, column csum_col of rows a_m0 + 16 (2 h + cs_par) + (l & 15).
template <int MI>
__device__ __forceinline__ void csum_store(const GemmArgs& p, const f32x4_t (&cs)[MI / 2],
                                           int a_m0, int lane, int split, int cs_par) {
  float* c32 = p.C32 + (int64_t)split * p.M * p.ldc32;
#pragma unroll
  for (int h = 0; h < MI / 2; ++h) {
    const int m = a_m0 + (2 * h + cs_par) * 16 + (lane & 15);
    if (lane < 16 && m < p.M) c32[(int64_t)m * p.ldc32 + p.csum_col] = cs[h][0];
  }
}

// ---------------------------------------------------------------------------
// Small-tile kernel: BMT x 128 x 64 (BMT = 128, or 64 for row-layout A when
// the 128-row grid leaves CUs idle), 4 waves (2x2 of (BMT/2)x64), 2-deep glds
// ring (2 x (BMT + 128) x 64 x 2 B of LDS) -> 2+ blocks per CU.
// Body of the small-tile kernel for block `bid` of this problem's grid (a
// paired launch runs two problems' bodies in one grid, gemm_pair_kernel).
template <int BMT, bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_small_body(const GemmArgs& p, int bid, char* smem_raw) {
  static_assert(BMT == 128 || !A_COL, "64-row tiles need a row-layout A");
  constexpr int MI = BMT / 32;                   // 16-row fragments per wave
  constexpr int A_BYTES = BMT * BK * 2;
  constexpr int ST = A_BYTES + TILE_BYTES;
  TDFO_LDS char* smem = (TDFO_LDS char*)smem_raw;

  const int tiles_m = (p.M + BMT - 1) / BMT, tiles_n = (p.N + BN - 1) / BN;
  const TileIdx ti = tile_of(tiles_m, tiles_n, p.splits, bid);
  const int m0 = ti.tm * BMT, n0 = ti.tn * BN;

  const int ktiles = p.K / BK;
  const int per = (ktiles + p.splits - 1) / p.splits;
  const int kt0 = ti.split * per;
  const int kt1 = min(ktiles, kt0 + per);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;

  f32x4_t acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int buf, int kt) {
    TDFO_LDS char* ta = smem + buf * ST;
    TDFO_LDS char* tb = ta + A_BYTES;
    const int k0 = kt * BK;
    if (A_COL) stage_col(p.A, p.lda, m0, p.M, k0, ta, w, lane);
    else {
#pragma unroll
      for (int i = 0; i < BMT / 32; ++i)
        glds_row(p.A, p.lda, m0, p.M, k0, ta, w * (BMT / 32) + i, lane);
    }
    if (B_COL) stage_col(p.B, p.ldb, n0, p.N, k0, tb, w, lane);
    else       stage_row(p.B, p.ldb, n0, p.N, k0, tb, w, lane);
  };

  // column sums of A (bias gradient) in the first column tile's blocks,
  // whose waves already hold every A fragment of their rows; the loop is
  // instantiated with and without them (block-uniform branch outside it)
  const bool csum = A_COL && p.csum_on && ti.tn == 0;
  const int cs_par = __builtin_amdgcn_readfirstlane(wc);
  f32x4_t cs[MI / 2];
#pragma unroll
  for (int h = 0; h < MI / 2; ++h) cs[h] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  auto kloop = [&](auto cs_on) {
    constexpr bool CS = decltype(cs_on)::value;
    if (kt0 < kt1) {
      stage(0, kt0);
      __syncthreads();
      int cur = 0;
      for (int kt = kt0; kt < kt1; ++kt) {
        if (kt + 1 < kt1) stage(cur ^ 1, kt + 1);
        const TDFO_LDS char* ta = smem + cur * ST;
        mfma_k64<A_COL, B_COL, MI, CS>(acc, ta, wr * (BMT / 2), ta + A_BYTES, wc * 64, lane, cs,
                                       cs_par);
        __syncthreads();
        cur ^= 1;
      }
    }
  };
  if (csum) {
    kloop(BoolC<true>{});
    csum_store<MI>(p, cs, m0 + wr * (BMT / 2), lane, ti.split, cs_par);
  } else {
    kloop(BoolC<false>{});
  }
  epilogue<BMT, 256, MI>(p, acc, smem_raw, m0, n0, wr, wc, lane, tid, ti.split);
}

template <int BMT, bool A_COL, bool B_COL>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_small_body<BMT, A_COL, B_COL>(p, blockIdx.x, smem_raw);
}

// ---------------------------------------------------------------------------
// Large-tile kernel: 256x128x64, 8 waves (4 along M x 2 along N, each 64x64),
// 3-deep glds ring (3 x 48 KiB = 144 KiB LDS, 1 block per CU, 2 waves per
// SIMD). Two K tiles stay in flight across each barrier: the wait before the
// barrier is a counted vmcnt (6 pieces per thread per tile), the barrier is a
// raw s_barrier (no vmcnt(0) drain, cdna_hip_programming.md "Pipelining
// across barriers"), and the ring slot being refilled is the one every wave
// finished reading before that barrier. Twice the FLOP per staged byte of the
// 128x128 tile: DCN-v2's 3456-wide GEMMs (>= 1024 128x128 tiles) and its
// weight grads run on it (profiles/r03/dcn_policy_ab.log).
constexpr int LBM = 256;
constexpr int LSTAGE = 3 * TILE_BYTES;             // A (2 images) + B
constexpr int LSMEM = 3 * LSTAGE;                  // 144 KiB >= 256x128 fp32 epilogue tile

template <bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_big_body(const GemmArgs& p, int bid, char* smem_raw) {
  constexpr int MI = 4, NW = 8;
  constexpr int APW = 32 / NW, BPW = 16 / NW;       // A / B pieces per wave per K tile
  TDFO_LDS char* smem = (TDFO_LDS char*)smem_raw;

  const int tiles_m = (p.M + LBM - 1) / LBM, tiles_n = (p.N + BN - 1) / BN;
  const TileIdx ti = tile_of(tiles_m, tiles_n, p.splits, bid);
  const int m0 = ti.tm * LBM, n0 = ti.tn * BN;

  const int ktiles = p.K / BK;
  const int per = (ktiles + p.splits - 1) / p.splits;
  const int kt0 = ti.split * per;
  const int nk = min(ktiles, kt0 + per) - kt0;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;

  f32x4_t acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // 48 pieces per K tile (A: 2 images x 16, B: 16) spread over the waves.
  auto stage = [&](int buf, int kt) {
    TDFO_LDS char* ta = smem + buf * LSTAGE;
    TDFO_LDS char* tb = ta + 2 * TILE_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int ii = w * APW + i, half = ii >> 4;
      glds_piece_asm<A_COL>(p.A, p.lda, m0 + half * 128, p.M, k0, ta + half * TILE_BYTES,
                            ii & 15, lane);
    }
#pragma unroll
    for (int i = 0; i < BPW; ++i)
      glds_piece_asm<B_COL>(p.B, p.ldb, n0, p.N, k0, tb, w * BPW + i, lane);
  };
  // all but the youngest K tile's pieces landed
  auto wait_one_ahead = [&]() { asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory"); };

  // Fragment-pipelined main loop: one raw barrier per K tile, in the middle
  // of it. Iteration t: issue tile t+2's DMA, read tile t's k=32..63
  // fragments, MFMAs on its k=0..31 fragments (read last iteration) hide that
  // read, then wait for tile t+1 + barrier, read tile t+1's k=0..31
  // fragments, and the k=32..63 MFMAs hide those. Ring-slot reuse: slot
  // (t+2)%3 was last read before iteration t-1's barrier (each wave drains
  // its LDS reads with lgkmcnt(0) before that barrier).
  if (nk > 0) {
    const TDFO_LDS char* tAo = smem + (wr >> 1) * TILE_BYTES;
    const TDFO_LDS char* tBo = smem + 2 * TILE_BYTES;
    const int a_r0 = (wr & 1) * 64, b_c0 = wc * 64;
    auto frags = [&](int buf, int ks, bf16x8_t (&af)[MI], bf16x8_t (&bfr)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = B_COL ? frag_col(tBo + buf * LSTAGE, b_c0 + j * 16, ks, lane)
                       : frag_row(tBo + buf * LSTAGE, b_c0 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = A_COL ? frag_col(tAo + buf * LSTAGE, a_r0 + i * 16, ks, lane)
                      : frag_row(tAo + buf * LSTAGE, a_r0 + i * 16, ks, lane);
    };
    auto mm = [&](const bf16x8_t (&af)[MI], const bf16x8_t (&bfr)[4]) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    };
    stage(0, kt0);
    if (nk > 1) stage(1, kt0 + 1);
    if (nk > 1) wait_one_ahead();
    else        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bf16x8_t a0[MI], b0[4], a1[MI], b1[4];
    frags(0, 0, a0, b0);
    int cur = 0;
    // steady state (straight-line body so the compiler's lgkmcnt waits only
    // cover the reads each MFMA group actually consumes); last tile peeled
    for (int t = 0; t + 1 < nk; ++t) {
      __builtin_amdgcn_sched_barrier(0);
      const bool pre = t + 2 < nk;
      if (pre) stage(cur == 0 ? 2 : cur - 1, kt0 + t + 2);
      frags(cur, 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mm(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (pre) wait_one_ahead();
      else     asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      cur = cur == 2 ? 0 : cur + 1;
      frags(cur, 0, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mm(a1, b1);
    }
    __builtin_amdgcn_sched_barrier(0);
    frags(cur, 1, a1, b1);
    mm(a0, b0);
    mm(a1, b1);
  }
  epilogue<LBM, NW * 64, MI>(p, acc, smem_raw, m0, n0, wr, wc, lane, tid, ti.split);
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_big_body<A_COL, B_COL>(p, blockIdx.x, smem_raw);
}

// Two problems in one 256x128 grid (see gemm_pp_pair_kernel).
template <bool AC0, bool BC0, bool AC1, bool BC1>
__global__ __launch_bounds__(512, 1) void gemm_big_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x < nb0) gemm_big_body<AC0, BC0>(p0, blockIdx.x, smem_raw);
  else                       gemm_big_body<AC1, BC1>(p1, blockIdx.x - nb0, smem_raw);
}

// ---------------------------------------------------------------------------
// Deep-pipelined 128x128 kernel: 4 waves (2x2 of 64x64), DNS-deep glds ring
// (DNS x 32 KiB, one block per CU) with DNS-2 K tiles of DMA in flight across
// each raw barrier (counted vmcnt, never 0 in the steady state). For GEMMs
// whose grid is ~one 128x128 tile per CU and whose K is long (DCN-v2 cross
// layers, K = 3456): the 2-stage kernel exposes a whole load round trip per
// K tile there (V fwd: 54 K tiles in 43 us, ~1900 cycles each, ~32 KiB in
// flight per CU).
#ifndef TDFO_GEMM_DNS
#define TDFO_GEMM_DNS 4
#endif
constexpr int DNS = TDFO_GEMM_DNS;
constexpr int DSMEM = DNS * STAGE_BYTES;

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(256, 1) void gemm_deep_kernel(GemmArgs p) {
  constexpr int MI = 4;
  constexpr int PPW = 8;                             // glds pieces per wave per K tile
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TDFO_LDS char* smem = (TDFO_LDS char*)smem_raw;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const TileIdx ti = tile_of(tiles_m, tiles_n, p.splits);
  const int m0 = ti.tm * BM, n0 = ti.tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.splits - 1) / p.splits;
  const int kt0 = ti.split * per;
  const int nk = min(ktiles, kt0 + per) - kt0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  f32x4_t acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // 32 pieces per K tile (A 16, B 16), 8 per wave
  auto stage = [&](int buf, int kt) {
    TDFO_LDS char* ta = smem + buf * STAGE_BYTES;
    TDFO_LDS char* tb = ta + TILE_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds_piece_asm<A_COL>(p.A, p.lda, m0, p.M, k0, ta, w * 4 + i, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds_piece_asm<B_COL>(p.B, p.ldb, n0, p.N, k0, tb, w * 4 + i, lane);
  };
  const bool csum = A_COL && p.csum_on && ti.tn == 0;
  const int cs_par = __builtin_amdgcn_readfirstlane(wc);
  f32x4_t cs[MI / 2];
#pragma unroll
  for (int h = 0; h < MI / 2; ++h) cs[h] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  auto kloop = [&](auto cs_on) {
    constexpr bool CS = decltype(cs_on)::value;
#pragma unroll
    for (int q = 0; q < DNS - 1; ++q)
      if (q < nk) stage(q, kt0 + q);
    for (int t = 0; t < nk; ++t) {
      // tile t landed for this thread: the younger tiles (up to DNS-2) may
      // still be in flight
      const int younger = min(nk - 1 - t, DNS - 2);
      if (younger >= 3)      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else if (younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else                   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // every thread's pieces of tile t landed, and every wave finished
      // reading slot (t-1) % DNS, which the stage below refills
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (t + DNS - 1 < nk) stage((t + DNS - 1) % DNS, kt0 + t + DNS - 1);
      const TDFO_LDS char* ta = smem + (t % DNS) * STAGE_BYTES;
      mfma_k64<A_COL, B_COL, MI, CS>(acc, ta, wr * 64, ta + TILE_BYTES, wc * 64, lane, cs,
                                     cs_par);
      // this wave's fragment reads of slot t % DNS done before the next
      // barrier (the slot is refilled DNS-1 iterations later)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  static_assert(DNS >= 2 && DNS <= 5, "ring depth");
  if (csum) {
    kloop(BoolC<true>{});
    csum_store<MI>(p, cs, m0 + wr * 64, lane, ti.split, cs_par);
  } else {
    kloop(BoolC<false>{});
  }
  __syncthreads();
  epilogue<BM, 256, MI>(p, acc, smem_raw, m0, n0, wr, wc, lane, tid, ti.split);
}

// ---------------------------------------------------------------------------
// Ping-pong tile kernel: 128x128x64 tiles, 8 waves, 2 blocks per CU.
//
// The waves form two groups of four (waves 0-3 and 4-7: one wave of each
// group per SIMD) owning the upper and lower 64 rows of the tile; each wave
// computes 64x32 (4x2 v_mfma_f32_16x16x32_bf16 fragments). Every wave
// alternates a READ segment (its share of the next K tile's global->LDS DMA,
// then its fragment ds_reads for one K tile) and an MFMA segment (16 MFMAs),
// each closed by a workgroup barrier; group 1 starts one barrier late, so on
// every SIMD one wave issues MFMAs while the other reads LDS and issues DMA
// (cdna_hip_programming.md §5 "8-phase template": groups staggered by a
// barrier; T3+T4 counted vmcnt, T5 setprio). Operands are staged by
// inline-asm global_load_lds into a 2-slot LDS ring (counted vmcnt, raw
// s_barrier: the DMA stays in flight across barriers); 64 KiB of LDS lets
// two blocks share a CU, so one block's prologue / epilogue overlaps the
// other's main loop -- which is what beat every one-block-per-CU variant
// measured (256x128 and 256x256 tiles, 3-4 slot rings, DMA in the MFMA
// segment, no stagger: profiles/r03/gemm_lab_variants.jsonl).
// Epilogue straight from the accumulators (bias, ReLU, ReLU mask, DCN
// Hadamard/residual second output, fp32 split-K slabs, bias-grad column sums).
template <int BMP, int NSTP, int BNP = 128>
struct PPGeom {
  static constexpr int BM = BMP, BN = BNP;
  static constexpr int GROWS = BM / 2;                  // rows per wave group
  static constexpr int WGN = (BN == 256 || BM == 128) ? 4 : 2;   // waves along N in a group
  static constexpr int WGM = 4 / WGN;
  static constexpr int WROWS = GROWS / WGM;             // 64 | 128
  static constexpr int WCOLS = BN / WGN;                // 64 | 32
  static constexpr int MI = WROWS / 16;
  static constexpr int NJ = WCOLS / 16;
  static constexpr int KS = MI * NJ >= 16 ? 1 : 2;      // k32 steps per segment
  static constexpr int SEGS = 2 / KS;                   // READ/MFMA segment pairs per K tile
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int STAGE = A_BYTES + BN * BK * 2;
  static constexpr int NST = NSTP;
  static constexpr int LDS = NST * STAGE;
  static constexpr int APW = BM / 64;                   // A glds pieces per wave per K tile
  static constexpr int BPW = BN / 64;
  static constexpr int PPW = APW + BPW;
  static constexpr int CSF = MI / WGN;                  // column-sum fragments per wave
  static_assert(PPW * (NST - 1) <= 63, "vmcnt range");
};

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(n * PPW), n in 0..3 (wave-uniform)
template <int PPW>
__device__ __forceinline__ void pp_wait_vm(int n) {
  if (n >= 3)      asm volatile("s_waitcnt vmcnt(%0)" :: "i"(3 * PPW) : "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(2 * PPW) : "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(PPW) : "memory");
  else             asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Epilogue of a wave's MI x NJ fragments (acc holds C transposed: lane l,
// register r of fragment (i, j) = C[mw + 16 i + (l & 15)][nw + 16 j + 4 (l >> 4) + r]).
template <int MI, int NJ>
__device__ __forceinline__ void pp_epilogue(const GemmArgs& p, const f32x4_t (&acc)[MI][NJ],
                                            int mw, int nw, int lane, int split) {
  const int rho = lane & 15, g = lane >> 4;
  float* c32 = p.C32 ? p.C32 + (int64_t)split * p.M * p.ldc32 : nullptr;
  const bool plain32 = c32 && !p.C && !p.C2 && !p.bias && !p.relu && !p.mask;
  const bool full = mw + MI * 16 <= p.M && nw + NJ * 16 <= p.N;
  if (plain32 && full && (p.ldc32 & 3) == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i)
        *(f32x4_t*)(c32 + (int64_t)(mw + 16 * i + rho) * p.ldc32 + nw + 16 * j + 4 * g) = acc[i][j];
    return;
  }
  const bool vec = full && (!p.C || (((p.ldc & 7) == 0) && al16(p.C))) &&
                   (!p.mask || (((p.ldm & 7) == 0) && al16(p.mask))) &&
                   (!p.C2 || (((p.ldc2 & 7) == 0) && al16(p.C2))) &&
                   (!p.mul || (((p.ldmul & 7) == 0) && al16(p.mul))) &&
                   (!p.add || (((p.ldadd & 7) == 0) && al16(p.add))) &&
                   (!c32 || (((p.ldc32 & 3) == 0) && al16(c32)));
  if (vec) {
    // rows i, i+1 paired: after a v_permlane16_swap per value every lane
    // holds 8 consecutive columns (16 B of bf16) of ONE row (guide T21)
    float bias[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bias[j][r] = p.bias ? p.bias[(int64_t)(nw + 16 * j + 4 * g + r) * p.bias_stride] : 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = nw + 16 * j + 8 * (g >> 1);
      // this column fragment's epilogue operands, all in flight before the first use
      uint4 mk[MI / 2], mv[MI / 2], av[MI / 2];
#pragma unroll
      for (int i = 0; i < MI; i += 2) {
        const int m = mw + (i + (g & 1)) * 16 + rho;
        if (p.mask) mk[i / 2] = *(const uint4*)(p.mask + (int64_t)m * p.ldm + n);
        if (p.C2 && p.mul) mv[i / 2] = *(const uint4*)(p.mul + (int64_t)m * p.ldmul + n);
        if (p.C2 && p.add) av[i / 2] = *(const uint4*)(p.add + (int64_t)m * p.ldadd + n);
      }
#pragma unroll
      for (int i = 0; i < MI; i += 2) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a = acc[i][j][r] + bias[j][r], b = acc[i + 1][j][r] + bias[j][r];
          if (p.relu) {
            a = fmaxf(a, 0.f);
            b = fmaxf(b, 0.f);
          }
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b),
                                                           false, false);
          v[r] = __uint_as_float(sw[0]);
          v[4 + r] = __uint_as_float(sw[1]);
        }
        const int m = mw + (i + (g & 1)) * 16 + rho;
        if (p.mask) {
          const uint4 q4 = mk[i / 2];
          const uint32_t mu[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!(bf2f((uint16_t)(mu[q] & 0xffff)) > 0.f)) v[2 * q] = 0.f;
            if (!(bf2f((uint16_t)(mu[q] >> 16)) > 0.f)) v[2 * q + 1] = 0.f;
          }
        }
        if (p.C)
          *(uint4*)(p.C + (int64_t)m * p.ldc + n) =
              make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]),
                         pack2bf(v[6], v[7]));
        if (p.C2) {
          float w2[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) w2[q] = v[q];
          if (p.mul) {
            const uint4 q4 = mv[i / 2];
            const uint32_t mu[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              w2[2 * q] *= bf2f((uint16_t)(mu[q] & 0xffff));
              w2[2 * q + 1] *= bf2f((uint16_t)(mu[q] >> 16));
            }
          }
          if (p.add) {
            const uint4 q4 = av[i / 2];
            const uint32_t au[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              w2[2 * q] += bf2f((uint16_t)(au[q] & 0xffff));
              w2[2 * q + 1] += bf2f((uint16_t)(au[q] >> 16));
            }
          }
          *(uint4*)(p.C2 + (int64_t)m * p.ldc2 + n) =
              make_uint4(pack2bf(w2[0], w2[1]), pack2bf(w2[2], w2[3]), pack2bf(w2[4], w2[5]),
                         pack2bf(w2[6], w2[7]));
        }
        if (c32) {
          float* o = c32 + (int64_t)m * p.ldc32 + n;
          *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
          *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    return;
  }
  // edge tiles / unaligned operands: element by element
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mw + 16 * i + rho, n = nw + 16 * j + 4 * g + r;
        if (m >= p.M || n >= p.N) continue;
        float x = acc[i][j][r] + (p.bias ? p.bias[(int64_t)n * p.bias_stride] : 0.f);
        if (p.relu) x = fmaxf(x, 0.f);
        if (p.mask && !(bf2f(p.mask[(int64_t)m * p.ldm + n]) > 0.f)) x = 0.f;
        if (p.C) p.C[(int64_t)m * p.ldc + n] = f2bf(x);
        if (c32) c32[(int64_t)m * p.ldc32 + n] = x;
        if (p.C2) {
          float x2 = x;
          if (p.mul) x2 *= bf2f(p.mul[(int64_t)m * p.ldmul + n]);
          if (p.add) x2 += bf2f(p.add[(int64_t)m * p.ldadd + n]);
          p.C2[(int64_t)m * p.ldc2 + n] = f2bf(x2);
        }
      }
}

template <int BMP, int NSTP, int BNP, bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_pp_body(const GemmArgs& p, int bid, char* smem_raw) {
  using G = PPGeom<BMP, NSTP, BNP>;
  constexpr int BN = BNP;
  constexpr int MI = G::MI, NJ = G::NJ, KS = G::KS, SEGS = G::SEGS, NST = G::NST;
  TDFO_LDS char* smem = (TDFO_LDS char*)smem_raw;
  const int tiles_m = (p.M + G::BM - 1) / G::BM, tiles_n = (p.N + BN - 1) / BN;
  const TileIdx ti = tile_of(tiles_m, tiles_n, p.splits, bid);
  const int m0 = ti.tm * G::BM, n0 = ti.tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.splits - 1) / p.splits;
  const int kt0 = ti.split * per;
  const int nk = max(0, min(ktiles, kt0 + per) - kt0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, q = w & 3;
  const int wr = q / G::WGN, wc = q - (q / G::WGN) * G::WGN;
  const int a_row = grp * G::GROWS + wr * G::WROWS;       // wave's first row in the tile
  const int a_img = a_row >> 7, a_r0 = a_row & 127;
  const int b_c0 = wc * G::WCOLS;
  const int b_img = b_c0 >> 7, b_cc = b_c0 & 127;
  const bool lag = grp == 1;

  f32x4_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // this wave's share of K tile kt's DMA into ring slot `slot`
  auto stage = [&](int slot, int kt) {
    TDFO_LDS char* ta = smem + slot * G::STAGE;
    TDFO_LDS char* tb = ta + G::A_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < G::APW; ++i) {
      const int ii = w * G::APW + i, img = ii >> 4;
      glds_piece_asm<A_COL>(p.A, p.lda, m0 + img * 128, p.M, k0, ta + img * TILE_BYTES, ii & 15,
                            lane);
    }
#pragma unroll
    for (int i = 0; i < G::BPW; ++i) {
      const int ii = w * G::BPW + i, img = ii >> 4;
      glds_piece_asm<B_COL>(p.B, p.ldb, n0 + img * 128, p.N, k0, tb + img * TILE_BYTES, ii & 15,
                            lane);
    }
  };
  // K tiles issued before the wait for tile T (at the end of the segment
  // holding half T*SEGS - 1) that are younger than T: tile X is issued in the
  // READ segment of half (X - NST + 1) * SEGS (the prologue for X < NST)
  auto younger = [&](int T) {
    int n = 0;
#pragma unroll
    for (int d = 1; d < NST; ++d) {
      const int X = T + d;
      if (X < nk && (X < NST || (X - NST + 1) * SEGS <= T * SEGS - 1)) ++n;
    }
    return n;
  };

  bf16x8_t af[KS][MI], bfr[KS][NJ];
  const bool csum = A_COL && p.csum_on && ti.tn == 0;
  f32x4_t cs[G::CSF];
#pragma unroll
  for (int c = 0; c < G::CSF; ++c) cs[c] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < NST; ++s)
      if (s < nk) stage(s, kt0 + s);
    pp_wait_vm<G::PPW>(younger(0));
    pp_barrier();
    if (lag) pp_barrier();                            // group 1 runs one segment behind
    const int H = nk * SEGS;
    for (int h = 0; h < H; ++h) {
      const int t = h / SEGS, s = h - t * SEGS;
      // ---- READ segment: DMA of tile t + NST - 1 (first half of tile t),
      // then this half's fragments
      if (s == 0 && t >= 1 && t + NST - 1 < nk) stage((t + NST - 1) % NST, kt0 + t + NST - 1);
      {
        const TDFO_LDS char* ta = smem + (t % NST) * G::STAGE + a_img * TILE_BYTES;
        const TDFO_LDS char* tb = smem + (t % NST) * G::STAGE + G::A_BYTES + b_img * TILE_BYTES;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int ks = s * KS + kk;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bfr[kk][j] = B_COL ? frag_col(tb, b_cc + 16 * j, ks, lane)
                               : frag_row(tb, b_cc + 16 * j, ks, lane);
#pragma unroll
          for (int i = 0; i < MI; ++i)
            af[kk][i] = A_COL ? frag_col(ta, a_r0 + 16 * i, ks, lane)
                              : frag_row(ta, a_r0 + 16 * i, ks, lane);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lag && s == SEGS - 1 && t + 1 < nk) pp_wait_vm<G::PPW>(younger(t + 1));
      pp_barrier();
      // ---- MFMA segment
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j],
                                                                0, 0, 0);
        if constexpr (A_COL) {
          if (csum) {
            const bf16x8_t ones = __builtin_bit_cast(
                bf16x8_t, (s16x8_t){0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80,
                                    0x3F80});
#pragma unroll
            for (int c = 0; c < G::CSF; ++c) {
              bf16x8_t a = af[kk][c * G::WGN];
#pragma unroll
              for (int u = 1; u < G::WGN; ++u)
                if (wc == u) a = af[kk][c * G::WGN + u];
              cs[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, a, cs[c], 0, 0, 0);
            }
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (!lag && s == SEGS - 1 && t + 1 < nk) pp_wait_vm<G::PPW>(younger(t + 1));
      pp_barrier();
    }
    if (grp == 0) pp_barrier();
  }
  if constexpr (A_COL) {
    if (csum) {
      float* c32 = p.C32 + (int64_t)ti.split * p.M * p.ldc32;
#pragma unroll
      for (int c = 0; c < G::CSF; ++c) {
        const int m = m0 + a_row + (c * G::WGN + wc) * 16 + (lane & 15);
        if (lane < 16 && m < p.M) c32[(int64_t)m * p.ldc32 + p.csum_col] = cs[c][0];
      }
    }
  }
  pp_epilogue<MI, NJ>(p, acc, m0 + a_row, n0 + b_c0, lane, ti.split);
}

using PPG = PPGeom<128, 2, 128>;

// ---------------------------------------------------------------------------
// Two-group split-K kernel ("p8"): 256x128 tiles, 8 waves in two groups of
// four (waves 0-3 / 4-7: one of each per SIMD), group 1 one barrier behind
// group 0, so on every SIMD one wave issues MFMAs while its partner reads
// fragments and issues LDS-DMA (cdna_hip_programming.md §5, the 8-phase
// template's staggered groups; T3/T4 counted vmcnt + raw barriers; T5
// setprio). Unlike that template's 256x256 tile, the block tile is 256x128
// (DLRM's 8192 x 1024 outputs are 256 such tiles: one per CU) and the two
// groups split each 64-deep K tile: group g computes its k32 half of every K
// tile on the WHOLE 256x128 tile (wave tile 128x64, 32 fragments, the
// cheapest LDS bytes per MFMA), and the two sums are added through LDS at
// the end. Two phases per K tile per group (one 64-row half of the wave tile
// x 4 column fragments = 16 MFMAs each); a 3-slot LDS ring (144 KiB) keeps
// two K tiles of DMA in flight (issued in phase 0, two tiles ahead).
// Measured (labs/probes/gemm_pp8.hip vs gemm_floor.hip, random bf16):
// compute floor 2.1 PF at 8192^3 vs 0.8-0.9 for the one-group loops.
// Epilogue: pp_epilogue (bias, ReLU, ReLU mask, DCN second output, fp32
// split-K slabs). No column-sum (bias-grad) support.
constexpr int P8_NST = 3;
constexpr int P8_STAGE = 3 * TILE_BYTES;                 // A 256x64 + B 128x64
constexpr int P8_LDS = P8_NST * P8_STAGE;                // 144 KiB (>= 128 KiB reduction)
static_assert(P8_LDS >= 128 * 1024, "p8 reduction buffer");

template <bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_p8_body(const GemmArgs& p, int bid, char* smem_raw) {
  constexpr int PPW = 6;                                  // 48 DMA pieces per K tile / 8 waves
  TDFO_LDS char* smem = (TDFO_LDS char*)smem_raw;
  const int tiles_m = (p.M + LBM - 1) / LBM, tiles_n = (p.N + BN - 1) / BN;
  const TileIdx ti = tile_of(tiles_m, tiles_n, p.splits, bid);
  const int m0 = ti.tm * LBM, n0 = ti.tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.splits - 1) / p.splits;
  const int kt0 = ti.split * per;
  const int nk = max(0, min(ktiles, kt0 + per) - kt0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, q = w & 3;
  const int ar = (q >> 1) * 128, bc = (q & 1) * 64;       // wave tile origin (128 x 64)

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int slot, int kt) {
    TDFO_LDS char* st = smem + slot * P8_STAGE;
    const int k0 = (kt0 + kt) * BK;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int ii = w * PPW + u, img = ii >> 4;
      if (img < 2)
        glds_piece_asm<A_COL>(p.A, p.lda, m0 + img * 128, p.M, k0, st + img * TILE_BYTES, ii & 15,
                              lane);
      else
        glds_piece_asm<B_COL>(p.B, p.ldb, n0, p.N, k0, st + 2 * TILE_BYTES, ii & 15, lane);
    }
  };
  bf16x8_t af[4], bfr[4];
  auto rd_a = [&](int slot, int half) {
    const TDFO_LDS char* img = smem + slot * P8_STAGE + (ar >> 7) * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = A_COL ? frag_col(img, half * 64 + i * 16, grp, lane)
                    : frag_row(img, half * 64 + i * 16, grp, lane);
  };
  auto rd_b = [&](int slot) {
    const TDFO_LDS char* img = smem + slot * P8_STAGE + 2 * TILE_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = B_COL ? frag_col(img, bc + j * 16, grp, lane) : frag_row(img, bc + j * 16, grp, lane);
  };
  auto mm = [&](int half) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[half * 4 + i][j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[half * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // the wait before tile t's first read: every thread's pieces of tile t
  // landed, tile t+1's (issued one tile later) may still be in flight
  auto wait_landed = [&](bool one_ahead) {
    if (one_ahead) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PPW) : "memory");
    else           asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  if (nk > 0) {
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    wait_landed(nk > 1);
  }
  pp_barrier();
  if (grp == 1) pp_barrier();                            // group 1: one interval behind
  for (int t = 0; t < nk; ++t) {
    const int slot = t % P8_NST;
    const bool ahead = t + 2 < nk;
    // phase 0: B fragments + upper A half; DMA of tile t+2 into the slot
    // every wave finished reading before this phase's opening barrier
    rd_b(slot);
    rd_a(slot, 0);
    if (ahead) stage((t + 2) % P8_NST, t + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();
    mm(0);
    pp_barrier();
    // phase 1: lower A half
    rd_a(slot, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp == 1 && t + 1 < nk) wait_landed(ahead);      // tile t+1 (group 1's pieces)
    pp_barrier();
    mm(1);
    if (grp == 0 && t + 1 < nk) wait_landed(ahead);      // tile t+1 (group 0's pieces)
    pp_barrier();
  }
  if (grp == 0) pp_barrier();                            // balance group 1's extra barrier
  // group 1's sums into LDS (lane-major, conflict-free), group 0 adds them
  __syncthreads();
  f32x4_t* red = (f32x4_t*)smem_raw;
  if (grp == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(q * 32 + i * 4 + j) * 64 + lane] = acc[i][j];
  }
  __syncthreads();
  if (grp == 1) return;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] += red[(q * 32 + i * 4 + j) * 64 + lane];
  pp_epilogue<8, 4>(p, acc, m0 + ar, n0 + bc, lane, ti.split);
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(512, 1) void gemm_p8_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_p8_body<A_COL, B_COL>(p, blockIdx.x, smem_raw);
}

template <bool AC0, bool BC0, bool AC1, bool BC1>
__global__ __launch_bounds__(512, 1) void gemm_p8_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x < nb0) gemm_p8_body<AC0, BC0>(p0, blockIdx.x, smem_raw);
  else                       gemm_p8_body<AC1, BC1>(p1, blockIdx.x - nb0, smem_raw);
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(512, 2) void gemm_pp_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_pp_body<128, 2, 128, A_COL, B_COL>(p, blockIdx.x, smem_raw);
}

// Two problems in one ping-pong grid (a layer's weight grad + dgrad, or two
// weight grads): blocks [0, nb0) run problem 0, the rest problem 1.
template <bool AC0, bool BC0, bool AC1, bool BC1>
// blocks [nb01, ...): a parked head_reduce (two 256-thread units per block)
__global__ __launch_bounds__(512, 2) void gemm_pp_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0,
                                                              int nb01, HeadReduceJob hr) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x >= nb01) {
    const int slice = threadIdx.x >> 8;
    head_reduce_unit(hr, ((int)blockIdx.x - nb01) * 2 + slice, threadIdx.x & 255,
                     (float(*)[RA_COLS])smem_raw + slice * RA_PH);
    return;
  }
  if ((int)blockIdx.x < nb0) gemm_pp_body<128, 2, 128, AC0, BC0>(p0, blockIdx.x, smem_raw);
  else                       gemm_pp_body<128, 2, 128, AC1, BC1>(p1, blockIdx.x - nb0, smem_raw);
}

int pp_grid(const GemmArgs& a) {
  return ((a.M + 127) / 128) * ((a.N + 127) / 128) * a.splits;
}

template <bool AC, bool BC>
void pp_launch(const GemmArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_pp_kernel<AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, PPG::LDS));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<AC, BC>), dim3(pp_grid(a)), dim3(512), PPG::LDS, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

template <bool AC0, bool BC0, bool AC1, bool BC1>
void pp_pair_launch(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  auto fn = gemm_pp_pair_kernel<AC0, BC0, AC1, BC1>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       PPG::LDS));
    attr = true;
  }
  const int g0 = pp_grid(a0), g01 = g0 + pp_grid(a1);
  HeadReduceJob hr{};
  const int side = head_reduce_take(&hr) ? (head_reduce_units(hr) + 1) / 2 : 0;
  hipLaunchKernelGGL(fn, dim3(g01 + side), dim3(512), PPG::LDS, s, a0, a1, g0, g01, hr);
  TDFO_CHECK_HIP(hipGetLastError());
}

// Kernel choice. Auto (policy 0), measured on the DLRM / DCN-v2 step shapes
// on random operands (labs/gemm_lab.py; profiles/r03/gemm_lab_*.jsonl):
//   * ping-pong 128x128 (2 blocks per CU): every weight grad and dgrad, and
//     the forwards whose 128x128 grid fills the CUs (DLRM-1TB MLP GEMMs
//     266.5 vs 285.2 us on the round-2 kernels, 0.455 vs 0.472 ms/step);
//   * deep-pipelined 128x128 (4-slot ring, one block per CU): non-weight-grad
//     GEMMs with >= 32 K tiles per split on <= 512 tiles (DCN-v2 V fwd and
//     U dgrad, K = 3456: 37 vs 45 us and 41 vs 49 us on the ping-pong kernel);
//   * 2-stage 64x128 tiles: forwards whose 128x128 grid leaves CUs idle
//     (N <= 256: bot1 / top3 fwd 8.3 vs 9.6 us).
//   * 256x128 tiles (8 waves, one block per CU) for GEMMs of >= 1024 128x128
//     tiles (DCN-v2's 3456-wide U fwd, V dgrad and top-0 dgrad), and, under
//     policy 5 (DCN-v2's default, DLRMConfig.gemm_big), for every GEMM
//     without bias column sums except the deep kernel's.
// Policies 1 / 2 / 3 / 4 force the 2-stage, deep, ping-pong or 256x128
// kernel (256x128: not for column-sum weight grads) (tests, A/B).
int g_policy = 0;

enum Kern { K_SMALL64 = 64, K_SMALL128 = 128, K_DEEP = 2, K_PP = 3, K_BIG = 4, K_P8 = 8 };

template <bool AC, bool BC>
int choose(const GemmArgs& a) {
  const int t128 = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.splits;
  const int ktps = (a.K / BK + a.splits - 1) / a.splits;
  const bool big_ok = !a.csum_on && a.K % BK == 0;
  switch (g_policy) {
    case 1: return (!AC && t128 < 256) ? K_SMALL64 : K_SMALL128;
    case 2: return K_DEEP;
    case 3: return K_PP;
    case 4: return big_ok ? K_BIG : K_PP;
    case 8: return big_ok ? K_P8 : K_PP;
    default: break;
  }
  if (g_policy == 5) {
    // DCN-v2: the deep kernel where a 256x128 grid would leave CUs idle while
    // a 128x128 one fills them about once, with long K (cross-layer V fwd /
    // U dgrad); 256x128 tiles for everything else without column sums, the
    // bottom MLP included: it runs beside the memory-bound embedding kernels
    // and its 144-KiB blocks wait there for whole free CUs (a 398-us backward
    // pair, profiles/r04/prof_dcn/step_lanes.txt), yet sending its GEMMs of
    // < 300 / 600 tiles to the 128x128 kernels ran the step at 2.64 / 2.66 vs
    // 2.36 ms (profiles/r04/notes.md); nor do the epilogue-heavy GEMMs (DCN
    // Hadamard / residual outputs, ReLU-masked dgrads) on the two-block
    // ping-pong kernel: 2.55-2.62 vs 2.37 ms
    const int t256 = ((a.M + LBM - 1) / LBM) * ((a.N + BN - 1) / BN) * a.splits;
    if (!AC && t256 < 256 && t128 <= 512 && ktps >= 16) return K_DEEP;
    if (big_ok) return K_BIG;
  } else {
    if (!AC && ktps >= 32 && t128 <= 512) return K_DEEP;
    if (big_ok && t128 >= 1024) return K_BIG;
  }
  if (AC || BC || t128 >= 256) return K_PP;
  return K_SMALL64;
}

template <bool AC, bool BC>
void launch(const GemmArgs& a, int k, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_kernel<128, AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_deep_kernel<AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, DSMEM));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_big_kernel<AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LSMEM));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_p8_kernel<AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, P8_LDS));
    attr = true;
  }
  const int tn = (a.N + BN - 1) / BN;
  switch (k) {
    case K_PP:
      pp_launch<AC, BC>(a, s);
      return;
    case K_BIG:
      hipLaunchKernelGGL((gemm_big_kernel<AC, BC>), dim3(((a.M + LBM - 1) / LBM) * tn * a.splits),
                         dim3(512), LSMEM, s, a);
      break;
    case K_P8:
      hipLaunchKernelGGL((gemm_p8_kernel<AC, BC>), dim3(((a.M + LBM - 1) / LBM) * tn * a.splits),
                         dim3(512), P8_LDS, s, a);
      break;
    case K_DEEP:
      hipLaunchKernelGGL((gemm_deep_kernel<AC, BC>), dim3(((a.M + BM - 1) / BM) * tn * a.splits),
                         dim3(256), DSMEM, s, a);
      break;
    case K_SMALL64:
      if constexpr (!AC) {
        hipLaunchKernelGGL((gemm_kernel<64, AC, BC>), dim3(((a.M + 63) / 64) * tn * a.splits),
                           dim3(256), 2 * (64 * BK * 2 + TILE_BYTES), s, a);
        break;
      }
      [[fallthrough]];
    default:
      hipLaunchKernelGGL((gemm_kernel<128, AC, BC>), dim3(((a.M + BM - 1) / BM) * tn * a.splits),
                         dim3(256), SMEM_BYTES, s, a);
      break;
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

int kernel_of(const GemmArgs& a) {
  if (a.a_col) return a.b_col ? choose<true, true>(a) : choose<true, false>(a);
  return a.b_col ? choose<false, true>(a) : choose<false, false>(a);
}

void launch_any(const GemmArgs& a, hipStream_t s) {
  const int k = kernel_of(a);
  if (a.a_col) {
    if (a.b_col) launch<true, true>(a, k, s); else launch<true, false>(a, k, s);
  } else {
    if (a.b_col) launch<false, true>(a, k, s); else launch<false, false>(a, k, s);
  }
}

// layout code of a problem: 0 row/row, 1 row/col, 3 col/col (col/row unused)
int layout_of(const GemmArgs& a) { return (a.a_col ? 2 : 0) | (a.b_col ? 1 : 0); }

// A layer's weight grad + dgrad (both read dy), or two weight grads, both on
// the ping-pong kernel: one grid (each small launch pays fill / drain, and
// the two problems' blocks fill each other's idle CUs). Bit-identical to
// two launches.
int big_grid(const GemmArgs& a) {
  return ((a.M + LBM - 1) / LBM) * ((a.N + BN - 1) / BN) * a.splits;
}

template <bool AC0, bool BC0, bool AC1, bool BC1>
void big_pair_launch(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  auto fn = gemm_big_pair_kernel<AC0, BC0, AC1, BC1>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       LSMEM));
    attr = true;
  }
  const int g0 = big_grid(a0);
  hipLaunchKernelGGL(fn, dim3(g0 + big_grid(a1)), dim3(512), LSMEM, s, a0, a1, g0);
  TDFO_CHECK_HIP(hipGetLastError());
}

template <bool AC0, bool BC0, bool AC1, bool BC1>
void p8_pair_launch(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  auto fn = gemm_p8_pair_kernel<AC0, BC0, AC1, BC1>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       P8_LDS));
    attr = true;
  }
  const int g0 = big_grid(a0);
  hipLaunchKernelGGL(fn, dim3(g0 + big_grid(a1)), dim3(512), P8_LDS, s, a0, a1, g0);
  TDFO_CHECK_HIP(hipGetLastError());
}

bool try_pair(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  const int k0 = kernel_of(a0), k1 = kernel_of(a1);
  const int l0 = layout_of(a0), l1 = layout_of(a1);
  if (k0 == K_P8 && k1 == K_P8) {
    if (l0 == 3 && l1 == 1) { p8_pair_launch<true, true, false, true>(a0, a1, s); return true; }
    if (l1 == 3 && l0 == 1) { p8_pair_launch<true, true, false, true>(a1, a0, s); return true; }
    if (l0 == 3 && l1 == 3) { p8_pair_launch<true, true, true, true>(a0, a1, s); return true; }
    return false;
  }
  // 256x128 pairs: a weight grad on that kernel takes its layer's dgrad
  // along onto it (also a deep-kernel one: one grid instead of two)
  const bool b0 = k0 == K_BIG || (k1 == K_BIG && k0 == K_DEEP && !a0.csum_on);
  const bool b1 = k1 == K_BIG || (k0 == K_BIG && k1 == K_DEEP && !a1.csum_on);
  if (b0 && b1) {
    if (l0 == 3 && l1 == 1) { big_pair_launch<true, true, false, true>(a0, a1, s); return true; }
    if (l1 == 3 && l0 == 1) { big_pair_launch<true, true, false, true>(a1, a0, s); return true; }
    if (l0 == 3 && l1 == 3) { big_pair_launch<true, true, true, true>(a0, a1, s); return true; }
    return false;
  }
  if (k0 != K_PP || k1 != K_PP) return false;
  if (l0 == 3 && l1 == 1) { pp_pair_launch<true, true, false, true>(a0, a1, s); return true; }
  if (l1 == 3 && l0 == 1) { pp_pair_launch<true, true, false, true>(a1, a0, s); return true; }
  if (l0 == 3 && l1 == 3) { pp_pair_launch<true, true, true, true>(a0, a1, s); return true; }
  return false;
}

int g_pair = 1;

}  // namespace

int gemm_policy(int p) {
  const int old = g_policy;
  if (p >= 0) g_policy = p;
  return old;
}

void gemm_bf16(const GemmArgs& a, hipStream_t s) { launch_any(a, s); }

int gemm_pairing(int v) {
  const int old = g_pair;
  if (v >= 0) g_pair = v ? 1 : 0;
  return old;
}

void gemm_group(const GemmArgs* a, int n, hipStream_t s) {
  for (int i = 0; i < n;) {
    if (g_pair && i + 1 < n && try_pair(a[i], a[i + 1], s)) {
      i += 2;
      continue;
    }
    gemm_bf16(a[i], s);
    ++i;
  }
}

}  // namespace tdfo
