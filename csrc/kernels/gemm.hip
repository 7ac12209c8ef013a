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
#include "tdfo_common.h"
#include "tdfo_kernels.h"

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
  if (p.abl & (224 | 256)) return false;           // ablations / forced LDS path
  // operand reads (ReLU mask, DCN mul/add) in this layout are 32-B row runs;
  // the LDS path reads them as 256-B rows (measured: DCN-v2 3.16 vs 3.05 ms)
  if (p.mul || p.add) return false;
  if (p.mask && !(p.abl & 512)) return false;      // abl 512: masked dgrads direct too (A/B)
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
      (p.N & 3) == 0 && !(p.abl & 224)) {   // abl 128: force the LDS path (A/B)
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
  const bool pf = !(p.abl & 1024) && (p.N & 7) == 0 &&
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
    if (p.abl & 64) {                  // perf ablation: LDS staging only, no global stores
      asm volatile("" :: "v"(lo.x), "v"(lo.y), "v"(lo.z), "v"(lo.w), "v"(hi.x), "v"(hi.y), "v"(hi.z), "v"(hi.w));
      continue;
    }
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

// Two independent small-tile GEMMs in one grid: blocks [0, nb0) run problem
// 0, the rest problem 1 (e.g. a layer's weight grad and its dgrad, both
// reading dy). Each small launch pays ~4-6 us of fill / drain / launch in the
// graph (profiles/gemm_step_ab.md: 5.9 us for a one-K-tile 256-block GEMM);
// paired, the two problems' blocks also fill each other's idle CUs.
template <int BM0, bool AC0, bool BC0, int BM1, bool AC1, bool BC1>
__global__ __launch_bounds__(256, 2) void gemm_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x < nb0) gemm_small_body<BM0, AC0, BC0>(p0, blockIdx.x, smem_raw);
  else                       gemm_small_body<BM1, AC1, BC1>(p1, blockIdx.x - nb0, smem_raw);
}

// ---------------------------------------------------------------------------
// Large-tile kernel: 256x128x64, 8 waves (4 along M x 2 along N, each 64x64),
// 3-deep glds ring (3 x 48 KiB = 144 KiB LDS, 1 block per CU, 2 waves per
// SIMD). Two K tiles stay in flight across each barrier: the wait before the
// barrier is a counted vmcnt (6 pieces per thread per tile), the barrier is a
// raw s_barrier (no vmcnt(0) drain, cdna_hip_programming.md "Pipelining
// across barriers"), and the ring slot being refilled is the one every wave
// finished reading before that barrier. Twice the FLOP per staged byte of the
// 128x128 tile, which is what bounds that kernel on these short-K problems.
constexpr int LBM = 256;
constexpr int LSTAGE = 3 * TILE_BYTES;             // A (2 images) + B
constexpr int LNSTAGE = 3;
constexpr int LSMEM = LNSTAGE * LSTAGE;            // 144 KiB >= 256x128 fp32 epilogue tile

// MI = 4: 8 waves (4 along M x 2 along N), 64x64 per wave, 2 waves per SIMD.
// MI = 8: 4 waves (2 x 2), 128x64 per wave (32 accumulators), 1 wave per
// SIMD: 1.33x the FLOP per LDS-read byte of the 64x64 wave tile (12 fragment
// reads per 32 MFMAs instead of 8 per 16), the wave hides its own reads
// between MFMAs (fragment double buffer) and the 3-deep ring keeps two K
// tiles of DMA in flight.
template <bool A_COL, bool B_COL, int MI>
__device__ __forceinline__ void gemm_big_body(const GemmArgs& p, int bid, char* smem_raw) {
  constexpr int NW = MI == 4 ? 8 : 4;               // waves
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
    if (!(p.abl & 1))
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int ii = w * APW + i, half = ii >> 4;
      glds_piece_asm<A_COL>(p.A, p.lda, m0 + half * 128, p.M, k0, ta + half * TILE_BYTES,
                            ii & 15, lane);
    }
    if (!(p.abl & 2))
#pragma unroll
    for (int i = 0; i < BPW; ++i)
      glds_piece_asm<B_COL>(p.B, p.ldb, n0, p.N, k0, tb, w * BPW + i, lane);
  };
  auto wait_one_ahead = [&]() {        // all but the youngest K tile's pieces landed
    if constexpr (NW == 8) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
  };

  // Fragment-pipelined main loop: one raw barrier per K tile, in the middle
  // of it. Iteration t: issue tile t+2's DMA, read tile t's k=32..63
  // fragments, MFMAs on its k=0..31 fragments (read last iteration) hide that
  // read, then wait for tile t+1 + barrier, read tile t+1's k=0..31
  // fragments, and the k=32..63 MFMAs hide those. Ring-slot reuse: slot
  // (t+2)%3 was last read before iteration t-1's barrier (each wave drains
  // its LDS reads with lgkmcnt(0) before that barrier).
  if (nk > 0 && !(p.abl & 16)) {
    const TDFO_LDS char* tAo = smem + (MI == 4 ? (wr >> 1) : wr) * TILE_BYTES;
    const TDFO_LDS char* tBo = smem + 2 * TILE_BYTES;
    const int a_r0 = MI == 4 ? (wr & 1) * 64 : 0, b_c0 = wc * 64;
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
  } else if (nk > 0) {
    stage(0, kt0);
    if (nk > 1) stage(1, kt0 + 1);
    int cur = 0;
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk && !(p.abl & 7)) wait_one_ahead();
      else            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nk && !(p.abl & 4)) stage(cur == 0 ? 2 : cur - 1, kt0 + t + 2);
      const TDFO_LDS char* ta = smem + cur * LSTAGE;
      mfma_k64<A_COL, B_COL, MI>(acc, ta + (MI == 4 ? (wr >> 1) : wr) * TILE_BYTES,
                                 MI == 4 ? (wr & 1) * 64 : 0, ta + 2 * TILE_BYTES, wc * 64, lane);
      cur = cur == 2 ? 0 : cur + 1;
    }
  }
  if (p.abl & 32) {                 // perf ablation: keep acc live, skip the epilogue
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  epilogue<LBM, NW * 64, MI>(p, acc, smem_raw, m0, n0, wr, wc, lane, tid, ti.split);
}

template <bool A_COL, bool B_COL, int MI>
__global__ __launch_bounds__(MI == 4 ? 512 : 256, 1) void gemm_big_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_big_body<A_COL, B_COL, MI>(p, blockIdx.x, smem_raw);
}

// Paired 256x128 launch (DCN-v2's one-block-per-CU kernel): see gemm_pair_kernel.
template <bool AC0, bool BC0, bool AC1, bool BC1>
__global__ __launch_bounds__(512, 1) void gemm_big_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x < nb0) gemm_big_body<AC0, BC0, 4>(p0, blockIdx.x, smem_raw);
  else                       gemm_big_body<AC1, BC1, 4>(p1, blockIdx.x - nb0, smem_raw);
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
// Ping-pong tile kernel (BM x 128 x 64, BM = 256 or 128, 8 waves).
//
// The waves form two groups of four (waves 0-3 and 4-7: one wave of each
// group per SIMD) that own the upper and lower half of the tile's rows. Each
// wave alternates a READ segment (its fragment ds_reads for the next k-chunk,
// plus its share of the global->LDS DMA) and an MFMA segment, every segment
// closed by a workgroup barrier; group 1 starts one barrier late, so on every
// SIMD one wave issues MFMAs while the other reads LDS and issues DMA -- the
// MFMA pipe sees one wave's back-to-back MFMAs in every interval
// (cdna_hip_programming.md §5 "8-phase template": per-phase interleave with
// the wave groups staggered by a barrier; T3+T4 counted vmcnt, T5 setprio).
// Operands are staged by inline-asm global_load_lds into an NST-deep LDS ring
// (counted vmcnt, raw s_barrier: DMA stays in flight across barriers).
//   BM = 256: waves 64x64 (2x2 per group), 16 MFMAs per segment, 3-slot ring
//             (144 KiB LDS).
//   BM = 128: waves 64x32 (1x4 per group), both k32 steps of a K tile per
//             segment (16 MFMAs), 4-slot ring (128 KiB LDS).
// Epilogue straight from the accumulators (bias, ReLU, ReLU mask, DCN
// Hadamard/residual second output, fp32 split-K slabs, bias-grad column sums).
template <int BMP, int NSTP = (BMP == 256 ? 3 : 4)>
struct PPGeom {
  static constexpr int BM = BMP;
  static constexpr int GROWS = BM / 2;                  // rows per wave group
  static constexpr int WGM = BM == 256 ? 2 : 1;         // waves along M in a group
  static constexpr int WGN = 4 / WGM;
  static constexpr int WROWS = GROWS / WGM;             // 64
  static constexpr int WCOLS = BN / WGN;                // 64 | 32
  static constexpr int MI = WROWS / 16;                 // 4
  static constexpr int NJ = WCOLS / 16;                 // 4 | 2
  static constexpr int KS = NJ == 4 ? 1 : 2;            // k32 steps per segment
  static constexpr int SEGS = 2 / KS;                   // READ/MFMA segment pairs per K tile
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int STAGE = A_BYTES + TILE_BYTES;
  static constexpr int NST = NSTP;
  static constexpr int LDS = NST * STAGE;
  static constexpr int APW = BM / 64;                   // A glds pieces per wave per K tile
  static constexpr int BPW = 2;
  static constexpr int PPW = APW + BPW;
  static constexpr int CSF = MI / WGN;                  // column-sum fragments per wave
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
    // epilogue operands first (all loads in flight before the first use)
    uint4 mk[MI / 2][NJ], mv[MI / 2][NJ], av[MI / 2][NJ];
#pragma unroll
    for (int i = 0; i < MI; i += 2)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = mw + (i + (g & 1)) * 16 + rho;
        const int n = nw + 16 * j + 8 * (g >> 1);
        if (p.mask) mk[i / 2][j] = *(const uint4*)(p.mask + (int64_t)m * p.ldm + n);
        if (p.C2 && p.mul) mv[i / 2][j] = *(const uint4*)(p.mul + (int64_t)m * p.ldmul + n);
        if (p.C2 && p.add) av[i / 2][j] = *(const uint4*)(p.add + (int64_t)m * p.ldadd + n);
      }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = nw + 16 * j + 8 * (g >> 1);
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
          const uint4 q4 = mk[i / 2][j];
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
            const uint4 q4 = mv[i / 2][j];
            const uint32_t mu[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              w2[2 * q] *= bf2f((uint16_t)(mu[q] & 0xffff));
              w2[2 * q + 1] *= bf2f((uint16_t)(mu[q] >> 16));
            }
          }
          if (p.add) {
            const uint4 q4 = av[i / 2][j];
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

template <int BMP, int NSTP, bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_pp_body(const GemmArgs& p, int bid, char* smem_raw) {
  using G = PPGeom<BMP, NSTP>;
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
  // A/B knobs (p.abl): 1 DMA issued in the MFMA segment (4: after its
  // MFMAs) instead of the READ segment; 2 no stagger (both groups in phase)
  const bool gm = p.abl & 1, gend = p.abl & 4, nopp = p.abl & 2;
  const bool lag = grp == 1 && !nopp;

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
    for (int i = 0; i < G::BPW; ++i)
      glds_piece_asm<B_COL>(p.B, p.ldb, n0, p.N, k0, tb, w * G::BPW + i, lane);
  };
  // K tiles issued before the wait for tile T (at the end of the segment
  // holding half T*SEGS - 1) that are younger than T: tile X is issued in the
  // READ segment of half (X - NST + 1) * SEGS (the prologue for X < NST)
  auto younger = [&](int T) {
    int n = 0;
#pragma unroll
    for (int d = 1; d < NST; ++d) {
      const int X = T + d;
      const int hx = (X - NST + 1) * SEGS;
      if (X < nk && (X < NST || hx < T * SEGS - 1 || (hx == T * SEGS - 1 && !(lag && gm)))) ++n;
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
      const bool dma = s == 0 && t >= 1 && t + NST - 1 < nk;
      if (dma && !gm) stage((t + NST - 1) % NST, kt0 + t + NST - 1);
      {
        const TDFO_LDS char* ta = smem + (t % NST) * G::STAGE + a_img * TILE_BYTES;
        const TDFO_LDS char* tb = smem + (t % NST) * G::STAGE + G::A_BYTES;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int ks = s * KS + kk;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bfr[kk][j] = B_COL ? frag_col(tb, b_c0 + 16 * j, ks, lane)
                               : frag_row(tb, b_c0 + 16 * j, ks, lane);
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
      if (dma && gm && !gend) stage((t + NST - 1) % NST, kt0 + t + NST - 1);
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
      if (dma && gm && gend) stage((t + NST - 1) % NST, kt0 + t + NST - 1);
      if (!lag && s == SEGS - 1 && t + 1 < nk) pp_wait_vm<G::PPW>(younger(t + 1));
      pp_barrier();
    }
    if (grp == 0 && !nopp) pp_barrier();
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

template <int BMP, int NSTP, int OCC, bool A_COL, bool B_COL>
__global__ __launch_bounds__(512, OCC) void gemm_pp_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  gemm_pp_body<BMP, NSTP, A_COL, B_COL>(p, blockIdx.x, smem_raw);
}

// Two problems in one ping-pong grid (a layer's weight grad + dgrad): blocks
// [0, nb0) run problem 0 on BM0-row tiles, the rest problem 1 on BM1-row tiles.
// (the production configuration: 128-row tiles, 2-slot ring, 2 blocks per CU)
template <bool AC0, bool BC0, bool AC1, bool BC1>
__global__ __launch_bounds__(512, 2) void gemm_pp_pair_kernel(GemmArgs p0, GemmArgs p1, int nb0) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  if ((int)blockIdx.x < nb0) gemm_pp_body<128, 2, AC0, BC0>(p0, blockIdx.x, smem_raw);
  else                       gemm_pp_body<128, 2, AC1, BC1>(p1, blockIdx.x - nb0, smem_raw);
}

template <int BMP, int NSTP, int OCC, bool AC, bool BC>
void pp_launch(const GemmArgs& a, hipStream_t s) {
  using G = PPGeom<BMP, NSTP>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_pp_kernel<BMP, NSTP, OCC, AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  const int tiles = ((a.M + BMP - 1) / BMP) * ((a.N + BN - 1) / BN) * a.splits;
  hipLaunchKernelGGL((gemm_pp_kernel<BMP, NSTP, OCC, AC, BC>), dim3(tiles), dim3(512), G::LDS, s,
                     a);
  TDFO_CHECK_HIP(hipGetLastError());
}

// 0 auto, 1 small tiles only (64-row tiles when 128-row ones underfill),
// 2 large tiles only, 3 128x128 tiles only, 4 = 1 with 256x128 tiles for
// the weight-grad (col-A) GEMMs, 5 = auto with 64-row tiles below 512
// 128x128 tiles (instead of 256). Auto (default) takes the 256x128 kernel only
// for GEMMs with >= 1024 128x128 tiles: in the graph-replayed DLRM-1TB step
// (<= 512 tiles per GEMM) 128x128 measured 0.725-0.728 ms/step vs 0.735 with
// the 256x128 kernel from 256 blocks up (profiles/gemm_tile_ab.md); on the
// DCN-v2 cross layers (1728 tiles) 256x128 is ahead (3.19 vs 3.28 ms/step).
int g_policy = 0;

// The launch a problem would get: bmt 64 / 128 small-tile kernel, 256 the
// 8-wave 256x128 kernel, 0 another kernel.
struct SmallPlan {
  int bmt, grid;
  GemmArgs args;
  int big_grid;   // deep-kernel problems: the 256x128 grid if paired instead (0: n/a)
};

// plan != nullptr: decide only; fill *plan (bmt 0 if the problem would not
// run on the small-tile kernel) and launch nothing.
template <bool AC, bool BC>
void launch(const GemmArgs& a, hipStream_t s, SmallPlan* plan = nullptr) {
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_kernel<128, AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       SMEM_BYTES));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_big_kernel<AC, BC, 4>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LSMEM));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_big_kernel<AC, BC, 8>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LSMEM));
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)gemm_deep_kernel<AC, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, DSMEM));
    attr = true;
  }
  if (g_policy >= 30 && g_policy < 70 && !plan) {
    // ping-pong kernel: 30 auto (256-row tiles when they fill the CUs), 31 256, 32 128;
    // A/B: 40+k 256-row with abl k, 50+k 128-row, 60+k 128-row 2-slot ring at 2 blocks/CU
    GemmArgs b = a;
    const int t256 = ((a.M + 255) / 256) * ((a.N + BN - 1) / BN) * a.splits;
    if (g_policy >= 40) b.abl = g_policy % 10;
    if (g_policy == 31 || (g_policy == 30 && t256 >= 240) || (g_policy >= 40 && g_policy < 50))
      pp_launch<256, 3, 1, AC, BC>(b, s);
    else if (g_policy >= 60)
      pp_launch<128, 2, 2, AC, BC>(b, s);
    else
      pp_launch<128, 4, 1, AC, BC>(b, s);
    return;
  }
  const int tn = (a.N + BN - 1) / BN;
  const int small_tiles = ((a.M + BM - 1) / BM) * tn;
  // auto: the ping-pong kernel (128-row tiles, 2 blocks per CU) for every
  // weight grad and dgrad and for forwards whose 128-row grid fills the CUs
  // (scripts/gemm_lab.py, profiles/gemm_lab_r03.md); GEMMs with >= 1024
  // tiles keep the 256x128 kernel below
  if (g_policy == 0 && small_tiles * a.splits < 1024 &&
      (AC || BC || small_tiles * a.splits >= 256)) {
    if (plan) {
      plan->bmt = 129;
      plan->grid = small_tiles * a.splits;
      plan->args = a;
      plan->big_grid = 0;
      return;
    }
    pp_launch<128, 2, 2, AC, BC>(a, s);
    return;
  }
  const int big_tiles = ((a.M + LBM - 1) / LBM) * tn;
  GemmArgs b = a;
  b.abl = (g_policy >= 8 && g_policy < 16) ? g_policy - 8 : 0;  // perf ablations (9..15), big kernel
  if (g_policy == 6) b.abl = 128;                // auto, every output through the LDS epilogue
  if (g_policy == 7) b.abl = 256;                // auto, bf16 outputs through the LDS epilogue
  if (g_policy == 17) b.abl = 512;               // auto, masked dgrads on the direct path
  const bool autop = g_policy == 0 || g_policy == 6 || g_policy == 7 || g_policy == 17 ||
                     g_policy == 21 || g_policy == 22 || g_policy == 24;
  bool big = (g_policy >= 2 && g_policy != 3 && g_policy != 4 && !autop) ||
             (g_policy == 4 && AC) || (autop && small_tiles * a.splits >= 1024);
  // the A column sums are produced by the 128x128 kernel only
  const bool small_only = a.csum_on != 0;
  if (small_only) big = false;
  // policy 20: the 4-wave 128x64-per-wave kernel for every GEMM; 21: auto
  // with it in place of the 8-wave kernel; 22: auto with it for every GEMM
  // that fills >= 128 CUs with 256x128 tiles
  // policy 23: the deep-pipelined 128x128 kernel for every GEMM; 24: auto,
  // with it in place of the 2-stage 128x128 kernel where the grid has at
  // most 2 tiles per CU and K spans >= 16 tiles per split
  // 25 (DCN-v2): policy 2 (256x128 everywhere), except the deep kernel for
  // non-weight-grad GEMMs whose 256x128 grid would leave CUs idle while a
  // 128x128 grid fills them once, with long K (cross-layer V fwd / U dgrad:
  // 36 vs 44 us and 39 vs 48 us, profiles/gemm_step_ab.md)
  const int ktps = (a.K / BK + a.splits - 1) / a.splits;
  const bool deep25 = g_policy == 25 && !AC && big_tiles * a.splits < 256 &&
                      small_tiles * a.splits <= 512 && ktps >= 16;
  if (g_policy == 25 && !deep25 && !small_only) big = true;
  const bool deep = g_policy == 23 || deep25 ||
                    (g_policy == 24 && !big && small_tiles * a.splits <= 512 && ktps >= 16);
  const bool w4 = !small_only && (g_policy == 20 || (g_policy == 22 && big_tiles * a.splits >= 128) ||
                                  (g_policy == 21 && small_tiles * a.splits >= 1024));
  if (plan) {
    plan->bmt = 0;
    plan->args = b;
    plan->big_grid = (deep && !small_only) ? big_tiles * a.splits : 0;
    if (deep || w4) return;
    if (big) {                                    // 256x128, 8 waves
      plan->bmt = 256;
      plan->grid = big_tiles * a.splits;
      return;
    }
    if constexpr (!AC) {
      const int thr64 = g_policy == 5 ? 512 : 256;
      if (small_tiles * a.splits < thr64 && g_policy != 3 && g_policy != 2) {
        plan->bmt = 64;
        plan->grid = ((a.M + 63) / 64) * tn * a.splits;
        return;
      }
    }
    plan->bmt = 128;
    plan->grid = small_tiles * a.splits;
    return;
  }
  if (deep) {
    dim3 grid(small_tiles * a.splits);
    hipLaunchKernelGGL((gemm_deep_kernel<AC, BC>), grid, dim3(256), DSMEM, s, b);
    TDFO_CHECK_HIP(hipGetLastError());
    return;
  }
  if (!small_only && (g_policy == 20 || (g_policy == 22 && big_tiles * a.splits >= 128))) {
    b.abl = 0;
    dim3 grid(big_tiles * a.splits);
    hipLaunchKernelGGL((gemm_big_kernel<AC, BC, 8>), grid, dim3(256), LSMEM, s, b);
    TDFO_CHECK_HIP(hipGetLastError());
    return;
  }
  if (!small_only && g_policy == 21 && small_tiles * a.splits >= 1024) {
    dim3 grid(big_tiles * a.splits);
    hipLaunchKernelGGL((gemm_big_kernel<AC, BC, 8>), grid, dim3(256), LSMEM, s, b);
    TDFO_CHECK_HIP(hipGetLastError());
    return;
  }
  if (big) {
    dim3 grid(big_tiles * a.splits);
    hipLaunchKernelGGL((gemm_big_kernel<AC, BC, 4>), grid, dim3(512), LSMEM, s, b);
  } else {
    if constexpr (!AC) {
      // 64-row tiles when 128-row tiles leave CUs idle (bottom MLP, top3)
      const int thr64 = g_policy == 5 ? 512 : 256;
      if (small_tiles * a.splits < thr64 && g_policy != 3 && g_policy != 2) {
        const int t64 = ((a.M + 63) / 64) * tn;
        dim3 grid(t64 * a.splits);
        hipLaunchKernelGGL((gemm_kernel<64, AC, BC>), grid, dim3(256),
                           2 * (64 * BK * 2 + TILE_BYTES), s, b);
        TDFO_CHECK_HIP(hipGetLastError());
        return;
      }
    }
    dim3 grid(small_tiles * a.splits);
    hipLaunchKernelGGL((gemm_kernel<128, AC, BC>), grid, dim3(256), SMEM_BYTES, s, b);
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace

int gemm_policy(int p) {
  const int old = g_policy;
  if (p >= 0) g_policy = p;
  return old;
}

void gemm_bf16(const GemmArgs& a, hipStream_t s) {
  if (a.a_col) {
    if (a.b_col) launch<true, true>(a, s); else launch<true, false>(a, s);
  } else {
    if (a.b_col) launch<false, true>(a, s); else launch<false, false>(a, s);
  }
}

namespace {
SmallPlan small_plan(const GemmArgs& a) {
  SmallPlan p{};
  if (a.a_col) {
    if (a.b_col) launch<true, true>(a, nullptr, &p); else launch<true, false>(a, nullptr, &p);
  } else {
    if (a.b_col) launch<false, true>(a, nullptr, &p); else launch<false, false>(a, nullptr, &p);
  }
  return p;
}

// layout code of a problem: 0 row/row, 1 row/col, 3 col/col (col/row unused)
int layout_of(const GemmArgs& a) { return (a.a_col ? 2 : 0) | (a.b_col ? 1 : 0); }

template <int BM0, bool AC0, bool BC0, int BM1, bool AC1, bool BC1>
void pair_launch(const SmallPlan& p0, const SmallPlan& p1, hipStream_t s) {
  auto fn = gemm_pair_kernel<BM0, AC0, BC0, BM1, AC1, BC1>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES));
    attr = true;
  }
  hipLaunchKernelGGL(fn, dim3(p0.grid + p1.grid), dim3(256), SMEM_BYTES, s, p0.args, p1.args,
                     p0.grid);
  TDFO_CHECK_HIP(hipGetLastError());
}

// The pairs the MLP backward issues: a layer's dgrad (row A, col B; 64- or
// 128-row tiles) with its weight grad (col A, col B, 128-row tiles), or two
// weight grads (the deferred ones of a multi-rank step).
template <bool AC0, bool BC0, bool AC1, bool BC1>
void big_pair_launch(const SmallPlan& p0, const SmallPlan& p1, hipStream_t s) {
  auto fn = gemm_big_pair_kernel<AC0, BC0, AC1, BC1>;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LSMEM));
    attr = true;
  }
  hipLaunchKernelGGL(fn, dim3(p0.grid + p1.grid), dim3(512), LSMEM, s, p0.args, p1.args,
                     p0.grid);
  TDFO_CHECK_HIP(hipGetLastError());
}

template <bool AC0, bool BC0, bool AC1, bool BC1>
void pp_pair_launch(const SmallPlan& p0, const SmallPlan& p1, hipStream_t s) {
  auto fn = gemm_pp_pair_kernel<AC0, BC0, AC1, BC1>;
  constexpr int lds = PPGeom<128, 2>::LDS;
  static bool attr = false;
  if (!attr) {
    TDFO_CHECK_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       lds));
    attr = true;
  }
  hipLaunchKernelGGL(fn, dim3(p0.grid + p1.grid), dim3(512), lds, s, p0.args, p1.args, p0.grid);
  TDFO_CHECK_HIP(hipGetLastError());
}

int g_pair_deep = 1;   // pair a deep-kernel dgrad on 256x128 tiles with its weight grad

bool try_pair(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  SmallPlan p0 = small_plan(a0), p1 = small_plan(a1);
  // a dgrad the deep 128x128 kernel would take alone (DCN-v2's U dgrad: the
  // 256x128 grid leaves CUs idle) runs on 256x128 tiles beside a 256x128
  // weight grad, whose blocks fill those CUs
  if (g_pair_deep && p0.bmt == 256 && !p1.bmt && p1.big_grid) { p1.bmt = 256; p1.grid = p1.big_grid; }
  if (g_pair_deep && p1.bmt == 256 && !p0.bmt && p0.big_grid) { p0.bmt = 256; p0.grid = p0.big_grid; }
  if (!p0.bmt || !p1.bmt) return false;
  const int l0 = layout_of(a0), l1 = layout_of(a1);
  if (p0.bmt == 129 || p1.bmt == 129) {           // ping-pong pairs
    if (p0.bmt != 129 || p1.bmt != 129) return false;
    if (l0 == 3 && l1 == 1) { pp_pair_launch<true, true, false, true>(p0, p1, s); return true; }
    if (l1 == 3 && l0 == 1) { pp_pair_launch<true, true, false, true>(p1, p0, s); return true; }
    if (l0 == 3 && l1 == 3) { pp_pair_launch<true, true, true, true>(p0, p1, s); return true; }
    return false;
  }
  if ((p0.bmt == 256) != (p1.bmt == 256)) return false;
  if (p0.bmt == 256) {                            // weight grad + dgrad on 256x128 tiles
    if (l0 == 3 && l1 == 1) { big_pair_launch<true, true, false, true>(p0, p1, s); return true; }
    if (l1 == 3 && l0 == 1) { big_pair_launch<true, true, false, true>(p1, p0, s); return true; }
    if (l0 == 3 && l1 == 3) { big_pair_launch<true, true, true, true>(p0, p1, s); return true; }
    return false;
  }
  if (l0 == 3 && l1 == 3 && p0.bmt == 128 && p1.bmt == 128) {   // two weight grads
    pair_launch<128, true, true, 128, true, true>(p0, p1, s);
    return true;
  }
  if (l0 == 3 && p0.bmt == 128 && l1 == 1) {
    if (p1.bmt == 64) pair_launch<128, true, true, 64, false, true>(p0, p1, s);
    else              pair_launch<128, true, true, 128, false, true>(p0, p1, s);
    return true;
  }
  if (l1 == 3 && p1.bmt == 128 && l0 == 1) {
    if (p0.bmt == 64) pair_launch<128, true, true, 64, false, true>(p1, p0, s);
    else              pair_launch<128, true, true, 128, false, true>(p1, p0, s);
    return true;
  }
  return false;
}
}  // namespace

int g_pair = 1;

int gemm_pairing(int v) {
  // 0 off, 1 on, 2 on but a deep-kernel dgrad is not moved to 256x128 tiles
  const int old = g_pair ? (g_pair_deep ? 1 : 2) : 0;
  if (v >= 0) {
    g_pair = v ? 1 : 0;
    g_pair_deep = v == 1 ? 1 : 0;
  }
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
