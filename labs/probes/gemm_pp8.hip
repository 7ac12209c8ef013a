// Two-group ping-pong GEMM lab (cdna_hip_programming.md §5 "256^2 8-phase
// template" structure, written for this repo's swizzled LDS images):
//   BM = 256, 8 waves in two groups of 4 (waves 0-3, 4-7; one of each per
//   SIMD), group 1 one barrier behind group 0, so on every SIMD one wave
//   issues MFMAs while the other reads LDS fragments / issues LDS-DMA.
//   Wave tile 128 x 64 (32 16x16x32 fragments), 16 MFMAs per phase.
//   KS = 1: BN = 256, the groups own the upper / lower 128 rows, 4 phases per
//           64-deep K tile (one 64x32 quadrant x both k32 steps each).
//   KS = 2: BN = 128, intra-block split-K: group g computes k32 step g of
//           every K tile on the whole 256x128 tile (2 phases per K tile: one
//           64-row half x 4 column fragments); the groups' sums are added
//           through LDS at the end.
//   Two LDS slots (K tile t+1's DMA issued in the first phase(s) of tile t,
//   drained by a vmcnt(0) in the last interval before tile t+1's first
//   read); every read interval ends with lgkmcnt(0) before its barrier.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 gemm_pp8.hip -o gemm_pp8
#include "lab_common.h"

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// SPREAD: 0 DMA issued in the first phase(s) of a tile, 1 spread over all
// phases, 2 register staging (global_load_dwordx4 of tile t+2 into VGPRs at
// phase 0 of tile t, ds_write_b128 of them at phase 0 of tile t+1 into the
// same lane-linear images; cdna_hip_programming.md T14)
template <int BN, int KS, int NST, bool AC, bool BC, int MODE, int SPREAD = 0>
__global__ __launch_bounds__(512, 1) void gpp(P p) {
  constexpr int BM = 256;
  constexpr int AI = 2, BI = BN / 128;
  constexpr int STAGE = (AI + BI) * IMG;
  constexpr int PIECES = (AI + BI) * 16;                // 1-KiB DMA pieces per K tile
  constexpr int PPW = PIECES / 8;                       // per wave
  constexpr int NPH = KS == 1 ? 4 : 2;                  // phases per K tile
  constexpr int LPH = SPREAD == 1 ? NPH : (KS == 1 ? 2 : 1);   // phases that issue DMA
  constexpr bool REG = SPREAD == 2;
  static_assert(PPW % LPH == 0, "pieces per phase");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  LDSP char* smem = (LDSP char*)smem_raw;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int nk = p.K / BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, q = w & 3;
  // wave tile origin in the block tile
  const int ar = KS == 1 ? grp * 128 : (q >> 1) * 128;
  const int bc = KS == 1 ? q * 64 : (q & 1) * 64;
  const int a_img = ar >> 7, b_img = bc >> 7, b_c0 = bc & 127;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto stage_part = [&](int slot, int kt, int part) {
    if (MODE == 2) return;
    LDSP char* st = smem + slot * STAGE;
    const int k0 = kt * BK;
#pragma unroll
    for (int u = 0; u < PPW / LPH; ++u) {
      const int ii = w * PPW + part * (PPW / LPH) + u, img = ii >> 4;
      if (img < AI)
        piece<AC>(p.A, p.lda, m0 + img * 128, p.M, k0, st + img * IMG, ii & 15, lane);
      else
        piece<BC>(p.B, p.ldb, n0 + (img - AI) * 128, p.N, k0, st + img * IMG, ii & 15, lane);
    }
  };

  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
  u32x4 stg[REG ? PPW : 1];
  auto src_of = [&](int kt, int ii) -> const uint16_t* {
    const int img = ii >> 4, pi = ii & 15, k0 = kt * BK;
    const bool col = img < AI ? AC : BC;
    const uint16_t* g = img < AI ? p.A : p.B;
    const int64_t ld = img < AI ? p.lda : p.ldb;
    const int x0 = img < AI ? m0 + img * 128 : n0 + (img - AI) * 128;
    const int xs = img < AI ? p.M : p.N;
    if (col) {
      const int kr = pi * 4 + (lane >> 4);
      const int c = (lane & 15) ^ swz_col(kr);
      int gc = x0 + c * 8;
      gc = gc <= xs - 8 ? gc : xs - 8;
      return g + (int64_t)(k0 + kr) * ld + gc;
    }
    const int r = pi * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int gr = x0 + r;
    gr = gr < xs ? gr : xs - 1;
    return g + (int64_t)gr * ld + k0 + c * 8;
  };
  auto reg_load = [&](int kt) {
#pragma unroll
    for (int u = 0; u < PPW; ++u) stg[u] = *(const u32x4*)src_of(kt, w * PPW + u);
  };
  auto reg_write = [&](int slot) {
    LDSP char* st = smem + slot * STAGE;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int ii = w * PPW + u;
      *(LDSP u32x4*)(st + (ii >> 4) * IMG + (ii & 15) * 1024 + lane * 16) = stg[u];
    }
  };

  // fragments: KS 1: a[ks][4] (one 64-row quadrant half), b[ks][2] (32 cols)
  //            KS 2: a[0][4], b[0][4] (k32 step = grp)
  bf16x8_t a[2][4], b[2][4];
  auto rdA = [&](int slot, int mq) {
    const LDSP char* img = smem + slot * STAGE + a_img * IMG;
#pragma unroll
    for (int s = 0; s < (KS == 1 ? 2 : 1); ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[s][i] = frag<AC>(img, (ar & 127) + mq * 64 + i * 16, KS == 1 ? s : grp, lane);
  };
  auto rdB = [&](int slot, int nq) {
    const LDSP char* img = smem + slot * STAGE + (AI + b_img) * IMG;
#pragma unroll
    for (int s = 0; s < (KS == 1 ? 2 : 1); ++s)
#pragma unroll
      for (int j = 0; j < (KS == 1 ? 2 : 4); ++j)
        b[s][j] = frag<BC>(img, b_c0 + (KS == 1 ? nq * 32 : 0) + j * 16, KS == 1 ? s : grp, lane);
  };
  auto mma = [&](int mq, int nq) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < (KS == 1 ? 2 : 1); ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < (KS == 1 ? 2 : 4); ++j) {
          f32x4_t& c = acc[mq * 4 + i][(KS == 1 ? nq * 2 : 0) + j];
          if (MODE == 3) asm volatile("" ::"v"(a[s][i]), "v"(b[s][j]));
          else c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[s][j], a[s][i], c, 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: tiles 0 .. NST-2 into their slots, wait for tile 0
  if (REG) {
    if (MODE != 2 && nk > 0) {
      reg_load(0);
      reg_write(0);
      if (nk > 1) reg_load(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
#pragma unroll
    for (int s0 = 0; s0 < NST - 1; ++s0)
      if (s0 < nk) {
#pragma unroll
        for (int part = 0; part < LPH; ++part) stage_part(s0, s0, part);
      }
    if (NST == 3 && nk > 1) vm_wait<PPW>();
    else vm_wait<0>();
  }
  bar();
  if (grp == 1) bar();                                  // group 1 runs one interval behind
  for (int kt = 0; kt < nk; ++kt) {
    const int slot = MODE == 2 ? 0 : kt % NST;
    const bool more = kt + NST - 1 < nk;            // tile kt+NST-1 to stage
    const bool ahead = kt + 2 < nk && NST == 3;     // tile kt+2 may stay in flight
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      // ---- read interval
      int mq, nq;
      if (KS == 1) {
        mq = (ph == 2 || ph == 3) ? 1 : 0;
        nq = (ph == 1 || ph == 2) ? 1 : 0;
        if (ph == 0) { rdB(slot, 0); rdA(slot, 0); }
        else if (ph == 1) rdB(slot, 1);
        else if (ph == 2) rdA(slot, 1);
        else rdB(slot, 0);
      } else {
        mq = ph;
        nq = 0;
        if (ph == 0) { rdB(slot, 0); rdA(slot, 0); }
        else rdA(slot, 1);
      }
      if (REG) {
        if (ph == 0 && MODE != 2) {
          if (kt + 1 < nk) reg_write((kt + 1) % NST);     // tile kt+1, loaded one tile ago
          if (kt + 2 < nk) reg_load(kt + 2);
        }
      } else if (ph < LPH && more) {
        stage_part((kt + NST - 1) % NST, kt + NST - 1, ph);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!REG && grp == 1 && ph == NPH - 1 && MODE != 2) {   // tile kt+1 landed (group 1's DMA)
        if (ahead) vm_wait<PPW>(); else vm_wait<0>();
      }
      bar();
      // ---- MFMA interval
      if (MODE != 1) mma(mq, nq);
      if (!REG && grp == 0 && ph == NPH - 1 && MODE != 2) {   // tile kt+1 landed (group 0's DMA)
        if (ahead) vm_wait<PPW>(); else vm_wait<0>();
      }
      bar();
    }
  }
  if (grp == 0) bar();                                  // balance group 1's extra barrier
  if constexpr (KS == 2) {
    // group 1's partial sums to LDS, group 0 adds them
    f32x4_t* red = (f32x4_t*)smem_raw;
    __syncthreads();
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[((q * 32) + i * 4 + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t o = red[((q * 32) + i * 4 + j) * 64 + lane];
        acc[i][j] += o;
      }
  }
  // epilogue (acc = C^T fragments: lane l reg r of (i,j) = C[16i + (l&15)][16j + 4(l>>4) + r])
  const int rho = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + ar + 16 * i + rho, n = n0 + bc + 16 * j + 4 * g;
      if (m < p.M && n + 3 < p.N) {
        uint2 u;
        u.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[i][j][0]) |
              ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[i][j][1]) << 16);
        u.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[i][j][2]) |
              ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[i][j][3]) << 16);
        *(uint2*)(p.C + (int64_t)m * p.ldc + n) = u;
      }
    }
}

template <int BN, int KS, int NST, bool AC, bool BC, int MODE, int SPREAD = 0>
float run(const P& p, int reps) {
  auto fn = gpp<BN, KS, NST, AC, BC, MODE, SPREAD>;
  constexpr int STAGE = (2 + BN / 128) * IMG;
  const int lds = std::max(KS == 2 ? 131072 : 0, NST * STAGE);
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int grid = ((p.M + 255) / 256) * ((p.N + BN - 1) / BN);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(512), lds, 0, p);
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(512), lds, 0, p);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1e3f / reps);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

template <int BN, int KS, int NST, bool AC, bool BC, int SPREAD = 0>
void variant(const char* shape, P p, float* R, bool check) {
  const double flop = 2.0 * p.M * p.N * p.K;
  const int reps = p.K >= 4096 && p.M * (double)p.N >= 8192.0 * 4096 ? 5 : 20;
  float t0 = run<BN, KS, NST, AC, BC, 0, SPREAD>(p, reps);
  double err = -1;
  if (check) {
    CK(hipMemset(p.C, 0, (size_t)p.M * p.ldc * 2));
    run<BN, KS, NST, AC, BC, 0, SPREAD>(p, 1);
    std::vector<uint16_t> c((size_t)p.M * p.ldc);
    std::vector<float> r((size_t)p.M * p.N);
    CK(hipMemcpy(c.data(), p.C, c.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), R, r.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, sc = 1e-6;
    for (int m = 0; m < p.M; ++m)
      for (int n = 0; n < p.N; ++n) {
        uint32_t u = (uint32_t)c[(size_t)m * p.ldc + n] << 16;
        float gv;
        memcpy(&gv, &u, 4);
        mx = std::max(mx, (double)std::fabs(gv - r[(size_t)m * p.N + n]));
        sc = std::max(sc, (double)std::fabs(r[(size_t)m * p.N + n]));
      }
    err = mx / sc;
  }
  float t1 = run<BN, KS, NST, AC, BC, 1, SPREAD>(p, reps);
  float t2 = run<BN, KS, NST, AC, BC, 2, SPREAD>(p, reps);
  printf("{\"shape\": \"%s\", \"MNK\": [%d, %d, %d], \"variant\": \"pp256x%d_ks%d_s%d_d%d\", "
         "\"full_us\": %.2f, \"TF\": %.0f, \"load_only_us\": %.2f, \"compute_only_us\": %.2f, "
         "\"compute_TF\": %.0f, \"rel_err\": %.2e}\n",
         shape, p.M, p.N, p.K, BN, KS, NST, SPREAD, t0, flop / t0 / 1e6, t1, t2, flop / t2 / 1e6, err);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const bool check = argc < 2 || std::string(argv[1]) != "nocheck";
  const size_t MAXE = (size_t)8192 * 8192;
  uint16_t *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, MAXE * 2));
  CK(hipMalloc(&B, MAXE * 2));
  CK(hipMalloc(&C, MAXE * 2));
  CK(hipMalloc(&R, MAXE * 4));
  {
    std::vector<uint16_t> h(MAXE);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& x : h) x = f2b(u(rng));
    CK(hipMemcpy(A, h.data(), MAXE * 2, hipMemcpyHostToDevice));
    for (auto& x : h) x = f2b(u(rng));
    CK(hipMemcpy(B, h.data(), MAXE * 2, hipMemcpyHostToDevice));
  }
  struct S {
    const char* name;
    int M, N, K, ac, bc;
  };
  std::vector<S> shapes = {
      {"sq8192", 8192, 8192, 8192, 0, 0}, {"sq4096", 4096, 4096, 4096, 0, 0},
      {"top1.fwd", 8192, 1024, 1024, 0, 0}, {"top0.fwd", 8192, 1024, 512, 0, 0},
      {"top2.fwd", 8192, 512, 1024, 0, 0},  {"top1.dgrad", 8192, 1024, 1024, 0, 1},
      {"dcnU.fwd", 8192, 3456, 512, 0, 0},  {"dcnV.fwd", 8192, 512, 3456, 0, 0},
      {"dcnT0.fwd", 8192, 1024, 3456, 0, 0},
  };
  for (auto& s : shapes) {
    P p{A, B, C, s.ac ? s.M : s.K, s.bc ? s.N : s.K, s.N, s.M, s.N, s.K};
    const bool ck = check && (double)s.M * s.N * s.K < 1e11;
    if (ck) {
      hipLaunchKernelGGL(ref_kernel, dim3((s.N + 255) / 256, s.M), dim3(256), 0, 0, p, s.ac, s.bc, R);
      CK(hipDeviceSynchronize());
    }
    if (s.bc) {
      variant<256, 1, 2, false, true, 2>(s.name, p, R, ck);
      variant<128, 2, 3, false, true, 0>(s.name, p, R, ck);
      variant<128, 2, 2, false, true, 2>(s.name, p, R, ck);
    } else {
      variant<256, 1, 2, false, false, 2>(s.name, p, R, ck);
      variant<128, 2, 3, false, false, 0>(s.name, p, R, ck);
      variant<128, 2, 2, false, false, 2>(s.name, p, R, ck);
    }
  }
  return 0;
}
