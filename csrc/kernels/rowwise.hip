// Row-wise (RW) sharded pooled embeddings: the fixed-capacity exchange that
// replaces TorchRec's RW input/output dist (reference call site: DMP sharding
// in torchrec/train.py:241-247). Every shape is
// static, so the whole exchange is hipGraph-capturable and no split sizes
// ever travel to the host:
//
//   requester  rw_bucketize : ids -> per-owner segments of a [W][cap+1]
//              int64 send buffer (slot cap holds the count), each entry
//              packing (bag key j*B+b) << 32 | owner-local row key; stable,
//              so every segment stays sorted by bag key. Rows are dealt
//              round-robin (owner = id mod W, local row = id div W), so a
//              hot head of low ids -- Zipf / frequency-ordered data --
//              spreads over every owner instead of landing on owner 0.
//   (RCCL)     all_to_all_single of the send buffer (equal splits)
//   owner      rw_pool      : per (requester, bag key) partial sum of the
//              rows it owns -> bf16 [W][B][nrw*D] (zeros where a bag has no
//              id here): the input of one RCCL reduce-scatter (bf16)
//   backward   all-gather of the [B][nrw*D] pooled gradients, then the
//              shared sort-based fused embedding backward, fed from the
//              received entries (embedding.hip: embedding_bwd_prepare_rw)
//
// The scan also records the largest per-owner count ("need"): the engine
// all-reduces it before the exchange and grows the capacity (re-bucketizing
// the batch) when a segment would overflow, so no lookup is ever dropped.
// Entries beyond a segment's capacity (only possible if that check is
// bypassed) raise a sticky device flag the engine checks on the host.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int RW_THREADS = 256;
constexpr int RW_CHUNK = 2048;                   // ids per block in bucketize
constexpr int RW_TILES = RW_CHUNK / RW_THREADS;

struct RwMeta {
  const int64_t* in_base; const int64_t* L; const int64_t* blk; const int64_t* lrow;
  const int64_t* cum;
};

__device__ __forceinline__ RwMeta rw_meta(const int64_t* m, int nrw) {
  return {m, m + nrw, m + 2 * nrw, m + 3 * nrw, m + 4 * nrw};
}

// table j of rw id q: last j with cum[j] <= q
__device__ __forceinline__ int rw_table(const RwMeta& M, int nrw, int64_t q) {
  int lo = 0, hi = nrw;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (M.cum[mid] <= q) lo = mid; else hi = mid;
  }
  return lo;
}

// owner and packed entry of rw id q
__device__ __forceinline__ int rw_route(const RwBucketArgs& a, const RwMeta& M, int64_t q,
                                        uint64_t& packed) {
  const int j = rw_table(M, a.nrw, q);
  const int64_t off = q - M.cum[j];
  const int64_t L = M.L[j];
  const int64_t b = off / L;
  const int64_t id = a.ids[M.in_base[j] + off];
  const int64_t o = id % a.W;
  const uint64_t row = (uint64_t)(M.lrow[j] + id / a.W);
  const uint64_t key = (uint64_t)j * (uint64_t)a.B + (uint64_t)b;
  packed = (key << 32) | (row & 0xffffffffull);
  return (int)o;
}

__global__ __launch_bounds__(RW_THREADS) void rw_hist_kernel(RwBucketArgs a, int32_t* hist) {
  __shared__ int32_t cnt[64];
  const RwMeta M = rw_meta(a.meta, a.nrw);
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RW_CHUNK;
  for (int t = 0; t < RW_TILES; ++t) {
    const int64_t q = base + t * RW_THREADS + threadIdx.x;
    if (q < a.n) {
      uint64_t pk;
      const int o = rw_route(a, M, q, pk);
      atomicAdd(&cnt[o], 1);                       // LDS integer atomic: order-free count
    }
  }
  __syncthreads();
  if (threadIdx.x < a.W) hist[(int64_t)blockIdx.x * a.W + threadIdx.x] = cnt[threadIdx.x];
}

// One block: per owner, exclusive scan of the chunk counts (in place) and the
// segment count into the send buffer's count slot; overflow is sticky.
__global__ __launch_bounds__(1024) void rw_scan_kernel(RwBucketArgs a, int32_t* hist, int nch) {
  __shared__ int32_t wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int32_t most = 0;
  for (int o = 0; o < a.W; ++o) {
    int32_t carry = 0;
    for (int c0 = 0; c0 < nch; c0 += 1024) {
      const int c = c0 + tid;
      const int32_t v = c < nch ? hist[(int64_t)c * a.W + o] : 0;
      int32_t incl = v;
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
      }
      if (lane == 63) wsum[w] = incl;
      __syncthreads();
      int32_t wbase = 0, tot = 0;
      for (int q = 0; q < 16; ++q) {
        if (q < w) wbase += wsum[q];
        tot += wsum[q];
      }
      if (c < nch) hist[(int64_t)c * a.W + o] = carry + wbase + incl - v;
      carry += tot;
      __syncthreads();
    }
    if (tid == 0) {
      a.send[(int64_t)o * (a.cap + 1) + a.cap] = carry < a.cap ? carry : a.cap;
      if (carry > a.cap) a.overflow[0] = 1;
      most = carry > most ? carry : most;
    }
  }
  if (tid == 0 && a.need) a.need[0] = most;
}

// Stable scatter: chunk order, then tile order, then wave order, then lane
// order -- i.e. exactly the input order inside every owner's segment.
__global__ __launch_bounds__(RW_THREADS) void rw_scatter_kernel(RwBucketArgs a,
                                                                const int32_t* hist) {
  __shared__ int32_t wcnt[RW_THREADS / 64][64];
  __shared__ int32_t run[64];
  const RwMeta M = rw_meta(a.meta, a.nrw);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 64) run[tid] = 0;
  int nbits = 1;
  while ((1 << nbits) < a.W + 1) ++nbits;          // owner ids + the "invalid" value W
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t base = (int64_t)blockIdx.x * RW_CHUNK;
  for (int t = 0; t < RW_TILES; ++t) {
    for (int i = tid; i < (RW_THREADS / 64) * 64; i += RW_THREADS) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const int64_t q = base + t * RW_THREADS + tid;
    uint64_t pk = 0;
    const int o = q < a.n ? rw_route(a, M, q, pk) : a.W;
    uint64_t peers = ~0ull;
    for (int b = 0; b < nbits; ++b) {
      const uint64_t bal = __ballot((o >> b) & 1);
      peers &= ((o >> b) & 1) ? bal : ~bal;
    }
    const int rank = __popcll(peers & lt);
    if (o < a.W && (peers & lt) == 0) wcnt[w][o] = __popcll(peers);
    __syncthreads();
    if (o < a.W) {
      int32_t pos = hist[(int64_t)blockIdx.x * a.W + o] + run[o] + rank;
      for (int q2 = 0; q2 < w; ++q2) pos += wcnt[q2][o];
      if (pos < a.cap) a.send[(int64_t)o * (a.cap + 1) + pos] = (int64_t)pk;
    }
    __syncthreads();
    if (tid < a.W) {
      int32_t s = 0;
      for (int q2 = 0; q2 < RW_THREADS / 64; ++q2) s += wcnt[q2][tid];
      run[tid] += s;
    }
    __syncthreads();
  }
}

// starts[r][k] = first entry of requester r's segment with bag key >= k
// (k in [0, K]; starts[r][K] = count): each entry writes the keys its gap
// covers, so every slot is written exactly once.
__global__ void rw_starts_kernel(RwPoolArgs a) {
  const int64_t K = (int64_t)a.nrw * a.B;
  const int64_t tot = (int64_t)a.W * (a.cap + 1);
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < tot;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(p / (a.cap + 1));
    const int64_t i = p - (int64_t)r * (a.cap + 1);
    const int64_t* seg = a.recv + (int64_t)r * (a.cap + 1);
    int64_t cnt = seg[a.cap];
    if (cnt > a.cap) cnt = a.cap;
    if (i > cnt) continue;
    const int64_t ki = i < cnt ? (int64_t)((uint64_t)seg[i] >> 32) : K;
    const int64_t kp = i > 0 ? (int64_t)((uint64_t)seg[i - 1] >> 32) : -1;
    int32_t* st = a.starts + (int64_t)r * (K + 1);
    for (int64_t k = kp + 1; k <= ki && k <= K; ++k) st[k] = (int32_t)i;
  }
}

// One lane group (D/4 lanes, 16-B row loads) per (requester, bag key) slot:
// sum of the owned rows of that bag, written bf16 (zeros if none).
template <int D>
__global__ __launch_bounds__(256) void rw_pool_kernel(RwPoolArgs a) {
  constexpr int LPB = (D / 4) < 64 ? (D / 4) : 64;
  constexpr int BPW = 64 / LPB;
  const RwMeta M = rw_meta(a.meta, a.nrw);
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPB, sl = lane - sub * LPB;
  const int64_t K = (int64_t)a.nrw * a.B;
  const int64_t nslots = (int64_t)a.W * K;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave0 * BPW + sub; s < nslots; s += nwaves * BPW) {
    const int r = (int)(s / K);
    const int64_t k = s - (int64_t)r * K;
    const int j = (int)(k / a.B);
    const int64_t b = k - (int64_t)j * a.B;
    const int32_t* st = a.starts + (int64_t)r * (K + 1);
    const int64_t s0 = st[k], s1 = st[k + 1];
    const int64_t* seg = a.recv + (int64_t)r * (a.cap + 1);
    const float sc = a.mean ? 1.f / (float)M.L[j] : 1.f;
    for (int c = sl * 4; c < D; c += LPB * 4) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int64_t p = s0;
      for (; p + 2 <= s1; p += 2) {
        const uint32_t r0 = (uint32_t)seg[p], r1 = (uint32_t)seg[p + 1];
        const float4 v0 = *(const float4*)(a.Wt + (int64_t)r0 * D + c);
        const float4 v1 = *(const float4*)(a.Wt + (int64_t)r1 * D + c);
        acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
        acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
      }
      if (p < s1) {
        const uint32_t r0 = (uint32_t)seg[p];
        const float4 v0 = *(const float4*)(a.Wt + (int64_t)r0 * D + c);
        acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
      }
      const int64_t o = ((int64_t)r * a.B + b) * a.out_ld + (int64_t)j * D + c;
      if (a.out_f32)
        *(float4*)((float*)a.out + o) = make_float4(acc.x * sc, acc.y * sc, acc.z * sc, acc.w * sc);
      else
        *(uint2*)((uint16_t*)a.out + o) = make_uint2(pack2bf(acc.x * sc, acc.y * sc),
                                                     pack2bf(acc.z * sc, acc.w * sc));
    }
  }
}

// ---- one-hot row-wise tables: the looked-up rows travel instead of pooled
// partials. With one id per bag the [W][B][nrw*D] partials of the pooled
// exchange are (W-1)/W zeros; returning each received entry's row in the
// layout of the id exchange moves ~W/1.25 x fewer bytes each way
// (config 3, W = 8: 21 vs 134 MB per direction per rank) and gives the same
// bf16 values (x + 0 + ... + 0 in the reduce-scatter is x).
//   owner      rw_rows_gather : rows[r][i] = bf16 W[row of entry (r, i)]
//   (RCCL)     all_to_all of rows (equal splits, [W][cap+1][D])
//   requester  rw_rows_scatter: pooled[b][j*D..] = received row of its slot
//              (o, i) (from its own send entry), and map[o][i] = that offset,
//              map[o][cap] = count -- the backward's gather map, so the
//              send buffer may be re-bucketized for the next batch meanwhile
//   backward   rw_grads_gather: g[o][i] = d_pooled[map[o][i]..] (requester),
//              all_to_all, and the owner's keys read entry (r, i)'s gradient
//              at (r*(cap+1) + i)*D (embedding_bwd_prepare_rw, rows = 1)
// One lane group of D/4 lanes per slot, 16-B fp32 / 8-B bf16 accesses.
template <int D>
__global__ __launch_bounds__(256) void rw_rows_gather_kernel(const float* __restrict__ Wt,
                                                             const int64_t* __restrict__ recv,
                                                             int W, int64_t cap,
                                                             uint16_t* __restrict__ out) {
  constexpr int LPR = (D / 4) < 64 ? (D / 4) : 64;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, sl = lane - sub * LPR;
  const int64_t nslots = (int64_t)W * (cap + 1);
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave0 * RPW + sub; s < nslots; s += nwaves * RPW) {
    const int r = (int)(s / (cap + 1));
    const int64_t i = s - (int64_t)r * (cap + 1);
    int64_t cnt = recv[(int64_t)r * (cap + 1) + cap];
    if (cnt > cap) cnt = cap;
    if (i >= cnt) continue;                  // padding / count slot: never read
    const uint32_t row = (uint32_t)recv[s];
    for (int c = sl * 4; c < D; c += LPR * 4) {
      const float4 v = *(const float4*)(Wt + (int64_t)row * D + c);
      *(uint2*)(out + s * D + c) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void rw_rows_scatter_kernel(const int64_t* __restrict__ send,
                                                              int W, int64_t cap, int B,
                                                              const uint16_t* __restrict__ rows,
                                                              uint16_t* __restrict__ region,
                                                              int64_t ld, int32_t* __restrict__ map) {
  constexpr int LPR = (D / 4) < 64 ? (D / 4) : 64;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, sl = lane - sub * LPR;
  const int64_t nslots = (int64_t)W * (cap + 1);
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave0 * RPW + sub; s < nslots; s += nwaves * RPW) {
    const int o = (int)(s / (cap + 1));
    const int64_t i = s - (int64_t)o * (cap + 1);
    int64_t cnt = send[(int64_t)o * (cap + 1) + cap];
    if (cnt > cap) cnt = cap;
    if (i == cap) {
      if (sl == 0) map[s] = (int32_t)cnt;
      continue;
    }
    if (i >= cnt) continue;
    const uint64_t k = (uint64_t)send[s] >> 32;
    const int64_t j = (int64_t)(k / (uint64_t)B), b = (int64_t)(k % (uint64_t)B);
    const int64_t off = b * ld + j * D;
    if (sl == 0) map[s] = (int32_t)off;
    for (int c = sl * 4; c < D; c += LPR * 4)
      *(uint2*)(region + off + c) = *(const uint2*)(rows + s * D + c);
  }
}

template <int D>
__global__ __launch_bounds__(256) void rw_grads_gather_kernel(const int32_t* __restrict__ map,
                                                              int W, int64_t cap,
                                                              const uint16_t* __restrict__ dregion,
                                                              uint16_t* __restrict__ gsend) {
  constexpr int LPR = (D / 4) < 64 ? (D / 4) : 64;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, sl = lane - sub * LPR;
  const int64_t nslots = (int64_t)W * (cap + 1);
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave0 * RPW + sub; s < nslots; s += nwaves * RPW) {
    const int o = (int)(s / (cap + 1));
    const int64_t i = s - (int64_t)o * (cap + 1);
    if (i >= (int64_t)map[(int64_t)o * (cap + 1) + cap]) continue;
    const int64_t off = map[s];
    for (int c = sl * 4; c < D; c += LPR * 4)
      *(uint2*)(gsend + s * D + c) = *(const uint2*)(dregion + off + c);
  }
}

int64_t rows_blocks(int64_t nslots, int D) {
  const int lpr = D / 4 < 64 ? D / 4 : 64;
  int64_t b = (nslots * lpr + 255) / 256;
  if (b > 8192) b = 8192;
  return b < 1 ? 1 : b;
}

}  // namespace

void rw_rows_gather(const float* Wt, int D, const int64_t* recv, int W, int64_t cap,
                    uint16_t* out, hipStream_t s) {
  const int64_t blocks = rows_blocks((int64_t)W * (cap + 1), D);
  switch (D) {
    case 16: hipLaunchKernelGGL(rw_rows_gather_kernel<16>, dim3(blocks), dim3(256), 0, s, Wt, recv, W, cap, out); break;
    case 32: hipLaunchKernelGGL(rw_rows_gather_kernel<32>, dim3(blocks), dim3(256), 0, s, Wt, recv, W, cap, out); break;
    case 64: hipLaunchKernelGGL(rw_rows_gather_kernel<64>, dim3(blocks), dim3(256), 0, s, Wt, recv, W, cap, out); break;
    case 128: hipLaunchKernelGGL(rw_rows_gather_kernel<128>, dim3(blocks), dim3(256), 0, s, Wt, recv, W, cap, out); break;
    case 256: hipLaunchKernelGGL(rw_rows_gather_kernel<256>, dim3(blocks), dim3(256), 0, s, Wt, recv, W, cap, out); break;
    default: throw std::runtime_error("rw_rows_gather: unsupported D");
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

void rw_rows_scatter(const int64_t* send, int W, int64_t cap, int B, int D, const uint16_t* rows,
                     uint16_t* region, int64_t ld, int32_t* map, hipStream_t s) {
  const int64_t blocks = rows_blocks((int64_t)W * (cap + 1), D);
  switch (D) {
    case 16: hipLaunchKernelGGL(rw_rows_scatter_kernel<16>, dim3(blocks), dim3(256), 0, s, send, W, cap, B, rows, region, ld, map); break;
    case 32: hipLaunchKernelGGL(rw_rows_scatter_kernel<32>, dim3(blocks), dim3(256), 0, s, send, W, cap, B, rows, region, ld, map); break;
    case 64: hipLaunchKernelGGL(rw_rows_scatter_kernel<64>, dim3(blocks), dim3(256), 0, s, send, W, cap, B, rows, region, ld, map); break;
    case 128: hipLaunchKernelGGL(rw_rows_scatter_kernel<128>, dim3(blocks), dim3(256), 0, s, send, W, cap, B, rows, region, ld, map); break;
    case 256: hipLaunchKernelGGL(rw_rows_scatter_kernel<256>, dim3(blocks), dim3(256), 0, s, send, W, cap, B, rows, region, ld, map); break;
    default: throw std::runtime_error("rw_rows_scatter: unsupported D");
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

void rw_grads_gather(const int32_t* map, int W, int64_t cap, int D, const uint16_t* dregion,
                     uint16_t* gsend, hipStream_t s) {
  const int64_t blocks = rows_blocks((int64_t)W * (cap + 1), D);
  switch (D) {
    case 16: hipLaunchKernelGGL(rw_grads_gather_kernel<16>, dim3(blocks), dim3(256), 0, s, map, W, cap, dregion, gsend); break;
    case 32: hipLaunchKernelGGL(rw_grads_gather_kernel<32>, dim3(blocks), dim3(256), 0, s, map, W, cap, dregion, gsend); break;
    case 64: hipLaunchKernelGGL(rw_grads_gather_kernel<64>, dim3(blocks), dim3(256), 0, s, map, W, cap, dregion, gsend); break;
    case 128: hipLaunchKernelGGL(rw_grads_gather_kernel<128>, dim3(blocks), dim3(256), 0, s, map, W, cap, dregion, gsend); break;
    case 256: hipLaunchKernelGGL(rw_grads_gather_kernel<256>, dim3(blocks), dim3(256), 0, s, map, W, cap, dregion, gsend); break;
    default: throw std::runtime_error("rw_grads_gather: unsupported D");
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

size_t rw_bucketize_workspace(int64_t n, int W) {
  const int64_t nch = (n + RW_CHUNK - 1) / RW_CHUNK;
  return (size_t)(nch < 1 ? 1 : nch) * W * sizeof(int32_t);
}

void rw_bucketize(const RwBucketArgs& a, void* ws, hipStream_t s) {
  if (a.W > 64) throw std::runtime_error("rw_bucketize: world size > 64");
  int32_t* hist = (int32_t*)ws;
  const int nch = (int)((a.n + RW_CHUNK - 1) / RW_CHUNK);
  if (nch == 0) {
    // no ids: every segment is empty
    hipLaunchKernelGGL(rw_scan_kernel, dim3(1), dim3(1024), 0, s, a, hist, 0);
    TDFO_CHECK_HIP(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(rw_hist_kernel, dim3(nch), dim3(RW_THREADS), 0, s, a, hist);
  TDFO_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(rw_scan_kernel, dim3(1), dim3(1024), 0, s, a, hist, nch);
  TDFO_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(rw_scatter_kernel, dim3(nch), dim3(RW_THREADS), 0, s, a, hist);
  TDFO_CHECK_HIP(hipGetLastError());
}

void rw_pool(const RwPoolArgs& a, hipStream_t s) {
  const int64_t tot = (int64_t)a.W * (a.cap + 1);
  int64_t sb = (tot + 255) / 256;
  if (sb > 4096) sb = 4096;
  hipLaunchKernelGGL(rw_starts_kernel, dim3(sb), dim3(256), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
  const int64_t nslots = (int64_t)a.W * a.nrw * a.B;
  const int lpb = a.D / 4 < 64 ? a.D / 4 : 64;
  int64_t blocks = (nslots * lpb + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return;
  switch (a.D) {
    case 16: hipLaunchKernelGGL(rw_pool_kernel<16>, dim3(blocks), dim3(256), 0, s, a); break;
    case 32: hipLaunchKernelGGL(rw_pool_kernel<32>, dim3(blocks), dim3(256), 0, s, a); break;
    case 64: hipLaunchKernelGGL(rw_pool_kernel<64>, dim3(blocks), dim3(256), 0, s, a); break;
    case 128: hipLaunchKernelGGL(rw_pool_kernel<128>, dim3(blocks), dim3(256), 0, s, a); break;
    case 256: hipLaunchKernelGGL(rw_pool_kernel<256>, dim3(blocks), dim3(256), 0, s, a); break;
    default: throw std::runtime_error("rw_pool: unsupported D");
  }
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
