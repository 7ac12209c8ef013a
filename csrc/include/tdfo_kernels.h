// Host-side launcher API of the tdfo_amd HIP kernels. Included by the torch
// bindings (csrc/bindings.cpp) and implemented in csrc/kernels/*.hip. Nothing
// here depends on torch, so kernel files compile in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdfo {

// ---------------------------------------------------------------- GEMM ----
// C[M,N] = op(A) * op(B), bf16 inputs, fp32 MFMA accumulation.
//   a_col == 0: A stored [M][K] (K contiguous, row stride lda)
//   a_col == 1: A stored [K][M] (M contiguous, row stride lda)
//   b_col == 0: B stored [N][K] (i.e. torch Linear weight layout)
//   b_col == 1: B stored [K][N]
// Epilogue (in order): +bias[n] (fp32), relu, *= (mask[m,n] > 0), then store
// bf16 C and/or fp32 C32 (C32 + z*M*ldc32 for split-K slice z).
struct GemmArgs {
  const uint16_t* A; int64_t lda; int a_col;
  const uint16_t* B; int64_t ldb; int b_col;
  int M, N, K, splits;
  const float* bias; int64_t bias_stride;   // bias[n * bias_stride]
  int relu;
  const uint16_t* mask; int64_t ldm;
  uint16_t* C; int64_t ldc;
  float* C32; int64_t ldc32;
  // optional second output C2 = (mul ? mul * v : v) + (add ? add : 0), used by
  // the DCN-v2 cross layer (x0 * (U h + b) + x_l) and residual dgrads.
  const uint16_t* mul; int64_t ldmul;
  const uint16_t* add; int64_t ldadd;
  uint16_t* C2; int64_t ldc2;
  // csum_on (col-layout A, fp32 C32 output): each split also writes the sum
  // over its K range of A's column m (= sum_k A[k][m]) into C32 row m, column
  // csum_col (>= N, so the GEMM tile never writes it). The weight-grad GEMM
  // uses it for the bias gradient (sum over the batch of dy), which lets the
  // GEMM's N stay at the 128-aligned input width.
  int csum_on, csum_col;
};
void gemm_bf16(const GemmArgs& a, hipStream_t s);


// Launch n independent GEMMs in order; consecutive (weight grad, dgrad)
// pairs on the small-tile kernel share one paired launch (gemm_pairing(0):
// never). Returns after enqueueing.
void gemm_group(const GemmArgs* a, int n, hipStream_t s);
int gemm_pairing(int v);
// Kernel policy for gemm_bf16 (0 auto; 1 2-stage 64/128-row tiles, 2 deep
// 4-slot ring, 3 ping-pong: forced, for tests / A/B); p < 0 just reads it.
// Returns the previous policy.
int gemm_policy(int p);

// ------------------------------------------------------ interaction ----
// DLRM dot interaction over F <= 32 features of width D (one of 16/32/64/128).
// Feature 0 comes from `dense` ([B, ld_dense]); feature f >= 1 from
// emb + off[f] + b * stride[f] (element units). Output row b of `out`
// ([B, ldo]) = [dense_b (D) | tril(X X^T, -1) (F(F-1)/2) | 0 ...].
struct SlotMap { int64_t off[32]; int64_t stride[32]; };
void interaction_fwd(const uint16_t* dense, int64_t ld_dense,
                     const uint16_t* emb, const SlotMap& slots, int F, int D,
                     int B, uint16_t* out, int64_t ldo, int ones_col, hipStream_t s);
// Backward: dZ [B, ldz] -> d_emb (same slot layout as forward emb) and
// d_dense = (passthrough + interaction grad) * (dense > 0 if relu_mask).
void interaction_bwd(const uint16_t* dz, int64_t ldz, const uint16_t* dense,
                     int64_t ld_dense, const uint16_t* emb,
                     const SlotMap& slots, int F, int D, int B,
                     uint16_t* d_dense, int64_t ld_ddense, uint16_t* d_emb,
                     const SlotMap& dslots, int relu_mask, hipStream_t s);

// ------------------------------------------------------ elementwise ----
// out[b, f*D + d] = f == 0 ? dense[b, d] : emb[off[f] + b*stride[f] + d]
void concat_features(const uint16_t* dense, int64_t ld_dense, const uint16_t* emb,
                     const SlotMap& slots, int F, int D, int B, uint16_t* out,
                     hipStream_t s);
// inverse of concat_features; the dense slot is multiplied by (dense > 0)
// when relu_mask (ReLU of the bottom MLP's last layer). Row b of dx starts at
// dx + b * ld_dx (F * D when packed).
void split_features(const uint16_t* dx, int64_t ld_dx, int F, int D, int B,
                    const uint16_t* dense, int64_t ld_dense, uint16_t* d_dense,
                    int64_t ld_ddense, uint16_t* d_emb, const SlotMap& dslots, int relu_mask,
                    hipStream_t s);
// DCN-v2 cross backward: dy = dout * x0 ;
// dx0 = (accumulate ? dx0 : 0) + dout * y + (add_dout ? dout : 0)
void cross_bwd(const uint16_t* dout, const uint16_t* x0, const uint16_t* y, int64_t n,
               uint16_t* dy, uint16_t* dx0, int accumulate, int add_dout, hipStream_t s);

// ------------------------------------------------------ radix sort ----
// Stable LSD radix sort of (key, value) pairs on the low `key_bits` bits.
// ka/va hold the input; kb/vb are scratch of the same size. Returns 1 if the
// sorted result ended in (kb, vb), 0 if in (ka, va). ws: radix_sort_workspace(n).
size_t radix_sort_workspace(int64_t n);
// digit bits per radix pass (4..10); returns the previous value (b < 4: read only)
int radix_sort_max_bits(int b);
// number of digit passes for key_bits at n keys (odd: the sorted result lands
// in (kb, vb))
int radix_sort_passes(int key_bits, int64_t n);
// 0: 1024-item tiles / 10-bit digits, 1: 4096-item tiles / <=8-bit digits
// from 2^19 keys up (default), 2: always 4096-item tiles; returns the old mode
int radix_sort_tiled(int v);
// 1: per-pass hist kernels, 0: next-pass hist counted by the scatter (atomics)
int radix_sort_sep_hist(int v);
int radix_sort_pairs_u32(uint32_t* ka, int32_t* va, uint32_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s);
int radix_sort_pairs_u64(uint64_t* ka, int32_t* va, uint64_t* kb, int32_t* vb, int64_t n,
                         int key_bits, void* ws, hipStream_t s);

// -------------------------------------------------------- embedding ----
// Table-batched pooled lookup. Bag j = t*B + b (t table, b sample) owns
// indices[offsets[j] .. offsets[j+1]); table t's rows start at
// row_offset[t] in the fused weight buffer W ([rows, D] fp32).
// out + b*out_stride + out_off[t] gets the pooled (sum or mean) row.
// step counters (fp32 or int64 scalars) each advanced by one
struct BumpArgs {
  void* p[8];
  int is_i64[8];
  int n;
};

struct EmbFwdArgs {
  const float* W; int D;
  const int64_t* row_offset;   // [T] (device)
  const int64_t* indices;      // [nnz] (device)
  const int64_t* offsets;      // [T*B+1] (device)
  const int64_t* out_off;      // [T] (device) element offsets
  const float* psw;            // per-sample weights [nnz] or null
  int T, B, mean;
  int64_t out_stride;
  void* out; int out_bf16;
  int onehot;                  // caller's promise: offsets[j] == j (one id per bag)
  // optional: step counters bumped by block 0 (a step's first launch takes
  // the bump launch along; nothing in the lookup reads them)
  BumpArgs bumps{};
};
void embedding_bag_fwd(const EmbFwdArgs& a, hipStream_t s);

// Fused backward + optimizer (no float atomics, deterministic):
//   1. keys = row_offset[t] + index, vals = bag id; radix sort by key;
//   2. fixed-size chunks of the sorted list segment-reduce grads (fp32);
//   3. rows whose run crosses a chunk edge are combined in chunk order;
//   4. the optimizer is applied once per unique row.
enum EmbOpt { EMB_SGD = 0, EMB_ROWWISE_ADAGRAD = 1, EMB_ADAM = 2,
              EMB_ADAGRAD = 3, EMB_DENSE_GRAD = 4 };
struct HeadBumps { float* p[4]; int n; };

// ------------------------------------------------------- two-tower ----
// Fused TwoTower step (two_tower.hip). X: [B, ldx] fp32 with the user
// embedding at cols [0,16) and the 98-wide item-tower input at [16,114).
// P: 2400 flat params. train=1 also writes dX (embedding grads, cols [0,112))
// and part[block][TT_PART_LD] = [dP (2400) | loss_sum].
constexpr int TT_NPARAM = 2400;
constexpr int TT_PART_LD = 2432;
struct TwoTowerArgs {
  const float* X; int64_t ldx;
  const float* P;
  const float* labels; float inv_n;
  const float* loss_scale;  // device scalar multiplying dlogit (dynamic loss scaling) or null
  int half;                 // fp16 compute: inputs, weights, activations and gradients
                            // rounded to fp16 at every layer boundary, fp32 accumulation
  int B;
  float* logits;
  float* dX; int64_t lddx;
  float* part;
  // optional (train): step counters bumped by block 0 (no bump launch)
  HeadBumps bumps{};
  // optional: the 7 embedding rows of every sample gathered here from the
  // table (emb_w [rows, 16] fp32, ids table-major ids[t * B + s], row_off[t])
  // instead of read from X[:, :112] -- the lookup launch folded in; X then
  // supplies only the two dense features (columns 112, 113)
  const float* emb_w = nullptr; const int64_t* ids = nullptr; const int64_t* row_off = nullptr;
};

// reduce_adam's arguments (declared with it below, in the loss section)
constexpr int REDUCE_ADAM_MAX_NB = 512;
struct ReduceAdamArgs {
  const float* part; int nparts; int n; int ld;
  float* grad; float* p; float* m; float* v;
  const float* hyper; float beta1, beta2, eps, wd; int adamw;
  double* loss_acc;
  const float* logits = nullptr; const float* labels = nullptr; int nlog = 0; int nb = 0;
  unsigned long long* hist = nullptr;
};

struct EmbBwdArgs {
  float* W; int D;
  const int64_t* row_offset; const int64_t* indices; const int64_t* offsets;
  const int64_t* grad_off;     // [T] element offsets into grad
  const float* psw;
  int T, B, mean; int64_t nnz; int key_bits;
  const void* grad; int grad_bf16; int64_t grad_stride;
  int opt;
  float* state1; float* state2;  // rowwise: state1[rows]; adam: m, v [rows, D]
  const float* hyper;          // device: [lr, step (, grad scale (, skip flag))]
  int hyper_n;                 // elements in hyper: > 2 -> grads x hyper[2] (loss-scale
                               // unscale), > 3 -> no update at all if hyper[3] > 0
  float eps, beta1, beta2, weight_decay;
  float* dense_grad;           // EMB_DENSE_GRAD: accumulate into [rows, D]
  void* workspace; size_t workspace_bytes;
  // one id per bag and T = R runs x Tp physical tables (virtual table v =
  // run * Tp + table, runs of a table share its rows): per-table LDS sorts
  // (+ a run merge when R > 1) replace the radix sort. 0: not applicable.
  int segsort;
  int goff_sorted;             // internal: grad offsets stored in sorted order
  // optional: every bag of virtual table v holds exactly bag_len[v] ids
  // (offsets[v*B + b] = offsets[v*B] + b*bag_len[v]; fixed multi-hot): the
  // keys pass finds a position's bag by division instead of a binary search
  // over all T*B bag offsets
  const int32_t* bag_len;
  // optional side job (side_on): a reduce_adam run by extra blocks of the
  // one-hot per-table sort launch, beside the sort (it needs nothing the
  // backward touches) -- or, when that launch carries the towers whose
  // partials it reads (tower_on), by extra blocks of the update launch (the
  // in-kernel-combine variant); run as its own launch where neither can.
  // TwoTower: the dense step hidden behind the sort / update.
  ReduceAdamArgs side{};
  int side_on = 0;
  // optional co-launched tower step (tower_on): the fused TwoTower
  // forward + backward run by extra blocks of the per-table sort launch
  // (one-hot, <= 2048 ids per table), else as its own launch before the sort
  TwoTowerArgs tower{};
  int tower_on = 0;
  int side_block0 = 0;         // internal: first side block of the update launch
};
size_t embedding_bwd_workspace(int64_t nnz, int D);
// One-hot batches (nnz == T*B, B <= 8192): per-table LDS sort in one launch
// (1, default) or the device-wide radix sort (0); v < 0 queries. Returns the
// previous setting.
int embedding_segsort(int v);
void embedding_bwd_fused(const EmbBwdArgs& a, hipStream_t s);
// The same in two halves around a workspace that persists between them:
// prepare needs only the ids (keys, sort, gradient offsets) and can run on a
// side stream while the dense forward/backward computes; apply does the
// segment reduction + optimizer once the gradient exists.
void embedding_bwd_prepare(const EmbBwdArgs& a, hipStream_t s);
void embedding_bwd_apply(const EmbBwdArgs& a, hipStream_t s);

// Dense optimizer step over rows [0, rows) of W from a dense fp32 gradient
// [rows, D] (a.opt, a.state1/2, a.hyper, eps/betas/wd as for the backward).
// clear: null, or grad itself (each row zeroed once read)
void embedding_dense_update(const EmbBwdArgs& a, int64_t rows, const float* grad, float* clear,
                            hipStream_t s);

// --------------------------------------------------- synthetic data ----
// (synthetic.hip) One fresh synthetic Criteo batch (device twin of
// csrc/data/synthetic.cpp): dense [B, num_dense] fp32, ids table-major (table
// t at base[t], B * pooling[t] ids; dist 0 uniform, 1 Zipf(alpha)), label [B].
// rows / base int64[T], pooling int32[T], w_dense [num_dense], table_bias
// [T, 64] all device-resident.
struct SynthArgs {
  uint64_t seed; int rank; int64_t batch_index;
  int B, num_dense, T;
  const int64_t* rows; const int* pooling; const int64_t* base;
  int dist; double alpha;
  const float* w_dense; const float* table_bias;
  float* dense; int64_t* ids; float* label;
  // in-step generation (synth_ids / synth_dense): batch index = batch_index +
  // (int64) index_ptr[0] read on the device (a step counter), so a captured
  // graph draws a fresh batch every replay; synth_dense writes bf16 features
  // into x0 (row pitch ldx) instead of fp32 `dense`
  const float* index_ptr; uint16_t* x0; int64_t ldx;
};
void synth_criteo(const SynthArgs& a, hipStream_t s);
// the ids of synth_criteo's batch only (one thread per (table, sample))
void synth_ids(const SynthArgs& a, hipStream_t s);
// its dense features (-> bf16 x0) and labels only (one thread per sample)
void synth_dense(const SynthArgs& a, hipStream_t s);

// ------------------------------------------------ fused bottom MLP ----
// (mlp_fused.hip) The default DLRM bottom stack (K0 = 64 padded input with
// the bias inside K, 512 -> 256 -> 128, ReLU everywhere) in one launch:
// y_i = relu(y_{i-1} W_i^T + b_i), bf16 activations written to y0 / y1 / y2
// (row strides ldy*), weights [N][ldw] bf16 (the first K columns used),
// biases fp32 with element stride bs* (nullptr: inside K). Bitwise equal to
// the three per-layer GEMMs.
struct BotMlpArgs {
  const uint16_t* x; int64_t ldx;
  const uint16_t* w0; const uint16_t* w1; const uint16_t* w2;
  int64_t ldw0, ldw1, ldw2;
  const float* b0; const float* b1; const float* b2;
  int64_t bs0, bs1, bs2;
  uint16_t* y0; uint16_t* y1; uint16_t* y2;
  int64_t ldy0, ldy1, ldy2;
  int M;
  // optional batch load folded in (dense != nullptr): columns [0, nd) of the
  // input come from fp32 dense[M][ld_dense], converted as batch_load does and
  // written back to x (x_out, the same buffer: the backward's weight grad
  // reads it); each block also copies its rows' labels label_src -> label_dst
  const float* dense = nullptr; int64_t ld_dense = 0; int nd = 0;
  uint16_t* x_out = nullptr;
  const float* label_src = nullptr; float* label_dst = nullptr;
};
bool bottom_mlp_fwd_supported(int k0, int n0, int n1, int n2);
void bottom_mlp_fwd(const BotMlpArgs& a, hipStream_t s);

// --------------------------------------------------- row-wise shards ----
// (rowwise.hip) Fixed-capacity row-wise exchange. meta (int64, device):
// [in_base (nrw) | L (nrw) | blk (nrw) | lrow (nrw) | cum (nrw + 1)]:
// table j's ids start at ids[in_base[j]], L[j] ids per bag, owner(id) =
// id mod W, owner-local row key = lrow[j] + id div W (blk[j] = ceil(rows/W)
// rows per owner), cum = prefix of B*L[j]. Buffers are [W][cap + 1] int64;
// entry = (j*B + b) << 32 | row key; slot cap of segment o holds its count.
// need (optional): the largest per-owner count of this batch.
struct RwBucketArgs {
  const int64_t* ids; const int64_t* meta;
  int nrw, W, B; int64_t cap; int64_t n;      // n = cum[nrw] rw ids
  int64_t* send; int32_t* overflow; int32_t* need;
};
size_t rw_bucketize_workspace(int64_t n, int W);
void rw_bucketize(const RwBucketArgs& a, void* ws, hipStream_t s);
// Owner side: out (bf16, or fp32 if out_f32; row (r*B + b), column j*D, row
// stride out_ld) = pooled owned rows of requester r's bag (j, b); starts:
// [W][nrw*B + 1] int32.
struct RwPoolArgs {
  const float* Wt; int D; const int64_t* recv; const int64_t* meta;
  int nrw, W, B; int64_t cap; int mean;
  int32_t* starts; void* out; int out_f32; int64_t out_ld;
};
void rw_pool(const RwPoolArgs& a, hipStream_t s);
// One-hot row-wise tables ("rows" exchange, rowwise.hip): the owner's bf16
// rows per received entry ([W][cap+1][D]), the requester's scatter of the
// received rows into its pooled region (row stride ld) plus the slot -> offset
// map ([W][cap+1] int32, slot cap = count) its backward gathers the gradient
// rows with.
void rw_rows_gather(const float* Wt, int D, const int64_t* recv, int W, int64_t cap,
                    uint16_t* out, hipStream_t s);
void rw_rows_scatter(const int64_t* send, int W, int64_t cap, int B, int D, const uint16_t* rows,
                     uint16_t* region, int64_t ld, int32_t* map, hipStream_t s);
void rw_grads_gather(const int32_t* map, int W, int64_t cap, int D, const uint16_t* dregion,
                     uint16_t* gsend, hipStream_t s);
// Backward, owner side: keys/positions/gradient offsets of every received
// entry into the embedding workspace (entry (r, i) reads its gradient row at
// grad + (r*B + b)*grad_ld + j*D; empty slots update row `dummy_row`, a
// scratch row the store keeps past its real rows), then the radix sort.
// embedding_bwd_apply then runs with a.nnz = W*cap, a.segsort = 0.
// rows = 1 ("rows" exchange): entry (r, i) reads its gradient row at
// grad + (r*(cap+1) + i)*grad_ld instead.
void embedding_bwd_prepare_rw(const EmbBwdArgs& a, const int64_t* recv, const int64_t* meta,
                              int nrw, int W, int64_t cap, int64_t grad_ld, int64_t dummy_row,
                              int rows, hipStream_t s);

// ------------------------------------------------------------ optim ----
// Flat fused optimizer over one contiguous fp32 parameter buffer.
enum DenseOpt { OPT_ADAMW = 0, OPT_ADAM = 1, OPT_SGD = 2, OPT_ADAGRAD = 3 };
struct DenseOptArgs {
  float* p; const float* g; float* m; float* v; uint16_t* p_bf16;
  int64_t n; int opt;
  const float* hyper;   // device: [lr, step, grad_scale]
  float beta1, beta2, eps, weight_decay, momentum;
  const float* found_inf;  // optional device flag: skip update if > 0
  // optional gradient segments: elements [seg_start, +seg_len) take their
  // gradient as the sum of seg_splits slabs seg_ptr[s * seg_len + j] (the
  // split-K partials of a weight-grad GEMM) instead of g
  int nseg;
  int64_t seg_start[16], seg_len[16];
  int seg_splits[16];
  const float* seg_ptr[16];
};
void dense_optimizer(const DenseOptArgs& a, hipStream_t s);
// found_inf[0] = any(!isfinite(g)) over n (caller zeroes it first).
void check_finite(const float* g, int64_t n, float* found_inf, hipStream_t s);
void cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s);
// Batch inputs in one launch: ids copy, label copy, dense fp32 -> bf16 x0[:, :nd].
void batch_load(const float* dense, int nd, int64_t ld_dense, uint16_t* x0, int64_t ldx,
                const int64_t* ids, int64_t* ids_dst, int64_t n, const float* label,
                float* label_dst, int B, hipStream_t s);
// MFMA load on `blocks` 256-thread blocks for `ticks` of the 100 MHz clock
void burn_ticks(uint64_t ticks, int blocks, hipStream_t s);
void spin_ticks(uint64_t ticks, hipStream_t s);

void bump(const BumpArgs& a, hipStream_t s);
void stamp(uint64_t* buf, int64_t* cnt, int seg, int nseg, int which, int64_t cap,
           hipStream_t s);
// dst[chunk.dst_off + i] = src[chunk.src_off + i], i < chunk.len, for every
// chunk of the device table chunks[nchunks][3] (one block per chunk)
void seg_copy(const int64_t* src, int64_t* dst, const int64_t* chunks, int nchunks,
              hipStream_t s);
// pieces[p] = (src_off, src_ld, dst_off, dst_ld) (device, elements): B rows x w
// bf16 (w % 8 == 0, 16-B aligned rows) copied within buf, all pieces in one launch
void piece_copy_bf16(uint16_t* buf, const int64_t* pieces, int npieces, int B, int w,
                     hipStream_t s);
// host mailbox: host_word[slot] = (++seq[slot]) << 32 | (uint32) value[0]
void host_publish(const int32_t* value, int32_t* seq, uint64_t* host_word, hipStream_t s);

// ---------------------------------------------------- loss / reduce ----
// Fused last layer (K -> 1) + sigmoid BCE-with-logits + backward:
//   logit = H.w + b; loss partials; dlogit = (sigmoid(logit) - y) * inv_n
//   dH = dlogit * w * (H > 0 if relu_mask) ; partials of dw, db.
// part: [gridDim, K + 2] fp32 rows = [dw (K) | db | loss_sum].
void head_bce(const uint16_t* H, int64_t ldh, int B, int K, const float* w,
              const float* b, const float* label, float inv_n, int relu_mask,
              float* logits, uint16_t* dH, int64_t lddh, float* part,
              int nparts, hipStream_t s);
int head_bce_parts(int B);
// grad[0..K] = sum over parts of part[:, 0..K]; loss_acc[0] += sum part[:, K+1];
// bump.p[i][1] += 1 for each step counter (fp32 [lr, step, ...] hyper vectors;
// HeadBumps: above EmbBwdArgs).
void head_reduce(const float* part, int nparts, int K, float* grad, float* loss_acc,
                 const HeadBumps& bumps, hipStream_t s);
// The same, parked (one per thread): the next paired 128x128 GEMM launch --
// the first top-MLP backward pair, which needs nothing it writes -- runs it
// in extra blocks (head_reduce_take); head_reduce_flush launches it on its
// own if nothing took it.
struct HeadReduceJob {
  const float* part; int nparts; int K; float* grad; float* loss_acc; HeadBumps bumps;
};
void head_reduce_park(const HeadReduceJob& j);
bool head_reduce_take(HeadReduceJob* j);
void head_reduce_flush(hipStream_t s);
// grad[j] = sum_r part[r * ld + j] for j < n (head_reduce's / reduce_rows'
// fixed order) followed by one Adam / AdamW step of p[j] from it (hyper =
// [lr, step, grad_scale], adam_elem: the flat optimizer's bits); column n is
// the loss partial: loss_acc[0] += (double)sum. Optionally one more block
// bins logits[0..nlog) into hist ([2 * nb] int64, auc_hist's buckets).
// Replaces reduce_rows + the flat optimizer + the loss add + auc_hist of a
// small model's step (TwoTower). (ReduceAdamArgs: above EmbBwdArgs, which
// can carry one as a side job.)
void reduce_adam(const ReduceAdamArgs& a, hipStream_t s);
// out[j] (=|+=) sum_r in[r*ld + j], j < n, fixed order (deterministic).
// idx (optional): out[idx[j]] instead of out[j] (a gather-free scatter into
// a flat gradient buffer whose layout differs from the packed order)
void reduce_rows(const float* in, int rows, int64_t n, int64_t ld, float* out,
                 int accumulate, float scale, hipStream_t s, const int64_t* idx = nullptr);
// several fp32 split-K slab sets reduced in one launch: seg k sums S slabs of
// n floats (n % 4 == 0, 16-B aligned) into out; start[] = prefix of n / 4
struct SlabSeg { const float* in; float* out; int64_t n; int S; };
constexpr int SLAB_MAX_SEGS = 16;
struct SlabReduceArgs { SlabSeg seg[SLAB_MAX_SEGS]; int64_t start[SLAB_MAX_SEGS + 1]; int nseg; };
void slab_reduce(const SlabReduceArgs& a, hipStream_t s);
// out[n] = sum_m x[m, n] (bf16 in). part must hold parts(M)*N floats.
void colsum_bf16(const uint16_t* x, int M, int N, int64_t ldx, float* part,
                 int nparts, float* out, int accumulate, hipStream_t s);
int colsum_parts(int M);
// AUC histogram: hist[2*nb]: [neg counts | pos counts] of sigmoid(logit)
// bucketed uniformly on [0, 1] (tf.keras.metrics.AUC-style thresholds).
void auc_hist(const float* logits, const float* labels, int n, int nb,
              unsigned long long* hist, hipStream_t s);


int two_tower_parts(int B);
void two_tower(const TwoTowerArgs& a, int train, hipStream_t s);

// ----------------------------------------------------- linear + xent ----
// Fused Linear(16 -> V) + CrossEntropy(ignore_index, label_smoothing=eps),
// forward and backward without materialising logits (linear_xent.hip).
struct LinearXentArgs {
  const float* H;          // [N, 16]
  const float* W;          // [V, 16]
  const float* bias;       // [V]
  const int64_t* labels;   // [N]
  int N; int64_t V; int ignore; float eps;
  float* dH;               // [N, 16] (scaled by 1/n_valid)
  float* lossv;            // [N] per-token loss (0 for ignored)
  float* dW; float* db;    // optional [V, 16], [V]
  float* loss;             // optional scalar: sum(lossv) / max(1, n_valid)
  double* loss_acc;        // optional running sum: += loss (device, fp64)
  void* workspace;
  // optional fused optimizer step of the output layer (okind OPT_ADAM /
  // OPT_ADAMW; -1: none): W and bias updated in place from their gradient
  // inside the kernels (dW / db then serve as scratch), moments mW/vW [V,16],
  // mb/vb [V], ohyper = the flat optimizer's [lr, step, grad_scale]
  int okind = -1;
  float* mW = nullptr; float* vW = nullptr; float* mb = nullptr; float* vb = nullptr;
  const float* ohyper = nullptr;
  float beta1 = 0.9f, beta2 = 0.999f, oeps = 1e-8f, owd = 0.f;
};
size_t linear_xent_workspace(int N, int64_t V);
// 1: f32-input MFMA pass1/wgrad (default), 0: VALU kernels; <0 queries.
// Returns the previous setting.
int linear_xent_impl(int impl);
void linear_xent(const LinearXentArgs& a, hipStream_t s);

// -------------------------------------------------------- attention ----
// Fused small-T MHA core (attention.hip): qkv [B,T,3E] fp32 (q|k|v, each
// H x dk), key-padding mask from ids != pad_id, dropout(rate) from a counter
// hash of (seed, *step, b, h, i, j). out/dout [B,T,E], dqkv [B,T,3E].
struct AttnArgs {
  const float* qkv; const int64_t* ids;
  const float* dout; float* out; float* dqkv;
  int B, T, H, dk; float scale, rate; int64_t seed; const int64_t* step; int64_t pad_id;
};
void attention_fwd(const AttnArgs& a, hipStream_t s);
void attention_bwd(const AttnArgs& a, hipStream_t s);

// --------------------------------------------------- encoder layer ----
// Fused Bert4Rec transformer block (encoder.hip), fp32, one workgroup per
// sequence. x/y/dx [B,T,E]; saves qkv [B,T,3E], ctx [B,T,E], x1 [B,T,E],
// f [B,T,FF]; part [B][encoder_param_count(E, FF)].
// A parameter-gradient reduction grad[gidx ? gidx[c] : c] = sum_b part[b][c]
// (c < P, rows in order: deterministic) parked by encoder_layer_bwd(defer)
// and run by extra blocks of the next encoder-backward or sequence-prologue
// backward launch -- or flushed as its own launch (encoder_reduce_flush).
struct EncRedJob {
  const float* part = nullptr;
  int B = 0, P = 0;
  float* grad = nullptr;
  const int64_t* gidx = nullptr;
};
__device__ __forceinline__ void enc_red_col(const EncRedJob& j, int c) {
  if (c >= j.P) return;
  float s = 0.f;
#pragma unroll 16
  for (int b = 0; b < j.B; ++b) s += j.part[(int64_t)b * j.P + c];
  j.grad[j.gidx ? j.gidx[c] : c] = s;
}
// take the parked job (true) or nothing (false); flush: run it standalone
bool encoder_reduce_take(EncRedJob* j);
void encoder_reduce_flush(hipStream_t s);

struct EncArgs {
  int B, T, E, H, FF; float rate; int64_t seed; const int64_t* step; int64_t pad_id; float eps;
  const float* x; const int64_t* ids;
  const float *wqkv, *bqkv, *wo, *bo, *g1, *be1, *g2, *be2, *w1, *b1, *w2, *b2;
  // optional: K / V projection weights and biases as separate tensors (then
  // wqkv / bqkv point at Q's alone)
  const float *wk = nullptr, *wv = nullptr, *bk = nullptr, *bv = nullptr;
  float *y, *qkv, *ctx, *x1, *f;
  const float* dy; float* dx; float* part;
  EncRedJob red{};             // internal: a parked reduction run by extra blocks
  int red_on = 0;
};
int encoder_param_count(int E, int FF);
bool encoder_layer_supported(int T, int E, int H, int FF);
void encoder_layer_fwd(const EncArgs& a, hipStream_t s);
// grad: [encoder_param_count] = [dWqkv | dbqkv | dWo | dbo | dg1 | dbe1 | dg2 |
// dbe2 | dW1 | db1 | dW2 | db2]
// gidx (optional): parameter gradient c goes to grad[gidx[c]] (the trainer's
// flat gradient buffer) instead of grad[c]
// defer: park this layer's reduction for the next encoder / prologue
// backward launch instead of launching it (the caller keeps `part` alive and
// flushes before the gradient is read)
void encoder_layer_bwd(const EncArgs& a, float* grad, hipStream_t s,
                       const int64_t* gidx = nullptr, bool defer = false);

// ------------------------------------------------------ ranking (eval) ----
// Bert4Rec-style candidate ranking: per sample b, scores of candidates
// cand[b, 0..C) = h[b] . W[cand] + bias[cand] (candidate 0 = the positive),
// rank = #negatives scoring >= the positive; out[0..2nk] = sums over samples
// of [rank < k_i (i < nk) | (rank < k_i) / log2(rank + 2) | 1].
struct RankKs { int k[8]; };
int rank_metrics_parts(int B);
void rank_metrics(const float* h, const float* W, const float* bias, const int64_t* cand, int B,
                  int C, int E, const RankKs& ks, int nk, float* part, float* out,
                  hipStream_t s);

// ------------------------------------------------------- layernorm ----
// Row LayerNorm over the last n <= 1024 elements (layernorm.hip).
int layernorm_parts(int64_t M);
void layernorm_fwd(const float* x, int64_t M, int n, float eps, const float* gamma,
                   const float* beta, float* y, float* mean, float* rstd, hipStream_t s);
// part: layernorm_parts(M) * 2n floats; dgamma_dbeta: [2n] = [dgamma | dbeta]
void layernorm_bwd(const float* x, const float* g, int64_t M, int n, const float* gamma,
                   const float* mean, const float* rstd, float* dx, float* part,
                   float* dgamma_dbeta, hipStream_t s);
// Bert4Rec input block y = dropout(LN(x + pos)) (pos [n] broadcast over rows;
// counter-hash dropout keyed by seed ^ f(step[0]), regenerated in backward).
// bwd: dx, and [dgamma | dbeta | dpos] (3n) reduced over rows in fixed order;
// part: layernorm_parts(M) * 3n floats.
void seq_prologue_fwd(const float* x, const float* pos, int64_t M, int n, float eps,
                      const float* gamma, const float* beta, float rate, uint32_t seed,
                      const int64_t* step, float* y, float* mean, float* rstd, hipStream_t s);
void seq_prologue_bwd(const float* x, const float* pos, const float* g, int64_t M, int n,
                      const float* gamma, const float* mean, const float* rstd, float rate,
                      uint32_t seed, const int64_t* step, float* dx, float* part,
                      float* dgamma_dbeta_dpos, hipStream_t s,
                      const int64_t* idx = nullptr);

// ------------------------------------------------------ batch gather ----
// out_c[i * dst_stride_c] = convert(src_c[idx ? idx[i] : row0 + i]) for every
// column c < ncols and row i < n. src dtype codes: 0 i8, 1 i16, 2 i32, 3 i64,
// 4 f32; dst is int64 (dst_int) or fp32.
struct GatherColsArgs {
  const void* src[16]; int src_dtype[16];
  void* dst[16]; int dst_int[16]; int64_t dst_stride[16];
  int ncols; int64_t n; const int64_t* idx; int64_t row0;
};
void gather_columns(const GatherColsArgs& a, hipStream_t s);

// ----------------------------------------------------------- jagged ----
void jagged_to_dense(const float* values, const int64_t* off, int B, int T, int D, float pad,
                     float* out, hipStream_t s);
void dense_to_jagged(const float* dense, const int64_t* off, int B, int T, int D, int64_t nnz,
                     float* vgrad, hipStream_t s);
void jagged_ids_to_dense(const int64_t* values, const int64_t* off, int B, int T, int64_t pad,
                         int64_t* out, hipStream_t s);

}  // namespace tdfo
