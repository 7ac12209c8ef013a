// torch op registrations for the tdfo_amd HIP kernels (namespace torch.ops.tdfo).
//
// Every op is an out-variant: callers own all buffers, so the ops can be
// captured into a hipGraph (torch.cuda.CUDAGraph) and replayed without
// allocation. Shapes, dtypes, strides and alignment are validated on the host
// before any launch (a mis-shaped launch can fault the GPU).
#include <cmath>
#include <cstring>

#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include "tdfo_kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

const uint16_t* bf16_ptr(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "expected bf16 tensor");
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
uint16_t* bf16_mut(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "expected bf16 tensor");
  return reinterpret_cast<uint16_t*>(t.data_ptr());
}
void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_2d_rowmajor(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must have unit inner stride");
}
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ------------------------------------------------------------------ gemm
// GEMM batching (ops.gemm_batch): while on, gemm() validates and records its
// launch instead of enqueueing it; gemm_batch_end() enqueues the recorded
// launches in order through tdfo::gemm_group (pairs share one launch). The
// operand tensors are kept alive until then.
struct GemmBatch {
  bool on = false;
  std::vector<tdfo::GemmArgs> args;
  std::vector<Tensor> keep;
};
thread_local GemmBatch g_gemm_batch;

void gemm_batch_begin() {
  TORCH_CHECK(!g_gemm_batch.on, "gemm_batch: already open");
  g_gemm_batch.on = true;
}

void gemm_batch_end() {
  GemmBatch& b = g_gemm_batch;
  b.on = false;
  if (!b.args.empty()) tdfo::gemm_group(b.args.data(), (int)b.args.size(), cur_stream());
  b.args.clear();
  b.keep.clear();
}

void gemm(const Tensor& a_in, bool a_col, const Tensor& b_in, bool b_col,
          const c10::optional<Tensor>& bias, bool relu,
          const c10::optional<Tensor>& mask, const c10::optional<Tensor>& out,
          const c10::optional<Tensor>& out32, int64_t splits, const c10::optional<Tensor>& mul,
          const c10::optional<Tensor>& add, const c10::optional<Tensor>& out2, int64_t ldc32,
          int64_t csum_col) {
  check_dev(a_in, "a"); check_dev(b_in, "b");
  check_2d_rowmajor(a_in, "a"); check_2d_rowmajor(b_in, "b");
  const int64_t Ka = a_col ? a_in.size(0) : a_in.size(1);
  const int64_t Kb = b_col ? b_in.size(0) : b_in.size(1);
  TORCH_CHECK(Ka == Kb && Ka > 0, "gemm: K mismatch ", Ka, " vs ", Kb);
  // The kernel consumes whole 64-deep K tiles. A K tail (only tiny layers:
  // e.g. the dgrad of a 16- or 32-wide layer) is zero-padded here, once,
  // instead of predicating the hot loop.
  Tensor a = a_in, b = b_in;
  if (Ka % 64) {
    const int64_t Kp = (Ka + 63) / 64 * 64;
    auto pad = [&](const Tensor& t, bool col) {
      Tensor z = col ? at::zeros({Kp, t.size(1)}, t.options()) : at::zeros({t.size(0), Kp}, t.options());
      if (col) z.narrow(0, 0, Ka).copy_(t); else z.narrow(1, 0, Ka).copy_(t);
      return z;
    };
    a = pad(a_in, a_col);
    b = pad(b_in, b_col);
  }
  const int64_t M = a_col ? a.size(1) : a.size(0);
  const int64_t K = a_col ? a.size(0) : a.size(1);
  const int64_t N = b_col ? b.size(1) : b.size(0);
  TORCH_CHECK(M > 0 && N > 0, "gemm: empty output");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm: ld must be multiple of 8");
  TORCH_CHECK(aligned16(a.data_ptr()) && aligned16(b.data_ptr()), "gemm: operands must be 16-B aligned");
  if (a_col) TORCH_CHECK(M % 8 == 0 && M >= 8, "gemm: col-layout A needs M % 8 == 0");
  if (b_col) TORCH_CHECK(N % 8 == 0 && N >= 8, "gemm: col-layout B needs N % 8 == 0");
  TORCH_CHECK(splits >= 1 && splits <= K / 64, "gemm: bad split count");
  tdfo::GemmArgs g{};
  g.A = bf16_ptr(a); g.lda = a.stride(0); g.a_col = a_col;
  g.B = bf16_ptr(b); g.ldb = b.stride(0); g.b_col = b_col;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.splits = (int)splits;
  if (bias) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->dim() == 1 && bias->numel() == N,
                "gemm: bias must be fp32 [N] (any stride)");
    g.bias = bias->data_ptr<float>(); g.bias_stride = bias->stride(0);
  }
  g.relu = relu;
  if (mask) {
    check_2d_rowmajor(*mask, "mask");
    TORCH_CHECK(mask->size(0) == M && mask->size(1) == N, "gemm: mask shape");
    g.mask = bf16_ptr(*mask); g.ldm = mask->stride(0);
  }
  TORCH_CHECK(out || out32 || out2, "gemm: need an output");
  if (out) {
    check_2d_rowmajor(*out, "out");
    TORCH_CHECK(out->size(0) == M && out->size(1) == N, "gemm: out shape");
    g.C = bf16_mut(*out); g.ldc = out->stride(0);
    TORCH_CHECK(splits == 1, "gemm: bf16 output requires splits == 1");
  }
  if (out32) {
    TORCH_CHECK(out32->scalar_type() == at::kFloat && out32->is_contiguous(), "gemm: out32 fp32 contiguous");
    // ldc32: row pitch of each [M, ldc32] split slab (>= N; 0 = N)
    const int64_t ld32 = ldc32 > 0 ? ldc32 : N;
    TORCH_CHECK(ld32 >= N && ld32 % 4 == 0, "gemm: ldc32 must be >= N and a multiple of 4");
    TORCH_CHECK(out32->numel() >= splits * M * ld32, "gemm: out32 too small");
    g.C32 = out32->data_ptr<float>(); g.ldc32 = ld32;
    if (csum_col >= 0) {
      TORCH_CHECK(a_col && csum_col >= N && csum_col < ld32,
                  "gemm: csum_col needs a col-layout A and N <= csum_col < ldc32");
      g.csum_on = 1; g.csum_col = (int)csum_col;
    }
  }
  TORCH_CHECK(csum_col < 0 || out32, "gemm: csum_col needs out32");
  auto check_mn = [&](const c10::optional<Tensor>& t, const char* name) {
    check_2d_rowmajor(*t, name);
    TORCH_CHECK(t->size(0) == M && t->size(1) == N && t->stride(0) % 8 == 0 &&
                aligned16(t->data_ptr()), "gemm: ", name, " must be [M, N], 16-B aligned rows");
  };
  if (mul) { check_mn(mul, "mul"); g.mul = bf16_ptr(*mul); g.ldmul = mul->stride(0); }
  if (add) { check_mn(add, "add"); g.add = bf16_ptr(*add); g.ldadd = add->stride(0); }
  if (out2) {
    check_mn(out2, "out2");
    TORCH_CHECK(splits == 1, "gemm: out2 requires splits == 1");
    g.C2 = bf16_mut(*out2); g.ldc2 = out2->stride(0);
  }
  TORCH_CHECK(!(mul || add) || out2, "gemm: mul/add need out2");
  if (g_gemm_batch.on) {
    g_gemm_batch.args.push_back(g);
    g_gemm_batch.keep.push_back(a);                // may be a zero-padded copy
    g_gemm_batch.keep.push_back(b);
    return;
  }
  tdfo::gemm_bf16(g, cur_stream());
}

// ----------------------------------------------------------- interaction
tdfo::SlotMap make_slots(at::IntArrayRef off, at::IntArrayRef stride, int64_t F) {
  TORCH_CHECK((int64_t)off.size() >= F && (int64_t)stride.size() >= F, "slot map too short");
  tdfo::SlotMap m{};
  for (int64_t i = 0; i < F && i < 32; ++i) { m.off[i] = off[i]; m.stride[i] = stride[i]; }
  return m;
}

void check_inter(int64_t F, int64_t D) {
  TORCH_CHECK(F >= 2 && F <= 32, "interaction: F must be in [2, 32]");
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256,
              "interaction: D must be 16/32/64/128/256");
}

void check_slots_fit(const Tensor& emb, const tdfo::SlotMap& m, int64_t F, int64_t D, int64_t B) {
  for (int64_t i = 1; i < F; ++i) {
    TORCH_CHECK(m.off[i] % 8 == 0 && m.stride[i] % 8 == 0, "slot offsets must be multiples of 8");
    TORCH_CHECK(m.off[i] >= 0 && m.off[i] + (B - 1) * m.stride[i] + D <= emb.numel(),
                "interaction: slot ", i, " out of range");
  }
}

void interaction_fwd(const Tensor& dense, const Tensor& emb, at::IntArrayRef off,
                     at::IntArrayRef stride, int64_t F, int64_t D, const Tensor& out,
                     int64_t ones_col) {
  check_dev(dense, "dense"); check_dev(emb, "emb"); check_dev(out, "out");
  check_inter(F, D); check_2d_rowmajor(dense, "dense"); check_2d_rowmajor(out, "out");
  const int64_t B = dense.size(0);
  TORCH_CHECK(dense.size(1) >= D && dense.stride(0) % 8 == 0, "dense shape");
  TORCH_CHECK(out.size(0) == B && out.size(1) >= D + F * (F - 1) / 2 && out.size(1) % 8 == 0 &&
              out.stride(0) == out.size(1), "interaction out must be [B, ldo] contiguous, ldo%8==0");
  TORCH_CHECK(emb.is_contiguous() && aligned16(emb.data_ptr()) && aligned16(dense.data_ptr()) &&
              aligned16(out.data_ptr()), "alignment");
  auto m = make_slots(off, stride, F);
  check_slots_fit(emb, m, F, D, B);
  tdfo::interaction_fwd(bf16_ptr(dense), dense.stride(0), bf16_ptr(emb), m, (int)F, (int)D,
                        (int)B, bf16_mut(out), out.stride(0), (int)ones_col, cur_stream());
}

void interaction_bwd(const Tensor& dz, const Tensor& dense, const Tensor& emb,
                     at::IntArrayRef off, at::IntArrayRef stride, int64_t F, int64_t D,
                     const Tensor& d_dense, const Tensor& d_emb, at::IntArrayRef doff,
                     at::IntArrayRef dstride, bool relu_mask) {
  check_dev(dz, "dz"); check_dev(dense, "dense"); check_dev(emb, "emb");
  check_dev(d_dense, "d_dense"); check_dev(d_emb, "d_emb");
  check_inter(F, D);
  check_2d_rowmajor(dz, "dz"); check_2d_rowmajor(dense, "dense"); check_2d_rowmajor(d_dense, "d_dense");
  const int64_t B = dense.size(0);
  TORCH_CHECK(dz.size(0) == B && dz.size(1) >= D + F * (F - 1) / 2, "dz shape");
  TORCH_CHECK(d_dense.size(0) == B && d_dense.size(1) >= D, "d_dense shape");
  TORCH_CHECK(dz.stride(0) % 8 == 0 && aligned16(dz.data_ptr()), "dz alignment");
  TORCH_CHECK(d_dense.stride(0) % 8 == 0 && aligned16(d_dense.data_ptr()) &&
              aligned16(d_emb.data_ptr()), "d_dense / d_emb alignment (16-B row stores)");
  TORCH_CHECK(emb.is_contiguous() && d_emb.is_contiguous(), "emb contiguous");
  auto m = make_slots(off, stride, F);
  auto dm = make_slots(doff, dstride, F);
  check_slots_fit(emb, m, F, D, B);
  check_slots_fit(d_emb, dm, F, D, B);
  tdfo::interaction_bwd(bf16_ptr(dz), dz.stride(0), bf16_ptr(dense), dense.stride(0),
                        bf16_ptr(emb), m, (int)F, (int)D, (int)B, bf16_mut(d_dense),
                        d_dense.stride(0), bf16_mut(d_emb), dm, relu_mask, cur_stream());
}

// ------------------------------------------------------------ attention
tdfo::AttnArgs attn_args(const Tensor& qkv, const Tensor& ids, int64_t H, double rate,
                         int64_t seed, const c10::optional<Tensor>& step, int64_t pad_id) {
  check_dev(qkv, "qkv"); check_dev(ids, "ids");
  TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.is_contiguous() && qkv.dim() == 3,
              "attention: qkv fp32 contiguous [B, T, 3E]");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.dim() == 2 &&
              ids.size(0) == qkv.size(0) && ids.size(1) == qkv.size(1), "attention: ids int64 [B, T]");
  const int64_t E3 = qkv.size(2);
  TORCH_CHECK(E3 % 3 == 0 && H > 0 && (E3 / 3) % H == 0, "attention: 3E must split into H heads");
  TORCH_CHECK(qkv.size(1) <= 64, "attention: T <= 64");
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "attention: dropout rate in [0, 1)");
  tdfo::AttnArgs a{};
  a.qkv = qkv.data_ptr<float>(); a.ids = ids.data_ptr<int64_t>();
  a.B = (int)qkv.size(0); a.T = (int)qkv.size(1); a.H = (int)H; a.dk = (int)(E3 / 3 / H);
  a.scale = 1.f / std::sqrt((float)a.dk); a.rate = (float)rate; a.seed = seed; a.pad_id = pad_id;
  if (step) {
    check_dev(*step, "step");
    TORCH_CHECK(step->scalar_type() == at::kLong && step->numel() >= 1, "attention: step int64");
    a.step = step->data_ptr<int64_t>();
  }
  return a;
}

void attention_fwd(const Tensor& qkv, const Tensor& ids, int64_t H, double rate, int64_t seed,
                   const c10::optional<Tensor>& step, int64_t pad_id, const Tensor& out) {
  auto a = attn_args(qkv, ids, H, rate, seed, step, pad_id);
  check_dev(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() &&
              out.numel() == qkv.numel() / 3, "attention: out fp32 [B, T, E]");
  a.out = out.data_ptr<float>();
  tdfo::attention_fwd(a, cur_stream());
}

void attention_bwd(const Tensor& qkv, const Tensor& ids, const Tensor& dout, int64_t H,
                   double rate, int64_t seed, const c10::optional<Tensor>& step, int64_t pad_id,
                   const Tensor& dqkv) {
  auto a = attn_args(qkv, ids, H, rate, seed, step, pad_id);
  check_dev(dout, "dout"); check_dev(dqkv, "dqkv");
  TORCH_CHECK(dout.scalar_type() == at::kFloat && dout.is_contiguous() &&
              dout.numel() == qkv.numel() / 3, "attention: dout fp32 [B, T, E]");
  TORCH_CHECK(dqkv.scalar_type() == at::kFloat && dqkv.is_contiguous() &&
              dqkv.numel() == qkv.numel(), "attention: dqkv fp32 [B, T, 3E]");
  a.dout = dout.data_ptr<float>(); a.dqkv = dqkv.data_ptr<float>();
  tdfo::attention_bwd(a, cur_stream());
}

void check_f32c(const Tensor& t, const char* name);
// ------------------------------------------------------- encoder layer
// params: [Wqkv [3E,E], bqkv, Wo [E,E], bo, g1, be1, g2, be2, W1 [FF,E], b1,
// W2 [E,FF], b2]; saved: [qkv, ctx, x1, f]
tdfo::EncArgs enc_args(const Tensor& x, const Tensor& ids, const c10::optional<Tensor>& step,
                       at::TensorList params, int64_t H, double rate, int64_t seed,
                       int64_t pad_id, double eps, at::TensorList saved) {
  TORCH_CHECK(x.dim() == 3, "encoder_layer: x [B, T, E]");
  const bool sep = params.size() == 16;       // Q / K / V weights and biases apart
  TORCH_CHECK((params.size() == 12 || sep) && saved.size() == 4,
              "encoder_layer: 12 (or 16: separate Q/K/V) params, 4 saved");
  const int64_t B = x.size(0), T = x.size(1), E = x.size(2);
  const int64_t FF = params[params.size() - 4].size(0);
  const int64_t want12[12] = {3 * E * E, 3 * E, E * E, E, E, E, E, E, FF * E, FF, E * FF, E};
  const int64_t want16[16] = {E * E, E * E, E * E, E, E, E, E * E, E, E, E, E, E,
                              FF * E, FF, E * FF, E};
  for (size_t i = 0; i < params.size(); ++i) {
    check_f32c(params[i], "encoder param");
    const int64_t want = sep ? want16[i] : want12[i];
    TORCH_CHECK(params[i].numel() == want, "encoder_layer: param ", i, " has ",
                params[i].numel(), " elements, expected ", want);
  }
  check_f32c(x, "x");
  check_dev(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.numel() == B * T,
              "encoder_layer: ids int64 [B, T]");
  const int64_t wsv[4] = {B * T * 3 * E, B * T * E, B * T * E, B * T * FF};
  for (int i = 0; i < 4; ++i) {
    check_f32c(saved[i], "encoder saved");
    TORCH_CHECK(saved[i].numel() == wsv[i], "encoder_layer: saved tensor ", i, " size");
  }
  TORCH_CHECK(tdfo::encoder_layer_supported((int)T, (int)E, (int)H, (int)FF),
              "encoder_layer: unsupported shape");
  tdfo::EncArgs a{};
  a.B = (int)B; a.T = (int)T; a.E = (int)E; a.H = (int)H; a.FF = (int)FF;
  a.rate = (float)rate; a.seed = seed; a.pad_id = pad_id; a.eps = (float)eps;
  if (step) {
    check_dev(*step, "step");
    TORCH_CHECK(step->scalar_type() == at::kLong, "encoder_layer: step int64");
    a.step = step->data_ptr<int64_t>();
  }
  a.x = x.data_ptr<float>(); a.ids = ids.data_ptr<int64_t>();
  if (params.size() == 16) {
    // [wq, wk, wv, bq, bk, bv, wo, bo, g1, be1, g2, be2, w1, b1, w2, b2]
    const float** pp[16] = {&a.wqkv, &a.wk, &a.wv, &a.bqkv, &a.bk, &a.bv, &a.wo, &a.bo,
                            &a.g1, &a.be1, &a.g2, &a.be2, &a.w1, &a.b1, &a.w2, &a.b2};
    for (int i = 0; i < 16; ++i) *pp[i] = params[i].data_ptr<float>();
  } else {
    const float** pp[12] = {&a.wqkv, &a.bqkv, &a.wo, &a.bo, &a.g1, &a.be1,
                            &a.g2, &a.be2, &a.w1, &a.b1, &a.w2, &a.b2};
    for (int i = 0; i < 12; ++i) *pp[i] = params[i].data_ptr<float>();
  }
  a.qkv = saved[0].data_ptr<float>(); a.ctx = saved[1].data_ptr<float>();
  a.x1 = saved[2].data_ptr<float>(); a.f = saved[3].data_ptr<float>();
  return a;
}

void encoder_layer_fwd(const Tensor& x, const Tensor& ids, const c10::optional<Tensor>& step,
                       at::TensorList params, int64_t H, double rate, int64_t seed,
                       int64_t pad_id, double eps, at::TensorList saved, const Tensor& y) {
  auto a = enc_args(x, ids, step, params, H, rate, seed, pad_id, eps, saved);
  check_f32c(y, "y");
  TORCH_CHECK(y.numel() == x.numel(), "encoder_layer: y [B, T, E]");
  a.y = y.data_ptr<float>();
  tdfo::encoder_layer_fwd(a, cur_stream());
}

void encoder_layer_bwd(const Tensor& x, const Tensor& ids, const c10::optional<Tensor>& step,
                       at::TensorList params, int64_t H, double rate, int64_t seed,
                       int64_t pad_id, double eps, at::TensorList saved, const Tensor& dy,
                       const Tensor& dx, const Tensor& part, const Tensor& grad,
                       const c10::optional<Tensor>& gidx, bool defer) {
  auto a = enc_args(x, ids, step, params, H, rate, seed, pad_id, eps, saved);
  check_f32c(dy, "dy"); check_f32c(dx, "dx"); check_f32c(part, "part"); check_f32c(grad, "grad");
  const int64_t P = tdfo::encoder_param_count(a.E, a.FF);
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "encoder_layer: dy/dx");
  TORCH_CHECK(part.numel() >= (int64_t)a.B * P && grad.numel() >= P, "encoder_layer: part/grad");
  a.dy = dy.data_ptr<float>(); a.dx = dx.data_ptr<float>(); a.part = part.data_ptr<float>();
  // gidx: flat-buffer positions of the P gradients, bounds-checked against
  // grad by the caller when it was built (ops.flat_scatter_index)
  const int64_t* gi = nullptr;
  if (gidx) {
    check_dev(*gidx, "gidx");
    TORCH_CHECK(gidx->scalar_type() == at::kLong && gidx->is_contiguous() && gidx->numel() == P,
                "encoder_layer: gidx int64 [P]");
    gi = gidx->data_ptr<int64_t>();
  }
  tdfo::encoder_layer_bwd(a, grad.data_ptr<float>(), cur_stream(), gi, defer);
}

void encoder_reduce_flush() { tdfo::encoder_reduce_flush(cur_stream()); }

// ------------------------------------------------------------ layernorm
void check_f32c(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be fp32 contiguous");
}

void layernorm_fwd(const Tensor& x, int64_t n, double eps, const Tensor& gamma, const Tensor& beta,
                   const Tensor& y, const Tensor& mean, const Tensor& rstd) {
  check_f32c(x, "x"); check_f32c(gamma, "gamma"); check_f32c(beta, "beta");
  check_f32c(y, "y"); check_f32c(mean, "mean"); check_f32c(rstd, "rstd");
  TORCH_CHECK(n > 0 && n <= 1024 && x.numel() % n == 0, "layernorm: n in (0, 1024] dividing x");
  const int64_t M = x.numel() / n;
  TORCH_CHECK(gamma.numel() == n && beta.numel() == n && y.numel() == x.numel() &&
              mean.numel() >= M && rstd.numel() >= M, "layernorm: shapes");
  tdfo::layernorm_fwd(x.data_ptr<float>(), M, (int)n, (float)eps, gamma.data_ptr<float>(),
                      beta.data_ptr<float>(), y.data_ptr<float>(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), cur_stream());
}

void layernorm_bwd(const Tensor& x, const Tensor& g, int64_t n, const Tensor& gamma,
                   const Tensor& mean, const Tensor& rstd, const Tensor& dx, const Tensor& part,
                   const Tensor& dgb) {
  check_f32c(x, "x"); check_f32c(g, "g"); check_f32c(gamma, "gamma"); check_f32c(mean, "mean");
  check_f32c(rstd, "rstd"); check_f32c(dx, "dx"); check_f32c(part, "part"); check_f32c(dgb, "dgb");
  TORCH_CHECK(n > 0 && n <= 1024 && x.numel() % n == 0, "layernorm: n");
  const int64_t M = x.numel() / n;
  TORCH_CHECK(g.numel() == x.numel() && dx.numel() == x.numel() && gamma.numel() == n &&
              mean.numel() >= M && rstd.numel() >= M && dgb.numel() == 2 * n &&
              part.numel() >= (int64_t)tdfo::layernorm_parts(M) * 2 * n, "layernorm_bwd: shapes");
  tdfo::layernorm_bwd(x.data_ptr<float>(), g.data_ptr<float>(), M, (int)n, gamma.data_ptr<float>(),
                      mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr<float>(),
                      part.data_ptr<float>(), dgb.data_ptr<float>(), cur_stream());
}

void seq_prologue_fwd(const Tensor& x, const Tensor& pos, int64_t n, double eps,
                      const Tensor& gamma, const Tensor& beta, double rate, int64_t seed,
                      const c10::optional<Tensor>& step, const Tensor& y, const Tensor& mean,
                      const Tensor& rstd) {
  check_f32c(x, "x"); check_f32c(pos, "pos"); check_f32c(gamma, "gamma"); check_f32c(beta, "beta");
  check_f32c(y, "y"); check_f32c(mean, "mean"); check_f32c(rstd, "rstd");
  TORCH_CHECK(n > 0 && n <= 1024 && x.numel() % n == 0, "seq_prologue: n in (0, 1024] dividing x");
  const int64_t M = x.numel() / n;
  TORCH_CHECK(pos.numel() == n && gamma.numel() == n && beta.numel() == n &&
              y.numel() == x.numel() && mean.numel() >= M && rstd.numel() >= M,
              "seq_prologue: shapes");
  const int64_t* sp = nullptr;
  if (step) {
    check_dev(*step, "step");
    TORCH_CHECK(step->scalar_type() == at::kLong && step->numel() >= 1, "step: int64 device scalar");
    sp = step->data_ptr<int64_t>();
  }
  tdfo::seq_prologue_fwd(x.data_ptr<float>(), pos.data_ptr<float>(), M, (int)n, (float)eps,
                         gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)rate,
                         (uint32_t)seed, sp, y.data_ptr<float>(), mean.data_ptr<float>(),
                         rstd.data_ptr<float>(), cur_stream());
}

void seq_prologue_bwd(const Tensor& x, const Tensor& pos, const Tensor& g, int64_t n,
                      const Tensor& gamma, const Tensor& mean, const Tensor& rstd, double rate,
                      int64_t seed, const c10::optional<Tensor>& step, const Tensor& dx,
                      const Tensor& part, const Tensor& out3, const c10::optional<Tensor>& gidx) {
  check_f32c(x, "x"); check_f32c(pos, "pos"); check_f32c(g, "g"); check_f32c(gamma, "gamma");
  check_f32c(mean, "mean"); check_f32c(rstd, "rstd"); check_f32c(dx, "dx");
  check_f32c(part, "part"); check_f32c(out3, "out3");
  TORCH_CHECK(n > 0 && n <= 1024 && x.numel() % n == 0, "seq_prologue: n");
  const int64_t M = x.numel() / n;
  TORCH_CHECK(pos.numel() == n && g.numel() == x.numel() && dx.numel() == x.numel() &&
              gamma.numel() == n && mean.numel() >= M && rstd.numel() >= M &&
              (gidx ? out3.numel() >= 3 * n : out3.numel() == 3 * n) &&
              part.numel() >= (int64_t)tdfo::layernorm_parts(M) * 3 * n, "seq_prologue_bwd: shapes");
  const int64_t* sp = nullptr;
  if (step) {
    check_dev(*step, "step");
    TORCH_CHECK(step->scalar_type() == at::kLong && step->numel() >= 1, "step: int64 device scalar");
    sp = step->data_ptr<int64_t>();
  }
  const int64_t* gi = nullptr;
  if (gidx) {        // out3 is then a flat gradient buffer: [dgamma|dbeta|dpos][j] -> out3[gidx[j]]
    check_dev(*gidx, "gidx");
    TORCH_CHECK(gidx->scalar_type() == at::kLong && gidx->is_contiguous() &&
                gidx->numel() == 3 * n, "seq_prologue_bwd: gidx int64 [3n]");
    gi = gidx->data_ptr<int64_t>();
  }
  tdfo::seq_prologue_bwd(x.data_ptr<float>(), pos.data_ptr<float>(), g.data_ptr<float>(), M,
                         (int)n, gamma.data_ptr<float>(), mean.data_ptr<float>(),
                         rstd.data_ptr<float>(), (float)rate, (uint32_t)seed, sp,
                         dx.data_ptr<float>(), part.data_ptr<float>(), out3.data_ptr<float>(),
                         cur_stream(), gi);
}

void rank_metrics(const Tensor& h, const Tensor& W, const Tensor& bias, const Tensor& cand,
                  at::IntArrayRef ks, const Tensor& out) {
  check_f32c(h, "h"); check_f32c(W, "W"); check_f32c(bias, "bias"); check_f32c(out, "out");
  check_dev(cand, "cand");
  TORCH_CHECK(h.dim() == 2 && W.dim() == 2 && h.size(1) == W.size(1), "rank_metrics: h [B,E], W [V,E]");
  const int64_t B = h.size(0), E = h.size(1);
  TORCH_CHECK(cand.scalar_type() == at::kLong && cand.dim() == 2 && cand.size(0) == B &&
              cand.is_contiguous() && cand.size(1) >= 1, "rank_metrics: cand int64 [B, C]");
  TORCH_CHECK(bias.numel() == W.size(0), "rank_metrics: bias [V]");
  TORCH_CHECK(aligned16(h.data_ptr()) && aligned16(W.data_ptr()), "rank_metrics: 16-B aligned rows");
  const int nk = (int)ks.size();
  TORCH_CHECK(nk >= 1 && nk <= 8 && out.numel() == 2 * nk + 1, "rank_metrics: 1..8 cutoffs, out [2nk+1]");
  tdfo::RankKs k{};
  for (int i = 0; i < nk; ++i) k.k[i] = (int)ks[i];
  Tensor part = at::empty({(int64_t)tdfo::rank_metrics_parts((int)B) * (2 * nk + 1)}, out.options());
  tdfo::rank_metrics(h.data_ptr<float>(), W.data_ptr<float>(), bias.data_ptr<float>(),
                     cand.data_ptr<int64_t>(), (int)B, (int)cand.size(1), (int)E, k, nk,
                     part.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
}

// A HIP stream whose kernels may only use the CUs set in mask_words (bit i
// of word w = CU 32 w + i). The embedding side stream uses it so its
// memory-bound, many-block kernels leave CUs to the latency-bound GEMMs.
// Returned as the raw handle for torch.cuda.ExternalStream (never destroyed:
// one per trainer).

// ---------------------------------------------------------- batch gather
void gather_columns(at::TensorList src, const c10::optional<Tensor>& idx, int64_t row0, int64_t n,
                    at::TensorList dst, at::IntArrayRef dst_stride) {
  TORCH_CHECK(src.size() == dst.size() && src.size() == dst_stride.size() && src.size() <= 16 &&
              !src.empty(), "gather_columns: 1..16 matching columns");
  tdfo::GatherColsArgs a{};
  a.ncols = (int)src.size(); a.n = n; a.row0 = row0;
  int64_t rows = -1;
  for (size_t c = 0; c < src.size(); ++c) {
    check_dev(src[c], "src"); check_dev(dst[c], "dst");
    TORCH_CHECK(src[c].is_contiguous() && src[c].dim() == 1, "gather_columns: 1-D contiguous columns");
    rows = rows < 0 ? src[c].numel() : rows;
    TORCH_CHECK(src[c].numel() == rows, "gather_columns: ragged columns");
    const auto st = src[c].scalar_type();
    a.src_dtype[c] = st == at::kChar ? 0 : st == at::kShort ? 1 : st == at::kInt ? 2 :
                     st == at::kLong ? 3 : st == at::kFloat ? 4 : -1;
    TORCH_CHECK(a.src_dtype[c] >= 0, "gather_columns: src dtype i8/i16/i32/i64/f32");
    const auto dt = dst[c].scalar_type();
    TORCH_CHECK(dt == at::kLong || dt == at::kFloat, "gather_columns: dst int64 or fp32");
    TORCH_CHECK(dst_stride[c] >= 1 && (n == 0 || dst[c].storage_offset() >= 0) &&
                (n - 1) * dst_stride[c] < dst[c].numel(), "gather_columns: dst too small");
    a.src[c] = src[c].data_ptr(); a.dst[c] = dst[c].data_ptr();
    a.dst_int[c] = dt == at::kLong; a.dst_stride[c] = dst_stride[c];
  }
  if (idx) {
    check_dev(*idx, "idx");
    TORCH_CHECK(idx->scalar_type() == at::kLong && idx->is_contiguous() && idx->numel() >= n,
                "gather_columns: idx int64 [n]");
    a.idx = idx->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(row0 >= 0 && row0 + n <= rows, "gather_columns: row range");
  }
  tdfo::gather_columns(a, cur_stream());
}

// ----------------------------------------------------------- elementwise
void concat_features(const Tensor& dense, const Tensor& emb, at::IntArrayRef off,
                     at::IntArrayRef stride, int64_t F, int64_t D, const Tensor& out) {
  check_dev(dense, "dense"); check_2d_rowmajor(dense, "dense");
  const int64_t B = dense.size(0);
  TORCH_CHECK(D % 8 == 0 && F <= 32 && F >= 1, "concat: D % 8 and F <= 32");
  TORCH_CHECK(out.is_contiguous() && out.numel() == B * F * D, "concat: out [B, F*D]");
  TORCH_CHECK(dense.stride(0) % 8 == 0 && aligned16(dense.data_ptr()), "concat alignment");
  auto m = make_slots(off, stride, F);
  check_slots_fit(emb, m, F, D, B);
  tdfo::concat_features(bf16_ptr(dense), dense.stride(0), bf16_ptr(emb), m, (int)F, (int)D,
                        (int)B, bf16_mut(out), cur_stream());
}

void split_features(const Tensor& dx, int64_t F, int64_t D, const Tensor& dense,
                    const Tensor& d_dense, const Tensor& d_emb, at::IntArrayRef doff,
                    at::IntArrayRef dstride, bool relu_mask) {
  check_dev(dx, "dx");
  const int64_t B = dense.size(0);
  // packed [B * F * D], or a row-major 2-D view whose rows hold >= F*D columns
  int64_t ld_dx = F * D;
  if (dx.dim() == 2) {
    check_2d_rowmajor(dx, "dx");
    TORCH_CHECK(dx.size(0) == B && dx.size(1) >= F * D && dx.stride(0) % 8 == 0 &&
                aligned16(dx.data_ptr()), "split: dx view [B, >= F*D], 16-B aligned rows");
    ld_dx = dx.stride(0);
  } else {
    TORCH_CHECK(dx.is_contiguous() && dx.numel() == B * F * D, "split: dx [B, F*D]");
  }
  TORCH_CHECK(D % 8 == 0, "split: D % 8");
  check_2d_rowmajor(d_dense, "d_dense");
  TORCH_CHECK(d_dense.stride(0) % 8 == 0 && dense.stride(0) % 8 == 0, "split alignment");
  auto m = make_slots(doff, dstride, F);
  check_slots_fit(d_emb, m, F, D, B);
  tdfo::split_features(bf16_ptr(dx), ld_dx, (int)F, (int)D, (int)B, bf16_ptr(dense), dense.stride(0),
                       bf16_mut(d_dense), d_dense.stride(0), bf16_mut(d_emb), m, relu_mask,
                       cur_stream());
}

void cross_bwd(const Tensor& dout, const Tensor& x0, const Tensor& y, const Tensor& dy,
               const Tensor& dx0, bool accumulate, bool add_dout) {
  const int64_t n = dout.numel();
  for (auto* t : {&dout, &x0, &y, &dy, &dx0}) {
    TORCH_CHECK(t->is_contiguous() && t->numel() == n && t->scalar_type() == at::kBFloat16 &&
                aligned16(t->data_ptr()), "cross_bwd: contiguous bf16 same-size tensors");
  }
  TORCH_CHECK(n % 8 == 0, "cross_bwd: numel % 8");
  tdfo::cross_bwd(bf16_ptr(dout), bf16_ptr(x0), bf16_ptr(y), n, bf16_mut(dy), bf16_mut(dx0),
                  accumulate, add_dout, cur_stream());
}

// ------------------------------------------------ cross-stream events
// Events for the per-stream step's cross-stream edges with a chosen release
// scope: a default hipEvent record performs a system-scope fence (L2
// writeback + invalidate); kernels already release to device scope when they
// end, so same-device consumers only need the ordering.
#define TDFO_HIP_OK(expr)                                                      \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e));        \
  } while (0)

int64_t sync_event_create(int64_t mode) {
  unsigned flags = hipEventDisableTiming;
  if (mode == 1) flags |= hipEventReleaseToDevice;
  if (mode == 2) flags |= hipEventDisableSystemFence;
  hipEvent_t e;
  TDFO_HIP_OK(hipEventCreateWithFlags(&e, flags));
  return reinterpret_cast<int64_t>(e);
}

// stream: a raw hipStream_t handle, or -1 for the current stream (the
// explicit handle spares the host a torch stream-context switch per call)
hipStream_t stream_or_cur(int64_t stream) {
  return stream == -1 ? cur_stream() : reinterpret_cast<hipStream_t>(stream);
}

void sync_event_record(int64_t e, int64_t stream) {
  TDFO_HIP_OK(hipEventRecord(reinterpret_cast<hipEvent_t>(e), stream_or_cur(stream)));
}

void sync_event_wait(int64_t e, int64_t stream) {
  TDFO_HIP_OK(hipStreamWaitEvent(stream_or_cur(stream), reinterpret_cast<hipEvent_t>(e), 0));
}

// dst <- src (same dtype / size, both contiguous on this device) as one async
// copy on an explicit stream (no torch stream-context switch on the host)
void copy_on(const Tensor& dst, const Tensor& src, int64_t stream) {
  check_dev(dst, "dst");
  check_dev(src, "src");
  TORCH_CHECK(dst.scalar_type() == src.scalar_type() && dst.numel() == src.numel() &&
              dst.is_contiguous() && src.is_contiguous(), "copy_on: same dtype / size, contiguous");
  if (dst.numel() == 0) return;
  TDFO_HIP_OK(hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), dst.nbytes(), hipMemcpyDeviceToDevice,
                             stream_or_cur(stream)));
}

bool sync_event_query(int64_t e) {
  const hipError_t r = hipEventQuery(reinterpret_cast<hipEvent_t>(e));
  if (r == hipErrorNotReady) return false;
  TDFO_HIP_OK(r);
  return true;
}

void sync_event_destroy(int64_t e) {
  TDFO_HIP_OK(hipEventDestroy(reinterpret_cast<hipEvent_t>(e)));
}

// ------------------------------------------------------- host mailbox
// Words of hipHostMalloc'd coherent + mapped memory wrapped as a CPU int64
// tensor (freed with it); the device writes them through their mapping
// (host_publish) and the host polls them (parallel/mailbox.py).
Tensor host_mailbox_alloc(int64_t n) {
  TORCH_CHECK(n >= 1 && n <= 4096, "host_mailbox_alloc: 1..4096 words");
  void* p = nullptr;
  TDFO_HIP_OK(hipHostMalloc(&p, (size_t)n * 8, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(p, 0, (size_t)n * 8);
  return at::from_blob(p, {n}, [](void* q) { (void)hipHostFree(q); },
                       at::TensorOptions().dtype(at::kLong));
}

void host_publish(const Tensor& value, const Tensor& seq, const Tensor& host, int64_t slot) {
  TORCH_CHECK(value.is_cuda() && value.scalar_type() == at::kInt && value.numel() >= 1,
              "host_publish: int32 GPU value");
  TORCH_CHECK(seq.is_cuda() && seq.scalar_type() == at::kInt && seq.numel() >= 1,
              "host_publish: int32 GPU sequence counter");
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == at::kLong && slot >= 0 &&
              slot < host.numel(), "host_publish: host mailbox word out of range");
  void* dptr = nullptr;
  TDFO_HIP_OK(hipHostGetDevicePointer(&dptr, host.data_ptr<int64_t>() + slot, 0));
  tdfo::host_publish(value.data_ptr<int32_t>(), seq.data_ptr<int32_t>(),
                     reinterpret_cast<uint64_t*>(dptr), cur_stream());
}

// A chain of captured graphs joined by event nodes, instantiated as ONE
// executable graph: kinds[i] = 0 child graph (handles[i] = hipGraph_t of a
// keep_graph capture), 1 wait on the event handles[i], 2 record it. Stream
// capture cannot create these event nodes on this ROCm (the external-flag
// record is refused, the wait crashes), so they are added explicitly.
// (Signal-memory value-wait nodes were measured and rejected: as graph nodes
// the wait did not hold the consumer, profiles/r04/notes.md.)
int64_t graph_compose(std::vector<int64_t> kinds, std::vector<int64_t> handles) {
  TORCH_CHECK(kinds.size() == handles.size() && !kinds.empty(), "graph_compose: bad parts");
  hipGraph_t g;
  TDFO_HIP_OK(hipGraphCreate(&g, 0));
  hipGraphNode_t prev = nullptr;
  for (size_t i = 0; i < kinds.size(); ++i) {
    hipGraphNode_t n;
    const hipGraphNode_t* dep = prev ? &prev : nullptr;
    const size_t nd = prev ? 1 : 0;
    if (kinds[i] == 0) {
      TDFO_HIP_OK(hipGraphAddChildGraphNode(&n, g, dep, nd,
                                            reinterpret_cast<hipGraph_t>(handles[i])));
    } else if (kinds[i] == 1) {
      TDFO_HIP_OK(hipGraphAddEventWaitNode(&n, g, dep, nd,
                                           reinterpret_cast<hipEvent_t>(handles[i])));
    } else if (kinds[i] == 2) {
      TDFO_HIP_OK(hipGraphAddEventRecordNode(&n, g, dep, nd,
                                             reinterpret_cast<hipEvent_t>(handles[i])));
    } else {
      TORCH_CHECK(false, "graph_compose: unknown part kind ", kinds[i]);
    }
    prev = n;
  }
  hipGraphExec_t ex;
  TDFO_HIP_OK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  TDFO_HIP_OK(hipGraphDestroy(g));
  return reinterpret_cast<int64_t>(ex);
}

void graph_exec_launch(int64_t ex, int64_t stream) {
  TDFO_HIP_OK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(ex), stream_or_cur(stream)));
}

void graph_exec_upload(int64_t ex) {
  TDFO_HIP_OK(hipGraphUpload(reinterpret_cast<hipGraphExec_t>(ex), cur_stream()));
}

// Node count of a captured (keep_graph) hipGraph: segments that captured
// no work are left out of the composed chains.
int64_t graph_num_nodes(int64_t g) {
  size_t n = 0;
  TDFO_HIP_OK(hipGraphGetNodes(reinterpret_cast<hipGraph_t>(g), nullptr, &n));
  return (int64_t)n;
}

void graph_exec_destroy(int64_t ex) {
  TDFO_HIP_OK(hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(ex)));
}

// ------------------------------------------------------- fused MLP


// ------------------------------------------------------------ radix sort
std::tuple<Tensor, Tensor> sort_pairs(const Tensor& keys, const Tensor& vals, int64_t key_bits) {
  check_dev(keys, "keys"); check_dev(vals, "vals");
  TORCH_CHECK(keys.is_contiguous() && vals.is_contiguous() && vals.scalar_type() == at::kInt &&
              keys.numel() == vals.numel(), "sort_pairs: contiguous keys, int32 vals");
  TORCH_CHECK(keys.scalar_type() == at::kLong || keys.scalar_type() == at::kInt, "keys int32/int64");
  const int64_t n = keys.numel();
  Tensor ka = keys.clone(), va = vals.clone();
  Tensor kb = at::empty_like(ka), vb = at::empty_like(va);
  Tensor ws = at::empty({(int64_t)tdfo::radix_sort_workspace(n)}, keys.options().dtype(at::kByte));
  int r;
  if (keys.scalar_type() == at::kLong)
    r = tdfo::radix_sort_pairs_u64(reinterpret_cast<uint64_t*>(ka.data_ptr()), va.data_ptr<int32_t>(),
                                   reinterpret_cast<uint64_t*>(kb.data_ptr()), vb.data_ptr<int32_t>(),
                                   n, (int)key_bits, ws.data_ptr(), cur_stream());
  else
    r = tdfo::radix_sort_pairs_u32(reinterpret_cast<uint32_t*>(ka.data_ptr()), va.data_ptr<int32_t>(),
                                   reinterpret_cast<uint32_t*>(kb.data_ptr()), vb.data_ptr<int32_t>(),
                                   n, (int)key_bits, ws.data_ptr(), cur_stream());
  return r ? std::make_tuple(kb, vb) : std::make_tuple(ka, va);
}

// ------------------------------------------------------------- embedding
void check_i64(const Tensor& t, const char* n) {
  check_dev(t, n);
  TORCH_CHECK(t.scalar_type() == at::kLong && t.is_contiguous(), n, " must be contiguous int64");
}

void embedding_bag_fwd(const Tensor& W, const Tensor& row_offset, const Tensor& indices,
                       const Tensor& offsets, const Tensor& out_off,
                       const c10::optional<Tensor>& psw, int64_t T, int64_t B, bool mean,
                       const Tensor& out, int64_t out_stride, bool onehot, at::TensorList bumps) {
  check_dev(W, "W"); check_2d_rowmajor(W, "W");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous(), "W must be contiguous fp32");
  const int64_t D = W.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256 || D == 512, "embedding D unsupported");
  check_i64(row_offset, "row_offset"); check_i64(indices, "indices");
  check_i64(offsets, "offsets"); check_i64(out_off, "out_off");
  TORCH_CHECK(row_offset.numel() == T && out_off.numel() == T && offsets.numel() == T * B + 1,
              "embedding: table/bag count mismatch");
  check_dev(out, "out"); TORCH_CHECK(out.is_contiguous(), "out contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out dtype");
  TORCH_CHECK(out_stride % 4 == 0, "out_stride must be a multiple of 4");
  tdfo::EmbFwdArgs a{};
  a.W = W.data_ptr<float>(); a.D = (int)D;
  a.row_offset = row_offset.data_ptr<int64_t>(); a.indices = indices.data_ptr<int64_t>();
  a.offsets = offsets.data_ptr<int64_t>(); a.out_off = out_off.data_ptr<int64_t>();
  if (psw) {
    TORCH_CHECK(psw->scalar_type() == at::kFloat && psw->numel() == indices.numel(), "psw");
    a.psw = psw->data_ptr<float>();
  }
  a.T = (int)T; a.B = (int)B; a.mean = mean; a.out_stride = out_stride;
  a.out = out.data_ptr(); a.out_bf16 = out.scalar_type() == at::kBFloat16;
  a.onehot = onehot && indices.numel() == T * B;
  TORCH_CHECK(bumps.size() <= 8, "embedding_bag_fwd: at most 8 counters");
  for (const auto& t : bumps) {
    TORCH_CHECK(t.is_cuda() && t.numel() >= 1 &&
                (t.scalar_type() == at::kFloat || t.scalar_type() == at::kLong),
                "embedding_bag_fwd: float32 / int64 GPU counters");
    a.bumps.p[a.bumps.n] = t.data_ptr();
    a.bumps.is_i64[a.bumps.n] = t.scalar_type() == at::kLong;
    ++a.bumps.n;
  }
  tdfo::embedding_bag_fwd(a, cur_stream());
}

tdfo::EmbBwdArgs emb_bwd_args(const Tensor& W, const Tensor& row_offset, const Tensor& indices,
                              const Tensor& offsets, const Tensor& grad_off,
                              const c10::optional<Tensor>& psw, int64_t T, int64_t B, bool mean,
                              int64_t key_bits, int64_t grad_stride, int64_t segsort) {
  check_dev(W, "W");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 2, "W fp32 2-D");
  const int64_t D = W.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256 || D == 512, "embedding D unsupported");
  check_i64(row_offset, "row_offset"); check_i64(indices, "indices");
  check_i64(offsets, "offsets"); check_i64(grad_off, "grad_off");
  TORCH_CHECK(offsets.numel() == T * B + 1 && grad_off.numel() == T && row_offset.numel() == T, "bwd counts");
  TORCH_CHECK(key_bits >= 1 && key_bits <= 64, "key_bits");
  const int64_t nnz = indices.numel();
  TORCH_CHECK(nnz < (1LL << 31), "nnz too large");
  tdfo::EmbBwdArgs a{};
  a.W = W.data_ptr<float>(); a.D = (int)D;
  a.row_offset = row_offset.data_ptr<int64_t>(); a.indices = indices.data_ptr<int64_t>();
  a.offsets = offsets.data_ptr<int64_t>(); a.grad_off = grad_off.data_ptr<int64_t>();
  if (psw) a.psw = psw->data_ptr<float>();
  a.T = (int)T; a.B = (int)B; a.mean = mean; a.nnz = nnz; a.key_bits = (int)key_bits;
  a.grad_stride = grad_stride;
  // caller's promise: one id per bag; virtual tables = segsort runs x
  // physical tables, run-major (only runs of the same table share rows)
  a.segsort = (segsort > 0 && nnz == T * B && T % segsort == 0) ? (int)segsort : 0;
  return a;
}

void emb_bwd_opt_args(tdfo::EmbBwdArgs& a, const Tensor& W, const Tensor& grad, int64_t opt,
                      const c10::optional<Tensor>& state1, const c10::optional<Tensor>& state2,
                      const Tensor& hyper, double eps, double beta1, double beta2,
                      double weight_decay, const c10::optional<Tensor>& dense_grad) {
  const int64_t D = W.size(1);
  TORCH_CHECK(grad.is_contiguous() && (grad.scalar_type() == at::kBFloat16 || grad.scalar_type() == at::kFloat), "grad");
  TORCH_CHECK(hyper.scalar_type() == at::kFloat && hyper.numel() >= 2 && hyper.is_cuda(), "hyper fp32[>=2] on device");
  a.grad = grad.data_ptr(); a.grad_bf16 = grad.scalar_type() == at::kBFloat16;
  a.opt = (int)opt;
  const int64_t rows = W.size(0);
  if (opt == tdfo::EMB_ROWWISE_ADAGRAD) {
    TORCH_CHECK(state1 && state1->numel() == rows && state1->scalar_type() == at::kFloat, "rowwise state [rows]");
  }
  if (opt == tdfo::EMB_ADAGRAD || opt == tdfo::EMB_ADAM) {
    TORCH_CHECK(state1 && state1->numel() == rows * D, "state1 [rows, D]");
  }
  if (opt == tdfo::EMB_ADAM) TORCH_CHECK(state2 && state2->numel() == rows * D, "state2 [rows, D]");
  if (opt == tdfo::EMB_DENSE_GRAD) TORCH_CHECK(dense_grad && dense_grad->numel() == rows * D, "dense_grad");
  if (state1) a.state1 = state1->data_ptr<float>();
  if (state2) a.state2 = state2->data_ptr<float>();
  if (dense_grad) a.dense_grad = dense_grad->data_ptr<float>();
  a.hyper = hyper.data_ptr<float>(); a.hyper_n = (int)hyper.numel();
  a.eps = (float)eps; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.weight_decay = (float)weight_decay;
}

void set_emb_ws(tdfo::EmbBwdArgs& a, const Tensor& work) {
  const size_t ws = tdfo::embedding_bwd_workspace(a.nnz, a.D);
  check_dev(work, "workspace");
  TORCH_CHECK(work.is_contiguous() && (size_t)work.nbytes() >= ws, "embedding workspace too small");
  a.workspace = work.data_ptr(); a.workspace_bytes = ws;
}

// reduce_adam(defer=true) parks its launch here; the next embedding_bwd of
// this thread runs it as side blocks of its sort launch (tdfo::EmbBwdArgs::
// side), flush_side_job() launches a still-parked one on its own.
thread_local bool g_side_pending = false;
thread_local tdfo::ReduceAdamArgs g_side{};
// two_tower(defer=true): the tower step parked the same way; the next
// embedding_bwd co-launches it with its per-table sort (or launches it first)
thread_local bool g_tower_pending = false;
thread_local tdfo::TwoTowerArgs g_tower{};

void embedding_bwd(const Tensor& W, const Tensor& row_offset, const Tensor& indices,
                   const Tensor& offsets, const Tensor& grad_off,
                   const c10::optional<Tensor>& psw, int64_t T, int64_t B, bool mean,
                   int64_t key_bits, const Tensor& grad, int64_t grad_stride, int64_t opt,
                   const c10::optional<Tensor>& state1, const c10::optional<Tensor>& state2,
                   const Tensor& hyper, double eps, double beta1, double beta2,
                   double weight_decay, const c10::optional<Tensor>& dense_grad, int64_t segsort) {
  auto a = emb_bwd_args(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, key_bits,
                        grad_stride, segsort);
  emb_bwd_opt_args(a, W, grad, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay,
                   dense_grad);
  const size_t ws = tdfo::embedding_bwd_workspace(a.nnz, a.D);
  Tensor work = at::empty({(int64_t)ws}, W.options().dtype(at::kByte));
  set_emb_ws(a, work);
  if (g_side_pending) {
    a.side = g_side;
    a.side_on = 1;
    g_side_pending = false;
  }
  if (g_tower_pending) {
    a.tower = g_tower;
    a.tower_on = 1;
    g_tower_pending = false;
  }
  tdfo::embedding_bwd_fused(a, cur_stream());
}

void embedding_bwd_prepare(const Tensor& W, const Tensor& row_offset, const Tensor& indices,
                           const Tensor& offsets, const Tensor& grad_off,
                           const c10::optional<Tensor>& psw, int64_t T, int64_t B, bool mean,
                           int64_t key_bits, int64_t grad_stride, int64_t segsort,
                           const Tensor& work, const c10::optional<Tensor>& bag_len) {
  auto a = emb_bwd_args(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, key_bits,
                        grad_stride, segsort);
  set_emb_ws(a, work);
  if (bag_len) {
    check_dev(*bag_len, "bag_len");
    TORCH_CHECK(bag_len->scalar_type() == at::kInt && bag_len->is_contiguous() &&
                bag_len->numel() >= T, "bag_len: int32 [T]");
    a.bag_len = bag_len->data_ptr<int32_t>();
  }
  tdfo::embedding_bwd_prepare(a, cur_stream());
}

void embedding_bwd_apply(const Tensor& W, const Tensor& row_offset, const Tensor& indices,
                         const Tensor& offsets, const Tensor& grad_off,
                         const c10::optional<Tensor>& psw, int64_t T, int64_t B, bool mean,
                         int64_t key_bits, const Tensor& grad, int64_t grad_stride, int64_t opt,
                         const c10::optional<Tensor>& state1, const c10::optional<Tensor>& state2,
                         const Tensor& hyper, double eps, double beta1, double beta2,
                         double weight_decay, const c10::optional<Tensor>& dense_grad,
                         int64_t segsort, const Tensor& work) {
  auto a = emb_bwd_args(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, key_bits,
                        grad_stride, segsort);
  emb_bwd_opt_args(a, W, grad, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay,
                   dense_grad);
  set_emb_ws(a, work);
  tdfo::embedding_bwd_apply(a, cur_stream());
}

void embedding_dense_update(const Tensor& W, const Tensor& grad, int64_t rows, int64_t opt,
                            const c10::optional<Tensor>& state1, const c10::optional<Tensor>& state2,
                            const Tensor& hyper, double eps, double beta1, double beta2,
                            double weight_decay, bool clear_grad) {
  check_dev(W, "W");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 2, "W fp32 2-D");
  const int64_t D = W.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256 || D == 512, "embedding D unsupported");
  TORCH_CHECK(rows >= 0 && rows <= W.size(0), "rows out of range");
  check_dev(grad, "grad");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.is_contiguous() && grad.numel() >= rows * D,
              "dense grad must be contiguous fp32 [rows, D]");
  TORCH_CHECK(opt != tdfo::EMB_DENSE_GRAD, "dense update needs a real optimizer");
  tdfo::EmbBwdArgs a{};
  a.W = W.data_ptr<float>(); a.D = (int)D;
  emb_bwd_opt_args(a, W, grad, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay,
                   c10::nullopt);
  tdfo::embedding_dense_update(a, rows, grad.data_ptr<float>(),
                               clear_grad ? const_cast<float*>(grad.data_ptr<float>()) : nullptr,
                               cur_stream());
}

// ------------------------------------------------------- row-wise shards
int64_t rw_meta_check(const Tensor& meta, int64_t nrw) {
  check_i64(meta, "rw meta");
  TORCH_CHECK(nrw >= 1 && meta.numel() == 5 * nrw + 1, "rw meta must hold 5*nrw+1 int64");
  return nrw;
}

int64_t rw_bucketize_workspace(int64_t n, int64_t W) {
  return (int64_t)tdfo::rw_bucketize_workspace(n, (int)W);
}

void rw_bucketize(const Tensor& ids, const Tensor& meta, int64_t nrw, int64_t W, int64_t B,
                  int64_t cap, int64_t n, const Tensor& send, const Tensor& work,
                  const Tensor& overflow) {
  check_i64(ids, "ids"); rw_meta_check(meta, nrw); check_i64(send, "send");
  TORCH_CHECK(W >= 1 && W <= 64, "rw: world size must be in [1, 64]");
  TORCH_CHECK(send.numel() == W * (cap + 1), "rw send buffer must be [W][cap+1]");
  TORCH_CHECK(nrw * B < (1LL << 31), "rw: bag keys must fit 31 bits");
  check_dev(work, "rw workspace");
  TORCH_CHECK((size_t)work.nbytes() >= tdfo::rw_bucketize_workspace(n, (int)W), "rw workspace too small");
  check_dev(overflow, "overflow");
  TORCH_CHECK(overflow.scalar_type() == at::kInt && overflow.numel() >= 1, "overflow int32[1]");
  tdfo::RwBucketArgs a{};
  a.ids = ids.data_ptr<int64_t>(); a.meta = meta.data_ptr<int64_t>();
  a.nrw = (int)nrw; a.W = (int)W; a.B = (int)B; a.cap = cap; a.n = n;
  a.send = send.data_ptr<int64_t>(); a.overflow = overflow.data_ptr<int32_t>();
  a.need = overflow.numel() >= 2 ? overflow.data_ptr<int32_t>() + 1 : nullptr;   // [flag, need]
  tdfo::rw_bucketize(a, work.data_ptr(), cur_stream());
}

void rw_pool(const Tensor& Wt, const Tensor& recv, const Tensor& meta, int64_t nrw, int64_t W,
             int64_t B, int64_t cap, bool mean, const Tensor& starts, const Tensor& out,
             int64_t out_ld) {
  check_dev(Wt, "W");
  TORCH_CHECK(Wt.scalar_type() == at::kFloat && Wt.is_contiguous() && Wt.dim() == 2, "W fp32 2-D");
  TORCH_CHECK(Wt.size(0) <= (1LL << 32), "rw: owner rows must fit 32-bit row keys");
  const int64_t D = Wt.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256, "rw_pool: D unsupported");
  check_i64(recv, "recv"); rw_meta_check(meta, nrw);
  TORCH_CHECK(recv.numel() == W * (cap + 1), "rw recv buffer must be [W][cap+1]");
  check_dev(starts, "starts");
  TORCH_CHECK(starts.scalar_type() == at::kInt && starts.numel() >= W * (nrw * B + 1), "starts int32");
  check_dev(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat,
              "rw_pool out must be bf16 or fp32");
  TORCH_CHECK(out_ld >= nrw * D && out_ld % 4 == 0 && out.numel() >= W * B * out_ld, "rw_pool out size");
  tdfo::RwPoolArgs a{};
  a.Wt = Wt.data_ptr<float>(); a.D = (int)D; a.recv = recv.data_ptr<int64_t>();
  a.meta = meta.data_ptr<int64_t>(); a.nrw = (int)nrw; a.W = (int)W; a.B = (int)B; a.cap = cap;
  a.mean = mean; a.starts = starts.data_ptr<int32_t>(); a.out = out.data_ptr();
  a.out_f32 = out.scalar_type() == at::kFloat; a.out_ld = out_ld;
  tdfo::rw_pool(a, cur_stream());
}

// fused bottom MLP forward (mlp_fused.hip)
bool bottom_mlp_fwd_ok(int64_t k0, int64_t n0, int64_t n1, int64_t n2) {
  return tdfo::bottom_mlp_fwd_supported((int)k0, (int)n0, (int)n1, (int)n2);
}

void bottom_mlp_fwd(const Tensor& x, const Tensor& w0, const Tensor& w1, const Tensor& w2,
                    const c10::optional<Tensor>& b0, const c10::optional<Tensor>& b1,
                    const c10::optional<Tensor>& b2, const Tensor& y0, const Tensor& y1,
                    const Tensor& y2, const c10::optional<Tensor>& dense,
                    const c10::optional<Tensor>& label_src,
                    const c10::optional<Tensor>& label_dst) {
  const Tensor* ts[7] = {&x, &w0, &w1, &w2, &y0, &y1, &y2};
  const char* nm[7] = {"x", "w0", "w1", "w2", "y0", "y1", "y2"};
  for (int i = 0; i < 7; ++i) {
    check_dev(*ts[i], nm[i]);
    TORCH_CHECK(ts[i]->scalar_type() == at::kBFloat16 && ts[i]->dim() == 2 &&
                ts[i]->stride(1) == 1 && ts[i]->stride(0) % 8 == 0 && aligned16(ts[i]->data_ptr()),
                "bottom_mlp_fwd: ", nm[i], " must be bf16 2-D, unit column stride, 16-B rows");
  }
  const int64_t M = x.size(0);
  TORCH_CHECK(tdfo::bottom_mlp_fwd_supported((int)x.size(1), (int)w0.size(0), (int)w1.size(0),
                                             (int)w2.size(0)), "bottom_mlp_fwd: unsupported dims");
  TORCH_CHECK(w0.size(1) >= x.size(1) && w1.size(1) >= w0.size(0) && w2.size(1) >= w1.size(0),
              "bottom_mlp_fwd: weight K");
  TORCH_CHECK(y0.size(0) == M && y1.size(0) == M && y2.size(0) == M && y0.size(1) >= w0.size(0) &&
              y1.size(1) >= w1.size(0) && y2.size(1) >= w2.size(0), "bottom_mlp_fwd: outputs");
  tdfo::BotMlpArgs a{};
  a.x = bf16_ptr(x); a.ldx = x.stride(0);
  a.w0 = bf16_ptr(w0); a.w1 = bf16_ptr(w1); a.w2 = bf16_ptr(w2);
  a.ldw0 = w0.stride(0); a.ldw1 = w1.stride(0); a.ldw2 = w2.stride(0);
  const c10::optional<Tensor>* bs[3] = {&b0, &b1, &b2};
  const int64_t nout[3] = {w0.size(0), w1.size(0), w2.size(0)};
  const float* bp[3] = {nullptr, nullptr, nullptr};
  int64_t bst[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    if (*bs[i]) {
      const Tensor& b = **bs[i];
      check_dev(b, "bias");
      TORCH_CHECK(b.scalar_type() == at::kFloat && b.dim() == 1 && b.size(0) >= nout[i],
                  "bottom_mlp_fwd: bias fp32 1-D");
      bp[i] = b.data_ptr<float>();
      bst[i] = b.stride(0);
    }
  }
  a.b0 = bp[0]; a.b1 = bp[1]; a.b2 = bp[2]; a.bs0 = bst[0]; a.bs1 = bst[1]; a.bs2 = bst[2];
  a.y0 = bf16_mut(y0); a.y1 = bf16_mut(y1); a.y2 = bf16_mut(y2);
  a.ldy0 = y0.stride(0); a.ldy1 = y1.stride(0); a.ldy2 = y2.stride(0);
  a.M = (int)M;
  if (dense) {
    check_dev(*dense, "dense");
    TORCH_CHECK(dense->scalar_type() == at::kFloat && dense->dim() == 2 && dense->size(0) == M &&
                dense->stride(1) == 1 && dense->size(1) <= 16 && dense->size(1) < x.size(1),
                "bottom_mlp_fwd: dense fp32 [M, nd < 16] rows");
    a.dense = dense->data_ptr<float>(); a.ld_dense = dense->stride(0);
    a.nd = (int)dense->size(1);
    a.x_out = bf16_mut(x);
    if (label_src) {
      TORCH_CHECK(label_dst && label_src->scalar_type() == at::kFloat &&
                  label_dst->scalar_type() == at::kFloat && label_src->is_contiguous() &&
                  label_dst->is_contiguous() && label_src->numel() >= M &&
                  label_dst->numel() >= M, "bottom_mlp_fwd: labels fp32 [M]");
      a.label_src = label_src->data_ptr<float>(); a.label_dst = label_dst->data_ptr<float>();
    }
  }
  tdfo::bottom_mlp_fwd(a, cur_stream());
}

// one-hot row-wise "rows" exchange (rowwise.hip)
void check_bf16_buf(const Tensor& t, int64_t n, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() >= n, name,
              ": bf16 contiguous buffer too small");
}

void rw_rows_gather(const Tensor& Wt, const Tensor& recv, int64_t W, int64_t cap, const Tensor& out) {
  check_dev(Wt, "W");
  TORCH_CHECK(Wt.scalar_type() == at::kFloat && Wt.is_contiguous() && Wt.dim() == 2, "W fp32 2-D");
  TORCH_CHECK(Wt.size(0) <= (1LL << 32), "rw: owner rows must fit 32-bit row keys");
  const int64_t D = Wt.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256, "rw_rows_gather: D unsupported");
  check_i64(recv, "recv");
  TORCH_CHECK(recv.numel() == W * (cap + 1), "rw recv buffer must be [W][cap+1]");
  check_bf16_buf(out, W * (cap + 1) * D, "rw rows out");
  tdfo::rw_rows_gather(Wt.data_ptr<float>(), (int)D, recv.data_ptr<int64_t>(), (int)W, cap,
                       bf16_mut(out), cur_stream());
}

void rw_rows_scatter(const Tensor& send, int64_t W, int64_t cap, int64_t B, int64_t D,
                     const Tensor& rows, const Tensor& region, int64_t ld, const Tensor& map,
                     int64_t nrw) {
  check_i64(send, "send");
  TORCH_CHECK(send.numel() == W * (cap + 1), "rw send buffer must be [W][cap+1]");
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256, "rw_rows_scatter: D unsupported");
  TORCH_CHECK(ld >= nrw * D && ld % 4 == 0, "rw_rows_scatter: row stride");
  TORCH_CHECK(B * ld < (1LL << 31), "rw_rows_scatter: region offsets must fit int32");
  check_bf16_buf(rows, W * (cap + 1) * D, "rw rows");
  check_bf16_buf(region, B * ld, "rw pooled region");
  check_dev(map, "rw map");
  TORCH_CHECK(map.scalar_type() == at::kInt && map.numel() >= W * (cap + 1), "rw map int32 [W][cap+1]");
  tdfo::rw_rows_scatter(send.data_ptr<int64_t>(), (int)W, cap, (int)B, (int)D, bf16_ptr(rows),
                        bf16_mut(region), ld, map.data_ptr<int32_t>(), cur_stream());
}

void rw_grads_gather(const Tensor& map, int64_t W, int64_t cap, int64_t D, const Tensor& dregion,
                     const Tensor& gsend) {
  check_dev(map, "rw map");
  TORCH_CHECK(map.scalar_type() == at::kInt && map.numel() >= W * (cap + 1), "rw map int32 [W][cap+1]");
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256, "rw_grads_gather: D unsupported");
  check_bf16_buf(dregion, D, "rw grad region");
  check_bf16_buf(gsend, W * (cap + 1) * D, "rw grad send");
  tdfo::rw_grads_gather(map.data_ptr<int32_t>(), (int)W, cap, (int)D, bf16_ptr(dregion),
                        bf16_mut(gsend), cur_stream());
}

tdfo::EmbBwdArgs emb_rw_args(const Tensor& W, int64_t Wsz, int64_t B, int64_t cap, bool mean,
                             int64_t key_bits) {
  check_dev(W, "W");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 2, "W fp32 2-D");
  const int64_t D = W.size(1);
  TORCH_CHECK(D == 16 || D == 32 || D == 64 || D == 128 || D == 256 || D == 512, "embedding D unsupported");
  TORCH_CHECK(key_bits >= 1 && key_bits <= 64, "key_bits");
  const int64_t nnz = Wsz * cap;
  TORCH_CHECK(nnz < (1LL << 31), "rw: W*cap too large");
  tdfo::EmbBwdArgs a{};
  a.W = W.data_ptr<float>(); a.D = (int)D; a.T = 1; a.B = (int)B; a.mean = mean; a.nnz = nnz;
  a.key_bits = (int)key_bits;
  return a;
}

void embedding_bwd_prepare_rw(const Tensor& W, const Tensor& recv, const Tensor& meta, int64_t nrw,
                              int64_t Wsz, int64_t B, int64_t cap, bool mean, int64_t key_bits,
                              int64_t grad_ld, int64_t dummy_row, const Tensor& work,
                              int64_t rows) {
  auto a = emb_rw_args(W, Wsz, B, cap, mean, key_bits);
  check_i64(recv, "recv"); rw_meta_check(meta, nrw);
  TORCH_CHECK(recv.numel() == Wsz * (cap + 1), "rw recv buffer must be [W][cap+1]");
  TORCH_CHECK(dummy_row >= 0 && dummy_row < W.size(0), "rw scratch row out of range");
  set_emb_ws(a, work);
  tdfo::embedding_bwd_prepare_rw(a, recv.data_ptr<int64_t>(), meta.data_ptr<int64_t>(), (int)nrw,
                                 (int)Wsz, cap, grad_ld, dummy_row, (int)rows, cur_stream());
}

void embedding_bwd_apply_rw(const Tensor& W, int64_t Wsz, int64_t B, int64_t cap, bool mean,
                            int64_t key_bits, const Tensor& grad, int64_t opt,
                            const c10::optional<Tensor>& state1, const c10::optional<Tensor>& state2,
                            const Tensor& hyper, double eps, double beta1, double beta2,
                            double weight_decay, const Tensor& work) {
  auto a = emb_rw_args(W, Wsz, B, cap, mean, key_bits);
  emb_bwd_opt_args(a, W, grad, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay,
                   c10::nullopt);
  set_emb_ws(a, work);
  tdfo::embedding_bwd_apply(a, cur_stream());
}

// --------------------------------------------------------------- optim
void dense_optimizer(const Tensor& p, const Tensor& g, const c10::optional<Tensor>& m,
                     const c10::optional<Tensor>& v, const c10::optional<Tensor>& p_bf16,
                     int64_t opt, const Tensor& hyper, double beta1, double beta2, double eps,
                     double wd, double momentum, const c10::optional<Tensor>& found_inf,
                     at::TensorList seg_slabs, at::IntArrayRef seg_start, at::IntArrayRef seg_splits) {
  check_dev(p, "p"); check_dev(g, "g");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat && p.is_contiguous() &&
              g.is_contiguous() && p.numel() == g.numel(), "p/g fp32 contiguous same size");
  TORCH_CHECK(p.numel() % 4 == 0, "flat buffer must be padded to a multiple of 4");
  TORCH_CHECK(hyper.is_cuda() && hyper.scalar_type() == at::kFloat && hyper.numel() >= 3, "hyper [lr, step, gscale]");
  tdfo::DenseOptArgs a{};
  a.p = p.data_ptr<float>(); a.g = g.data_ptr<float>(); a.n = p.numel(); a.opt = (int)opt;
  const bool need_m = opt == tdfo::OPT_ADAMW || opt == tdfo::OPT_ADAM || opt == tdfo::OPT_ADAGRAD ||
                      (opt == tdfo::OPT_SGD && momentum != 0.0);
  if (need_m) { TORCH_CHECK(m && m->numel() == p.numel(), "m state"); a.m = m->data_ptr<float>(); }
  if (opt == tdfo::OPT_ADAMW || opt == tdfo::OPT_ADAM) {
    TORCH_CHECK(v && v->numel() == p.numel(), "v state"); a.v = v->data_ptr<float>();
  }
  if (p_bf16) { TORCH_CHECK(p_bf16->numel() == p.numel(), "p_bf16 size"); a.p_bf16 = bf16_mut(*p_bf16); }
  a.hyper = hyper.data_ptr<float>();
  a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)wd; a.momentum = (float)momentum;
  if (found_inf) a.found_inf = found_inf->data_ptr<float>();
  TORCH_CHECK(seg_slabs.size() <= 16 && seg_start.size() == seg_slabs.size() &&
              seg_splits.size() == seg_slabs.size(), "dense_optimizer: <= 16 matching segments");
  a.nseg = (int)seg_slabs.size();
  for (size_t k = 0; k < seg_slabs.size(); ++k) {
    const Tensor& sl = seg_slabs[k];
    check_dev(sl, "seg slab");
    TORCH_CHECK(sl.scalar_type() == at::kFloat && sl.is_contiguous() && aligned16(sl.data_ptr()),
                "seg slab fp32 contiguous 16-B aligned");
    const int64_t S = seg_splits[k], len = S > 0 ? sl.numel() / S : 0;
    TORCH_CHECK(S >= 1 && len * S == sl.numel() && len % 4 == 0 && seg_start[k] % 4 == 0 &&
                seg_start[k] + len <= p.numel(), "dense_optimizer: segment shape/alignment");
    a.seg_start[k] = seg_start[k]; a.seg_len[k] = len; a.seg_splits[k] = (int)S;
    a.seg_ptr[k] = sl.data_ptr<float>();
  }
  tdfo::dense_optimizer(a, cur_stream());
}

void check_finite(const Tensor& g, const Tensor& found) {
  check_dev(g, "g");
  TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous(), "g fp32");
  tdfo::check_finite(g.data_ptr<float>(), g.numel(), found.data_ptr<float>(), cur_stream());
}

void cast_bf16(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "cast shapes");
  tdfo::cast_f32_bf16(x.data_ptr<float>(), bf16_mut(y), x.numel(), cur_stream());
}

void batch_load(const Tensor& dense, const Tensor& x0, const Tensor& ids, const Tensor& ids_dst,
                const Tensor& label, const Tensor& label_dst) {
  check_dev(dense, "dense"); check_dev(x0, "x0");
  TORCH_CHECK(dense.dim() == 2 && dense.scalar_type() == at::kFloat && dense.stride(1) == 1,
              "batch_load: dense fp32 [B, nd] row-major");
  TORCH_CHECK(x0.dim() == 2 && x0.scalar_type() == at::kBFloat16 && x0.stride(1) == 1 &&
              x0.size(0) == dense.size(0) && x0.size(1) >= dense.size(1), "batch_load: x0 bf16");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids_dst.scalar_type() == at::kLong &&
              ids.is_contiguous() && ids_dst.is_contiguous() && ids.numel() == ids_dst.numel(),
              "batch_load: ids int64, same size");
  TORCH_CHECK(aligned16(ids.data_ptr()) && aligned16(ids_dst.data_ptr()), "batch_load: ids alignment");
  TORCH_CHECK(label.scalar_type() == at::kFloat && label_dst.scalar_type() == at::kFloat &&
              label.is_contiguous() && label_dst.is_contiguous() &&
              label.numel() == dense.size(0) && label_dst.numel() == dense.size(0),
              "batch_load: label fp32 [B]");
  TORCH_CHECK(ids.device() == x0.device() && label.device() == x0.device() &&
              ids_dst.device() == x0.device() && label_dst.device() == x0.device(),
              "batch_load: one device");
  tdfo::batch_load(dense.data_ptr<float>(), (int)dense.size(1), dense.stride(0), bf16_mut(x0),
                   x0.stride(0), ids.data_ptr<int64_t>(), ids_dst.data_ptr<int64_t>(), ids.numel(),
                   label.data_ptr<float>(), label_dst.data_ptr<float>(), (int)dense.size(0),
                   cur_stream());
}

// ------------------------------------------------------- synthetic data
void synth_criteo(int64_t seed, int64_t rank, int64_t batch_index, int64_t B,
                  const Tensor& rows, const Tensor& pooling, const Tensor& base, int64_t dist,
                  double alpha, const Tensor& w_dense, const Tensor& table_bias,
                  const Tensor& dense, const Tensor& ids, const Tensor& label) {
  check_dev(dense, "dense");
  const int64_t T = rows.numel();
  TORCH_CHECK(rows.scalar_type() == at::kLong && base.scalar_type() == at::kLong &&
              pooling.scalar_type() == at::kInt && pooling.numel() == T && base.numel() == T &&
              rows.is_contiguous() && base.is_contiguous() && pooling.is_contiguous(),
              "synth_criteo: rows/base int64[T], pooling int32[T]");
  TORCH_CHECK(dense.scalar_type() == at::kFloat && dense.is_contiguous() && dense.dim() == 2 &&
              dense.size(0) == B, "synth_criteo: dense fp32 [B, nd]");
  TORCH_CHECK(w_dense.scalar_type() == at::kFloat && w_dense.numel() == dense.size(1) &&
              table_bias.scalar_type() == at::kFloat && table_bias.numel() == T * 64 &&
              w_dense.is_contiguous() && table_bias.is_contiguous(), "synth_criteo: teacher");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() &&
              label.scalar_type() == at::kFloat && label.numel() == B, "synth_criteo: outputs");
  for (const Tensor* t : {&rows, &pooling, &base, &w_dense, &table_bias, &ids, &label})
    TORCH_CHECK(t->device() == dense.device(), "synth_criteo: one device");
  tdfo::SynthArgs a{};
  a.seed = (uint64_t)seed; a.rank = (int)rank; a.batch_index = batch_index;
  a.B = (int)B; a.num_dense = (int)dense.size(1); a.T = (int)T;
  a.rows = rows.data_ptr<int64_t>(); a.pooling = pooling.data_ptr<int32_t>();
  a.base = base.data_ptr<int64_t>(); a.dist = (int)dist; a.alpha = alpha;
  a.w_dense = w_dense.data_ptr<float>(); a.table_bias = table_bias.data_ptr<float>();
  a.dense = dense.data_ptr<float>(); a.ids = ids.data_ptr<int64_t>();
  a.label = label.data_ptr<float>();
  tdfo::synth_criteo(a, cur_stream());
}

// In-step generation: the batch index is index_base + counter[0] (a float
// step counter on the device), read by the kernel -> a fresh batch per replay.
static tdfo::SynthArgs synth_in_step_args(int64_t seed, int64_t rank, int64_t index_base,
                                          int64_t B, const Tensor& rows, const Tensor& pooling,
                                          const Tensor& base, int64_t dist, double alpha,
                                          const Tensor& counter) {
  const int64_t T = rows.numel();
  check_dev(rows, "rows"); check_dev(counter, "counter");
  TORCH_CHECK(rows.scalar_type() == at::kLong && base.scalar_type() == at::kLong &&
              pooling.scalar_type() == at::kInt && pooling.numel() == T && base.numel() == T &&
              rows.is_contiguous() && base.is_contiguous() && pooling.is_contiguous() &&
              base.device() == rows.device() && pooling.device() == rows.device(),
              "synth in-step: rows/base int64[T], pooling int32[T] on one device");
  TORCH_CHECK(counter.scalar_type() == at::kFloat && counter.numel() >= 1 &&
              counter.device() == rows.device(), "synth in-step: float step counter");
  tdfo::SynthArgs a{};
  a.seed = (uint64_t)seed; a.rank = (int)rank; a.batch_index = index_base;
  a.B = (int)B; a.T = (int)T;
  a.rows = rows.data_ptr<int64_t>(); a.pooling = pooling.data_ptr<int32_t>();
  a.base = base.data_ptr<int64_t>(); a.dist = (int)dist; a.alpha = alpha;
  a.index_ptr = counter.data_ptr<float>();
  return a;
}

void synth_ids(int64_t seed, int64_t rank, int64_t index_base, int64_t B, const Tensor& rows,
               const Tensor& pooling, const Tensor& base, int64_t dist, double alpha,
               const Tensor& counter, int64_t nnz, const Tensor& ids) {
  tdfo::SynthArgs a = synth_in_step_args(seed, rank, index_base, B, rows, pooling, base, dist,
                                         alpha, counter);
  check_dev(ids, "ids");
  // nnz = sum_t B * pooling[t] (the host knows it; pooling lives on the device)
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.numel() == nnz &&
              ids.device() == rows.device(), "synth_ids: ids int64 [nnz]");
  a.ids = ids.data_ptr<int64_t>();
  tdfo::synth_ids(a, cur_stream());
}

void synth_dense(int64_t seed, int64_t rank, int64_t index_base, int64_t B, const Tensor& rows,
                 const Tensor& pooling, const Tensor& base, int64_t dist, double alpha,
                 const Tensor& counter, const Tensor& w_dense, const Tensor& table_bias,
                 const Tensor& x0, const Tensor& label) {
  tdfo::SynthArgs a = synth_in_step_args(seed, rank, index_base, B, rows, pooling, base, dist,
                                         alpha, counter);
  check_dev(x0, "x0"); check_dev(label, "label");
  TORCH_CHECK(x0.scalar_type() == at::kBFloat16 && x0.dim() == 2 && x0.size(0) == B &&
              x0.stride(1) == 1 && x0.size(1) >= w_dense.numel(), "synth_dense: x0 bf16 [B, >= nd]");
  TORCH_CHECK(w_dense.scalar_type() == at::kFloat && w_dense.is_contiguous() &&
              table_bias.scalar_type() == at::kFloat && table_bias.numel() == rows.numel() * 64 &&
              table_bias.is_contiguous() && label.scalar_type() == at::kFloat &&
              label.numel() == B && label.is_contiguous(), "synth_dense: teacher / label");
  for (const Tensor* t : {&w_dense, &table_bias, &x0, &label})
    TORCH_CHECK(t->device() == rows.device(), "synth_dense: one device");
  a.num_dense = (int)w_dense.numel();
  a.w_dense = w_dense.data_ptr<float>(); a.table_bias = table_bias.data_ptr<float>();
  a.x0 = reinterpret_cast<uint16_t*>(x0.data_ptr()); a.ldx = x0.stride(0);
  a.label = label.data_ptr<float>();
  tdfo::synth_dense(a, cur_stream());
}

// ------------------------------------------------------------ loss etc.
void head_bce(const Tensor& H, const Tensor& w, const Tensor& b, const Tensor& label,
              double inv_n, bool relu_mask, const Tensor& logits, const Tensor& dH,
              const Tensor& part) {
  check_dev(H, "H"); check_2d_rowmajor(H, "H"); check_2d_rowmajor(dH, "dH");
  const int64_t B = H.size(0), K = H.size(1);
  TORCH_CHECK(K == 16 || K == 32 || K == 64 || K == 128 || K == 256 || K == 512 || K == 1024,
              "head K unsupported");
  TORCH_CHECK(w.numel() == K && b.numel() == 1 && label.numel() == B && logits.numel() == B, "head shapes");
  TORCH_CHECK(label.scalar_type() == at::kFloat && logits.scalar_type() == at::kFloat, "head fp32 label/logits");
  TORCH_CHECK(dH.size(0) == B && dH.size(1) == K, "dH shape");
  const int nparts = tdfo::head_bce_parts((int)B);
  TORCH_CHECK(part.numel() >= nparts * (K + 2), "part too small");
  tdfo::head_bce(bf16_ptr(H), H.stride(0), (int)B, (int)K, w.data_ptr<float>(), b.data_ptr<float>(),
                 label.data_ptr<float>(), (float)inv_n, relu_mask, logits.data_ptr<float>(),
                 bf16_mut(dH), dH.stride(0), part.data_ptr<float>(), nparts, cur_stream());
}

void head_reduce(const Tensor& part, int64_t nparts, int64_t K, const Tensor& grad,
                 const Tensor& loss_acc, at::TensorList bumps, bool defer) {
  check_f32c(part, "part"); check_f32c(grad, "grad"); check_f32c(loss_acc, "loss_acc");
  TORCH_CHECK(part.numel() >= nparts * (K + 2) && grad.numel() >= K + 1 && loss_acc.numel() >= 1,
              "head_reduce: shapes");
  TORCH_CHECK(bumps.size() <= 4, "head_reduce: at most 4 step counters");
  tdfo::HeadBumps hb{};
  hb.n = (int)bumps.size();
  for (size_t i = 0; i < bumps.size(); ++i) {
    check_f32c(bumps[i], "bump");
    TORCH_CHECK(bumps[i].numel() >= 2, "head_reduce: counters are [lr, step, ...]");
    hb.p[i] = bumps[i].data_ptr<float>();
  }
  if (defer) {
    // run by the next paired 128x128 GEMM launch (flush_side_job otherwise)
    tdfo::head_reduce_park(tdfo::HeadReduceJob{part.data_ptr<float>(), (int)nparts, (int)K,
                                               grad.data_ptr<float>(),
                                               loss_acc.data_ptr<float>(), hb});
    return;
  }
  tdfo::head_reduce(part.data_ptr<float>(), (int)nparts, (int)K, grad.data_ptr<float>(),
                    loss_acc.data_ptr<float>(), hb, cur_stream());
}

void reduce_rows(const Tensor& inp, int64_t rows, int64_t n, int64_t ld, const Tensor& out,
                 bool accumulate, double scale) {
  // it would run ahead of the GEMMs a gemm_batch holds back (wrong order)
  TORCH_CHECK(!g_gemm_batch.on, "reduce_rows inside ops.gemm_batch");
  check_dev(inp, "inp");
  TORCH_CHECK(inp.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat, "fp32");
  TORCH_CHECK(inp.numel() >= (rows - 1) * ld + n && out.numel() >= n, "reduce_rows bounds");
  tdfo::reduce_rows(inp.data_ptr<float>(), (int)rows, n, ld, out.data_ptr<float>(), accumulate,
                    (float)scale, cur_stream());
}

void seg_copy(const Tensor& src, const Tensor& dst, const Tensor& chunks, int64_t src_n,
              int64_t dst_n) {
  check_dev(src, "src"); check_dev(dst, "dst"); check_dev(chunks, "chunks");
  TORCH_CHECK(src.scalar_type() == at::kLong && dst.scalar_type() == at::kLong &&
              chunks.scalar_type() == at::kLong && src.is_contiguous() && dst.is_contiguous() &&
              chunks.is_contiguous() && chunks.dim() == 2 && chunks.size(1) == 3,
              "seg_copy: contiguous int64 src / dst and int64 [n, 3] chunks");
  // the chunk table was bounds-checked on the host against (src_n, dst_n)
  TORCH_CHECK(src.numel() >= src_n && dst.numel() >= dst_n, "seg_copy: buffers smaller than "
              "the extents the segment map was built for");
  tdfo::seg_copy(src.data_ptr<int64_t>(), dst.data_ptr<int64_t>(), chunks.data_ptr<int64_t>(),
                 (int)chunks.size(0), cur_stream());
}

void piece_copy(const Tensor& buf, const Tensor& pieces, int64_t B, int64_t w, int64_t extent) {
  check_dev(buf, "buf"); check_dev(pieces, "pieces");
  TORCH_CHECK(buf.scalar_type() == at::kBFloat16 && buf.is_contiguous() &&
              pieces.scalar_type() == at::kLong && pieces.is_contiguous() && pieces.dim() == 2 &&
              pieces.size(1) == 4 && w % 8 == 0 && aligned16(buf.data_ptr()),
              "piece_copy: contiguous bf16 buffer, int64 [n, 4] pieces, w % 8 == 0");
  // the piece table was bounds- and alignment-checked on the host against extent
  TORCH_CHECK(buf.numel() >= extent, "piece_copy: buffer smaller than its piece table's extent");
  tdfo::piece_copy_bf16(reinterpret_cast<uint16_t*>(buf.data_ptr()), pieces.data_ptr<int64_t>(),
                        (int)pieces.size(0), (int)B, (int)w, cur_stream());
}

void slab_reduce(const std::vector<Tensor>& ins, const std::vector<int64_t>& splits,
                 const std::vector<Tensor>& outs) {
  TORCH_CHECK(!g_gemm_batch.on, "slab_reduce inside ops.gemm_batch");
  TORCH_CHECK(ins.size() == splits.size() && ins.size() == outs.size() &&
              (int)ins.size() <= tdfo::SLAB_MAX_SEGS, "slab_reduce: 1..16 matching segments");
  tdfo::SlabReduceArgs a{};
  a.nseg = (int)ins.size();
  a.start[0] = 0;
  for (int k = 0; k < a.nseg; ++k) {
    const Tensor &in = ins[k], &out = outs[k];
    check_dev(in, "slab"); check_dev(out, "out");
    TORCH_CHECK(in.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat &&
                in.is_contiguous() && out.is_contiguous(), "slab_reduce: contiguous fp32");
    const int64_t n = out.numel(), S = splits[k];
    TORCH_CHECK(S >= 1 && n % 4 == 0 && in.numel() >= S * n && aligned16(in.data_ptr()) &&
                aligned16(out.data_ptr()), "slab_reduce: S >= 1, n % 4, bounds, 16-B alignment");
    a.seg[k] = {in.data_ptr<float>(), out.data_ptr<float>(), n, (int)S};
    a.start[k + 1] = a.start[k] + n / 4;
  }
  tdfo::slab_reduce(a, cur_stream());
}

void colsum(const Tensor& x, const Tensor& out, bool accumulate) {
  check_dev(x, "x"); check_2d_rowmajor(x, "x");
  const int64_t M = x.size(0), N = x.size(1);
  TORCH_CHECK(N % 8 == 0 && x.stride(0) % 8 == 0 && aligned16(x.data_ptr()), "colsum alignment");
  TORCH_CHECK(out.numel() == N && out.scalar_type() == at::kFloat, "colsum out");
  const int np = tdfo::colsum_parts((int)M);
  Tensor part = at::empty({np, N}, out.options());
  tdfo::colsum_bf16(bf16_ptr(x), (int)M, (int)N, x.stride(0), part.data_ptr<float>(), np,
                    out.data_ptr<float>(), accumulate, cur_stream());
}

void auc_hist(const Tensor& logits, const Tensor& labels, int64_t nb, const Tensor& hist) {
  TORCH_CHECK(hist.scalar_type() == at::kLong && hist.numel() == 2 * nb, "hist int64 [2*nb]");
  TORCH_CHECK(logits.numel() == labels.numel(), "auc sizes");
  tdfo::auc_hist(logits.data_ptr<float>(), labels.data_ptr<float>(), (int)logits.numel(), (int)nb,
                 reinterpret_cast<unsigned long long*>(hist.data_ptr<int64_t>()), cur_stream());
}

void two_tower(const Tensor& X, const Tensor& P, const Tensor& labels, double inv_n,
               const Tensor& logits, const c10::optional<Tensor>& dX,
               const c10::optional<Tensor>& part, const c10::optional<Tensor>& loss_scale,
               bool half, at::TensorList bumps, const c10::optional<Tensor>& emb_w,
               const c10::optional<Tensor>& ids, const c10::optional<Tensor>& row_off,
               bool defer) {
  check_dev(X, "X"); check_2d_rowmajor(X, "X");
  const int64_t B = X.size(0);
  TORCH_CHECK(X.scalar_type() == at::kFloat && X.size(1) >= 114 && X.stride(0) % 4 == 0 &&
              aligned16(X.data_ptr()), "two_tower: X fp32 [B, >=114], 16B-aligned rows");
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.numel() >= tdfo::TT_NPARAM &&
              aligned16(P.data_ptr()), "two_tower: P fp32 [>= 2400], 16B-aligned");
  TORCH_CHECK(logits.scalar_type() == at::kFloat && logits.numel() == B, "two_tower: logits");
  tdfo::TwoTowerArgs a{};
  a.X = X.data_ptr<float>(); a.ldx = X.stride(0);
  a.P = P.data_ptr<float>();
  a.B = (int)B; a.inv_n = (float)inv_n;
  a.half = half;
  if (loss_scale) {
    check_dev(*loss_scale, "loss_scale");
    TORCH_CHECK(loss_scale->scalar_type() == at::kFloat && loss_scale->numel() >= 1, "loss_scale fp32");
    a.loss_scale = loss_scale->data_ptr<float>();
  }
  a.logits = logits.data_ptr<float>();
  if (emb_w) {
    // ids / row offsets come from the trainer's own validated buffers (the
    // same ones the lookup kernel it replaces read)
    TORCH_CHECK(ids && row_off, "two_tower: emb_w needs ids and row_off");
    check_f32c(*emb_w, "emb_w"); check_dev(*ids, "ids"); check_dev(*row_off, "row_off");
    TORCH_CHECK(emb_w->dim() == 2 && emb_w->size(1) == 16 && aligned16(emb_w->data_ptr()) &&
                ids->scalar_type() == at::kLong && ids->is_contiguous() && ids->numel() >= 7 * B &&
                row_off->scalar_type() == at::kLong && row_off->is_contiguous() &&
                row_off->numel() >= 7, "two_tower: emb_w [rows, 16] fp32, ids int64 [7 * B], "
                "row_off int64 [7]");
    a.emb_w = emb_w->data_ptr<float>();
    a.ids = ids->data_ptr<int64_t>();
    a.row_off = row_off->data_ptr<int64_t>();
  }
  const bool train = dX.has_value();
  if (train) {
    TORCH_CHECK(part.has_value(), "two_tower: train needs part");
    const Tensor& d = *dX;
    check_2d_rowmajor(d, "dX");
    TORCH_CHECK(d.scalar_type() == at::kFloat && d.size(0) == B && d.size(1) >= 112 &&
                d.stride(0) % 4 == 0 && aligned16(d.data_ptr()), "two_tower: dX");
    TORCH_CHECK(labels.scalar_type() == at::kFloat && labels.numel() == B, "two_tower: labels");
    TORCH_CHECK(part->scalar_type() == at::kFloat &&
                part->numel() >= (int64_t)tdfo::two_tower_parts((int)B) * tdfo::TT_PART_LD &&
                aligned16(part->data_ptr()), "two_tower: part");
    a.labels = labels.data_ptr<float>();
    a.dX = d.data_ptr<float>(); a.lddx = d.stride(0);
    a.part = part->data_ptr<float>();
    TORCH_CHECK(bumps.size() <= 4, "two_tower: at most 4 step counters");
    a.bumps.n = (int)bumps.size();
    for (size_t i = 0; i < bumps.size(); ++i) {
      check_f32c(bumps[i], "bump");
      TORCH_CHECK(bumps[i].numel() >= 2, "two_tower: counters are [lr, step, ...]");
      a.bumps.p[i] = bumps[i].data_ptr<float>();
    }
  } else {
    TORCH_CHECK(bumps.size() == 0, "two_tower: bumps are a train-step option");
  }
  if (defer) {
    TORCH_CHECK(train && !half && !g_tower_pending && !g_side_pending,
                "two_tower(defer): an fp32 train step, parked before its reduce_adam, one at "
                "a time (flush_side_job)");
    g_tower = a;
    g_tower_pending = true;
    return;
  }
  tdfo::two_tower(a, train ? 1 : 0, cur_stream());
}

void reduce_adam(const Tensor& part, int64_t nparts, int64_t n, int64_t ld, const Tensor& grad,
                 const Tensor& p, const Tensor& m, const Tensor& v, const Tensor& hyper,
                 double beta1, double beta2, double eps, double wd, bool adamw,
                 const Tensor& loss_acc, const c10::optional<Tensor>& logits,
                 const c10::optional<Tensor>& labels, int64_t nb,
                 const c10::optional<Tensor>& hist, bool defer) {
  check_f32c(part, "part"); check_f32c(grad, "grad"); check_f32c(p, "p"); check_f32c(m, "m");
  check_f32c(v, "v"); check_f32c(hyper, "hyper");
  check_dev(loss_acc, "loss_acc");
  TORCH_CHECK(loss_acc.scalar_type() == at::kDouble && loss_acc.numel() >= 1,
              "reduce_adam: loss_acc fp64");
  TORCH_CHECK(nparts >= 1 && n >= 1 && ld >= n + 1 && part.numel() >= (nparts - 1) * ld + n + 1 &&
              grad.numel() >= n + 1 && p.numel() >= n && m.numel() >= n && v.numel() >= n &&
              hyper.numel() >= 3, "reduce_adam: shapes");
  tdfo::ReduceAdamArgs a{};
  a.part = part.data_ptr<float>(); a.nparts = (int)nparts; a.n = (int)n; a.ld = (int)ld;
  a.grad = grad.data_ptr<float>(); a.p = p.data_ptr<float>(); a.m = m.data_ptr<float>();
  a.v = v.data_ptr<float>(); a.hyper = hyper.data_ptr<float>();
  a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps; a.wd = (float)wd;
  a.adamw = adamw ? 1 : 0;
  a.loss_acc = loss_acc.data_ptr<double>();
  if (hist) {
    TORCH_CHECK(logits && labels, "reduce_adam: hist needs logits and labels");
    check_f32c(*logits, "logits"); check_f32c(*labels, "labels"); check_dev(*hist, "hist");
    TORCH_CHECK(hist->scalar_type() == at::kLong && hist->is_contiguous() && nb > 0 &&
                nb <= tdfo::REDUCE_ADAM_MAX_NB && hist->numel() == 2 * nb &&
                labels->numel() == logits->numel(), "reduce_adam: hist int64 [2 * nb], nb <= 512");
    a.logits = logits->data_ptr<float>(); a.labels = labels->data_ptr<float>();
    a.nlog = (int)logits->numel(); a.nb = (int)nb;
    a.hist = reinterpret_cast<unsigned long long*>(hist->data_ptr<int64_t>());
  }
  if (defer) {
    TORCH_CHECK(!g_side_pending, "reduce_adam: a deferred job is already waiting for its "
                "embedding_bwd (flush_side_job)");
    g_side = a;
    g_side_pending = true;
    return;
  }
  tdfo::reduce_adam(a, cur_stream());
}

void flush_side_job() {
  tdfo::head_reduce_flush(cur_stream());
  if (g_tower_pending) {             // (before the reduce: it reads the towers' partials)
    g_tower_pending = false;
    tdfo::two_tower(g_tower, 1, cur_stream());
  }
  if (!g_side_pending) return;
  g_side_pending = false;
  tdfo::reduce_adam(g_side, cur_stream());
}

void linear_xent(const Tensor& H, const Tensor& W, const Tensor& bias, const Tensor& labels,
                 double eps, int64_t ignore, const Tensor& dH, const Tensor& lossv,
                 const c10::optional<Tensor>& dW, const c10::optional<Tensor>& db,
                 const c10::optional<Tensor>& loss, const c10::optional<Tensor>& loss_acc,
                 const std::vector<Tensor>& ostate, const c10::optional<Tensor>& ohyper,
                 const std::vector<double>& oparams, int64_t okind) {
  check_dev(H, "H");
  TORCH_CHECK(H.scalar_type() == at::kFloat && H.dim() == 2 && H.size(1) == 16 &&
              H.is_contiguous() && aligned16(H.data_ptr()), "linear_xent: H fp32 [N,16]");
  const int64_t N = H.size(0), V = W.size(0);
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.dim() == 2 && W.size(1) == 16 &&
              W.is_contiguous() && aligned16(W.data_ptr()), "linear_xent: W fp32 [V,16]");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == V && bias.is_contiguous(),
              "linear_xent: bias [V]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == N && labels.is_contiguous(),
              "linear_xent: labels int64 [N]");
  TORCH_CHECK(dH.scalar_type() == at::kFloat && dH.sizes() == H.sizes() && dH.is_contiguous() &&
              aligned16(dH.data_ptr()), "linear_xent: dH");
  TORCH_CHECK(lossv.scalar_type() == at::kFloat && lossv.numel() == N, "linear_xent: lossv");
  TORCH_CHECK(N < (1 << 30) && V < (1ll << 31), "linear_xent: sizes");
  tdfo::LinearXentArgs a{};
  a.H = H.data_ptr<float>(); a.W = W.data_ptr<float>(); a.bias = bias.data_ptr<float>();
  a.labels = labels.data_ptr<int64_t>();
  a.N = (int)N; a.V = V; a.ignore = (int)ignore; a.eps = (float)eps;
  a.dH = dH.data_ptr<float>(); a.lossv = lossv.data_ptr<float>();
  if (dW.has_value()) {
    TORCH_CHECK(db.has_value() && dW->sizes() == W.sizes() && dW->is_contiguous() &&
                dW->scalar_type() == at::kFloat && aligned16(dW->data_ptr()) &&
                db->numel() == V && db->scalar_type() == at::kFloat, "linear_xent: dW/db");
    a.dW = dW->data_ptr<float>(); a.db = db->data_ptr<float>();
  }
  if (loss) {
    check_dev(*loss, "loss");
    TORCH_CHECK(loss->scalar_type() == at::kFloat && loss->numel() >= 1, "linear_xent: loss fp32 [1]");
    a.loss = loss->data_ptr<float>();
  }
  if (loss_acc) {
    check_dev(*loss_acc, "loss_acc");
    TORCH_CHECK(loss && loss_acc->scalar_type() == at::kDouble && loss_acc->numel() >= 1,
                "linear_xent: loss_acc fp64 [1] (with loss)");
    a.loss_acc = loss_acc->data_ptr<double>();
  }
  if (okind >= 0) {
    // fused output-layer step: W / bias updated in place from moments
    // ostate = [mW, vW, mb, vb]; oparams = [beta1, beta2, eps, weight_decay]
    TORCH_CHECK(okind == tdfo::OPT_ADAM || okind == tdfo::OPT_ADAMW, "linear_xent: okind");
    TORCH_CHECK(ostate.size() == 4 && ohyper.has_value() && oparams.size() == 4 &&
                a.dW != nullptr, "linear_xent: fused step needs [mW, vW, mb, vb], hyper, 4 "
                "params and dW / db scratch");
    for (int k = 0; k < 4; ++k) {
      check_dev(ostate[k], "ostate");
      TORCH_CHECK(ostate[k].scalar_type() == at::kFloat && ostate[k].is_contiguous() &&
                  ostate[k].numel() == (k < 2 ? V * 16 : V) && aligned16(ostate[k].data_ptr()),
                  "linear_xent: moments");
    }
    check_dev(*ohyper, "ohyper");
    TORCH_CHECK(ohyper->scalar_type() == at::kFloat && ohyper->numel() >= 3,
                "linear_xent: hyper fp32 [lr, step, grad_scale]");
    TORCH_CHECK(aligned16(bias.data_ptr()), "linear_xent: bias alignment");
    a.okind = (int)okind;
    a.mW = ostate[0].data_ptr<float>(); a.vW = ostate[1].data_ptr<float>();
    a.mb = ostate[2].data_ptr<float>(); a.vb = ostate[3].data_ptr<float>();
    a.ohyper = ohyper->data_ptr<float>();
    a.beta1 = (float)oparams[0]; a.beta2 = (float)oparams[1];
    a.oeps = (float)oparams[2]; a.owd = (float)oparams[3];
  }
  Tensor ws = at::empty({(int64_t)tdfo::linear_xent_workspace((int)N, V)},
                        H.options().dtype(at::kByte));
  a.workspace = ws.data_ptr();
  tdfo::linear_xent(a, cur_stream());
}

void check_offsets(const Tensor& off, int64_t B) {
  check_dev(off, "offsets");
  TORCH_CHECK(off.scalar_type() == at::kLong && off.is_contiguous() && off.numel() == B + 1,
              "offsets must be int64 [B+1]");
}

void jagged_to_dense(const Tensor& values, const Tensor& offsets, int64_t T, double pad,
                     const Tensor& out) {
  check_dev(values, "values");
  const int64_t B = out.size(0);
  check_offsets(offsets, B);
  TORCH_CHECK(values.scalar_type() == at::kFloat && values.dim() == 2 && values.is_contiguous(),
              "values fp32 [nnz, D]");
  const int64_t D = values.size(1);
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 3 &&
              out.size(1) == T && out.size(2) == D, "out fp32 [B, T, D]");
  TORCH_CHECK(D % 4 != 0 || (aligned16(values.data_ptr()) && aligned16(out.data_ptr())),
              "jagged_to_dense alignment");
  tdfo::jagged_to_dense(values.data_ptr<float>(), offsets.data_ptr<int64_t>(), (int)B, (int)T,
                        (int)D, (float)pad, out.data_ptr<float>(), cur_stream());
}

void dense_to_jagged(const Tensor& dense, const Tensor& offsets, const Tensor& vgrad) {
  check_dev(dense, "dense");
  TORCH_CHECK(dense.scalar_type() == at::kFloat && dense.dim() == 3 && dense.is_contiguous(),
              "dense fp32 [B, T, D]");
  const int64_t B = dense.size(0), T = dense.size(1), D = dense.size(2);
  check_offsets(offsets, B);
  TORCH_CHECK(vgrad.scalar_type() == at::kFloat && vgrad.dim() == 2 && vgrad.size(1) == D &&
              vgrad.is_contiguous(), "vgrad fp32 [nnz, D]");
  TORCH_CHECK(D % 4 != 0 || (aligned16(vgrad.data_ptr()) && aligned16(dense.data_ptr())),
              "dense_to_jagged alignment");
  tdfo::dense_to_jagged(dense.data_ptr<float>(), offsets.data_ptr<int64_t>(), (int)B, (int)T,
                        (int)D, vgrad.size(0), vgrad.data_ptr<float>(), cur_stream());
}

void jagged_ids_to_dense(const Tensor& values, const Tensor& offsets, int64_t pad,
                         const Tensor& out) {
  check_dev(values, "values");
  TORCH_CHECK(values.scalar_type() == at::kLong && values.is_contiguous(), "ids int64");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.dim() == 2 && out.is_contiguous(),
              "out int64 [B, T]");
  const int64_t B = out.size(0), T = out.size(1);
  check_offsets(offsets, B);
  tdfo::jagged_ids_to_dense(values.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(), (int)B,
                            (int)T, pad, out.data_ptr<int64_t>(), cur_stream());
}

}  // namespace

TORCH_LIBRARY(tdfo, m) {
  m.def("gemm(Tensor a, bool a_col, Tensor b, bool b_col, Tensor? bias, bool relu, Tensor? mask, "
        "Tensor(a!)? out, Tensor(b!)? out32, int splits, Tensor? mul=None, Tensor? add=None, "
        "Tensor(c!)? out2=None, int ldc32=0, int csum_col=-1) -> ()");
  m.def("radix_sort_sep_hist(int v) -> int",
        [](int64_t v) { return (int64_t)tdfo::radix_sort_sep_hist((int)v); });
  m.def("sync_event_create(int mode) -> int", sync_event_create);
  m.def("stamp(Tensor(a!) buf, Tensor(b!) cnt, int seg, int nseg, int which) -> ()",
        [](const Tensor& buf, const Tensor& cnt, int64_t seg, int64_t nseg, int64_t which) {
    TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kLong && cnt.is_cuda() &&
                cnt.scalar_type() == at::kLong && seg >= 0 && seg < cnt.numel() &&
                seg < nseg && (which == 0 || which == 1), "stamp: int64 GPU buffers");
    tdfo::stamp(reinterpret_cast<uint64_t*>(buf.data_ptr()), cnt.data_ptr<int64_t>(), (int)seg,
                (int)nseg, (int)which, buf.numel(), cur_stream());
  });
  m.def("bump(Tensor[] counters) -> ()", [](const std::vector<Tensor>& ts) {
    TORCH_CHECK(ts.size() <= 8, "bump: at most 8 counters");
    tdfo::BumpArgs a{};
    for (const auto& t : ts) {
      TORCH_CHECK(t.is_cuda() && t.numel() >= 1 &&
                  (t.scalar_type() == at::kFloat || t.scalar_type() == at::kLong),
                  "bump: float32 / int64 GPU counters");
      a.p[a.n] = t.data_ptr();
      a.is_i64[a.n] = t.scalar_type() == at::kLong;
      ++a.n;
    }
    tdfo::bump(a, cur_stream());
  });
  m.def("spin_us(float us) -> ()", [](double us) {
    static const double ticks_per_us = [] {
      int dev = 0, khz = 0;
      TDFO_HIP_OK(hipGetDevice(&dev));
      TDFO_HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
      return khz > 0 ? khz / 1000.0 : 100.0;
    }();
    tdfo::spin_ticks(us > 0 ? (uint64_t)(us * ticks_per_us) : 0, cur_stream());
  });
  m.def("burn_us(float us) -> ()", [](double us) {
    int dev = 0, khz = 0, cus = 0;
    TDFO_HIP_OK(hipGetDevice(&dev));
    TDFO_HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    TDFO_HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const double tpu = khz > 0 ? khz / 1000.0 : 100.0;
    tdfo::burn_ticks(us > 0 ? (uint64_t)(us * tpu) : 0, 2 * cus, cur_stream());
  });
  m.def("host_mailbox_alloc(int n) -> Tensor", host_mailbox_alloc);
  m.def("host_publish(Tensor value, Tensor(a!) seq, Tensor host, int slot) -> ()", host_publish);
  m.def("sync_event_record(int e, int stream=-1) -> ()", sync_event_record);
  m.def("copy_on(Tensor(a!) dst, Tensor src, int stream=-1) -> ()", copy_on);
  m.def("sync_event_wait(int e, int stream=-1) -> ()", sync_event_wait);
  m.def("sync_event_destroy(int e) -> ()", sync_event_destroy);
  m.def("sync_event_query(int e) -> bool", sync_event_query);
  m.def("graph_compose(int[] kinds, int[] handles) -> int", graph_compose);
  m.def("graph_exec_launch(int ex, int stream=-1) -> ()", graph_exec_launch);
  m.def("graph_exec_destroy(int ex) -> ()", graph_exec_destroy);
  m.def("graph_num_nodes(int g) -> int", graph_num_nodes);
  m.def("graph_exec_upload(int ex) -> ()", graph_exec_upload);
  m.def("gemm_batch_begin() -> ()", gemm_batch_begin);
  m.def("gemm_batch_end() -> ()", gemm_batch_end);
  m.def("gemm_pairing(int v) -> int",
        [](int64_t v) { return (int64_t)tdfo::gemm_pairing((int)v); });
  m.def("radix_sort_tiled(int v) -> int",
        [](int64_t v) { return (int64_t)tdfo::radix_sort_tiled((int)v); });
  m.def("radix_sort_max_bits(int b) -> int",
        [](int64_t v) { return (int64_t)tdfo::radix_sort_max_bits((int)v); });
  m.def("gemm_policy(int p) -> int", [](int64_t p) { return (int64_t)tdfo::gemm_policy((int)p); });
  m.def("embedding_segsort(int v) -> int",
        [](int64_t v) { return (int64_t)tdfo::embedding_segsort((int)v); });
  m.def("linear_xent_impl(int p) -> int",
        [](int64_t p) { return (int64_t)tdfo::linear_xent_impl((int)p); });
  m.def("encoder_param_count(int E, int FF) -> int",
        [](int64_t E, int64_t FF) { return (int64_t)tdfo::encoder_param_count((int)E, (int)FF); });
  m.def("encoder_layer_supported(int T, int E, int H, int FF) -> bool",
        [](int64_t T, int64_t E, int64_t H, int64_t FF) {
          return tdfo::encoder_layer_supported((int)T, (int)E, (int)H, (int)FF);
        });
  m.def("encoder_layer_fwd(Tensor x, Tensor ids, Tensor? step, Tensor[] params, int H, float rate, "
        "int seed, int pad_id, float eps, Tensor(a!)[] saved, Tensor(b!) y) -> ()");
  m.def("encoder_layer_bwd(Tensor x, Tensor ids, Tensor? step, Tensor[] params, int H, float rate, "
        "int seed, int pad_id, float eps, Tensor[] saved, Tensor dy, Tensor(a!) dx, "
        "Tensor(b!) part, Tensor(c!) grad, Tensor? gidx, bool defer=False) -> ()");
  m.def("encoder_reduce_flush() -> ()", encoder_reduce_flush);
  m.def("attention_fwd(Tensor qkv, Tensor ids, int H, float rate, int seed, Tensor? step, int pad_id, "
        "Tensor(a!) out) -> ()");
  m.def("attention_bwd(Tensor qkv, Tensor ids, Tensor dout, int H, float rate, int seed, Tensor? step, "
        "int pad_id, Tensor(a!) dqkv) -> ()");
  m.def("layernorm_fwd(Tensor x, int n, float eps, Tensor gamma, Tensor beta, Tensor(a!) y, "
        "Tensor(b!) mean, Tensor(c!) rstd) -> ()");
  m.def("layernorm_bwd(Tensor x, Tensor g, int n, Tensor gamma, Tensor mean, Tensor rstd, "
        "Tensor(a!) dx, Tensor(b!) part, Tensor(c!) dgb) -> ()");
  m.def("seq_prologue_fwd(Tensor x, Tensor pos, int n, float eps, Tensor gamma, Tensor beta, "
        "float rate, int seed, Tensor? step, Tensor(a!) y, Tensor(b!) mean, Tensor(c!) rstd) -> ()");
  m.def("seq_prologue_bwd(Tensor x, Tensor pos, Tensor g, int n, Tensor gamma, Tensor mean, "
        "Tensor rstd, float rate, int seed, Tensor? step, Tensor(a!) dx, Tensor(b!) part, "
        "Tensor(c!) out3, Tensor? gidx) -> ()");
  m.def("rank_metrics(Tensor h, Tensor W, Tensor bias, Tensor cand, int[] ks, Tensor(a!) out) -> ()");
  m.def("layernorm_parts(int M) -> int", [](int64_t M) { return (int64_t)tdfo::layernorm_parts(M); });
  m.def("gather_columns(Tensor[] src, Tensor? idx, int row0, int n, Tensor(a!)[] dst, int[] dst_stride) -> ()");
  m.def("concat_features(Tensor dense, Tensor emb, int[] off, int[] stride, int F, int D, "
        "Tensor(a!) out) -> ()");
  m.def("split_features(Tensor dx, int F, int D, Tensor dense, Tensor(a!) d_dense, "
        "Tensor(b!) d_emb, int[] doff, int[] dstride, bool relu_mask) -> ()");
  m.def("cross_bwd(Tensor dout, Tensor x0, Tensor y, Tensor(a!) dy, Tensor(b!) dx0, "
        "bool accumulate, bool add_dout) -> ()");
  m.def("interaction_fwd(Tensor dense, Tensor emb, int[] off, int[] stride, int F, int D, Tensor(a!) out, "
        "int ones_col=-1) -> ()");
  m.def("interaction_bwd(Tensor dz, Tensor dense, Tensor emb, int[] off, int[] stride, int F, int D, "
        "Tensor(a!) d_dense, Tensor(b!) d_emb, int[] doff, int[] dstride, bool relu_mask) -> ()");
  m.def("embedding_bag_fwd(Tensor W, Tensor row_offset, Tensor indices, Tensor offsets, Tensor out_off, "
        "Tensor? psw, int T, int B, bool mean, Tensor(a!) out, int out_stride, bool onehot, "
        "Tensor(b!)[] bumps) -> ()");
  m.def("embedding_bwd(Tensor(a!) W, Tensor row_offset, Tensor indices, Tensor offsets, Tensor grad_off, "
        "Tensor? psw, int T, int B, bool mean, int key_bits, Tensor grad, int grad_stride, int opt, "
        "Tensor(b!)? state1, Tensor(c!)? state2, Tensor hyper, float eps, float beta1, float beta2, "
        "float weight_decay, Tensor(d!)? dense_grad, int segsort) -> ()");
  m.def("embedding_bwd_workspace(int nnz, int D) -> int", [](int64_t nnz, int64_t D) {
    return (int64_t)tdfo::embedding_bwd_workspace(nnz < 1 ? 1 : nnz, (int)D);
  });
  m.def("embedding_bwd_prepare(Tensor W, Tensor row_offset, Tensor indices, Tensor offsets, "
        "Tensor grad_off, Tensor? psw, int T, int B, bool mean, int key_bits, int grad_stride, "
        "int segsort, Tensor(a!) workspace, Tensor? bag_len=None) -> ()");
  m.def("embedding_bwd_apply(Tensor(a!) W, Tensor row_offset, Tensor indices, Tensor offsets, "
        "Tensor grad_off, Tensor? psw, int T, int B, bool mean, int key_bits, Tensor grad, "
        "int grad_stride, int opt, Tensor(b!)? state1, Tensor(c!)? state2, Tensor hyper, "
        "float eps, float beta1, float beta2, float weight_decay, Tensor(d!)? dense_grad, "
        "int segsort, Tensor(e!) workspace) -> ()");
  m.def("embedding_dense_update(Tensor(a!) W, Tensor(d!) grad, int rows, int opt, Tensor(b!)? state1, "
        "Tensor(c!)? state2, Tensor hyper, float eps, float beta1, float beta2, "
        "float weight_decay, bool clear_grad) -> ()");
  m.def("rw_bucketize_workspace(int n, int W) -> int", rw_bucketize_workspace);
  m.def("rw_bucketize(Tensor ids, Tensor meta, int nrw, int W, int B, int cap, int n, "
        "Tensor(a!) send, Tensor(b!) workspace, Tensor(c!) overflow) -> ()");
  m.def("rw_pool(Tensor Wt, Tensor recv, Tensor meta, int nrw, int W, int B, int cap, bool mean, "
        "Tensor(a!) starts, Tensor(b!) out, int out_ld) -> ()");
  m.def("embedding_bwd_prepare_rw(Tensor W, Tensor recv, Tensor meta, int nrw, int Wsz, int B, "
        "int cap, bool mean, int key_bits, int grad_ld, int dummy_row, Tensor(a!) workspace, "
        "int rows=0) -> ()");
  m.def("rw_rows_gather(Tensor Wt, Tensor recv, int W, int cap, Tensor(a!) out) -> ()");
  m.def("bottom_mlp_fwd_ok(int k0, int n0, int n1, int n2) -> bool", bottom_mlp_fwd_ok);
  m.def("bottom_mlp_fwd(Tensor x, Tensor w0, Tensor w1, Tensor w2, Tensor? b0, Tensor? b1, "
        "Tensor? b2, Tensor(a!) y0, Tensor(b!) y1, Tensor(c!) y2, Tensor? dense, Tensor? label_src, "
        "Tensor(d!)? label_dst) -> ()");
  m.def("rw_rows_scatter(Tensor send, int W, int cap, int B, int D, Tensor rows, Tensor(a!) region, "
        "int ld, Tensor(b!) map, int nrw) -> ()");
  m.def("rw_grads_gather(Tensor map, int W, int cap, int D, Tensor dregion, Tensor(a!) gsend) -> ()");
  m.def("embedding_bwd_apply_rw(Tensor(a!) W, int Wsz, int B, int cap, bool mean, int key_bits, "
        "Tensor grad, int opt, Tensor(b!)? state1, Tensor(c!)? state2, Tensor hyper, float eps, "
        "float beta1, float beta2, float weight_decay, Tensor(d!) workspace) -> ()");
  m.def("dense_optimizer(Tensor(a!) p, Tensor g, Tensor(b!)? m, Tensor(c!)? v, Tensor(d!)? p_bf16, int opt, "
        "Tensor hyper, float beta1, float beta2, float eps, float wd, float momentum, Tensor? found_inf, "
        "Tensor[] seg_slabs, int[] seg_start, int[] seg_splits) -> ()");
  m.def("check_finite(Tensor g, Tensor(a!) found) -> ()");
  m.def("sort_pairs(Tensor keys, Tensor vals, int key_bits) -> (Tensor, Tensor)");
  m.def("cast_bf16(Tensor x, Tensor(a!) y) -> ()");
  m.def("synth_criteo(int seed, int rank, int batch_index, int B, Tensor rows, Tensor pooling, "
        "Tensor base, int dist, float alpha, Tensor w_dense, Tensor table_bias, Tensor(a!) dense, "
        "Tensor(b!) ids, Tensor(c!) label) -> ()");
  m.def("synth_ids(int seed, int rank, int index_base, int B, Tensor rows, Tensor pooling, "
        "Tensor base, int dist, float alpha, Tensor counter, int nnz, Tensor(a!) ids) -> ()");
  m.def("synth_dense(int seed, int rank, int index_base, int B, Tensor rows, Tensor pooling, "
        "Tensor base, int dist, float alpha, Tensor counter, Tensor w_dense, Tensor table_bias, "
        "Tensor(a!) x0, Tensor(b!) label) -> ()");
  m.def("batch_load(Tensor dense, Tensor(a!) x0, Tensor ids, Tensor(b!) ids_dst, Tensor label, "
        "Tensor(c!) label_dst) -> ()");
  m.def("head_bce(Tensor H, Tensor w, Tensor b, Tensor label, float inv_n, bool relu_mask, "
        "Tensor(a!) logits, Tensor(b!) dH, Tensor(c!) part) -> ()");
  m.def("head_reduce(Tensor part, int nparts, int K, Tensor(a!) grad, Tensor(b!) loss_acc, "
        "Tensor(c!)[] bumps, bool defer) -> ()");
  m.def("reduce_rows(Tensor inp, int rows, int n, int ld, Tensor(a!) out, bool accumulate, float scale) -> ()");
  m.def("colsum(Tensor x, Tensor(a!) out, bool accumulate) -> ()");
  m.def("slab_reduce(Tensor[] slabs, int[] splits, Tensor(a!)[] outs) -> ()");
  m.def("seg_copy(Tensor src, Tensor(a!) dst, Tensor chunks, int src_n, int dst_n) -> ()");
  m.def("piece_copy(Tensor(a!) buf, Tensor pieces, int B, int w, int extent) -> ()");
  m.def("auc_hist(Tensor logits, Tensor labels, int nb, Tensor(a!) hist) -> ()");
  m.def("linear_xent(Tensor H, Tensor W, Tensor bias, Tensor labels, float eps, int ignore, "
        "Tensor(a!) dH, Tensor(b!) lossv, Tensor(c!)? dW, Tensor(d!)? db, Tensor(e!)? loss, "
        "Tensor(f!)? loss_acc, Tensor(g!)[] ostate, Tensor? ohyper, float[] oparams, "
        "int okind) -> ()");
  m.def("jagged_to_dense(Tensor values, Tensor offsets, int T, float pad, Tensor(a!) out) -> ()");
  m.def("dense_to_jagged(Tensor dense, Tensor offsets, Tensor(a!) vgrad) -> ()");
  m.def("jagged_ids_to_dense(Tensor values, Tensor offsets, int pad, Tensor(a!) out) -> ()");
  m.def("two_tower(Tensor X, Tensor P, Tensor labels, float inv_n, Tensor(a!) logits, "
        "Tensor(b!)? dX, Tensor(c!)? part, Tensor? loss_scale, bool half, "
        "Tensor(d!)[] bumps, Tensor? emb_w, Tensor? ids, Tensor? row_off, bool defer) -> ()");
  m.def("reduce_adam(Tensor part, int nparts, int n, int ld, Tensor(a!) grad, Tensor(b!) p, "
        "Tensor(c!) m, Tensor(d!) v, Tensor hyper, float beta1, float beta2, float eps, "
        "float wd, bool adamw, Tensor(e!) loss_acc, Tensor? logits, Tensor? labels, int nb, "
        "Tensor(f!)? hist, bool defer) -> ()");
  m.def("flush_side_job() -> ()", flush_side_job);
}

TORCH_LIBRARY_IMPL(tdfo, CUDA, m) {
  m.impl("gemm", gemm);
  m.impl("attention_fwd", attention_fwd);
  m.impl("encoder_layer_fwd", encoder_layer_fwd);
  m.impl("encoder_layer_bwd", encoder_layer_bwd);
  m.impl("attention_bwd", attention_bwd);
  m.impl("layernorm_fwd", layernorm_fwd);
  m.impl("layernorm_bwd", layernorm_bwd);
  m.impl("seq_prologue_fwd", seq_prologue_fwd);
  m.impl("rank_metrics", rank_metrics);
  m.impl("seq_prologue_bwd", seq_prologue_bwd);
  m.impl("gather_columns", gather_columns);
  m.impl("concat_features", concat_features);
  m.impl("batch_load", batch_load);
  m.impl("synth_criteo", synth_criteo);
  m.impl("split_features", split_features);
  m.impl("cross_bwd", cross_bwd);
  m.impl("interaction_fwd", interaction_fwd);
  m.impl("interaction_bwd", interaction_bwd);
  m.impl("embedding_bag_fwd", embedding_bag_fwd);
  m.impl("embedding_bwd", embedding_bwd);
  m.impl("embedding_bwd_prepare", embedding_bwd_prepare);
  m.impl("embedding_bwd_apply", embedding_bwd_apply);
  m.impl("embedding_dense_update", embedding_dense_update);
  m.impl("rw_bucketize", rw_bucketize);
  m.impl("rw_pool", rw_pool);
  m.impl("embedding_bwd_prepare_rw", embedding_bwd_prepare_rw);
  m.impl("rw_rows_gather", rw_rows_gather);
  m.impl("bottom_mlp_fwd", bottom_mlp_fwd);
  m.impl("rw_rows_scatter", rw_rows_scatter);
  m.impl("rw_grads_gather", rw_grads_gather);
  m.impl("embedding_bwd_apply_rw", embedding_bwd_apply_rw);
  m.impl("dense_optimizer", dense_optimizer);
  m.impl("check_finite", check_finite);
  m.impl("sort_pairs", sort_pairs);
  m.impl("cast_bf16", cast_bf16);
  m.impl("slab_reduce", slab_reduce);
  m.impl("synth_ids", synth_ids);
  m.impl("synth_dense", synth_dense);
  m.impl("seg_copy", seg_copy);
  m.impl("piece_copy", piece_copy);
  m.impl("head_bce", head_bce);
  m.impl("reduce_rows", reduce_rows);
  m.impl("head_reduce", head_reduce);
  m.impl("colsum", colsum);
  m.impl("auc_hist", auc_hist);
  m.impl("two_tower", two_tower);
  m.impl("reduce_adam", reduce_adam);
  m.impl("linear_xent", linear_xent);
  m.impl("jagged_to_dense", jagged_to_dense);
  m.impl("dense_to_jagged", dense_to_jagged);
  m.impl("jagged_ids_to_dense", jagged_ids_to_dense);
}
