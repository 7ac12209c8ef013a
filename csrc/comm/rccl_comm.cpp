// Native collective layer over RCCL (torch.ops.tdfo.rccl_*).
//
// the sharded engine's exchanges (pooled-embedding / id
// all-to-alls, row-wise reduce-scatter / all-gathers, the bucketed
// dense-gradient all-reduce) issued straight from C++ on a communicator of
// our own, instead of through c10d's per-call Python + work-object path
// (~25-37 us of host time per collective, profiles/r03/emu/rccl_cost.log).
// The role of the reference's DMP input/output dists and DDP reducer
// (torchrec/train.py:241-260), built for one process per MI355X over xGMI.
//
// Every op is enqueued on a stream and never blocks the host, so a whole
// multi-rank training step -- collectives included -- can be captured into
// ONE hipGraph and replayed with a single launch per step:
//
//  * async_op=false: the collective runs on the caller's current stream;
//  * async_op=true: it is forked onto the communicator's own stream (event
//    record on the caller's stream + wait on the comm stream) and a token is
//    returned; rccl_wait(token) orders the caller's current stream after it.
//    Under stream capture the fork / join become graph edges.
//
// All collectives of one communicator are serialised on its stream in issue
// order, which is identical on every rank (the NCCL ordering contract).
// Buffers must stay alive until the collective has run (the trainers own
// static buffers; nothing is allocated here per call).
//
// The library is the RCCL torch itself links (torch/lib/librccl.so, found via
// this library's rpath), so there is one RCCL in the process.
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/library.h>

namespace {

using at::Tensor;

#define TDFO_NCCL_OK(x)                                                                   \
  do {                                                                                    \
    ncclResult_t r_ = (x);                                                                \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error in " #x ": ", ncclGetErrorString(r_));     \
  } while (0)
#define TDFO_HIPC_OK(x)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    TORCH_CHECK(e_ == hipSuccess, "HIP error in " #x ": ", hipGetErrorString(e_));        \
  } while (0)

constexpr int kSlots = 256;   // in-flight async collectives per communicator

struct Communicator {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0, device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t fork[kSlots], done[kSlots];
  int next = 0;
  int64_t calls = 0, bytes = 0;
};

std::mutex g_mu;
std::vector<std::unique_ptr<Communicator>> g_comms;

Communicator& get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h], "rccl: bad communicator ", h);
  return *g_comms[h];
}

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

ncclDataType_t nccl_type(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
}

void check_buf(const Communicator& c, const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "rccl: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "rccl: ", name, " must be contiguous");
  TORCH_CHECK(t.get_device() == c.device, "rccl: ", name, " is on device ", t.get_device(),
              ", the communicator on ", c.device);
}

// Stream for one collective: the caller's (sync) or the comm stream forked
// off it (async; returns the slot of the token).
hipStream_t begin(Communicator& c, bool async_op, int* slot) {
  hipStream_t s = cur_stream();
  if (!async_op) {
    *slot = -1;
    return s;
  }
  const int k = c.next;
  c.next = (c.next + 1) % kSlots;
  TDFO_HIPC_OK(hipEventRecord(c.fork[k], s));
  TDFO_HIPC_OK(hipStreamWaitEvent(c.stream, c.fork[k], 0));
  *slot = k;
  return c.stream;
}

int64_t end(Communicator& c, int slot, int64_t nbytes) {
  c.calls += 1;
  c.bytes += nbytes;
  if (slot < 0) return -1;
  TDFO_HIPC_OK(hipEventRecord(c.done[slot], c.stream));
  return slot;
}

Tensor rccl_unique_id() {
  ncclUniqueId id;
  TDFO_NCCL_OK(ncclGetUniqueId(&id));
  Tensor t = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), id.internal, NCCL_UNIQUE_ID_BYTES);
  return t;
}

int64_t rccl_init(const Tensor& id, int64_t world, int64_t rank) {
  TORCH_CHECK(id.device().is_cpu() && id.scalar_type() == at::kByte &&
              id.numel() == NCCL_UNIQUE_ID_BYTES, "rccl_init: id must be a CPU uint8[128]");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl_init: bad rank ", rank, "/", world);
  auto c = std::make_unique<Communicator>();
  TDFO_HIPC_OK(hipGetDevice(&c->device));
  c->world = (int)world;
  c->rank = (int)rank;
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  TDFO_NCCL_OK(ncclCommInitRank(&c->comm, (int)world, uid, (int)rank));
  // default priority: high-priority streams slowed the multi-stream step
  // ~3x (models/dlrm_multirank.py)
  TDFO_HIPC_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (int k = 0; k < kSlots; ++k) {
    TDFO_HIPC_OK(hipEventCreateWithFlags(&c->fork[k], hipEventDisableTiming));
    TDFO_HIPC_OK(hipEventCreateWithFlags(&c->done[k], hipEventDisableTiming));
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size() - 1;
}

void rccl_destroy(int64_t h) {
  std::unique_ptr<Communicator> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h], "rccl: bad communicator ", h);
    c = std::move(g_comms[h]);
  }
  TDFO_HIPC_OK(hipStreamSynchronize(c->stream));
  TDFO_NCCL_OK(ncclCommDestroy(c->comm));
  for (int k = 0; k < kSlots; ++k) {
    TDFO_HIPC_OK(hipEventDestroy(c->fork[k]));
    TDFO_HIPC_OK(hipEventDestroy(c->done[k]));
  }
  TDFO_HIPC_OK(hipStreamDestroy(c->stream));
}

void rccl_wait(int64_t h, int64_t token) {
  if (token < 0) return;
  Communicator& c = get(h);
  TORCH_CHECK(token < kSlots, "rccl_wait: bad token ", token);
  TDFO_HIPC_OK(hipStreamWaitEvent(cur_stream(), c.done[token], 0));
}

// out[slot r] = what rank r sends here; inp[slot r] goes to rank r. Splits
// in elements (empty: equal split).
int64_t rccl_all_to_all(int64_t h, const Tensor& out, const Tensor& inp,
                        std::vector<int64_t> out_splits, std::vector<int64_t> in_splits,
                        bool async_op) {
  Communicator& c = get(h);
  check_buf(c, out, "out");
  check_buf(c, inp, "inp");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type(), "rccl_all_to_all: dtype mismatch");
  const int W = c.world;
  const bool equal = out_splits.empty() && in_splits.empty();
  if (out_splits.empty()) {
    TORCH_CHECK(out.numel() % W == 0, "rccl_all_to_all: out not divisible by world");
    out_splits.assign(W, out.numel() / W);
  }
  if (in_splits.empty()) {
    TORCH_CHECK(inp.numel() % W == 0, "rccl_all_to_all: inp not divisible by world");
    in_splits.assign(W, inp.numel() / W);
  }
  TORCH_CHECK((int)out_splits.size() == W && (int)in_splits.size() == W, "rccl_all_to_all: splits");
  std::vector<size_t> sc(W), sd(W), rc(W), rd(W);
  int64_t so = 0, ro = 0;
  for (int r = 0; r < W; ++r) {
    TORCH_CHECK(in_splits[r] >= 0 && out_splits[r] >= 0, "rccl_all_to_all: negative split");
    sc[r] = (size_t)in_splits[r]; sd[r] = (size_t)so; so += in_splits[r];
    rc[r] = (size_t)out_splits[r]; rd[r] = (size_t)ro; ro += out_splits[r];
  }
  TORCH_CHECK(so == inp.numel() && ro == out.numel(), "rccl_all_to_all: splits do not sum to sizes");
  int slot;
  hipStream_t s = begin(c, async_op, &slot);
  const ncclDataType_t dt = nccl_type(inp);
  bool uniform = equal;
  if (!uniform) {
    uniform = true;
    for (int r = 0; r < W; ++r) uniform &= (sc[r] == sc[0] && rc[r] == sc[0]);
  }
  if (uniform)
    TDFO_NCCL_OK(ncclAllToAll(inp.data_ptr(), out.data_ptr(), sc[0], dt, c.comm, s));
  else
    TDFO_NCCL_OK(ncclAllToAllv(inp.data_ptr(), sc.data(), sd.data(), out.data_ptr(), rc.data(),
                               rd.data(), dt, c.comm, s));
  return end(c, slot, inp.numel() * inp.element_size());
}

ncclRedOp_t red_op(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    default: TORCH_CHECK(false, "rccl: unknown reduction ", op);
  }
}

int64_t rccl_all_reduce(int64_t h, const Tensor& t, int64_t op, bool async_op) {
  Communicator& c = get(h);
  check_buf(c, t, "t");
  int slot;
  hipStream_t s = begin(c, async_op, &slot);
  TDFO_NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_type(t),
                             red_op(op), c.comm, s));
  return end(c, slot, t.numel() * t.element_size());
}

// out = sum over ranks of their inp chunk [rank] (equal chunks, sum).
int64_t rccl_reduce_scatter(int64_t h, const Tensor& out, const Tensor& inp, bool async_op) {
  Communicator& c = get(h);
  check_buf(c, out, "out");
  check_buf(c, inp, "inp");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type(), "rccl_reduce_scatter: dtype mismatch");
  TORCH_CHECK(inp.numel() == out.numel() * c.world, "rccl_reduce_scatter: inp must be W x out");
  int slot;
  hipStream_t s = begin(c, async_op, &slot);
  TDFO_NCCL_OK(ncclReduceScatter(inp.data_ptr(), out.data_ptr(), (size_t)out.numel(),
                                 nccl_type(inp), ncclSum, c.comm, s));
  return end(c, slot, inp.numel() * inp.element_size());
}

// out = concat over ranks of inp (rank-major).
int64_t rccl_all_gather(int64_t h, const Tensor& out, const Tensor& inp, bool async_op) {
  Communicator& c = get(h);
  check_buf(c, out, "out");
  check_buf(c, inp, "inp");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type(), "rccl_all_gather: dtype mismatch");
  TORCH_CHECK(out.numel() == inp.numel() * c.world, "rccl_all_gather: out must be W x inp");
  int slot;
  hipStream_t s = begin(c, async_op, &slot);
  TDFO_NCCL_OK(ncclAllGather(inp.data_ptr(), out.data_ptr(), (size_t)inp.numel(), nccl_type(inp),
                             c.comm, s));
  return end(c, slot, out.numel() * out.element_size());
}

void rccl_broadcast(int64_t h, const Tensor& t, int64_t root) {
  Communicator& c = get(h);
  check_buf(c, t, "t");
  TORCH_CHECK(root >= 0 && root < c.world, "rccl_broadcast: bad root ", root);
  TDFO_NCCL_OK(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_type(t),
                             (int)root, c.comm, cur_stream()));
  c.calls += 1;
  c.bytes += t.numel() * t.element_size();
}

std::vector<int64_t> rccl_info(int64_t h) {
  Communicator& c = get(h);
  return {c.world, c.rank, c.device, c.calls, c.bytes};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tdfo, m) {
  m.def("rccl_unique_id() -> Tensor", rccl_unique_id);
  m.def("rccl_init(Tensor id, int world, int rank) -> int", rccl_init);
  m.def("rccl_destroy(int h) -> ()", rccl_destroy);
  m.def("rccl_wait(int h, int token) -> ()", rccl_wait);
  m.def("rccl_all_to_all(int h, Tensor(a!) out, Tensor inp, int[] out_splits, int[] in_splits, "
        "bool async_op) -> int", rccl_all_to_all);
  m.def("rccl_all_reduce(int h, Tensor(a!) t, int op, bool async_op) -> int", rccl_all_reduce);
  m.def("rccl_reduce_scatter(int h, Tensor(a!) out, Tensor inp, bool async_op) -> int",
        rccl_reduce_scatter);
  m.def("rccl_all_gather(int h, Tensor(a!) out, Tensor inp, bool async_op) -> int",
        rccl_all_gather);
  m.def("rccl_broadcast(int h, Tensor(a!) t, int root) -> ()", rccl_broadcast);
  m.def("rccl_info(int h) -> int[]", rccl_info);
}
