// Native RCCL communicator for the bucketed gradient reducer.
//
// Reference: the reference reduces gradients through DDP's NCCL reducer
// (multi_gpu_trainer.py:88 DistributedDataParallel, :128 backward hooks) and
// broadcasts the initial weights through DDP's constructor (X2 in SURVEY §2.5).
// Here the train engine (train/engine.py) owns one ncclComm_t per process:
//
// * bootstrap: rank 0 draws the ncclUniqueId (comm_unique_id), the Python
//   side ships its 128 bytes through the torch.distributed TCPStore, every rank
//   calls comm_init (ncclCommInitRank on its own device);
// * collectives are enqueued directly on the CALLER's current HIP stream (the
//   engine's communication stream), so they are captured into the step's
//   hipGraph like any kernel, with no ProcessGroup work objects, internal
//   streams or cross-stream events in between;
// * the bf16 wire format packs the fp32 gradient range into a bf16 scratch
//   range (comm_wire.hip), all-reduces ncclBfloat16 in place and unpacks back:
//   three graph nodes per bucket instead of the cast/copy chain, half the xGMI
//   bytes.
//
// RCCL is the one PyTorch already loaded (torch/lib/librccl.so, linked by the
// same name), so there is a single RCCL instance in the process.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "kernels.h"

using at::Tensor;

namespace {

std::mutex g_mu;
std::vector<ncclComm_t> g_comms;  // handle -> communicator (nullptr once destroyed)

#define NCCL_CHECK(cmd)                                                                         \
  do {                                                                                          \
    ncclResult_t r_ = (cmd);                                                                    \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", (int)r_, " (", ncclGetErrorString(r_), ") at ", \
                #cmd);                                                                          \
  } while (0)

ncclComm_t get_comm(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "invalid communicator handle ", h);
  return g_comms[h];
}

ncclDataType_t nccl_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
}

ncclRedOp_t nccl_op(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    default: TORCH_CHECK(false, "reduce op must be 0 (sum), 1 (max) or 2 (min)");
  }
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_buf(const Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "communicator buffers must be GPU tensors");
  TORCH_CHECK(t.is_contiguous(), "communicator buffers must be contiguous");
}

Tensor comm_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  auto out = at::empty({(int64_t)sizeof(id.internal)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr<uint8_t>(), id.internal, sizeof(id.internal));
  return out;
}

// ncclCommInitRank blocks until every rank has joined and the transports are up; a
// rank whose peers never arrive (or a transport setup that never completes) would
// block the process forever.  The init runs on a helper thread and the caller waits
// at most timeout_ms (0: no bound): on timeout this raises "comm_init timed out" and
// the caller falls back to torch.distributed's communicator.  The helper thread is
// detached and left behind (there is no handle to abort before the init returns);
// comm_init_leaked() counts them.  A nonblocking communicator (config.blocking = 0)
// would give an abortable handle, but it also makes every later RCCL call
// asynchronous -- group launches from an RCCL thread -- which a thread-local
// hipGraph capture of the step cannot record.
// test_hang (testing only): the helper thread sleeps past the bound instead of
// initialising (exercises the timeout / fallback path on one rank).
struct InitJob {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  ncclResult_t res = ncclSuccess;
  ncclComm_t comm = nullptr;
};
std::atomic<int> g_init_leaked{0};

int64_t comm_init(Tensor uid, int64_t world, int64_t rank, int64_t device, int64_t timeout_ms, bool test_hang) {
  TORCH_CHECK(!uid.is_cuda() && uid.scalar_type() == at::kByte && uid.numel() == NCCL_UNIQUE_ID_BYTES,
              "uid must be a CPU uint8 tensor of ", NCCL_UNIQUE_ID_BYTES, " bytes");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "bad world/rank");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr<uint8_t>(), sizeof(id.internal));
  auto job = std::make_shared<InitJob>();
  const int dev = (int)device, nr = (int)world, r = (int)rank;
  const int64_t sleep_ms = test_hang ? std::max<int64_t>(2 * timeout_ms, 1000) : 0;
  std::thread th([job, id, dev, nr, r, sleep_ms]() {
    ncclComm_t comm = nullptr;
    ncclResult_t res = ncclSuccess;
    if (sleep_ms > 0) {
      std::this_thread::sleep_for(std::chrono::milliseconds(sleep_ms));
      res = ncclInternalError;
    } else {
      (void)hipSetDevice(dev);
      res = ncclCommInitRank(&comm, nr, id, r);
    }
    std::lock_guard<std::mutex> lk(job->mu);
    job->res = res;
    job->comm = comm;
    job->done = true;
    job->cv.notify_all();
  });
  bool done;
  {
    std::unique_lock<std::mutex> lk(job->mu);
    if (timeout_ms > 0)
      done = job->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return job->done; });
    else {
      job->cv.wait(lk, [&] { return job->done; });
      done = true;
    }
  }
  if (!done) {
    th.detach();
    g_init_leaked.fetch_add(1);
    TORCH_CHECK(false, "comm_init timed out after ", timeout_ms, " ms (rank ", rank, " of ", world,
                "): ncclCommInitRank did not return");
  }
  th.join();
  TORCH_CHECK(job->res == ncclSuccess, "RCCL error ", (int)job->res, " (", ncclGetErrorString(job->res),
              ") at ncclCommInitRank");
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(job->comm);
  return (int64_t)g_comms.size() - 1;
}

int64_t comm_init_leaked() { return g_init_leaked.load(); }

// In-place all-reduce of a contiguous GPU buffer on the current stream.
void comm_all_reduce_(Tensor buf, int64_t h, int64_t op) {
  check_buf(buf);
  const c10::DeviceGuard guard(buf.device());
  NCCL_CHECK(ncclAllReduce(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), nccl_dtype(buf), nccl_op(op),
                           get_comm(h), cur_stream()));
}

// Several in-place all-reduces as ONE RCCL group (one fused launch instead of one per
// buffer): a gradient bucket whose range is split around the time-embedding rows no
// sample can select is two ranges of one arena
void comm_all_reduce_many_(std::vector<Tensor> bufs, int64_t h, int64_t op) {
  TORCH_CHECK(!bufs.empty(), "all_reduce_many: no buffers");
  for (const auto& b : bufs) check_buf(b);
  const c10::DeviceGuard guard(bufs[0].device());
  ncclComm_t c = get_comm(h);
  hipStream_t s = cur_stream();
  NCCL_CHECK(ncclGroupStart());
  for (const auto& b : bufs)
    NCCL_CHECK(ncclAllReduce(b.data_ptr(), b.data_ptr(), (size_t)b.numel(), nccl_dtype(b), nccl_op(op), c, s));
  NCCL_CHECK(ncclGroupEnd());
}

// In-place SUM all-reduce of an fp32 range over a bf16 wire:
// pack fp32 -> bf16 scratch, all-reduce bf16, unpack back into the fp32 range.
void comm_all_reduce_bf16_wire_(Tensor buf, Tensor scratch, int64_t h) {
  check_buf(buf);
  check_buf(scratch);
  TORCH_CHECK(buf.scalar_type() == at::kFloat && scratch.scalar_type() == at::kBFloat16, "fp32 buf, bf16 scratch");
  TORCH_CHECK(scratch.numel() >= buf.numel(), "scratch too small");
  TORCH_CHECK(((uintptr_t)buf.data_ptr() % 16) == 0 && ((uintptr_t)scratch.data_ptr() % 16) == 0,
              "wire buffers must be 16-B aligned");
  const c10::DeviceGuard guard(buf.device());
  const int64_t n = buf.numel();
  hipStream_t s = cur_stream();
  wire_pack_launch(buf.data_ptr<float>(), scratch.data_ptr(), n, s);
  NCCL_CHECK(ncclAllReduce(scratch.data_ptr(), scratch.data_ptr(), (size_t)n, ncclBfloat16, ncclSum, get_comm(h), s));
  wire_unpack_launch(scratch.data_ptr(), buf.data_ptr<float>(), n, s);
}

// out[r * n : (r + 1) * n] = rank r's `in` (n = in.numel()), on the current stream
// (the sparse time-embedding gradient exchange: (t, row) pairs of every rank)
void comm_all_gather_(Tensor out, Tensor in, int64_t h) {
  check_buf(out);
  check_buf(in);
  TORCH_CHECK(out.scalar_type() == in.scalar_type(), "all_gather: dtype mismatch");
  int n = 0;
  ncclComm_t c = get_comm(h);
  NCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(out.numel() == in.numel() * n, "all_gather: out must hold world x in.numel() elements");
  const c10::DeviceGuard guard(in.device());
  NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), c, cur_stream()));
}

void comm_broadcast_(Tensor buf, int64_t h, int64_t root) {
  check_buf(buf);
  const c10::DeviceGuard guard(buf.device());
  NCCL_CHECK(ncclBroadcast(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), nccl_dtype(buf), (int)root,
                           get_comm(h), cur_stream()));
}

std::tuple<int64_t, int64_t> comm_info(int64_t h) {
  int n = 0, r = 0;
  ncclComm_t c = get_comm(h);
  NCCL_CHECK(ncclCommCount(c, &n));
  NCCL_CHECK(ncclCommUserRank(c, &r));
  return {n, r};
}

void comm_destroy(int64_t h) {
  ncclComm_t c = get_comm(h);
  NCCL_CHECK(ncclCommDestroy(c));
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms[h] = nullptr;
}

// ---- external graph events (the engine's event-split step, engine.py comm_events)
// A compute graph records one event per gradient bucket as an event-record node
// appended to the capture by hand (hipGraphAddEventRecordNode on the capturing
// stream's current dependencies, which then become that node): the graph stays a
// single chain, and the host-issued collectives on the comm stream wait on those
// events after the replay is enqueued.  (torch.cuda.Event(external=True) is refused
// on ROCm builds, and hipEventRecordWithFlags(.., hipEventRecordExternal) returns
// invalid-argument inside a capture on this runtime.)
#define HIP_CHECK(cmd)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (cmd);                                                               \
    TORCH_CHECK(e_ == hipSuccess, "HIP error ", hipGetErrorString(e_), " at ", #cmd);    \
  } while (0)

// flags: extra hipEventCreateWithFlags bits on top of hipEventDisableTiming, e.g.
// hipEventReleaseToDevice (device-scope release: visible to the comm queue of the
// same GPU, which is all the bucket's collective needs) or hipEventDisableSystemFence
// -- the default system-scope fence writes back AND invalidates the L2s, and the
// compute kernels after it refill them.
int64_t event_create(int64_t flags) {
  hipEvent_t ev;
  HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | static_cast<unsigned>(flags)));
  return reinterpret_cast<int64_t>(ev);
}

void event_record_external(int64_t ev) {
  hipStream_t s = c10::hip::getCurrentHIPStream().stream();
  hipEvent_t e = reinterpret_cast<hipEvent_t>(ev);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &st, nullptr, &g, &deps, &nd));
  if (st != hipStreamCaptureStatusActive) {
    HIP_CHECK(hipEventRecord(e, s));
    return;
  }
  std::vector<hipGraphNode_t> dv(deps, deps + nd);
  hipGraphNode_t node;
  HIP_CHECK(hipGraphAddEventRecordNode(&node, g, dv.data(), dv.size(), e));
  HIP_CHECK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
}

void stream_wait_event(int64_t ev) {
  HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), reinterpret_cast<hipEvent_t>(ev), 0));
}

void event_destroy(int64_t ev) { HIP_CHECK(hipEventDestroy(reinterpret_cast<hipEvent_t>(ev))); }

// ---- counter hand-off (engine.py comm_signal="flag"): the compute graph bumps a
// per-bucket uint32 counter with a kernel node; the comm stream waits until the
// counter reaches the replay number (wait-value packet, >=).
void flag_bump(Tensor flags, int64_t k) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.is_contiguous(), "flags: int32 cuda");
  TORCH_CHECK(k >= 0 && k < flags.numel(), "flag index out of range");
  flag_bump_launch(flags.data_ptr(), (int)k, c10::hip::getCurrentHIPStream().stream());
}

void stream_wait_flag(Tensor flags, int64_t k, int64_t value) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.is_contiguous(), "flags: int32 cuda");
  TORCH_CHECK(k >= 0 && k < flags.numel(), "flag index out of range");
  HIP_CHECK(hipStreamWaitValue32(c10::hip::getCurrentHIPStream().stream(),
                                 reinterpret_cast<uint32_t*>(flags.data_ptr<int>() + k),
                                 static_cast<uint32_t>(value), hipStreamWaitValueGte, 0xFFFFFFFFu));
}

// the same wait as a 1-lane polling kernel of ours (bounded, raises err[0] on timeout)
void flag_wait(Tensor flags, int64_t k, int64_t value, Tensor err, int64_t timeout_us) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.is_contiguous(), "flags: int32 cuda");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 1, "err: int32 cuda");
  TORCH_CHECK(k >= 0 && k < flags.numel(), "flag index out of range");
  flag_wait_launch(flags.data_ptr(), (int)k, static_cast<unsigned int>(value), err.data_ptr(),
                   c10::hip::getCurrentHIPStream().stream(), timeout_us);
}

// in-process loopback all-reduce (LoopbackPair): endpoint e of two, on the current stream
void pair_all_reduce_(Tensor buf, Tensor stage, Tensor flags, int64_t e, Tensor err, int64_t timeout_us) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kFloat && buf.is_contiguous(), "buf: fp32 cuda contiguous");
  TORCH_CHECK(stage.is_cuda() && stage.scalar_type() == at::kFloat && stage.is_contiguous() && stage.dim() == 2 &&
                  stage.size(0) == 2 && stage.size(1) >= buf.numel(),
              "stage: [2, >= numel] fp32");
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.numel() >= pair_allreduce_flags(),
              "flags: int32 cuda, pair_allreduce_flags() entries");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 1, "err: int32 cuda");
  TORCH_CHECK(e == 0 || e == 1, "endpoint must be 0 or 1");
  TORCH_CHECK(buf.device() == stage.device() && buf.device() == flags.device() && buf.device() == err.device(),
              "one device");
  pair_allreduce_launch(buf.data_ptr<float>(), buf.numel(), stage.data_ptr<float>(), stage.size(1), flags.data_ptr(),
                        (int)e, err.data_ptr(), timeout_us, c10::hip::getCurrentHIPStream().stream());
}

int64_t pair_flags_size() { return pair_allreduce_flags(); }

bool stream_wait_value_supported(int64_t device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, (int)device) != hipSuccess) return false;
  return v != 0;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ddim_cold, m) {
  m.def("event_create(int flags=0) -> int", &event_create);
  m.def("event_record_external(int event) -> ()", &event_record_external);
  m.def("stream_wait_event(int event) -> ()", &stream_wait_event);
  m.def("event_destroy(int event) -> ()", &event_destroy);
  m.def("flag_bump(Tensor(a!) flags, int k) -> ()", &flag_bump);
  m.def("stream_wait_flag(Tensor flags, int k, int value) -> ()", &stream_wait_flag);
  m.def("stream_wait_value_supported(int device) -> bool", &stream_wait_value_supported);
  m.def("flag_wait(Tensor flags, int k, int value, Tensor(a!) err, int timeout_us=0) -> ()", &flag_wait);
  m.def("pair_all_reduce_(Tensor(a!) buf, Tensor(b!) stage, Tensor(c!) flags, int e, Tensor(d!) err, "
        "int timeout_us=0) -> ()", &pair_all_reduce_);
  m.def("pair_flags_size() -> int", &pair_flags_size);
  m.def("comm_unique_id() -> Tensor", &comm_unique_id);
  m.def("comm_init(Tensor uid, int world, int rank, int device, int timeout_ms=0, bool test_hang=False) -> int",
        &comm_init);
  m.def("comm_init_leaked() -> int", &comm_init_leaked);
  m.def("comm_all_reduce_(Tensor(a!) buf, int handle, int op=0) -> ()", &comm_all_reduce_);
  m.def("comm_all_reduce_many_(Tensor(a!)[] bufs, int handle, int op=0) -> ()", &comm_all_reduce_many_);
  m.def("comm_all_reduce_bf16_wire_(Tensor(a!) buf, Tensor(b!) scratch, int handle) -> ()",
        &comm_all_reduce_bf16_wire_);
  m.def("comm_broadcast_(Tensor(a!) buf, int handle, int root=0) -> ()", &comm_broadcast_);
  m.def("comm_all_gather_(Tensor(a!) out, Tensor inp, int handle) -> ()", &comm_all_gather_);
  m.def("comm_info(int handle) -> (int, int)", &comm_info);
  m.def("comm_destroy(int handle) -> ()", &comm_destroy);
}
