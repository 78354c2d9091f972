// RCCL communicator engine for elastic data parallelism over xGMI.
//
// Replaces the NCCL data plane that Horovod drives inside the reference's user
// containers (hvd.DistributedOptimizer in
// examples/py/pytorch/pytorch_mnist_elastic.py:185-188).  Design points:
//   * one communicator per (job, membership epoch): the 128-byte unique id is published
//     through the job's rendezvous store by the epoch's rank 0, every member calls
//     init_rank; on resize the old communicator is finalized (or aborted when a member
//     died) and a new one is built — RCCL communicators are static.
//   * communicators are created NON-BLOCKING (ncclConfig_t.blocking = 0) so that init and
//     every enqueue can be bounded by a timeout and a hung peer turns into an error
//     instead of a wedged process; abort() can be called from a watchdog thread.
//   * collectives are enqueued on the caller's HIP stream (the DDP engine passes its
//     dedicated comm stream), so they overlap backward compute on the compute stream.
#include "host_common.h"
#include "ops.h"

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>

namespace voda {

static ncclDataType_t to_nccl_dtype(int dt) {
  switch (dt) {
    case kF32: return ncclFloat32;
    case kBF16: return ncclBfloat16;
    case kF16: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    default: throw std::invalid_argument("unsupported dtype for RCCL");
  }
}

static ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclProd;
    default: throw std::invalid_argument("unsupported reduction op");
  }
}

static void nccl_throw(ncclResult_t r, const char* what) {
  throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r) + " (" +
                           (ncclGetLastError(nullptr) ? ncclGetLastError(nullptr) : "") + ")");
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) nccl_throw(r, "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

RcclComm::RcclComm(const std::string& uid, int nranks, int rank, int device, double timeout_s, bool wait)
    : nranks_(nranks), rank_(rank), timeout_s_(timeout_s) {
  VODA_CHECK(uid.size() == sizeof(ncclUniqueId), "unique id must be 128 bytes");
  VODA_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
  if (device >= 0) VODA_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) nccl_throw(r, "ncclCommInitRankConfig");
  if (wait) wait_ready("init");
}

template <typename F>
int RcclComm::locked_call(F&& f) {
  std::lock_guard<std::mutex> g(mu_);
  check_live();
  return static_cast<int>(f());
}

bool RcclComm::poll_ready() {
  std::lock_guard<std::mutex> g(mu_);
  check_live();
  ncclResult_t st = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError(comm_, &st);
  if (r != ncclSuccess) nccl_throw(r, "ncclCommGetAsyncError");
  if (st == ncclSuccess) return true;
  if (st == ncclInProgress) return false;
  aborted_ = true;
  nccl_throw(st, "init");
  return false;
}

RcclComm::~RcclComm() {
  std::lock_guard<std::mutex> g(mu_);
  if (comm_ != nullptr) {
    // destructor must not throw; abort is the only call that never blocks on peers
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::wait_ready(const char* what) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  int spins = 0;
  while (true) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (comm_ == nullptr || aborted_) throw std::runtime_error(std::string("RCCL ") + what + ": communicator aborted");
      ncclResult_t st = ncclSuccess;
      ncclResult_t r = ncclCommGetAsyncError(comm_, &st);
      if (r != ncclSuccess) nccl_throw(r, "ncclCommGetAsyncError");
      if (st == ncclSuccess) return;
      if (st != ncclInProgress) {
        aborted_ = true;
        nccl_throw(st, what);
      }
      if (timeout_s_ > 0 && std::chrono::duration<double>(clock::now() - t0).count() > timeout_s_) {
        ncclCommAbort(comm_);
        comm_ = nullptr;
        aborted_ = true;
        throw std::runtime_error(std::string("RCCL ") + what + " timed out");
      }
    }
    // lock released between polls: a watchdog abort() can get in
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclComm::check_live() const {
  if (comm_ == nullptr || aborted_) throw std::runtime_error("RCCL communicator is aborted/destroyed");
}

void RcclComm::finish(int r_, const char* what) {
  const ncclResult_t r = static_cast<ncclResult_t>(r_);
  if (r == ncclSuccess) return;
  if (r == ncclInProgress) {
    wait_ready(what);
    return;
  }
  nccl_throw(r, what);
}

void RcclComm::allreduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
  const ncclDataType_t dt = to_nccl_dtype(dtype);
  const ncclRedOp_t rop = to_nccl_op(op);
  finish(locked_call([&] {
           return ncclAllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count), dt,
                                rop, comm_, as_stream(stream));
         }),
         "allreduce");
}

void RcclComm::broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream) {
  const ncclDataType_t dt = to_nccl_dtype(dtype);
  finish(locked_call([&] {
           return ncclBroadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count), dt,
                                root, comm_, as_stream(stream));
         }),
         "broadcast");
}

void RcclComm::allgather(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream) {
  const ncclDataType_t dt = to_nccl_dtype(dtype);
  finish(locked_call([&] {
           return ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count), dt,
                                comm_, as_stream(stream));
         }),
         "allgather");
}

void RcclComm::reduce_scatter(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
  const ncclDataType_t dt = to_nccl_dtype(dtype);
  const ncclRedOp_t rop = to_nccl_op(op);
  finish(locked_call([&] {
           return ncclReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count),
                                    dt, rop, comm_, as_stream(stream));
         }),
         "reduce_scatter");
}

void RcclComm::alltoall(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream) {
  const ncclDataType_t dt = to_nccl_dtype(dtype);
  finish(locked_call([&] {
           return ncclAllToAll(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count), dt,
                               comm_, as_stream(stream));
         }),
         "alltoall");
}

void RcclComm::group_start() { finish(ncclGroupStart(), "group_start"); }
void RcclComm::group_end() {
  ncclResult_t r = ncclGroupEnd();
  if (r == ncclInProgress) {
    wait_ready("group_end");
    return;
  }
  if (r != ncclSuccess) nccl_throw(r, "group_end");
}

std::string RcclComm::async_error() const {
  std::lock_guard<std::mutex> g(mu_);
  if (comm_ == nullptr) return aborted_ ? "aborted" : "destroyed";
  ncclResult_t st = ncclSuccess;
  ncclCommGetAsyncError(comm_, &st);
  if (st == ncclSuccess || st == ncclInProgress) return "";
  return ncclGetErrorString(st);
}

void RcclComm::abort() {
  // Safe from a watchdog thread: waits for any in-progress NCCL call on this communicator
  // (all of them return promptly in non-blocking mode), then aborts -- kernels of this
  // communicator spinning on a dead peer observe the abort flag and exit.
  aborted_ = true;
  std::lock_guard<std::mutex> g(mu_);
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::destroy() {
  std::unique_lock<std::mutex> g(mu_);
  if (comm_ == nullptr) return;
  ncclResult_t r = ncclCommFinalize(comm_);
  g.unlock();
  if (r == ncclInProgress) {
    try {
      wait_ready("finalize");
    } catch (...) {
      // wait_ready aborted the communicator on timeout / abort
      return;
    }
  }
  g.lock();
  if (comm_ != nullptr) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  aborted_ = true;  // no longer usable
}

}  // namespace voda
