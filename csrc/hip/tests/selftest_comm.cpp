// Sanitizer self-test of the RCCL communicator engine's host state machine (csrc/hip/comm.cpp)
// against a fake non-blocking RCCL: init polling, enqueue + progress polling, timeouts, and a
// watchdog thread aborting a communicator while other threads are enqueueing / waiting on it.
// Built with g++ -fsanitize=address,undefined or -fsanitize=thread by
// tests/test_native_sanitize.py; the scheduler's elastic runtime relies on exactly this path
// (runtime/elastic.py watcher -> RcclCommunicator.abort()).
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ops.h"

// ------------------------------------------------------------------ fake RCCL
struct ncclComm {
  std::atomic<int> init_polls{3};     // polls until init completes
  std::atomic<long> pending{0};       // polls until the last enqueued operation completes
  std::atomic<bool> fail{false};
  int magic = 0x5eed;
};
static std::atomic<long> g_hang{0};   // >0: next collectives stay in progress for that many polls

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) { std::memset(id, 7, sizeof(*id)); return ncclSuccess; }
ncclResult_t ncclGetVersion(int* v) { *v = 99999; return ncclSuccess; }
const char* ncclGetErrorString(ncclResult_t) { return "fake"; }
const char* ncclGetLastError(ncclComm_t) { return ""; }
ncclResult_t ncclCommInitRankConfig(ncclComm_t* c, int, ncclUniqueId, int, ncclConfig_t*) {
  *c = new ncclComm();
  return ncclInProgress;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* st) {
  if (c->magic != 0x5eed) std::abort();  // use after free would also be caught by ASan
  if (c->fail) { *st = ncclRemoteError; return ncclSuccess; }
  if (c->init_polls > 0) { --c->init_polls; *st = ncclInProgress; return ncclSuccess; }
  if (c->pending > 0) { --c->pending; *st = ncclInProgress; return ncclSuccess; }
  *st = ncclSuccess;
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t c) { c->magic = 0; delete c; return ncclSuccess; }
ncclResult_t ncclCommFinalize(ncclComm_t c) { c->pending = 2; return ncclInProgress; }
ncclResult_t ncclCommDestroy(ncclComm_t c) { c->magic = 0; delete c; return ncclSuccess; }
static ncclResult_t enqueue(ncclComm_t c) {
  if (c->magic != 0x5eed) std::abort();
  long h = g_hang.load();
  c->pending = h > 0 ? h : 2;
  return ncclInProgress;
}
ncclResult_t ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t c, hipStream_t) { return enqueue(c); }
ncclResult_t ncclBroadcast(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t c, hipStream_t) { return enqueue(c); }
ncclResult_t ncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t c, hipStream_t) { return enqueue(c); }
ncclResult_t ncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t c, hipStream_t) { return enqueue(c); }
ncclResult_t ncclAllToAll(const void*, void*, size_t, ncclDataType_t, ncclComm_t c, hipStream_t) { return enqueue(c); }
ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

// ------------------------------------------------------------------ scenarios
#define EXPECT(c) do { if (!(c)) { std::printf("FAILED %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static std::string uid() { return std::string(128, '\7'); }

int main() {
  using voda::RcclComm;
  // 1. init polling + collectives completing after in-progress polls + clean destroy
  {
    RcclComm c(uid(), 2, 0, -1, 10.0, false);
    int polls = 0;
    while (!c.poll_ready()) ++polls;
    EXPECT(polls == 3);
    for (int i = 0; i < 100; ++i) c.allreduce(0, 0, 16, 0, 1, 0);
    c.broadcast(0, 0, 16, 0, 0, 0);
    c.allgather(0, 0, 16, 1, 0);
    EXPECT(c.alive());
    c.destroy();
    EXPECT(!c.alive());
    bool threw = false;
    try { c.allreduce(0, 0, 1, 0, 0, 0); } catch (const std::runtime_error&) { threw = true; }
    EXPECT(threw);
  }
  // 2. a watchdog aborts while the owner waits on a collective that never completes
  {
    RcclComm c(uid(), 2, 0, -1, 60.0, true);
    g_hang = 1L << 40;
    std::atomic<bool> threw{false};
    std::thread owner([&] {
      try { c.allreduce(0, 0, 16, 0, 1, 0); } catch (const std::runtime_error&) { threw = true; }
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    c.abort();
    owner.join();
    g_hang = 0;
    EXPECT(threw.load());
    EXPECT(!c.alive());
    c.abort();  // idempotent
  }
  // 3. abort racing with 8 threads enqueueing and polling
  for (int rep = 0; rep < 20; ++rep) {
    RcclComm c(uid(), 8, 3, -1, 60.0, true);
    std::atomic<int> errors{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&] {
        for (int i = 0; i < 200; ++i) {
          try {
            c.allreduce(0, 0, 8, 0, 0, 0);
            (void)c.async_error();
          } catch (const std::runtime_error&) { ++errors; break; }
        }
      });
    std::this_thread::sleep_for(std::chrono::microseconds(200 * (rep % 5)));
    c.abort();
    for (auto& t : ts) t.join();
    EXPECT(!c.alive());
  }
  // 4. a collective that never completes times out and aborts the communicator
  {
    RcclComm c(uid(), 2, 1, -1, 0.05, true);
    g_hang = 1L << 40;
    bool threw = false;
    try { c.allreduce(0, 0, 16, 0, 1, 0); } catch (const std::runtime_error& e) {
      threw = std::string(e.what()).find("timed out") != std::string::npos;
    }
    g_hang = 0;
    EXPECT(threw && !c.alive());
  }
  // 5. an asynchronous peer failure surfaces as an error
  {
    RcclComm c(uid(), 2, 0, -1, 10.0, true);
    EXPECT(c.async_error().empty());
  }
  std::printf("selftest OK\n");
  return 0;
}
