// qpb_workspace.hip -- cached device scratch for the kernels that need one
// (the n <= 128 Gram kernel's spilled rows and work queue, the reference
// replicas' matrices at 64 < n <= 128).
//
// One buffer per (device, stream), grown on demand and never shrunk: a solve
// reuses it instead of a hipMallocAsync / hipFreeAsync pair per call.  Work on
// one stream runs in order, so a buffer handed to consecutive launches on the
// same stream is never used by two of them at once; different streams get
// different buffers.  Growing frees the old buffer stream-ordered (after the
// launches already queued on that stream).
//
// The buffer is only ever handed to a callback that queues its launches
// while the entry's lock is held (qpb_with_workspace): two host threads
// sharing a stream (the null stream, say) cannot have one grow -- free --
// the buffer between the other's lookup and its launch.  Each (device,
// stream) entry has its own lock; the map's lock is held only for the lookup,
// so launches on unrelated streams do not wait for each other.  A stream must be
// released (qpb_release_stream_workspace, or qpb_release_workspaces) before
// the caller destroys it: the cache frees its buffers stream-ordered on it.
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <utility>

#include "qpb_common.h"  // qpb_with_workspace's declaration

namespace {
struct Entry {
  std::mutex mu;  // held while the buffer is grown and the launch is queued
  void *p = nullptr;
  size_t bytes = 0;
  bool dead = false;  // released and erased from the map: look the stream up again
};
std::mutex g_mu;  // the map itself
std::map<std::pair<int, hipStream_t>, std::shared_ptr<Entry>> g_ws;

// frees one entry's buffer stream-ordered on its stream and waits for it; the
// caller holds the entry's lock
bool free_entry(int dev, hipStream_t st, Entry &w) {
  if (!w.p) {
    w.dead = true;
    return true;
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(dev);
  const bool ok = hipFreeAsync(w.p, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
  (void)hipSetDevice(cur);
  w.p = nullptr;
  w.bytes = 0;
  w.dead = true;
  return ok;
}
}  // namespace

hipError_t qpb_with_workspace(hipStream_t stream, size_t bytes, const std::function<hipError_t(void *)> &launch) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  // A release may free and erase the entry between the lookup and the entry's
  // lock: it then marks the entry dead, and the lookup is repeated (a dead
  // entry is in no map, so a buffer allocated through it would never be freed)
  std::shared_ptr<Entry> sp;
  std::unique_lock<std::mutex> lock;
  for (;;) {
    {
      std::lock_guard<std::mutex> ml(g_mu);
      auto &slot = g_ws[{dev, stream}];
      if (!slot) slot = std::make_shared<Entry>();
      sp = slot;
    }
    lock = std::unique_lock<std::mutex>(sp->mu);
    if (!sp->dead) break;
    lock.unlock();
  }
  Entry &w = *sp;
  if (w.bytes < bytes) {
    if (w.p) (void)hipFreeAsync(w.p, stream);
    w.p = nullptr;
    w.bytes = 0;
    // round up to 1 MiB so that a slowly growing batch does not reallocate every call
    const size_t want = (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    e = hipMallocAsync(&w.p, want, stream);
    if (e != hipSuccess) {
      w.p = nullptr;
      return e;
    }
    w.bytes = want;
  }
  return launch(w.p);  // queued on `stream` before any other thread can touch w
}

extern "C" int qpb_release_stream_workspace(void *stream) {
  const hipStream_t st = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(g_mu);
  int failed = 0;
  for (auto it = g_ws.begin(); it != g_ws.end();) {
    if (it->first.second != st) {
      ++it;
      continue;
    }
    {
      std::lock_guard<std::mutex> el(it->second->mu);  // waits for a launch being queued
      if (!free_entry(it->first.first, st, *it->second)) ++failed;
    }
    it = g_ws.erase(it);
  }
  return failed ? -3 : 0;  // QPB_ERR_HIP
}

extern "C" int qpb_release_workspaces(void) {
  std::lock_guard<std::mutex> lock(g_mu);
  int failed = 0;
  for (auto &kv : g_ws) {
    std::lock_guard<std::mutex> el(kv.second->mu);
    if (!free_entry(kv.first.first, kv.first.second, *kv.second)) ++failed;
  }
  g_ws.clear();
  return failed ? -3 : 0;  // QPB_ERR_HIP
}
