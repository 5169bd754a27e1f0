// Deferred IPC launches of ProcessGroupMI355X (IpcLauncher, process_group.h): the
// zero-copy record exchange of an IPC call runs on a per-device helper thread, so the
// caller's host never lines up with its peers' (the gradient all-reduce of a training
// step -- the use the reference motivates, README.md:5 -- overlaps with backward).
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include "../device/comm_util.h"
#include "process_group.h"

namespace pdcc {

// The exchange channel of the thread running a launcher job (nullptr on callers' threads):
// ipc_zero_copy exchanges through it instead of the group's shm(), which the caller's
// thread keeps using for CPU collectives meanwhile.
thread_local host::ShmComm* tls_xchg = nullptr;

bool capturing_stream(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

bool ProcessGroupMI355X::zc_exchanges(DeviceState& ds, Algo a, Coll c, size_t bytes) const {
  if (!is_ipc(a) || !ds.zc_ok || !cfg_.ipc_zc || bytes < cfg_.ipc_zc_min) return false;
  if (ds.ll_ok && bytes_in_ll_range(bytes)) return false;
  // the (all-)reduce and broadcast take the zero-copy path with their 2-shot protocols only
  if ((c == Coll::ALLREDUCE || c == Coll::REDUCE || c == Coll::BROADCAST) && bytes <= cfg_.ipc_1shot_max)
    return false;
  return c != Coll::SEND && c != Coll::RECV && c != Coll::BARRIER;
}

IpcLauncher& ProcessGroupMI355X::launcher(DeviceState& ds) {
  std::lock_guard<std::mutex> lk(init_mu_);
  if (ds.launcher) return *ds.launcher;
  auto L = std::make_unique<IpcLauncher>();
  c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)ds.device);
  L->zs = c10::hip::getStreamFromPoolMasqueradingAsCUDA(/*isHighPriority=*/false, (c10::DeviceIndex)ds.device);
  L->done = ds.sync->alloc();
  TORCH_CHECK(L->done, "pdcc: the IPC launcher needs signal memory (hipMallocSignalMemory)");
  L->thr = std::thread([this, p = &ds, l = L.get()] { launcher_loop(p, l); });
  ds.launcher = std::move(L);
  return *ds.launcher;
}

void ProcessGroupMI355X::launcher_loop(DeviceState* dsp, IpcLauncher* lp) {
  DeviceState& ds = *dsp;
  IpcLauncher& L = *lp;
  // the caller's thread may capture a graph while this one opens mappings / grows staging
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipSetDevice(ds.device);
  // never a device-synchronising release on this thread (streams wait for its launches)
  IpcComm::set_thread_defers_frees(true);
  for (;;) {
    IpcLauncher::Job job;
    {
      std::unique_lock<std::mutex> lk(L.mu);
      L.cv.wait(lk, [&] { return L.stop || !L.q.empty(); });
      if (L.q.empty()) return;  // stop, nothing left
      job = std::move(L.q.front());
      L.q.pop_front();
      L.busy = true;
    }
    const hipStream_t zs = L.zs->stream();
    if (cfg_.log_level >= 3) fprintf(stderr, "[pdcc r%d] launcher: job %llu start\n", rank_, (unsigned long long)job.ticket);
    std::string err;
    try {
      if (!L.shm) {  // collective: every rank's helper builds it at its first job
        host::ShmConfig sc;
        sc.slot_bytes = 64u << 10;  // records only
        sc.spin_us = cfg_.shm_spin_us;
        sc.chan_bytes = 4096;
        sc.timeout = timeout_;
        L.shm = std::make_unique<host::ShmComm>(store_, "pdcc/shm_xchg", rank_, size_, sc);
      }
      if (health_->poisoned.load()) throw std::runtime_error(health_->message());
      PDCC_HIP(hipStreamWaitValue64(zs, job.ready, job.ready_tick, hipStreamWaitValueGte, ~0ull));
      c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)ds.device);
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(*L.zs);
      tls_xchg = L.shm.get();
      job.fn(zs);
      tls_xchg = nullptr;
    } catch (const std::exception& e) {
      tls_xchg = nullptr;
      err = e.what();
    }
    if (!err.empty()) {
      // the streams waiting for this job must not hang: poison the group (every later
      // collective and wait() raises), stop IPC kernels in flight, then release the ticket
      fprintf(stderr, "[pdcc r%d] IPC launcher job failed: %s\n", rank_, err.c_str());
      health_->poison("IPC launcher job failed: " + err);
      if (ds.ipc) ds.ipc->abort();
    }
    (void)hipStreamWriteValue64(zs, L.done, job.ticket, 0);
    if (cfg_.log_level >= 3) fprintf(stderr, "[pdcc r%d] launcher: job %llu launched\n", rank_, (unsigned long long)job.ticket);
    {
      std::lock_guard<std::mutex> lk(L.mu);
      L.busy = false;
      ++L.jobs;
      if (!err.empty() && L.error.empty()) L.error = err;
      if (L.q.empty()) L.idle_cv.notify_all();
    }
  }
}

void ProcessGroupMI355X::ipc_issue(DeviceState& ds, Algo a, hipStream_t s, bool exchanges,
                                   std::function<void(hipStream_t)> fn) {
  if (!is_ipc(a) || !cfg_.ipc_zc_async) {
    fn(s);
    return;
  }
  const bool cap = capturing_stream(s);
  if (!ds.launcher && (!exchanges || cap)) {  // nothing deferred yet: the launcher may never be needed
    fn(s);
    return;
  }
  IpcLauncher& L = launcher(ds);
  std::unique_lock<std::mutex> lk(L.mu);
  const bool idle = L.q.empty() && !L.busy;
  // evicted mappings pile up on the launcher's thread (it never closes them): with the
  // launcher idle, close the ones whose last launch is done, here, now and then (every
  // 4 x PDCC_IPC_ZC_CACHE evictions; hipIpcCloseMemHandle synchronises the device)
  if (idle && !cap && ds.ipc && ds.ipc->zc_closing() >= 4 * cfg_.ipc_zc_cache) ds.ipc->reap_closing(false);
  if (cap || tuning_.load() || (!exchanges && idle)) {
    // inline: after every job the launcher took (host: launched; device: s waits for them)
    L.idle_cv.wait(lk, [&] { return L.q.empty() && !L.busy; });
    uint64_t& seen = L.seen[s];
    if (!cap && seen < L.next_ticket) {
      PDCC_HIP(hipStreamWaitValue64(s, L.done, L.next_ticket, hipStreamWaitValueGte, ~0ull));
      seen = L.next_ticket;
    }
    ++L.direct;
    fn(s);  // (L.mu held: the helper cannot start a job meanwhile; jobs are only queued here)
    return;
  }
  SignalWord& r = L.ready[s];
  if (!r.ptr) r.ptr = ds.sync->alloc();
  TORCH_CHECK(r.ptr, "pdcc: the IPC launcher needs signal memory (hipMallocSignalMemory)");
  const uint64_t rt = ++r.next;
  PDCC_HIP(hipStreamWriteValue64(s, r.ptr, rt, 0));
  const uint64_t ticket = ++L.next_ticket;
  PDCC_HIP(hipStreamWaitValue64(s, L.done, ticket, hipStreamWaitValueGte, ~0ull));
  L.seen[s] = ticket;
  L.q.push_back({std::move(fn), r.ptr, rt, ticket});
  L.cv.notify_one();
}

void ProcessGroupMI355X::launcher_quiesce(DeviceState& ds, hipStream_t s) {
  if (!ds.launcher) return;
  IpcLauncher& L = *ds.launcher;
  std::unique_lock<std::mutex> lk(L.mu);
  L.idle_cv.wait(lk, [&] { return L.q.empty() && !L.busy; });
  uint64_t& seen = L.seen[s];
  if (seen < L.next_ticket && !capturing_stream(s)) {
    PDCC_HIP(hipStreamWaitValue64(s, L.done, L.next_ticket, hipStreamWaitValueGte, ~0ull));
    seen = L.next_ticket;
  }
}

void ProcessGroupMI355X::stop_launchers() {
  std::vector<IpcLauncher*> ls;
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_)
      if (kv.second->launcher) ls.push_back(kv.second->launcher.get());
  }
  for (IpcLauncher* L : ls) {
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->stop = true;
    }
    L->cv.notify_all();
    if (health_->poisoned.load() && L->shm) L->shm->abort();  // a job stuck in an exchange leaves it
    if (L->thr.joinable()) L->thr.join();
  }
}

}  // namespace pdcc
