// Zero-copy exchanges off the caller's thread (PDCC_IPC_ZC_ASYNC, see IpcLauncher in
// process_group.h). A zero-copy IPC call is launched at once, in stream order, as a
// *gated* launch (kern::GateSlot): its kernels wait on the device until the call's
// buffer records have been exchanged with the peers and mapped, which this per-device
// exchange thread does and then publishes in the call's gate slot. The caller's host never
// lines up with its peers' -- the gradient all-reduce of a training step (the use the
// reference motivates, README.md:5) overlaps with backward -- and stream semantics stay
// those of any kernel (torch.cuda.synchronize() covers the call). The thread makes no
// stream operation and no device-synchronising call (hipFree / hipIpcCloseMemHandle), so
// no kernel ever waits on work that itself waits for the device.
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <cstring>

#include "../device/comm_util.h"
#include "process_group.h"

namespace pdcc {

bool capturing_stream(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

IpcLauncher& ProcessGroupMI355X::launcher(DeviceState& ds) {
  std::lock_guard<std::mutex> lk(init_mu_);
  if (ds.launcher) return *ds.launcher;
  auto L = std::make_unique<IpcLauncher>();
  L->thr = std::thread([this, p = &ds, l = L.get()] { launcher_loop(p, l); });
  ds.launcher = std::move(L);
  return *ds.launcher;
}

void ProcessGroupMI355X::launcher_loop(DeviceState* dsp, IpcLauncher* lp) {
  DeviceState& ds = *dsp;
  IpcLauncher& L = *lp;
  // the caller's thread may capture a graph while this one opens mappings
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipSetDevice(ds.device);
  // never a device-synchronising release on this thread (kernels wait for its exchanges)
  IpcComm::set_thread_defers_frees(true);
  // A gated kernel whose buffers are not in the device-side mapping table waits for its job,
  // and a thread woken from a condition-variable sleep costs 60-200 us per job on a busy box
  // (r3 host_path): PDCC_XCHG_SPIN_US lets the thread spin that long after its last job before
  // it sleeps (default 0: in steady state the kernels do not wait for the thread at all).
  const auto spin = std::chrono::microseconds(std::max(0, cfg_.xchg_spin_us));
  uint64_t seen = 0;
  for (;;) {
    std::function<void()> job;
    if (spin.count() > 0 && L.pushed.load(std::memory_order_acquire) == seen) {
      const auto t0 = std::chrono::steady_clock::now();
      while (L.pushed.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() - t0 < spin)
        __builtin_ia32_pause();
    }
    {
      std::unique_lock<std::mutex> lk(L.mu);
      L.cv.wait(lk, [&] { return L.stop || !L.q.empty(); });
      if (L.q.empty()) return;  // stop, nothing left
      job = std::move(L.q.front());
      L.q.pop_front();
      L.depth_sum += L.q.size();
      ++seen;
      L.busy = true;
    }
    job();  // (never throws: a job publishes its gate slot whatever happens)
    {
      std::lock_guard<std::mutex> lk(L.mu);
      L.busy = false;
      ++L.jobs;
      if (L.q.empty()) L.idle_cv.notify_all();
    }
  }
}

bool ProcessGroupMI355X::launcher_idle(DeviceState& ds) {
  if (!ds.launcher) return true;
  IpcLauncher& L = *ds.launcher;
  std::lock_guard<std::mutex> lk(L.mu);
  return L.q.empty() && !L.busy;
}

void ProcessGroupMI355X::launcher_quiesce(DeviceState& ds) {
  if (!ds.launcher) return;
  IpcLauncher& L = *ds.launcher;
  std::unique_lock<std::mutex> lk(L.mu);
  L.idle_cv.wait(lk, [&] { return L.q.empty() && !L.busy; });
}

host::ShmComm& ProcessGroupMI355X::exchange_channel(DeviceState& ds) {
  std::lock_guard<std::mutex> lk(ds.xchg_mu);
  if (!ds.xchg) {  // collective: every rank reaches its first zero-copy exchange in the same order
    host::ShmConfig sc;
    sc.slot_bytes = 64u << 10;  // records only
    sc.spin_us = cfg_.shm_spin_us;
    sc.chan_bytes = 4096;
    sc.timeout = timeout_;
    ds.xchg = std::make_unique<host::ShmComm>(store_, "pdcc/shm_xchg", rank_, size_, sc);
  }
  return *ds.xchg;
}

// The zero-copy body of `call` (`body` bytes, whole `unit`s) as gated launches on `s`, now;
// the exchange that opens the gates as a job of the exchange thread. Launches are chunked
// so that the staged fallback of each fits a staging window of at most kGateChunk.
constexpr size_t kGateChunk = 256u << 20;

uint64_t ProcessGroupMI355X::ipc_gated(DeviceState& ds, const kern::IpcCall& call, const void* zbuf, size_t zlen,
                                       size_t unit, size_t body, size_t per_call_max, hipStream_t s) {
  IpcComm& ic = ipc(ds);
  hp_.lap(HostStage::ENQUEUE);
  // Evicted mappings are only queued on the launcher's thread; close the finished ones here, on the
  // submitting thread, before this call's export: with every call gated (no inline exchange, no
  // barrier) the closing lists otherwise only grow, and at W = 8 (seven peers' entries per eviction)
  // a run of fresh buffers filled them within ~30 calls and every later fresh export was refused
  // (staged; conformance's op checks, profiles/r6/plan_rehearsal_w8_conformance_before.jsonl). Only
  // while the launcher is idle: a close synchronises the device, and with no exchange job queued or
  // running no kernel in flight waits on a host thread (and no mapping is being opened meanwhile) --
  // the state an inline exchange closes in (design.md §3, "Evictions without a safe point").
  if (ic.zc_closing() > 0 && launcher_idle(ds)) ic.reap_closing(false);
  const IpcComm::ZcRec mine = ic.zc_export(zbuf, zlen, false);
  hp_.lap(HostStage::ZC_EXPORT);
  const uint64_t t = ic.gate_reserve();
  hp_.lap(HostStage::ZC_RESERVE);
  size_t chunk = std::min(per_call_max, kGateChunk) / unit * unit;
  if (chunk == 0) chunk = unit;
  for (size_t off = 0; off < body; off += chunk) {
    kern::IpcCall c = call;
    c.bytes = std::min(chunk, body - off);
    for (int k = 0; k < kern::kMaxRanks; ++k) {
      if (call.in[k]) c.in[k] = static_cast<const char*>(call.in[k]) + off;
      if (call.out[k]) c.out[k] = static_cast<char*>(call.out[k]) + off;
    }
    ic.launch_gated(c, t, off, mine, zbuf, s);
  }
  hp_.lap(HostStage::ZC_LAUNCH);
  auto ev = ic.gate_mark(t, s);  // the launches that read the slot (and the mappings)
  hp_.lap(HostStage::ZC_MARK);
  std::shared_ptr<IpcComm> icp = ds.ipc;
  IpcLauncher& L = launcher(ds);
  std::lock_guard<std::mutex> lk(L.mu);
  L.q.push_back([this, dsp = &ds, icp, mine, zbuf, t, ev, t_q = std::chrono::steady_clock::now()] {
    const auto t_run = std::chrono::steady_clock::now();
    std::vector<char*> ptrs;
    double gather_ns = 0;
    bool ok = false;
    std::string err;
    try {
      if (health_->poisoned.load()) throw std::runtime_error(health_->message());
      host::ShmComm& xc = exchange_channel(*dsp);
      std::vector<IpcComm::ZcRec> all(size_);
      std::vector<void*> outs;
      for (auto& r : all) outs.push_back(&r);
      const auto g0 = std::chrono::steady_clock::now();
      xc.allgather(&mine, outs, sizeof(mine), timeout_);
      gather_ns = (double)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - g0)
                      .count();
      bool all_ok = true, fresh = false;
      for (const auto& r : all) {
        all_ok = all_ok && r.ok;
        fresh = fresh || r.fresh;
      }
      ok = icp->zc_import(all, zbuf, all_ok, ptrs);
      if (all_ok && fresh) {  // agree that every mapping of a fresh export worked
        double f = ok ? 1.0 : 0.0;
        xc.allreduce(&f, 1, at::kDouble, c10d::ReduceOp::MIN, timeout_);
        ok = f > 0.0;
      }
      ok = ok && all_ok;
      icp->zc_settle(mine, ok);
      if (ok) icp->zc_note_launch(ev);
    } catch (const std::exception& e) {
      err = e.what();
      ok = false;
    }
    if (!err.empty()) {
      // the gated kernels fall back to staging and then spin on the barriers with a peer
      // that never comes: poison the group and abort them, so they leave and wait() raises
      fprintf(stderr, "[pdcc r%d] zero-copy exchange failed: %s\n", rank_, err.c_str());
      health_->poison("zero-copy exchange failed: " + err);
      icp->abort();
    } else if (!ok) {
      std::lock_guard<std::mutex> lk2(dsp->launcher->mu);
      ++dsp->launcher->fallbacks;  // a rank could not export / map: this call runs staged
    }
    {  // the call's engine label (record()) is settled from this, not from the intent
      IpcLauncher& L2 = *dsp->launcher;
      std::lock_guard<std::mutex> lk2(L2.mu);
      if (L2.outcome.size() >= 4096)  // abandoned tickets (autotune races' scratch calls): keep it bounded
        for (auto it = L2.outcome.begin(); it != L2.outcome.end();)
          it = it->first + 2048 < t ? L2.outcome.erase(it) : std::next(it);
      L2.outcome[t] = ok;
      L2.done_hi = std::max(L2.done_hi, t);
    }
    dsp->launcher->outcome_cv.notify_all();
    icp->gate_publish(t, ok, ptrs);
    const auto t_end = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lk3(dsp->launcher->mu);
    dsp->launcher->wait_ns += (double)std::chrono::duration_cast<std::chrono::nanoseconds>(t_run - t_q).count();
    dsp->launcher->run_ns += (double)std::chrono::duration_cast<std::chrono::nanoseconds>(t_end - t_run).count();
    dsp->launcher->gather_ns += gather_ns;
  });
  L.pushed.fetch_add(1, std::memory_order_release);
  L.cv.notify_one();
  hp_.lap(HostStage::ZC_JOB);
  return t;
}

void ProcessGroupMI355X::stop_launchers() {
  std::vector<IpcLauncher*> ls;
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) {
      if (kv.second->launcher) ls.push_back(kv.second->launcher.get());
      // a job stuck in an exchange (a peer is gone) leaves it
      if (health_->poisoned.load() && kv.second->xchg) kv.second->xchg->abort();
    }
  }
  for (IpcLauncher* L : ls) {
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->stop = true;
    }
    L->cv.notify_all();
    if (L->thr.joinable()) L->thr.join();
  }
}

}  // namespace pdcc
