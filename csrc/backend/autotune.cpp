// Online autotuner of ProcessGroupMI355X: per (collective, dtype, op, power-of-two size
// bucket), the first call races every feasible engine on scratch copies of the caller's
// data, checks each result against the reference engine's, times interleaved runs and
// adopts the fastest on every rank (SURVEY.md §3.3 algorithm selection); decisions can
// be persisted per topology (PDCC_AUTOTUNE_FILE).
#include <sys/file.h>

#include "gpu_util.h"

namespace pdcc {

using namespace gpu;

// =================================================================== autotuner
std::vector<Algo> ProcessGroupMI355X::tune_candidates(Coll c, size_t bytes, bool rccl_can, bool ipc_can,
                                                      bool zc_can, bool ll_can) const {
  std::vector<Algo> v;
  if (!cfg_.autotune || cfg_.force_algo != Algo::AUTO || !ipc_can || !same_host_ || coalescing_) return v;
  if ((int)c >= 32 || !(cfg_.autotune_colls & (1u << (int)c))) return v;
  if (bytes < cfg_.autotune_min || bytes > cfg_.autotune_max) return v;
  // LL sizes keep the static choice: a race there would time the LL kernel and then apply
  // the verdict to the staged protocol the rest of the power-of-two bucket takes
  if (ll_can && bytes_in_ll_range(bytes)) return v;
  // reference engine: RCCL; without it (ranks sharing a GPU, or a reduction RCCL lacks:
  // BAND/BOR/BXOR, integer AVG) the host transport for small keys, and above kHostTuneMax the
  // static IPC engine itself -- checked against the host transport on a <= kHostTuneMax
  // prefix of the caller's data once per key (autotune(): `ref_check`) -- so the IPC variants
  // are still raced where the host path is too slow to time against
  if (rccl_can) v.push_back(Algo::RCCL);
  else if (bytes <= kHostTuneMax) v.push_back(Algo::HOST);
  // RCCL with more channels than its topology tuner picks (large all_reduce keys)
  if (c == Coll::ALLREDUCE && rccl_can && cfg_.rccl_wide_ctas > 0 && bytes >= cfg_.rccl_wide_min)
    v.push_back(Algo::RCCL_WIDE);
  v.push_back(Algo::IPC);
  // the pull all-reduce with more workgroups (distinct GPUs: rccl_can; shared devices are
  // capped for co-residency anyway)
  if (c == Coll::ALLREDUCE && rccl_can && cfg_.ipc_wide_grid > cfg_.ipc_grid && bytes >= cfg_.rccl_wide_min)
    v.push_back(Algo::IPC_WIDE);
  // the same IPC protocols without zero copy (zero-copy sizes): measured, not assumed, where the
  // staging copy beats the per-call record exchange
  if (zc_can && cfg_.ipc_zc && bytes >= cfg_.ipc_zc_min) v.push_back(Algo::IPC_STAGED);
  // the push all-reduce (zero-copy sizes): every remote access a write instead of a read
  if (c == Coll::ALLREDUCE && cfg_.ipc_push && zc_can && cfg_.ipc_zc && bytes >= cfg_.ipc_zc_min &&
      bytes > cfg_.ipc_1shot_max)
    v.push_back(Algo::IPC_PUSH);
  // the dynamic protocols (zero-copy sizes): work items claimed per workgroup -- the 2-shot
  // all-reduce, the all-gather, the reduce-scatter
  const bool dyn_coll = (c == Coll::ALLREDUCE && bytes > cfg_.ipc_1shot_max) || c == Coll::ALLGATHER ||
                        c == Coll::REDUCE_SCATTER;
  if (dyn_coll && cfg_.ipc_dyn > 0 && zc_can && cfg_.ipc_zc && bytes >= cfg_.ipc_zc_min)
    v.push_back(Algo::IPC_DYN);
  // the copy collectives on the copy engines (zero-copy sizes): no CU moves their bytes
  const bool sdma_coll = c == Coll::BROADCAST || c == Coll::ALLGATHER || c == Coll::GATHER || c == Coll::SCATTER ||
                         c == Coll::ALLTOALL;
  if (sdma_coll && cfg_.ipc_sdma && zc_can && cfg_.ipc_zc && bytes >= cfg_.ipc_zc_min) v.push_back(Algo::IPC_SDMA);
  if (v.size() < 2) return {};  // nothing to race
  return v;
}

Algo ProcessGroupMI355X::tuned(const TuneKey& k) {
  std::lock_guard<std::mutex> lk(tune_mu_);
  auto it = tune_.find(k);
  return it == tune_.end() ? Algo::AUTO : it->second.algo;
}

// The engine for one call. A decision for this key is used only if that engine is a
// candidate of this call too; everything here depends on group-wide facts only
// (topology, dtype/op support, the consensus table), so every rank picks the same.
Algo ProcessGroupMI355X::decide(Coll c, int dtype, int op, size_t bytes, DeviceState& ds, Algo a0, bool rccl_can,
                                bool ipc_can, const std::function<Algo(const TuneKey&, const std::vector<Algo>&)>& tune) {
  auto cands = tune_candidates(c, bytes, rccl_can, ipc_can, ds.zc_ok, ds.ll_ok);
  if (cands.empty()) return a0;
  // an async call whose IPC launches run the capped grid (PDCC_IPC_ASYNC_GRID) is a key of its own
  // (bucket + kAsyncBucket): a verdict timed at one grid is never applied at the other
  const int bucket = size_bucket(bytes) + (runs_capped(ds.device) ? kAsyncBucket : 0);
  const TuneKey key{(int)c, dtype, op, bucket};
  const Algo t = tuned(key);
  const bool cap = capturing_on(ds.device);
  if (t != Algo::AUTO) {
    // (HOST also stands for "the IPC reference engine failed its host check": always feasible)
    if (t != Algo::HOST && std::find(cands.begin(), cands.end(), t) == cands.end()) return a0;
    if (t == Algo::HOST && cap) return Algo::IPC;  // tuned to the host engine, which cannot be captured
    return t;
  }
  if (!cfg_.autotune_file.empty()) {  // a decision recorded by an earlier run (same topology)
    const Algo f = file_decision(key, ds);
    if (f != Algo::AUTO && std::find(cands.begin(), cands.end(), f) != cands.end() && !(f == Algo::HOST && cap)) {
      TuneEntry te;
      te.ref = cands[0];
      te.valid = true;
      te.algo = f;  // iters = 0: from the file
      std::lock_guard<std::mutex> lk(tune_mu_);
      tune_[key] = te;
      return f;
    }
  }
  if (cap) return a0;  // no timing runs inside a graph capture: static choice
  // every engine of the race exists before the clock starts (communicator setup is not timed)
  for (Algo a : cands) {
    if (a == Algo::RCCL) rccl(ds);
    if (is_ipc(a)) ipc(ds);
  }
  if (std::find(cands.begin(), cands.end(), Algo::RCCL_WIDE) != cands.end()) {
    // an optional candidate: a wide child communicator this RCCL build refuses (a channel count it
    // does not take) leaves the race on every rank -- and the group's later keys -- instead of
    // poisoning the group the headline runs on
    double ok = 1.0;
    std::string why;
    try {
      rccl_wide(ds, /*fatal=*/false);
    } catch (const std::exception& e) {
      ok = 0.0;
      why = e.what();
    }
    shm().allreduce(&ok, 1, at::kDouble, RedOpType::MIN, timeout_);
    if (ok <= 0.0) {
      fprintf(stderr, "[pdcc r%d] wide RCCL communicator (%d CTAs) unavailable, dropped from the autotuner: %s\n",
              rank_, cfg_.rccl_wide_ctas, why.empty() ? "failed on another rank" : why.c_str());
      cfg_.rccl_wide_ctas = 0;  // (every rank: agreed above)
      cands.erase(std::remove(cands.begin(), cands.end(), Algo::RCCL_WIDE), cands.end());
      if (cands.size() < 2) return a0;
    }
  }
  // the race runs on the caller's stream: it must not overlap an async collective of this
  // group still in flight on the comm stream (IPC kernels of one rank share the per-block
  // counters, the staging buffer and the LL epoch word)
  order_after_async(ds, current_stream(ds.device));
  return tune(key, cands);
}

Algo ProcessGroupMI355X::autotune(const TuneKey& key, size_t bytes, DeviceState& ds, const std::vector<Algo>& cands,
                                  const std::function<void(size_t)>& run,
                                  const std::function<bool(size_t, size_t)>& same,
                                  const std::function<bool()>& ref_check) {
  c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)ds.device);
  const hipStream_t s = current_stream(ds.device);
  const size_t n = cands.size();
  auto elapsed_us = [](hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    PDCC_HIP(hipEventElapsedTime(&ms, a, b));
    return 1e3 * (double)ms;
  };
  // IPC runs of the race get a short spin bound: a run that cannot complete here
  // disqualifies IPC for this key (below) instead of hanging the group
  struct Spin {
    IpcComm* ic;
    uint64_t saved;
    std::atomic<bool>& flag;
    Spin(IpcComm* c, uint64_t ms, std::atomic<bool>& f) : ic(c), saved(c ? c->timeout_ms() : 0), flag(f) {
      flag.store(true);
      if (ic) ic->set_timeout_ms(std::max<uint64_t>(1, std::min<uint64_t>(ms, saved)));
    }
    ~Spin() {
      if (ic) ic->set_timeout_ms(saved);
      flag.store(false);
    }
  };
  bool has_ipc = false;
  for (Algo a : cands) has_ipc = has_ipc || is_ipc(a);
  Spin spin(has_ipc ? ds.ipc.get() : nullptr, (uint64_t)cfg_.autotune_spin_ms, tuning_);
  // an async call's key is raced with the grid its IPC launches will run at (PDCC_IPC_ASYNC_GRID):
  // the verdict must hold for the capped engine next to compute, not for the full grid
  IpcComm::AsyncScope async_cap(has_ipc ? ds.ipc.get() : nullptr, runs_capped(ds.device));
  // The IPC engine as the reference (no RCCL, above kHostTuneMax): first its result on a prefix
  // of the caller's data against the host transport's, agreed on every rank. A failure (or an
  // IPC spin timeout in the reference run below) sends the key to the host engine: slow, exact.
  auto host_fallback = [&](const char* why) {
    if (ds.ipc) ds.ipc->clear_error();
    fprintf(stderr, "[pdcc r%d] autotune %s %zu B: reference IPC engine %s; using the host engine for this key\n",
            rank_, coll_name((Coll)std::get<0>(key)), bytes, why);
    TuneEntry te;
    te.ref = cands[0];
    te.valid = false;
    te.algo = Algo::HOST;
    std::lock_guard<std::mutex> lk(tune_mu_);
    tune_[key] = te;
    return Algo::HOST;
  };
  const bool ipc_ref = is_ipc(cands[0]);
  if (ipc_ref && ref_check) {
    bool ok = false;
    try {
      ok = ref_check();
      PDCC_HIP(hipStreamSynchronize(s));
      ok = ok && !(ds.ipc && ds.ipc->error_word() != 0);
    } catch (const std::exception& e) {
      ok = false;
    }
    double f = ok ? 1.0 : 0.0;
    shm().allreduce(&f, 1, at::kDouble, RedOpType::MIN, timeout_);
    if (f <= 0.0) return host_fallback("disagrees with the host transport on a prefix");
  }
  // 0) warm-up: one run each (staging growth, first-touch), then check every result
  //    against the reference engine's on identical data
  for (size_t k = 0; k < n; ++k) {
    if (is_ipc(cands[k]))
      if (const char* d = std::getenv("PDCC_TEST_AUTOTUNE_DELAY"))  // test hook "rank:ms": a late peer
        if (std::atoi(d) == rank_) {
          PDCC_HIP(hipStreamSynchronize(s));
          std::this_thread::sleep_for(std::chrono::milliseconds(std::atoi(std::strchr(d, ':') + 1)));
        }
    run(k);
  }
  PDCC_HIP(hipStreamSynchronize(s));
  std::vector<double> v(2 * n, 0.0);  // [estimate_us x n, mismatch x n], MAX-reduced across ranks
  const bool ipc_fault = has_ipc && ds.ipc && ds.ipc->error_word() != 0;
  if (ipc_ref && ipc_fault) v[n] = 2.0;  // the reference itself timed out
  for (size_t k = 1; k < n; ++k)
    v[n + k] = (is_ipc(cands[k]) && ipc_fault) ? 2.0 : (same(0, k) ? 0.0 : 1.0);
  {  // agree on faults first (every rank's stream is drained: no IPC kernel is running)
    std::vector<double> f(v.begin() + n, v.end());
    shm().allreduce(f.data(), f.size(), at::kDouble, RedOpType::MAX, timeout_);
    std::copy(f.begin(), f.end(), v.begin() + n);
  }
  if (v[n] >= 2.0) return host_fallback("timed out");
  std::vector<bool> live(n, true);
  for (size_t k = 1; k < n; ++k)
    if (v[n + k] >= 2.0) {
      live[k] = false;  // an IPC barrier timed out on some rank: drop IPC from the race
      if (ds.ipc) ds.ipc->clear_error();
      fprintf(stderr, "[pdcc r%d] autotune %s %zu B: IPC run timed out (>%lld ms); using %s for this key\n", rank_,
              coll_name((Coll)std::get<0>(key)), bytes, (long long)cfg_.autotune_spin_ms, algo_name(cands[0]));
    }
  // Every timed run is isolated: start / stop events around it, the stream drained, then a host
  // barrier, so no rank starts run k+1 while a peer still executes run k. Back-to-back runs of
  // DIFFERENT engines overlapped across ranks: a rank's zero-copy kernel waited in its entry
  // exchange for a peer still inside the previous (staged) run, and on a shared GPU its waiting
  // workgroups slowed that run down -- the race timed the 1 GiB zero-copy broadcast at 3853 us,
  // isolated it takes 2242 (W = 4, scripts/race_probe.py, profiles/r5/), and adopted the slower
  // staged engine. Isolated, each engine is timed the way a collective between other work runs.
  hipEvent_t ea = nullptr, eb = nullptr;
  PDCC_HIP(hipEventCreate(&ea));
  PDCC_HIP(hipEventCreate(&eb));
  const std::function<double(size_t)> timed = [&](size_t k) {
    PDCC_HIP(hipEventRecord(ea, s));
    if (live[k]) run(k);
    PDCC_HIP(hipEventRecord(eb, s));
    PDCC_HIP(hipEventSynchronize(eb));
    const double us = elapsed_us(ea, eb);
    shm().barrier(timeout_);
    return us;
  };
  // 1) one timed run each: sizes the measurement (same count on every rank: MAX-reduced inputs)
  for (size_t k = 0; k < n; ++k) v[k] = timed(k);
  shm().allreduce(v.data(), v.size(), at::kDouble, RedOpType::MAX, timeout_);
  double slow = 1.0;
  for (size_t k = 0; k < n; ++k) slow = std::max(slow, v[k]);
  const int iters = (int)std::max(3.0, std::min(25.0, std::ceil(30000.0 / slow)));
  // 2) interleaved timed runs (ref, ipc, ref, ipc, ...): drift hits both engines alike
  std::vector<std::vector<double>> t(n);
  for (int i = 0; i < iters; ++i)
    for (size_t k = 0; k < n; ++k) t[k].push_back(timed(k));
  hipEventDestroy(ea);
  hipEventDestroy(eb);
  std::vector<double> med(n);
  for (size_t k = 0; k < n; ++k) {
    std::nth_element(t[k].begin(), t[k].begin() + t[k].size() / 2, t[k].end());
    med[k] = t[k][t[k].size() / 2];
  }
  // 3) every rank adopts the same engine: slowest rank's median, any rank's mismatch
  shm().allreduce(med.data(), med.size(), at::kDouble, RedOpType::MAX, timeout_);
  size_t best = 0;
  for (size_t k = 1; k < n; ++k)
    if (live[k] && v[n + k] == 0.0 && med[k] < med[best]) best = k;
  TuneEntry te;
  te.ref = cands[0];
  te.iters = iters;
  te.valid = true;
  te.rccl_us = med[0];  // the reference engine's time (RCCL, the host transport, or static IPC)
  for (size_t k = 0; k < n; ++k) {
    if (is_ipc(cands[k])) {
      (cands[k] == Algo::IPC          ? te.ipc_us
       : cands[k] == Algo::IPC_WIDE   ? te.ipc_wide_us
       : cands[k] == Algo::IPC_STAGED ? te.staged_us
       : cands[k] == Algo::IPC_DYN    ? te.dyn_us
       : cands[k] == Algo::IPC_SDMA   ? te.sdma_us
                                      : te.push_us) = med[k];
      te.valid = te.valid && v[n + k] == 0.0;
    } else if (cands[k] == Algo::RCCL_WIDE) {
      te.wide_us = med[k];
      te.valid = te.valid && v[n + k] == 0.0;
    }
  }
  te.algo = cands[best];
  {
    std::lock_guard<std::mutex> lk(tune_mu_);
    tune_[key] = te;
  }
  if (!cfg_.autotune_file.empty() && rank_ == 0 && te.valid) file_append(key, te, ds);
  if (cfg_.log_level >= 1 && rank_ == 0)
    fprintf(stderr,
            "[pdcc r0] autotune %s %zu B: %s %.1f us, rccl_wide %.1f us, ipc %.1f us, ipc_wide %.1f us, ipc_push %.1f us,"
            " ipc_staged %.1f us, ipc_dyn %.1f us, ipc_sdma %.1f us%s (%d runs each) -> %s\n",
            coll_name((Coll)std::get<0>(key)), bytes, algo_name(cands[0]), te.rccl_us, te.wide_us, te.ipc_us,
            te.ipc_wide_us, te.push_us, te.staged_us, te.dyn_us, te.sdma_us,
            te.valid ? "" : " (MISMATCH)", iters, algo_name(te.algo));
  return te.algo;
}

// ---- PDCC_AUTOTUNE_FILE: one line per decision,
//   pdcc-tune v1 <signature> <coll> <dtype> <op> <size bucket> <engine> [# times]
// The signature names what the verdict depends on: world size, distinct or shared GPUs,
// the GPU architecture and the IPC grid cap.
std::string ProcessGroupMI355X::tune_sig(const DeviceState& ds) const {
  hipDeviceProp_t p{};
  std::string arch = hipGetDeviceProperties(&p, ds.device) == hipSuccess ? std::string(p.gcnArchName) : "?";
  arch = arch.substr(0, arch.find(':'));
  std::ostringstream o;
  o << "w" << size_ << "-" << (ds.shared_device ? "shared" : "distinct") << "-" << arch << "-g" << cfg_.ipc_grid;
  return o.str();
}

Algo ProcessGroupMI355X::file_decision(const TuneKey& key, DeviceState& ds) {
  if (!tune_file_read_) {
    tune_file_read_ = true;
    const std::string sig = tune_sig(ds);
    if (FILE* f = std::fopen(cfg_.autotune_file.c_str(), "r")) {
      char line[512];
      while (std::fgets(line, sizeof(line), f)) {
        char tag[16], ver[8], sg[128], eng[32];
        int c, dt, op, b;
        if (std::sscanf(line, "%15s %7s %127s %d %d %d %d %31s", tag, ver, sg, &c, &dt, &op, &b, eng) != 8) continue;
        if (std::strcmp(tag, "pdcc-tune") != 0 || std::strcmp(ver, "v1") != 0 || sig != sg) continue;
        const Algo a = algo_from_name(eng);
        if (a != Algo::AUTO) tune_file_[TuneKey{c, dt, op, b}] = a;  // later lines win
      }
      std::fclose(f);
    }
  }
  const auto it = tune_file_.find(key);
  double v[2] = {it == tune_file_.end() ? 0.0 : (double)(int)it->second, 0.0};
  v[1] = -v[0];
  shm().allreduce(v, 2, at::kDouble, RedOpType::MAX, timeout_);  // max and -min: agree only if equal
  return v[0] == -v[1] ? (Algo)(int)v[0] : Algo::AUTO;
}

void ProcessGroupMI355X::file_append(const TuneKey& key, const TuneEntry& e, const DeviceState& ds) {
  FILE* f = std::fopen(cfg_.autotune_file.c_str(), "a");
  if (!f) {
    fprintf(stderr, "[pdcc r%d] PDCC_AUTOTUNE_FILE %s: cannot append\n", rank_, cfg_.autotune_file.c_str());
    return;
  }
  flock(fileno(f), LOCK_EX);
  std::fprintf(f, "pdcc-tune v1 %s %d %d %d %d %s # %s %s %zu-%zu B: ref %.1f us, rccl_wide %.1f, ipc %.1f, "
               "ipc_wide %.1f, ipc_push %.1f, ipc_staged %.1f, ipc_dyn %.1f, ipc_sdma %.1f\n",
               tune_sig(ds).c_str(), std::get<0>(key), std::get<1>(key), std::get<2>(key), std::get<3>(key),
               algo_name(e.algo), coll_name((Coll)std::get<0>(key)), algo_name(e.ref),
               (size_t)1 << (std::get<3>(key) % kAsyncBucket), (size_t)2 << (std::get<3>(key) % kAsyncBucket), e.rccl_us, e.wide_us, e.ipc_us, e.ipc_wide_us, e.push_us, e.staged_us,
               e.dyn_us, e.sdma_us);
  std::fflush(f);
  flock(fileno(f), LOCK_UN);
  std::fclose(f);
}

std::vector<ProcessGroupMI355X::TuneRecord> ProcessGroupMI355X::autotune_table() {
  std::lock_guard<std::mutex> lk(tune_mu_);
  std::vector<TuneRecord> out;
  for (const auto& kv : tune_) {
    const TuneEntry& e = kv.second;
    const int dt = std::get<1>(kv.first), op = std::get<2>(kv.first), b = std::get<3>(kv.first) % kAsyncBucket;
    TuneRecord r;
    r.coll = coll_name((Coll)std::get<0>(kv.first));
    r.dtype = dt < 0 ? "-" : c10::toString((at::ScalarType)dt);
    r.op = op == kLayoutFlat ? "flat" : op == kLayoutList ? "list" : op < 0 ? "-" : op_name(op);
    r.lo = 1ull << b;
    r.hi = 2ull << b;
    r.ref = algo_name(e.ref);
    r.rccl_us = e.rccl_us;
    r.ipc_us = e.ipc_us;
    r.push_us = e.push_us;
    r.ipc_wide_us = e.ipc_wide_us;
    r.staged_us = e.staged_us;
    r.dyn_us = e.dyn_us;
    r.sdma_us = e.sdma_us;
    r.wide_us = e.wide_us;
    r.valid = e.valid;
    r.algo = algo_name(e.algo);
    r.iters = e.iters;
    r.async_capped = std::get<3>(kv.first) >= kAsyncBucket;
    out.push_back(r);
  }
  return out;
}

}  // namespace pdcc
