// GPU setup of ProcessGroupMI355X: per-device state, the group topology exchange,
// the RCCL communicators (fresh / split / shared / wide / point-to-point pairs), the
// IPC communicator and its self-test (the reference's
// init_process_group + new_group, main.py:11,21,31,46,63,75,94).
#include <cstring>

#include "gpu_util.h"

namespace pdcc {

using namespace gpu;

namespace {

// IPC self-test verdicts of earlier groups with the same member set on the same devices:
// the topology did not change, so later groups skip the test when every rank has one.
// 'A' + bits: bit 0 IPC, bit 1 zero-copy, bit 2 LL, bit 3 device-side exchange ('?' = none).
std::mutex g_verdict_mu;
std::map<std::string, char> g_ipc_verdict;

}  // namespace

std::string ProcessGroupMI355X::make_members_key(const std::vector<int64_t>& global_ranks, int size) {
  return members_key(global_ranks, size);
}

// =================================================================== device state
DeviceState& ProcessGroupMI355X::dev_local(const at::Tensor& t) { return dev_local_idx(t.device().index()); }

DeviceState& ProcessGroupMI355X::dev_local_idx(int d) {
  std::lock_guard<std::mutex> lk(init_mu_);
  auto it = devs_.find(d);
  if (it != devs_.end()) return *it->second;
  TORCH_CHECK(devs_.empty(), "pdcc: one GPU per rank per process group (got a tensor on cuda:", d,
              " after using cuda:", devs_.begin()->first, ")");
  c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)d);
  auto ds = std::make_unique<DeviceState>(
      c10::hip::getStreamFromPoolMasqueradingAsCUDA(/*isHighPriority=*/cfg_.stream_mode == 1, (c10::DeviceIndex)d));
  ds->device = d;
  (void)ds->sync->prealloc();  // signal words for stream hand-offs (see StreamSync::alloc)
  // this rank's device record, for point-to-point peers (non-blocking: set only; a
  // peer reads it after posting its own, so a ring of first ops cannot wait in a cycle)
  store_->set("pdcc/devrec/" + std::to_string(rank_), [&] {
    char bus[64] = {0};
    PDCC_HIP(hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, d));
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    const std::string rec = std::string(host) + "|" + bus;
    return std::vector<uint8_t>(rec.begin(), rec.end());
  }());
  DeviceState& ref = *ds;
  devs_[d] = std::move(ds);
  return ref;
}

DeviceState& ProcessGroupMI355X::dev_state(const at::Tensor& t) {
  DeviceState& ds = dev_local(t);
  std::lock_guard<std::mutex> lk(init_mu_);
  if (!ds.topo) init_topology(ds);
  return ds;
}

// PDCC_EAGER_INIT=1: everything the first GPU collective would set up (topology,
// IPC self-test, RCCL communicator) happens in init_process_group / new_group,
// on the current device -- so the first collective is not the one paying for
// it, and a graph can be captured right away.
void ProcessGroupMI355X::eager_init(int device) {
  DeviceState& ds = dev_local_idx(device);
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    if (!ds.topo) init_topology(ds);
  }
  if ((size_ > 1 || !cfg_.world1_local) && ds.rccl_ok) rccl(ds);
}

// Collective over the group (init_mu_ held): where is every rank, can RCCL run (one
// rank per device) and can the IPC path run (same host, every peer reachable, and
// the protocol self-test passes on this topology).
void ProcessGroupMI355X::init_topology(DeviceState& ds) {
  const int d = ds.device;
  c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)d);
  char bus[64] = {0};
  PDCC_HIP(hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, d));
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  const std::string rec = std::string(host) + "|" + bus;
  const std::string vkey = members_key_ + "@" + rec;
  char cached = '?';
  {
    std::lock_guard<std::mutex> lk(g_verdict_mu);
    auto it = g_ipc_verdict.find(vkey);
    if (it != g_ipc_verdict.end()) cached = it->second;
  }
  const std::string mine = rec + "#" + cached;
  const auto all = store_allgather(store_, "pdcc/dev", rank_, size_, std::vector<uint8_t>(mine.begin(), mine.end()));
  std::vector<std::string> recs;
  bool all_cached = true;
  for (const auto& v : all) {
    const std::string s(v.begin(), v.end());
    const size_t h = s.rfind('#');
    recs.push_back(s.substr(0, h));
    const char c = h + 1 < s.size() ? s[h + 1] : '?';
    all_cached = all_cached && c != '?' && c == cached;
  }
  bool shared = false;
  for (int a = 0; a < size_; ++a)
    for (int b = a + 1; b < size_; ++b) shared = shared || recs[a] == recs[b];
  bool ok = cfg_.ipc_enable && same_host_ && size_ >= 2 && size_ <= kern::kMaxRanks;
  for (int r = 0; r < size_ && ok; ++r) {
    if (recs[r] == rec) continue;
    const std::string pb = recs[r].substr(recs[r].find('|') + 1);
    int idx = -1;
    if (hipDeviceGetByPCIBusId(&idx, pb.c_str()) != hipSuccess) {
      (void)hipGetLastError();
      ok = false;
      break;
    }
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, d, idx) != hipSuccess || !can) ok = false;
  }
  // every rank must agree (a rank that cannot see its peers vetoes the IPC path)
  const auto votes = store_allgather(store_, "pdcc/dev_ipc", rank_, size_, std::vector<uint8_t>{(uint8_t)ok});
  for (const auto& v : votes) ok = ok && !v.empty() && v[0] == 1;

  // The IPC workgroup caps must be the same on every rank (the block-pairwise protocol pairs block b of
  // every rank): a rank started with different PDCC_IPC_GRID / _WIDE_GRID / _ASYNC_GRID settings is
  // brought to the group's minimum instead of hanging its peers' barriers. PDCC_IPC_DYN likewise: it
  // sets the dynamic all-reduce's chunk size (every rank must number the chunks alike) and whether the
  // autotuner races it (every rank must race the same candidates). The zero-copy size guard too: a
  // guarded rank must never import a record a rank without the guard exported (the stall the guard
  // exists to prevent), so it is lifted only if every rank lifts it (slot 5: 1 = lifted, min-voted).
  {
    constexpr int kN = 6;
    const int32_t mine3[kN] = {cfg_.ipc_grid, cfg_.ipc_wide_grid, cfg_.ipc_async_grid, cfg_.ipc_dyn,
                               cfg_.ipc_dyn_min_rows, cfg_.ipc_zc_size_guard ? 0 : 1};
    const auto gv = store_allgather(store_, "pdcc/dev_grids", rank_, size_,
                                    std::vector<uint8_t>(reinterpret_cast<const uint8_t*>(mine3),
                                                         reinterpret_cast<const uint8_t*>(mine3) + sizeof(mine3)));
    int32_t lo[kN];
    std::memcpy(lo, mine3, sizeof(lo));
    for (const auto& v : gv) {
      TORCH_CHECK(v.size() == sizeof(mine3), "pdcc: malformed IPC settings vote");
      int32_t t[kN];
      std::memcpy(t, v.data(), sizeof(t));
      for (int k = 0; k < kN; ++k) lo[k] = std::min(lo[k], t[k]);
    }
    if (std::memcmp(lo, mine3, sizeof(lo)) != 0)
      fprintf(stderr, "[pdcc r%d] IPC grid caps / PDCC_IPC_DYN / _DYN_MIN_ROWS / _ZC_SIZE_GUARD differ between ranks: "
              "using the group minimum %d/%d/%d/%d/%d, size guard %s\n", rank_, lo[0], lo[1], lo[2], lo[3], lo[4],
              lo[5] ? "lifted" : "on");
    cfg_.ipc_grid = std::max(1, lo[0]);
    cfg_.ipc_wide_grid = lo[1];
    cfg_.ipc_async_grid = lo[2];
    cfg_.ipc_dyn = lo[3];
    cfg_.ipc_dyn_min_rows = lo[4];
    cfg_.ipc_zc_size_guard = lo[5] == 0;
    // (as Config::from_env does for a guarded rank: its own staging window must not need the guard)
    if (cfg_.ipc_zc_size_guard && cfg_.ipc_max_staging >= (size_t{1} << 31)) cfg_.ipc_max_staging = size_t{1} << 30;
  }
  ds.recs = recs;
  ds.shared_device = shared;
  ds.rccl_ok = !shared;
  // test hook: claim RCCL on ranks sharing a GPU (the communicator-creation deadline test: one
  // rank never joins, so RCCL's duplicate-device check is never reached)
  if (const char* f = std::getenv("PDCC_TEST_RCCL_SHARED"))
    if (*f == '1') ds.rccl_ok = true;
  if (!ok) {
    ds.ipc_ok = false;
  } else if (!cfg_.ipc_selftest) {
    ds.ipc_ok = true;
    ds.zc_ok = cfg_.ipc_zc;
    ds.ll_ok = cfg_.ipc_ll_max > 0;
    // (no self-test: the device-side exchange still needs every rank's consent)
    const auto zv = store_allgather(store_, "pdcc/dev_zx", rank_, size_, std::vector<uint8_t>{(uint8_t)cfg_.ipc_zx});
    ds.zx_ok = true;
    for (const auto& v : zv) ds.zx_ok = ds.zx_ok && !v.empty() && v[0] == 1;
  } else if (all_cached) {
    const int bits = cached - 'A';  // an earlier group with these members tested this topology
    ds.ipc_ok = (bits & 1) != 0;
    ds.zc_ok = (bits & 2) != 0;
    ds.ll_ok = (bits & 4) != 0;
    ds.zx_ok = (bits & 8) != 0;
  } else {
    ds.ipc_ok = ipc_selftest(ds);
    if (!ds.ipc_ok) ds.zc_ok = ds.ll_ok = ds.zx_ok = false;
    std::lock_guard<std::mutex> lk(g_verdict_mu);
    g_ipc_verdict[vkey] = (char)('A' + (ds.ipc_ok ? 1 : 0) + (ds.zc_ok ? 2 : 0) + (ds.ll_ok ? 4 : 0) +
                                 (ds.zx_ok ? 8 : 0));
  }
  ds.topo = true;
  if (cfg_.log_level >= 1)
    fprintf(stderr, "[pdcc r%d] device %d (%s): rccl_ok=%d ipc_ok=%d zc_ok=%d ll_ok=%d shared_device=%d%s\n", rank_, d,
            bus, (int)ds.rccl_ok, (int)ds.ipc_ok, (int)ds.zc_ok, (int)ds.ll_ok, (int)shared,
            all_cached ? " (cached IPC verdict)" : "");
}

RcclOpts ProcessGroupMI355X::rccl_opts() const {
  RcclOpts o;
  o.min_ctas = cfg_.rccl_min_ctas;
  o.max_ctas = cfg_.rccl_max_ctas;
  o.split_share = cfg_.rccl_split_share ? 1 : 0;
  o.init_timeout_ms = std::max<int64_t>(1, std::min<int64_t>(cfg_.rccl_init_timeout_ms, timeout_.count()));
  o.nonblocking = cfg_.rccl_nonblocking;
  return o;
}

// The group's RCCL communicator (lazy, collective over the group). A group whose
// members equal those of a live communicator on this device (every demo of the
// reference builds new_group(range(size)), main.py:11,21,31,46,63,75) splits
// from it instead of bootstrapping a new one. All ranks vote first, so a rank
// that has no such parent (or a different one) sends everyone down the fresh path.
RcclComm& ProcessGroupMI355X::rccl(DeviceState& ds) {
  if (ds.rccl) return *ds.rccl;
  try {
    return rccl_create(ds);
  } catch (const std::exception& e) {
    // a peer that died or never arrived: this group is unusable from now on, and its later
    // calls fail at once (before_op) instead of each waiting out another creation deadline
    health_->poison(std::string("RCCL communicator creation failed: ") + e.what());
    throw;
  }
}

RcclComm& ProcessGroupMI355X::rccl_create(DeviceState& ds) {
  const auto t0 = std::chrono::steady_clock::now();
  const std::string mk = members_key_ + "@" + std::to_string(ds.device);
  std::shared_ptr<RcclComm> c;
  const char* how = "init";
  if (cfg_.group_comm != 2) {
    auto parent = rccl_registry_get(mk);
    const std::string tag = parent ? parent->tag : std::string();
    const auto all = store_allgather(store_, "pdcc/rccl_parent", rank_, size_, std::vector<uint8_t>(tag.begin(), tag.end()));
    bool agree = !tag.empty();
    for (const auto& v : all) agree = agree && std::string(v.begin(), v.end()) == tag;
    if (agree) {
      if (cfg_.group_comm == 1) {
        c = parent;
        c->add_user();  // from now on its issue order is enforced across streams (RcclComm::enter)
        how = "share";
      } else {
        c = std::make_shared<RcclComm>(*parent, rank_, rccl_opts());
        c->tag = parent->tag;
        how = "split";
      }
    }
  }
  if (!c) {
    if (const char* h = std::getenv("PDCC_TEST_RCCL_INIT_SKIP"))  // test hook: this rank never joins RCCL
      if (*h && std::atoi(h) == rank_) {
        std::this_thread::sleep_for(std::chrono::milliseconds(std::max<int64_t>(0, cfg_.rccl_init_timeout_ms) + 5000));
        throw std::runtime_error("PDCC_TEST_RCCL_INIT_SKIP: this rank skipped its communicator");
      }
    c = std::make_shared<RcclComm>(store_, "pdcc/rccl", rank_, size_, ds.device, rccl_opts());
    c->tag = group_name_ + "#" + mk;
  }
  rccl_registry_put(mk, c);
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    ds.rccl = c;
  }
  record_setup(std::string("rccl_comm/") + how, t0);
  if (cfg_.log_level >= 1 && rank_ == 0)
    fprintf(stderr, "[pdcc r0] group '%s': RCCL communicator (%s) in %.1f ms\n", group_name_.c_str(), how,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return *ds.rccl;
}

// The wide child of the group's communicator (collective over the group: created by
// decide() on every rank when a key races it, or by a forced PDCC_ALGO=rccl_wide).
RcclComm& ProcessGroupMI355X::rccl_wide(DeviceState& ds, bool fatal) {
  if (ds.rccl_wide) return *ds.rccl_wide;
  RcclComm& base = rccl(ds);
  const auto t0 = std::chrono::steady_clock::now();
  RcclOpts o = rccl_opts();
  o.min_ctas = std::max(cfg_.rccl_wide_ctas, 1);
  o.max_ctas = std::max(o.max_ctas, o.min_ctas);
  o.split_share = 0;  // its own channels and buffers
  std::shared_ptr<RcclComm> c;
  try {
    c = std::make_shared<RcclComm>(base, rank_, o);
  } catch (const std::exception& e) {
    if (fatal) health_->poison(std::string("RCCL (wide) communicator creation failed: ") + e.what());
    throw;
  }
  c->tag = base.tag + "#wide";
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    ds.rccl_wide = c;
  }
  record_setup("rccl_comm/wide", t0);
  return *ds.rccl_wide;
}

// The send/recv channel to `peer` (created on first use; its communicator is
// built by the channel's own thread, see PairChan).
std::shared_ptr<PairChan> ProcessGroupMI355X::pair_chan(DeviceState& ds, int peer) {
  std::lock_guard<std::mutex> lk(init_mu_);
  auto it = ds.pairs.find(peer);
  if (it != ds.pairs.end()) return it->second;
  auto pc = std::make_shared<PairChan>(
      c10::hip::getStreamFromPoolMasqueradingAsCUDA(/*isHighPriority=*/false, (c10::DeviceIndex)ds.device));
  ds.pairs[peer] = pc;
  return pc;
}

// Are this rank and `peer` on different GPUs of one host? From the group topology when a
// collective already exchanged it, else from the peer's device record (posted by its
// first GPU op in this group, before it waits on anybody).
bool ProcessGroupMI355X::pair_on_distinct_devices(DeviceState& ds, int peer) {
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    if (ds.topo) return ds.recs[peer] != ds.recs[rank_];
    auto it = ds.pair_distinct.find(peer);
    if (it != ds.pair_distinct.end()) return it->second;
  }
  const auto mine = store_->get("pdcc/devrec/" + std::to_string(rank_));
  const auto theirs = store_->get("pdcc/devrec/" + std::to_string(peer));
  const std::string a(mine.begin(), mine.end()), b(theirs.begin(), theirs.end());
  const bool distinct = a.substr(0, a.find('|')) == b.substr(0, b.find('|')) && a != b;
  std::lock_guard<std::mutex> lk(init_mu_);
  ds.pair_distinct[peer] = distinct;
  return distinct;
}

IpcComm& ProcessGroupMI355X::ipc(DeviceState& ds) {
  if (!ds.ipc) {
    const uint64_t spin = (uint64_t)std::max<int64_t>(1, std::min<int64_t>(cfg_.ipc_spin_ms, timeout_.count()));
    auto c = std::make_shared<IpcComm>(store_, "pdcc/ipc", rank_, size_, ds.device, cfg_.ipc_max_staging, spin,
                                       ds.shared_device, cfg_.ipc_zc_cache);
    c->set_grid_max(cfg_.ipc_grid);
    c->set_async_grid(cfg_.ipc_async_grid);
    c->set_zx(ds.zx_ok);
    c->set_zc_size_guard(cfg_.ipc_zc_size_guard);
    std::lock_guard<std::mutex> lk(init_mu_);
    ds.ipc = c;
  }
  return *ds.ipc;
}

// PDCC_IPC_SELFTEST (default on): before a group's first GPU collective, every
// rank runs the IPC protocol once on known data -- 1-shot all-reduce, 2-shot
// all-reduce over rows of W tiles with a partial last row and a ragged tail, and
// an all-gather -- with a short spin timeout. Two store votes decide (after the
// communicator is built, after the checks): one failure on any rank (handle
// export or mapping, spin timeout, wrong data) turns IPC off for the whole group,
// so a topology the protocol does not work on falls back to RCCL (or the host
// path) instead of hanging or corrupting data. Called from init_topology() with
// init_mu_ held, on the group's comm stream (never a capturing one).
bool ProcessGroupMI355X::ipc_selftest(DeviceState& ds) {
  auto vote = [&](const std::string& key, bool mine) {
    const auto v = store_allgather(store_, key, rank_, size_, std::vector<uint8_t>{(uint8_t)mine});
    bool all = true;
    for (const auto& x : v) all = all && !x.empty() && x[0] == 1;
    return all;
  };
  const int64_t spin_ms = std::max<int64_t>(1, std::min<int64_t>(cfg_.ipc_selftest_ms, timeout_.count()));
  std::string why;
  bool ok = true;
  try {
    ds.ipc = std::make_shared<IpcComm>(store_, "pdcc/ipc", rank_, size_, ds.device, cfg_.ipc_max_staging,
                                       (uint64_t)spin_ms, ds.shared_device, cfg_.ipc_zc_cache);
    ds.ipc->set_grid_max(cfg_.ipc_grid);
    ds.ipc->set_async_grid(cfg_.ipc_async_grid);
    ds.ipc->set_zc_size_guard(cfg_.ipc_zc_size_guard);
  } catch (const std::exception& e) {
    ok = false;
    why = e.what();
  }
  bool all = vote("pdcc/ipc_selftest/built", ok);
  if (all) {
    try {
      IpcComm& ic = *ds.ipc;
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(ds.stream);
      const hipStream_t s = ds.stream.stream();
      const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
      const double tri = size_ * (size_ + 1) / 2.0;
      for (const int64_t n : {int64_t{1000}, int64_t{3} * size_ * 1024 + 257}) {
        const at::Tensor base = at::arange(n, opt).remainder(7);
        at::Tensor x = base + (double)(rank_ + 1);
        kern::IpcCall c{};
        c.coll = n == 1000 ? kern::IpcColl::ALLREDUCE_1SHOT : kern::IpcColl::ALLREDUCE_2SHOT;
        c.dtype = kern::DType::F32;
        c.op = kern::RedOp::SUM;
        c.avg_div = size_;
        c.bytes = x.nbytes();
        c.in[0] = x.data_ptr();
        c.out[0] = x.data_ptr();
        ic.launch(c, s);
        ok = at::equal(x, base * (double)size_ + tri) && ok;
      }
      const int64_t m = 780;  // 3120 B per rank: whole 16-B vectors, one partial tile
      const at::Tensor in = at::full({m}, (double)rank_, opt);
      at::Tensor out = at::full({m * size_}, -1.0, opt);
      kern::IpcCall c{};
      c.coll = kern::IpcColl::ALLGATHER;
      c.dtype = kern::DType::U8;
      c.op = kern::RedOp::COPY;
      c.bytes = in.nbytes();
      c.in[0] = in.data_ptr();
      for (int r = 0; r < size_; ++r) c.out[r] = static_cast<char*>(out.data_ptr()) + r * in.nbytes();
      ic.launch(c, s);
      ok = at::equal(out, at::arange(size_, opt).repeat_interleave(m)) && ok;
      if (ic.error_word() != 0) {
        ok = false;
        why = "a cross-GPU barrier timed out";
      } else if (!ok) {
        why = "wrong data";
      }
    } catch (const std::exception& e) {
      ok = false;
      why = e.what();
    }
    if (const char* f = std::getenv("PDCC_IPC_SELFTEST_FAIL"))  // test hook: this rank reports a failure
      if (*f && std::atoi(f) == rank_) {
        ok = false;
        why = "PDCC_IPC_SELFTEST_FAIL";
      }
    all = vote("pdcc/ipc_selftest/result", ok);
  }
  if (!all) {
    fprintf(stderr, "[pdcc r%d] IPC self-test failed (%s): group '%s' runs without the peer-memory path\n", rank_,
            ok ? "on another rank" : why.c_str(), group_name_.c_str());
    // every rank voted after its own kernels finished: nothing touches these buffers any more
    if (ds.ipc) ds.ipc->release(std::chrono::milliseconds(std::max<int64_t>(1, std::min<int64_t>(timeout_.count(), 30000))));
    ds.ipc.reset();
    return false;
  }
  // zero-copy IPC (user buffers mapped per call and read in place): whole rows /
  // tiles zero-copy plus a staged rest, twice on one buffer (first and cached
  // mapping), all-gather with a ragged tail, reduce-scatter of a flat input
  ds.zc_ok = false;
  if (cfg_.ipc_zc) {
    bool zok = true;
    std::string zwhy;
    IpcComm& ic = *ds.ipc;
    try {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(ds.stream);
      const hipStream_t s = ds.stream.stream();
      const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
      const int64_t tile_f = kern::kTileBytes / 4;
      const int64_t n = 3 * size_ * tile_f + 257;
      const at::Tensor base = at::arange(n, opt).remainder(5);
      at::Tensor x = base + (double)(rank_ + 1);
      const double tri = size_ * (size_ + 1) / 2.0;
      for (int k = 0; k < 2; ++k) {
        kern::IpcCall c{};
        c.coll = kern::IpcColl::ALLREDUCE_2SHOT;
        c.dtype = kern::DType::F32;
        c.op = kern::RedOp::SUM;
        c.avg_div = size_;
        c.bytes = x.nbytes();
        c.in[0] = x.data_ptr();
        c.out[0] = x.data_ptr();
        ipc_run(ds, c, x.data_ptr(), x.nbytes(), (size_t)size_ * kern::kTileBytes, ic.max_staging(), s,
                k == 0 ? "pdcc/ipc_selftest/zc_ar0" : "pdcc/ipc_selftest/zc_ar1");
        const at::Tensor want = k == 0 ? base * (double)size_ + tri : (base * (double)size_ + tri) * (double)size_;
        zok = at::equal(x, want) && zok;
      }
      const int64_t m = 2 * tile_f + 5;
      const at::Tensor in = at::full({m}, (double)rank_, opt);
      at::Tensor out = at::full({m * size_}, -1.0, opt);
      {
        kern::IpcCall c{};
        c.coll = kern::IpcColl::ALLGATHER;
        c.dtype = kern::DType::U8;
        c.op = kern::RedOp::COPY;
        c.bytes = in.nbytes();
        c.in[0] = in.data_ptr();
        for (int r = 0; r < size_; ++r) c.out[r] = static_cast<char*>(out.data_ptr()) + r * in.nbytes();
        ipc_run(ds, c, in.data_ptr(), in.nbytes(), kern::kTileBytes, ic.max_staging(), s, "pdcc/ipc_selftest/zc_ag");
        zok = at::equal(out, at::arange(size_, opt).repeat_interleave(m)) && zok;
      }
      {
        const at::Tensor rin = at::arange(size_ * 2 * tile_f, opt).remainder(3) + (double)rank_;
        at::Tensor rout = at::full({2 * tile_f}, -1.0, opt);
        kern::IpcCall c{};
        c.coll = kern::IpcColl::REDUCE_SCATTER;
        c.dtype = kern::DType::F32;
        c.op = kern::RedOp::SUM;
        c.avg_div = size_;
        c.bytes = rout.nbytes();
        c.zstride = rout.nbytes();
        for (int r = 0; r < size_; ++r) c.in[r] = static_cast<const char*>(rin.data_ptr()) + r * rout.nbytes();
        c.out[0] = rout.data_ptr();
        ipc_run(ds, c, rin.data_ptr(), rin.nbytes(), kern::kTileBytes, ic.max_staging(), s, "pdcc/ipc_selftest/zc_rs");
        const at::Tensor mine = rin.narrow(0, rank_ * 2 * tile_f, 2 * tile_f) - (double)rank_;
        zok = at::equal(rout, mine * (double)size_ + (size_ - 1) * size_ / 2.0) && zok;
      }
      PDCC_HIP(hipStreamSynchronize(s));
      if (ic.error_word() != 0) {
        zok = false;
        zwhy = "a cross-GPU barrier timed out";
        ic.clear_error();
      } else if (!zok) {
        zwhy = "wrong data";
      }
    } catch (const std::exception& e) {
      zok = false;
      zwhy = e.what();
    }
    if (const char* f = std::getenv("PDCC_IPC_ZC_SELFTEST_FAIL"))  // test hook: this rank reports a failure
      if (*f && std::atoi(f) == rank_) {
        zok = false;
        zwhy = "PDCC_IPC_ZC_SELFTEST_FAIL";
      }
    ds.zc_ok = vote("pdcc/ipc_selftest/zc", zok);
    if (!ds.zc_ok)
      fprintf(stderr, "[pdcc r%d] zero-copy IPC self-test failed (%s): group '%s' stages every IPC call\n", rank_,
              zok ? "on another rank" : zwhy.c_str(), group_name_.c_str());
  }
  // Device-side record exchange of gated zero-copy launches (design.md §3): a gated all-reduce
  // on a buffer every rank has mapped now must resolve on the device -- its host gate is not
  // opened unless the kernel is still running after a grace period (then: staged fallback,
  // and the device exchange stays off for the group)
  // (every rank votes, also one whose PDCC_IPC_ZX=0 skips the test: the ranks agree without
  // depending on the environment being the same everywhere)
  ds.zx_ok = false;
  if (ds.zc_ok) {
    bool xok = cfg_.ipc_zx;
    std::string xwhy = xok ? "" : "PDCC_IPC_ZX=0";
    IpcComm& ic = *ds.ipc;
    ic.set_zx(cfg_.ipc_zx);
    if (xok) try {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(ds.stream);
      const hipStream_t s = ds.stream.stream();
      const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
      const int64_t row = (int64_t)size_ * (kern::kTileBytes / 4);
      const at::Tensor base = at::arange(4 * row, opt).remainder(7);
      at::Tensor x = base + (double)rank_;
      // map x everywhere first (inline exchange through the store, like the zc self-test)
      kern::IpcCall c{};
      c.coll = kern::IpcColl::ALLREDUCE_2SHOT;
      c.dtype = kern::DType::F32;
      c.op = kern::RedOp::SUM;
      c.avg_div = size_;
      c.bytes = x.nbytes();
      c.in[0] = x.data_ptr();
      c.out[0] = x.data_ptr();
      ipc_run(ds, c, x.data_ptr(), x.nbytes(), (size_t)size_ * kern::kTileBytes, ic.max_staging(), s,
              "pdcc/ipc_selftest/zx_map");
      const IpcComm::ZcRec mine = ic.zc_export(x.data_ptr(), x.nbytes(), false);
      const uint64_t t = ic.gate_reserve();
      ic.launch_gated(c, t, 0, mine, x.data_ptr(), s);
      auto ev = ic.gate_mark(t, s);
      const uint64_t tag = ic.zx_last_tag();
      const auto t0 = std::chrono::steady_clock::now();
      while (hipEventQuery(ev->ev) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(std::max<int64_t>(2000, spin_ms / 4)))
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      (void)hipGetLastError();
      ic.gate_publish(t, false, {});  // (a kernel still waiting for the host gate runs staged now)
      PDCC_HIP(hipStreamSynchronize(s));
      const at::Tensor once = base * (double)size_ + size_ * (size_ - 1) / 2.0;  // after the mapping call
      const bool data_ok = at::equal(x, once * (double)size_);
      const uint32_t verdict = ic.zx_verdict(tag);
      if (ic.error_word() != 0) {
        xok = false;
        xwhy = "the device exchange or a barrier timed out";
        ic.clear_error();
      } else if (verdict != 1u) {
        xok = false;
        xwhy = "the kernel did not resolve the buffers on the device (verdict " + std::to_string(verdict) + ")";
      } else if (!data_ok) {
        xok = false;
        xwhy = "wrong data";
      }
    } catch (const std::exception& e) {
      xok = false;
      xwhy = e.what();
    }
    if (const char* f = std::getenv("PDCC_IPC_ZX_SELFTEST_FAIL"))  // test hook: this rank reports a failure
      if (*f && std::atoi(f) == rank_) {
        xok = false;
        xwhy = "PDCC_IPC_ZX_SELFTEST_FAIL";
      }
    const bool zx = vote("pdcc/ipc_selftest/zx", xok);
    ic.set_zx(zx);
    ds.zx_ok = zx;
    if (!zx && cfg_.ipc_zx)
      fprintf(stderr, "[pdcc r%d] device-side zero-copy exchange self-test failed (%s): group '%s' gates zero-copy "
              "calls on the host\n", rank_, xok ? "on another rank" : xwhy.c_str(), group_name_.c_str());
  }
  // LL all-reduce: payloads with a partial last line and the largest one, each twice
  // (both slot parities), bf16 and f32
  ds.ll_ok = false;
  if (cfg_.ipc_ll_max > 0) {
    bool lok = true;
    std::string lwhy;
    IpcComm& ic = *ds.ipc;
    try {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(ds.stream);
      const hipStream_t s = ds.stream.stream();
      const double tri = size_ * (size_ + 1) / 2.0;
      const int64_t full = (int64_t)(kern::kLLMaxBytes / 4);
      for (const int64_t n : {int64_t{1}, int64_t{1001}, full, full}) {
        for (const auto dt : {at::kFloat, at::kBFloat16}) {
          const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(dt);
          const int64_t ne = dt == at::kFloat ? n : std::max<int64_t>(1, n / 2 - 1);  // bf16: odd byte counts too
          const at::Tensor base = at::arange(ne, opt).remainder(3);
          at::Tensor x = base + (double)(rank_ + 1);
          kern::IpcCall c{};
          c.coll = kern::IpcColl::ALLREDUCE_LL;
          c.dtype = dt == at::kFloat ? kern::DType::F32 : kern::DType::BF16;
          c.op = kern::RedOp::SUM;
          c.avg_div = size_;
          c.bytes = x.nbytes();
          c.in[0] = x.data_ptr();
          c.out[0] = x.data_ptr();
          ic.launch(c, s);
          lok = at::equal(x, base * (double)size_ + tri) && lok;
        }
      }
      for (const int64_t m : {int64_t{3}, full}) {  // all-gather: a partial line, the maximum
        const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
        const at::Tensor in = at::full({m}, (double)rank_, opt);
        at::Tensor out = at::full({m * size_}, -1.0, opt);
        kern::IpcCall c{};
        c.coll = kern::IpcColl::ALLGATHER_LL;
        c.dtype = kern::DType::U8;
        c.op = kern::RedOp::COPY;
        c.bytes = in.nbytes();
        c.in[0] = in.data_ptr();
        for (int r = 0; r < size_; ++r) c.out[r] = static_cast<char*>(out.data_ptr()) + r * in.nbytes();
        ic.launch(c, s);
        lok = at::equal(out, at::arange(size_, opt).repeat_interleave(m)) && lok;
      }
      // rooted kinds (tokens on the pairs without data), first and last rank as root, a partial line
      for (const int root : {0, size_ - 1}) {
        const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
        const int64_t m = 1001;
        const bool am_root = rank_ == root;
        kern::IpcCall c{};
        c.dtype = kern::DType::U8;
        c.op = kern::RedOp::COPY;
        c.root = root;
        c.bytes = (size_t)m * 4;
        at::Tensor b = at::full({m}, am_root ? 7.0 : -1.0, opt);  // broadcast
        c.coll = kern::IpcColl::BROADCAST_LL;
        c.in[0] = b.data_ptr();
        c.out[0] = b.data_ptr();
        ic.launch(c, s);
        lok = at::equal(b, at::full({m}, 7.0, opt)) && lok;
        const at::Tensor src = at::arange(size_ * m, opt).view({size_, m}).add((double)rank_);  // scatter
        at::Tensor sc = at::full({m}, -1.0, opt);
        c.coll = kern::IpcColl::SCATTER_LL;
        for (int r = 0; r < size_; ++r) c.in[r] = am_root ? src[r].data_ptr() : nullptr;
        c.out[0] = sc.data_ptr();
        ic.launch(c, s);
        lok = at::equal(sc, at::arange(m, opt).add((double)(rank_ * m + root))) && lok;
        const at::Tensor gi = at::full({m}, (double)rank_, opt);  // gather
        at::Tensor go = at::full({size_, m}, -1.0, opt);
        c.coll = kern::IpcColl::GATHER_LL;
        c.in[0] = gi.data_ptr();
        for (int r = 0; r < size_; ++r) c.out[r] = am_root ? go[r].data_ptr() : nullptr;
        ic.launch(c, s);
        lok = (am_root ? at::equal(go, at::arange(size_, opt).view({size_, 1}).expand({size_, m}))
                       : at::equal(go, at::full({size_, m}, -1.0, opt))) && lok;
        const at::Tensor rb = at::arange(m, opt).remainder(5);  // reduce (non-root tensors untouched)
        at::Tensor rx = rb + (double)(rank_ + 1);
        c.coll = kern::IpcColl::REDUCE_LL;
        c.dtype = kern::DType::F32;
        c.op = kern::RedOp::SUM;
        c.avg_div = size_;
        c.in[0] = rx.data_ptr();
        c.out[0] = rx.data_ptr();
        ic.launch(c, s);
        const double tri = size_ * (size_ + 1) / 2.0;
        lok = at::equal(rx, am_root ? rb * (double)size_ + tri : rb + (double)(rank_ + 1)) && lok;
      }
      {  // reduce-scatter and all-to-all: chunk q to rank q (a partial line per chunk)
        const auto opt = at::TensorOptions().device(at::kCUDA, ds.device).dtype(at::kFloat);
        const int64_t m = 333;
        const at::Tensor src = at::arange(size_, opt).view({size_, 1}).add((double)(100 * rank_)).expand({size_, m})
                                   .contiguous();  // chunk q = 100 * rank + q
        at::Tensor rs = at::full({m}, -1.0, opt);
        at::Tensor a2a = at::full({size_, m}, -1.0, opt);
        kern::IpcCall c{};
        c.coll = kern::IpcColl::REDUCE_SCATTER_LL;
        c.dtype = kern::DType::F32;
        c.op = kern::RedOp::SUM;
        c.avg_div = size_;
        c.bytes = (size_t)m * 4;
        for (int r = 0; r < size_; ++r) c.in[r] = src[r].data_ptr();
        c.out[0] = rs.data_ptr();
        ic.launch(c, s);
        lok = at::equal(rs, at::full({m}, 100.0 * (tri - size_) + (double)(size_ * rank_), opt)) && lok;
        c.coll = kern::IpcColl::ALLTOALL_LL;
        c.dtype = kern::DType::U8;
        c.op = kern::RedOp::COPY;
        for (int r = 0; r < size_; ++r) c.out[r] = a2a[r].data_ptr();
        ic.launch(c, s);
        lok = at::equal(a2a, at::arange(size_, opt).mul(100.0).add((double)rank_).view({size_, 1}).expand({size_, m}))
              && lok;
      }
      PDCC_HIP(hipStreamSynchronize(s));
      if (ic.error_word() != 0) {
        lok = false;
        lwhy = "an LL poll timed out";
        ic.clear_error();
      } else if (!lok) {
        lwhy = "wrong data";
      }
    } catch (const std::exception& e) {
      lok = false;
      lwhy = e.what();
    }
    if (const char* f = std::getenv("PDCC_IPC_LL_SELFTEST_FAIL"))  // test hook: this rank reports a failure
      if (*f && std::atoi(f) == rank_) {
        lok = false;
        lwhy = "PDCC_IPC_LL_SELFTEST_FAIL";
      }
    ds.ll_ok = vote("pdcc/ipc_selftest/ll", lok);
    if (!ds.ll_ok)
      fprintf(stderr, "[pdcc r%d] LL all-reduce self-test failed (%s): group '%s' uses the 1-shot protocol\n", rank_,
              lok ? "on another rank" : lwhy.c_str(), group_name_.c_str());
  }
  ds.ipc->set_timeout_ms((uint64_t)std::max<int64_t>(1, std::min<int64_t>(cfg_.ipc_spin_ms, timeout_.count())));
  return true;
}

}  // namespace pdcc
