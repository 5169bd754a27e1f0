#include "ipc_comm.h"

#include <hip/hip_runtime_api.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <utility>

#include "comm_util.h"

namespace pdcc {

namespace {

// A hipIpc handle names the runtime's underlying allocation, which may be larger
// than (and start before) the pointer we exported: the runtime is free to
// sub-allocate. Export (handle, offset of p from its allocation base) and add the
// offset back after opening -- without it a second group's buffers would alias
// the first group's on the peer side.
//
// Every exported buffer also carries a random 64-bit nonce in its last 8 bytes, published with the
// handle: the importer reads it back through the mapping it was given, so a mapping that does not show
// the exporter's fresh buffer (a stale one the runtime handed back) is caught before any kernel uses it;
// it is closed and opened again (`ipc_stale_maps`). Added while chasing wrong sums in re-made groups on a
// shared GPU; none was ever seen -- the cause was elsewhere (release(), profiles/r6/regroup/README.md).
constexpr size_t kNonceBytes = 64;  // reserved at the end of every exported buffer
std::atomic<uint64_t> g_stale_maps{0};

uint64_t fresh_nonce() {
  static std::atomic<uint64_t> ctr{0};
  static const uint64_t seed = [] {
    std::random_device rd;
    return ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)getpid() << 17);
  }();
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (++ctr);  // splitmix64
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return (z ^ (z >> 31)) | 1u;  // (never 0: zeroed memory never matches)
}

// PDCC_IPC_VA_LOG=1 (debug): every IPC buffer this process allocates, maps, frees or unmaps, with its
// address range, on stderr
bool va_log_on() {
  static const bool on = [] {
    const char* e = std::getenv("PDCC_IPC_VA_LOG");
    return e && *e == '1';
  }();
  return on;
}
void va_note(const char* what, void* p) {
  if (!va_log_on() || !p) return;
  hipDeviceptr_t base = nullptr;
  size_t range = 0;
  if (hipMemGetAddressRange(&base, &range, reinterpret_cast<hipDeviceptr_t>(p)) != hipSuccess) (void)hipGetLastError();
  fprintf(stderr, "[pdcc va %d] %s %p base %p range %zu\n", (int)getpid(), what, p, (void*)base, range);
}
hipError_t ipc_close(void* m) {
  va_note("close", m);
  return hipIpcCloseMemHandle(m);
}
hipError_t dev_free(void* p) {
  va_note("free", p);
  return hipFree(p);
}

std::vector<uint8_t> handle_bytes(void* p, size_t bytes) {
  hipIpcMemHandle_t h;
  PDCC_HIP(hipIpcGetMemHandle(&h, p));
  hipDeviceptr_t base = nullptr;
  size_t range = 0;
  PDCC_HIP(hipMemGetAddressRange(&base, &range, reinterpret_cast<hipDeviceptr_t>(p)));
  const uint64_t off = static_cast<uint64_t>(static_cast<char*>(p) - static_cast<char*>(base));
  const uint64_t nonce = fresh_nonce(), at = bytes - sizeof(uint64_t);
  PDCC_HIP(hipMemcpy(static_cast<char*>(p) + at, &nonce, sizeof(nonce), hipMemcpyHostToDevice));
  std::vector<uint8_t> out(sizeof(h) + 3 * sizeof(uint64_t));
  std::memcpy(out.data(), &h, sizeof(h));
  std::memcpy(out.data() + sizeof(h), &off, sizeof(off));
  std::memcpy(out.data() + sizeof(h) + 8, &nonce, sizeof(nonce));
  std::memcpy(out.data() + sizeof(h) + 16, &at, sizeof(at));
  return out;
}

// returns {mapping to close later, usable pointer}
std::pair<void*, void*> open_handle(const std::vector<uint8_t>& b) {
  hipIpcMemHandle_t h;
  uint64_t off = 0, nonce = 0, at = 0;
  if (b.size() != sizeof(h) + 3 * sizeof(uint64_t)) throw std::runtime_error("pdcc: malformed hipIpc handle in store");
  std::memcpy(&h, b.data(), sizeof(h));
  std::memcpy(&off, b.data() + sizeof(h), sizeof(off));
  std::memcpy(&nonce, b.data() + sizeof(h) + 8, sizeof(nonce));
  std::memcpy(&at, b.data() + sizeof(h) + 16, sizeof(at));
  for (int attempt = 0;; ++attempt) {
    void* p = nullptr;
    PDCC_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    uint64_t seen = 0;
    PDCC_HIP(hipMemcpy(&seen, static_cast<char*>(p) + off + at, sizeof(seen), hipMemcpyDeviceToHost));
    if (seen == nonce) {
      va_note("open", p);
      return {p, static_cast<char*>(p) + off};
    }
    ++g_stale_maps;
    (void)ipc_close(p);
    if (attempt >= 50)
      throw std::runtime_error("pdcc: hipIpcOpenMemHandle keeps returning a stale mapping of a peer's IPC buffer");
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

// Allocate `bytes` of device memory and export it. With two ranks on one device
// the runtime can hand back a range it just unmapped for a closed peer import,
// and then refuses to export it (hipIpcGetMemHandle: invalid argument). Such a
// block is held (so the next try gets a different range) and freed once an
// exportable one is found. `uncached` selects fine-grained memory (signals).
void* alloc_exportable(size_t bytes, bool uncached, std::vector<uint8_t>& blob, std::vector<void*>* defer = nullptr) {
  std::vector<void*> refused;
  auto release = [&] {  // (deferred: hipFree synchronises the device, see IpcComm::defer_frees)
    for (void* q : refused) {
      if (defer) defer->push_back(q);
      else dev_free(q);
    }
  };
  for (int attempt = 0; attempt < 6; ++attempt) {
    void* p = nullptr;
    hipError_t e = uncached ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) : hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      release();
      PDCC_HIP(e);
    }
    try {
      blob = handle_bytes(p, bytes);
      va_note(uncached ? "alloc-uncached" : "alloc", p);
      release();
      return p;
    } catch (const std::exception&) {
      (void)hipGetLastError();
      refused.push_back(p);
    }
  }
  release();
  throw std::runtime_error("pdcc: hipIpcGetMemHandle refused 6 fresh allocations of " + std::to_string(bytes) +
                           " bytes");
}

// own allocations in whole 2 MiB granules, so the runtime never packs two of
// them (or anybody else's) into one IPC-exported allocation
constexpr size_t kGranule = 2u << 20;
size_t granule(size_t b) { return (b + kGranule - 1) / kGranule * kGranule; }

struct DeviceScope {
  int prev = 0;
  explicit DeviceScope(int d) {
    PDCC_HIP(hipGetDevice(&prev));
    if (prev != d) PDCC_HIP(hipSetDevice(d));
  }
  ~DeviceScope() { hipSetDevice(prev); }
};

// An empty blob in the store means "this rank could not export": every rank
// checks all blobs before opening any, so the whole group fails the same step
// instead of some ranks waiting on the store for a handle that never comes.
void check_blobs(const std::vector<std::vector<uint8_t>>& all, int self, const char* what) {
  for (size_t r = 0; r < all.size(); ++r)
    if ((int)r != self && all[r].empty())
      throw std::runtime_error("pdcc: rank " + std::to_string(r) + " could not export its IPC " + what);
}

}  // namespace

uint64_t IpcComm::stale_mappings() { return g_stale_maps.load(); }

IpcComm::IpcComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
                 int device, size_t max_staging, uint64_t timeout_ms, bool shared_device, size_t zc_cache)
    : store_(store),
      key_(key),
      rank_(rank),
      world_(world),
      device_(device),
      max_staging_(std::max<size_t>(max_staging, 1u << 20)),
      timeout_ticks_(timeout_ms * 100000ull),  // s_memrealtime runs at 100 MHz
      shared_device_(shared_device) {
  zc_imports_.assign(world, {});
  keep_exports_ = shared_device;
  if (const char* lv = std::getenv("PDCC_LOG_LEVEL")) log_ = std::atoi(lv);
  shared_grid_ = std::max(1, 256 / std::max(1, world));
  shared_wide_grid_ = std::max(1, kSharedWideSlots / std::max(1, world) - 1);
  zc_cache_ = std::max<size_t>(zc_cache, 1);
  closing_limit_ = std::max<size_t>(2, (size_t)kern::kZcTab > zc_cache_ ? (size_t)kern::kZcTab - zc_cache_ : 0);
  if (world < 2 || world > kern::kMaxRanks)
    throw std::runtime_error("pdcc: the IPC path supports 2..8 ranks per group");
  DeviceScope ds(device);
  std::vector<uint8_t> mine;
  std::string err;
  try {
    const size_t sig = granule(kern::ipc_signal_bytes() + kNonceBytes);
    my_flags_ = static_cast<uint32_t*>(alloc_exportable(sig, true, mine));
    PDCC_HIP(hipMemset(my_flags_, 0, sig - kNonceBytes));  // (not the nonce at the end)
    // the dynamic protocols' own control words: ordinary device memory (only this device's blocks)
    PDCC_HIP(hipMalloc(reinterpret_cast<void**>(&dyn_ctl_), kern::kDynCtlBytes));
    PDCC_HIP(hipMemset(dyn_ctl_, 0, kern::kDynCtlBytes));
    if (const char* ep = std::getenv("PDCC_TEST_ZX_EPOCH")) {  // test hook: start the exchange epoch near the wrap
      const uint32_t v = (uint32_t)std::strtoul(ep, nullptr, 0);
      PDCC_HIP(hipMemcpy(reinterpret_cast<char*>(my_flags_) + kern::kZxEpochOffset, &v, sizeof(v),
                         hipMemcpyHostToDevice));
    }
    PDCC_HIP(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 64, hipHostMallocMapped | hipHostMallocCoherent));
    *err_host_ = 0;
    PDCC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0));
    PDCC_HIP(hipHostMalloc(reinterpret_cast<void**>(&gates_host_), kern::kGateSlots * sizeof(kern::GateSlot),
                           hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(gates_host_, 0, kern::kGateSlots * sizeof(kern::GateSlot));
    PDCC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&gates_dev_), gates_host_, 0));
    gate_last_.assign(kern::kGateSlots, nullptr);
    PDCC_HIP(hipHostMalloc(reinterpret_cast<void**>(&ztab_host_), sizeof(kern::ZcTable),
                           hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(ztab_host_, 0, sizeof(kern::ZcTable));
    PDCC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&ztab_dev_), ztab_host_, 0));
    if (const char* tr = std::getenv("PDCC_IPC_TRACE")) {
      const long n = std::atol(tr);
      if (n > 0) {
        trace_cap_ = (uint32_t)std::min<long>(n, 1 << 20);
        const size_t tb = (size_t)trace_cap_ * kern::kTraceRecWords * sizeof(uint64_t);
        PDCC_HIP(hipHostMalloc(reinterpret_cast<void**>(&trace_host_), tb, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(trace_host_, 0, tb);
        PDCC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&trace_dev_), trace_host_, 0));
      }
    }
    PDCC_HIP(hipStreamSynchronize(nullptr));  // the memset (null stream) is done before peers map it
  } catch (const std::exception& e) {
    err = e.what();
    mine.clear();  // published empty: the peers fail this step with us
  }
  const auto all = store_allgather(store_, key_ + "/ipc_sig", rank_, world_, mine);
  if (!err.empty()) throw std::runtime_error(err);
  check_blobs(all, rank_, "signal area");
  peer_flags_.assign(world_, nullptr);
  flags_maps_.assign(world_, nullptr);
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      peer_flags_[r] = my_flags_;
      continue;
    }
    auto m = open_handle(all[r]);
    flags_maps_[r] = m.first;
    peer_flags_[r] = static_cast<uint32_t*>(m.second);
  }
}

void IpcComm::drop_map(void* m) {
  if (m) (void)ipc_close(m);
}

IpcComm::~IpcComm() {
  release(std::chrono::milliseconds(0));
  if (err_host_) hipHostFree(err_host_);
}

// Teardown order across the group: every rank closes its mappings of the peers' buffers, the ranks
// meet, and only then does each free what it exported -- never a free under a peer's mapping. Without
// the meeting (no deadline given, or a peer that never arrives) the exported buffers are kept (a leak
// of the signal area and staging). Ranks sharing one GPU never free them at all (keep_exports_): there,
// a buffer a peer had mapped, once unmapped and freed -- in either order, with the meeting too -- came
// back to both processes at once (the next group's fresh tensor zeroed by a peer's memset;
// tests/_workers.py::regroup_probe / bulk_pre_diag, profiles/r6/regroup/README.md).
void IpcComm::release(std::chrono::milliseconds deadline) {
  if (released_) return;
  released_ = true;
  try {
    DeviceScope ds(device_);
    graph_mode_ = false;  // the group is gone: staging retired for captured graphs goes too
    // 1. this rank's mappings of the peers' memory
    for (void* m : staging_maps_)
      if (m) drop_map(m);
    staging_maps_.clear();
    peer_staging_.clear();
    for (auto& r : retired_) {
      for (void* m : r.maps)
        if (m) drop_map(m);
      r.maps.clear();
      if (r.mine) parked_.push_back(r.mine);
    }
    retired_.clear();
    reap_closing(true);
    {
      std::lock_guard<std::mutex> il(imports_mu_);
      for (auto& peer : zc_imports_)
        for (auto& im : peer) {
          if (im.last && im.last->ev) (void)hipEventSynchronize(im.last->ev);
          if (im.map) drop_map(im.map);
        }
      zc_imports_.clear();
    }
    for (void* m : flags_maps_)
      if (m) drop_map(m);
    flags_maps_.clear();
    peer_flags_.clear();
    // 2. never exported: free now
    for (void* q : deferred_free_) dev_free(q);
    deferred_free_.clear();
    if (dyn_ctl_) dev_free(dyn_ctl_);
    dyn_ctl_ = nullptr;
    gate_last_.clear();
    if (gates_host_) hipHostFree(gates_host_);
    gates_host_ = nullptr;
    if (ztab_host_) hipHostFree(ztab_host_);
    ztab_host_ = nullptr;
    if (trace_host_) hipHostFree(trace_host_);
    trace_host_ = nullptr;
    // 3. exported: once every rank has closed its mappings of them
    if (my_staging_) parked_.push_back(my_staging_);
    my_staging_ = nullptr;
    cap_ = 0;
    if (my_flags_) parked_.push_back(reinterpret_cast<char*>(my_flags_));
    my_flags_ = nullptr;
    const bool met = !keep_exports_ && deadline.count() > 0 && store_barrier_for(store_, key_ + "/ipc_release", rank_, world_, deadline);
    if (met) {
      for (char* q : parked_) dev_free(q);
    } else if (keep_exports_) {
      kept_exports_ += parked_.size();  // ranks sharing one GPU: see keep_exports_
    } else if (!parked_.empty() && log_ >= 1) {
      fprintf(stderr, "[pdcc r%d] ipc: the group ended without every rank's teardown: its %zu exported buffer(s) "
              "stay allocated\n", rank_, parked_.size());
    }
    parked_.clear();
  } catch (...) {
  }
}

thread_local bool IpcComm::tls_defer_frees_ = false;

void IpcComm::map_staging(size_t cap) {
  // the new buffer is allocated and exported while the old one and the peers'
  // old mappings still hold their ranges, so it cannot land on a just-closed import
  std::vector<uint8_t> mine;
  std::string err;
  char* fresh = nullptr;
  try {
    fresh = static_cast<char*>(
        alloc_exportable(granule(cap + kNonceBytes), false, mine, tls_defer_frees_ ? &deferred_free_ : nullptr));
  } catch (const std::exception& e) {
    err = e.what();
    mine.clear();
  }
  // the old staging goes before the exchange: this rank's mappings of the peers' old buffers closed, its
  // own old buffer freed (kept instead while a captured graph or the launcher's thread may use it). This
  // order is the one measured clean on a shared GPU: keeping the old buffers until the new ones were
  // mapped everywhere, then closing / freeing (or parking) them, was followed by wrong results in later
  // calls (profiles/r6/regroup/README.md)
  if (graph_mode_ || tls_defer_frees_) {
    if (my_staging_) retired_.push_back({my_staging_, staging_maps_});
  } else {
    for (void* m : staging_maps_)
      if (m) drop_map(m);
    if (my_staging_ && keep_exports_) ++kept_exports_;
    else if (my_staging_) dev_free(my_staging_);
  }
  staging_maps_.clear();
  peer_staging_.clear();
  my_staging_ = nullptr;
  cap_ = 0;
  const auto all = store_allgather(store_, key_ + "/ipc_stg/" + std::to_string(staging_gen_), rank_, world_, mine);
  try {
    if (!err.empty()) throw std::runtime_error(err);
    check_blobs(all, rank_, "staging buffer");
  } catch (...) {
    if (fresh) dev_free(fresh);  // nobody opened it: every rank stops before opening
    throw;
  }
  my_staging_ = fresh;
  cap_ = cap;
  peer_staging_.assign(world_, nullptr);
  staging_maps_.assign(world_, nullptr);
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      peer_staging_[r] = my_staging_;
      continue;
    }
    auto m = open_handle(all[r]);
    staging_maps_[r] = m.first;
    peer_staging_[r] = static_cast<char*>(m.second);
  }
}

void IpcComm::ensure_staging(size_t bytes, hipStream_t stream) {
  bytes = (bytes + kern::kTileBytes - 1) / kern::kTileBytes * kern::kTileBytes;
  if (bytes <= cap_) return;
  if (bytes > max_staging_) throw std::runtime_error("pdcc: IPC call larger than PDCC_IPC_MAX_STAGING");
  DeviceScope ds(device_);
  size_t cap = std::max<size_t>(bytes, 4u << 20);
  cap = std::max(cap, std::min(max_staging_, cap_ * 2));
  if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: staging %zu -> %zu B\n", rank_, cap_, cap);
  // nobody may still read the old buffers: drain locally, then agree globally
  PDCC_HIP(hipStreamSynchronize(stream));
  ++staging_gen_;
  store_barrier(store_, key_ + "/ipc_grow/" + std::to_string(staging_gen_), rank_, world_);
  map_staging(cap);
}

void IpcComm::launch(kern::IpcCall call, hipStream_t stream) {
  call.zc = 0;
  prepare_staging(call, stream);
  launch_view(view(peer_staging_), call, stream);
}

void IpcComm::prepare_staging(const kern::IpcCall& call, hipStream_t stream) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  PDCC_HIP(hipStreamIsCapturing(stream, &cs));
  const bool capturing = cs != hipStreamCaptureStatusNone;
  const size_t need = kern::ipc_staging_bytes(call, world_);
  if (need > 0) {
    if (capturing && (need + kern::kTileBytes - 1) / kern::kTileBytes * kern::kTileBytes > cap_)
      throw std::runtime_error(
          "pdcc: this IPC collective needs more staging than the group has, and staging cannot grow while the "
          "stream is being captured into a graph: run the collective once before capturing it "
          "(parallel.graphs.capture does)");
    if (tls_defer_frees_ && (need + kern::kTileBytes - 1) / kern::kTileBytes * kern::kTileBytes > cap_)
      throw std::runtime_error("pdcc: an IPC launcher job needs " + std::to_string(need) + " B of staging, the group "
                               "has " + std::to_string(cap_) + " (staging is grown by the submitting thread only)");
    ensure_staging(need, stream);
  }
  // A captured graph bakes the staging pointers into its kernel arguments: from
  // now on staging is retired, never freed, when it grows.
  if (capturing) graph_mode_ = true;
}

kern::IpcView IpcComm::view(const std::vector<char*>& bufs) const {
  kern::IpcView v{};
  for (int r = 0; r < world_; ++r) {
    v.buf[r] = bufs.empty() ? nullptr : bufs[r];
    v.stg[r] = peer_staging_.empty() ? nullptr : peer_staging_[r];
    v.flags[r] = peer_flags_[r];
  }
  v.err = err_dev_;
  v.counters = my_flags_ + kern::kCountWord;
  v.dctl = dyn_ctl_;
  v.cap = cap_;
  v.rank = rank_;
  v.world = world_;
  v.timeout_ticks = timeout_ticks_;
  v.trace = trace_dev_;
  v.trace_cap = trace_cap_;
  return v;
}

void IpcComm::launch_view(const kern::IpcView& v, kern::IpcCall call, hipStream_t stream) {
  ++seq_;  // launches so far (informational: the kernels keep their own per-block call counters)
  if (shared_device_) {
    // All ranks' grids run on ONE device (test setups, rehearsals): small calls at 256 / W workgroups per
    // rank; from kSharedWideMin bytes per launch W x (cap + exchange block) = kSharedWideSlots in all, within
    // the 2-per-CU x 256-CU residency of the heaviest IPC kernels (65 KiB of LDS at W = 8). More workgroups
    // keep more loads in flight: 1 GiB all_reduce 1411 -> 1213 us (W = 2), 3842 -> 2850 (W = 4, static),
    // 6745 -> 5140 (W = 8); calls of 4-16 MiB lose 5-15 % with them (profiles/r5/shared_grid_*.jsonl)
    call.grid_cap = call.bytes >= kSharedWideMin ? shared_wide_grid_ : shared_grid_;
  } else if (grid_max_ > 0 && call.grid_cap <= 0) {  // (a call may carry its own cap: IPC_WIDE)
    call.grid_cap = grid_max_;
  }
  if (async_now_ && async_grid_ > 0) {  // overlapped with compute: leave CU slots to it
    call.grid_cap = call.grid_cap > 0 ? std::min(call.grid_cap, async_grid_) : async_grid_;
    ++async_capped_;
  }
  DeviceScope ds(device_);
  if (!v.trace) {
    PDCC_HIP(kern::ipc_launch(v, call, stream));
    return;
  }
  kern::IpcView tv = v;  // PDCC_IPC_TRACE: every block of this launch files into one record
  tv.trace_slot = seq_ % trace_cap_;
  PDCC_HIP(kern::ipc_launch(tv, call, stream));
}

// ------------------------------------------------------------------ zero copy
IpcComm::ZcRec IpcComm::zc_export(const void* p, size_t len, bool capturing) {
  std::lock_guard<std::mutex> zl(zc_mu_);
  ZcRec r{};
  r.full = zc_closing() >= closing_limit_ ? 1 : 0;
  if (!p && len == 0) {  // this rank has nothing the peers read (a scatter's non-root)
    r.ok = 1;
    return r;
  }
  if (!p || len == 0 || (reinterpret_cast<uintptr_t>(p) & 15u) != 0) return r;
  DeviceScope ds(device_);
  hipDeviceptr_t base = nullptr;
  size_t range = 0;
  if (hipMemGetAddressRange(&base, &range, reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) != hipSuccess) {
    (void)hipGetLastError();
    return r;
  }
  const uint64_t off = static_cast<uint64_t>(static_cast<const char*>(p) - static_cast<char*>(base));
  if (off + len > range) return r;  // the readable span must lie inside one allocation
  // An allocation whose size has bit 31 set (2-4 GiB, 6-8 GiB, ...) is never exported: a peer's
  // hipIpcOpenMemHandle of it does not return (this ROCm 7 image, dmabuf IPC) -- the exchange stalls and
  // every rank's gated kernels spin to their timeout, or, exchanging on the caller's thread, the group
  // hangs. Measured with one process per rank on one MI355X (scripts/ag_probe.py, profiles/r5/
  // zc_size_rule.md): 1024 / 2046 / 4096 / 5120 / 8192 MiB inputs map at once; 2048 / 2050 / 3072 /
  // 6144 MiB stall. Such a buffer runs the staged protocol (PDCC_IPC_ZC_SIZE_GUARD=0 lifts the guard).
  if (size_guard_ && (range & (size_t{1} << 31)) != 0) {
    ++size_refusals_;
    return r;
  }
  uint64_t id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, base) != hipSuccess || id == 0) {
    (void)hipGetLastError();
    return r;
  }
  const bool full = zc_closing() >= closing_limit_;
  r.full = full ? 1 : 0;
  auto it = std::find_if(zc_exports_.begin(), zc_exports_.end(),
                         [&](const ZcExport& e) { return e.id == id && e.base == static_cast<char*>(base); });
  if (it == zc_exports_.end() && (full || peer_full_.load()) && !capturing) {
    ++full_refusals_;  // no fresh export (and so no eviction) until a safe point drains the lists
    return r;          // ok = 0: this call runs staged
  }
  if (it == zc_exports_.end()) {
    ZcExport e{};
    e.id = id;
    e.base = static_cast<char*>(base);
    if (hipIpcGetMemHandle(&e.handle, base) != hipSuccess) {
      (void)hipGetLastError();  // e.g. a range the runtime refuses to export (ranks sharing a device)
      ++export_failures_;
      return r;
    }
    // LRU eviction (never while capturing: importers could not drain their streams
    // before unmapping, and the graph may hold the pointers)
    if (zc_exports_.size() >= zc_cache_ && !capturing) {
      auto victim = zc_exports_.end();
      for (auto v = zc_exports_.begin(); v != zc_exports_.end(); ++v)
        if (!v->pinned && (victim == zc_exports_.end() || v->last < victim->last)) victim = v;
      if (victim != zc_exports_.end()) {
        if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: evict export id %llu\n", rank_, (unsigned long long)victim->id);
        r.evict = victim->id;
        zc_exports_.erase(victim);
      }
    }
    zc_exports_.push_back(e);
    it = zc_exports_.end() - 1;
  }
  it->last = ++zc_tick_;
  if (capturing) it->pinned = true;
  r.ok = 1;
  r.fresh = it->confirmed ? 0 : 1;
  r.id = id;
  r.off = off;
  r.len = len;
  r.handle = it->handle;
  return r;
}

IpcComm::LaunchEvent::~LaunchEvent() {
  if (!ev) return;
  if (pool) {
    std::lock_guard<std::mutex> lk(pool->mu);
    if (pool->free.size() < 256) {
      pool->free.push_back(ev);
      return;
    }
  }
  (void)hipEventDestroy(ev);
}

IpcComm::EventPool::~EventPool() {
  for (hipEvent_t e : free) (void)hipEventDestroy(e);
}

std::shared_ptr<IpcComm::LaunchEvent> IpcComm::new_launch_event(hipStream_t stream) {
  auto le = std::make_shared<LaunchEvent>();
  le->pool = ev_pool_;
  {
    std::lock_guard<std::mutex> lk(ev_pool_->mu);
    if (!ev_pool_->free.empty()) {
      le->ev = ev_pool_->free.back();
      ev_pool_->free.pop_back();
    }
  }
  DeviceScope ds(device_);
  if (!le->ev) PDCC_HIP(hipEventCreateWithFlags(&le->ev, hipEventDisableTiming));
  PDCC_HIP(hipEventRecord(le->ev, stream));
  return le;
}

void IpcComm::reap_closing(bool wait_all) {
  // pick the finished entries under the lock, close them outside it: a close synchronises
  // the device, and the launcher's thread must stay free to queue more meanwhile
  std::vector<Closing> done;
  {
    std::lock_guard<std::mutex> lk(closing_mu_);
    size_t keep = 0;
    for (size_t i = 0; i < zc_closing_.size(); ++i) {
      Closing& c = zc_closing_[i];
      bool fin = true;
      for (const auto& le : c.last) {
        if (!le || !le->ev) continue;
        const hipError_t e = wait_all ? hipEventSynchronize(le->ev) : hipEventQuery(le->ev);
        (void)hipGetLastError();
        if (e == hipErrorNotReady) {
          fin = false;
          break;
        }
      }
      if (fin) done.push_back(std::move(c));
      else zc_closing_[keep++] = std::move(c);
    }
    zc_closing_.resize(keep);
  }
  for (auto& c : done) {
    if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: close %p\n", rank_, c.map);
    if (c.map) drop_map(c.map);
  }
  if (!done.empty()) {
    std::lock_guard<std::mutex> lk(closing_mu_);
    for (auto& c : done) tab_release(c.tab_peer, c.tab_slot);
  }
}

bool IpcComm::zc_import(const std::vector<ZcRec>& all, const void* mine, bool all_ok, std::vector<char*>& ptrs) {
  DeviceScope ds(device_);
  std::lock_guard<std::mutex> il(imports_mu_);
  if (!tls_defer_frees_) reap_closing(false);
  // evictions first, whatever the outcome of this exchange (keeps the caches in step); an
  // in-flight kernel of this rank may still read through the mapping: the close waits for
  // the last launch that used it (reap_closing), not for the whole device
  for (int r = 0; r < world_; ++r) {
    if (r == rank_ || all[r].evict == 0) continue;
    auto& peer = zc_imports_[r];
    auto it = std::find_if(peer.begin(), peer.end(), [&](const ZcImport& im) { return im.id == all[r].evict; });
    if (it == peer.end()) continue;
    tab_drop(r, it->tab);  // no kernel launched from now on finds it
    {
      auto last = latest_gated();  // ... and the ones launched so far may still read through it
      last.push_back(it->last);
      std::lock_guard<std::mutex> lk(closing_mu_);
      zc_closing_.push_back({it->map, std::move(last), it->tab >= 0 ? r : -1, it->tab});
    }
    peer.erase(it);
  }
  if (!tls_defer_frees_) reap_closing(false);
  zc_cur_ids_.assign(world_, 0);
  bool any_full = false, fresh = false;
  for (int r = 0; r < world_; ++r) {
    any_full = any_full || all[r].full;
    fresh = fresh || (all[r].fresh && all[r].id != 0);
  }
  peer_full_.store(any_full);
  if (!all_ok) return false;
  if (any_full && fresh) {  // a rank cannot take another mapping before a safe point: staged
    ++full_refusals_;
    return false;
  }
  ptrs.assign(world_, nullptr);
  if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: import (%zu closing)\n", rank_, zc_closing_.size());
  bool ok = true;
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      ptrs[r] = static_cast<char*>(const_cast<void*>(mine));
      continue;
    }
    if (all[r].id == 0) continue;  // nothing to read from this rank
    auto& peer = zc_imports_[r];
    auto it = std::find_if(peer.begin(), peer.end(), [&](const ZcImport& im) { return im.id == all[r].id; });
    if (it == peer.end()) {
      void* m = nullptr;
      if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: open id %llu of rank %d\n", rank_, (unsigned long long)all[r].id, r);
      if (hipIpcOpenMemHandle(&m, all[r].handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !m) {
        (void)hipGetLastError();
        ++map_failures_;
        if (!all[r].fresh)  // every rank mapped it when it was fresh: this cannot be agreed on any more
          throw std::runtime_error("pdcc: zero-copy IPC: re-mapping a confirmed peer buffer failed on rank " +
                                   std::to_string(rank_));
        ok = false;
        continue;
      }
      va_note("open-zc", m);
      peer.push_back({all[r].id, m, nullptr, tab_insert(r, all[r].id, m)});
      it = peer.end() - 1;
    }
    zc_cur_ids_[r] = all[r].id;
    ptrs[r] = static_cast<char*>(it->map) + all[r].off;
    if (va_log_on())
      fprintf(stderr, "[pdcc va %d] zc r%d<-r%d id %llu map %p off %llu ptr %p mine %p\n", (int)getpid(), rank_, r,
              (unsigned long long)all[r].id, it->map, (unsigned long long)all[r].off, (void*)ptrs[r], mine);
  }
  return ok;
}

void IpcComm::zc_settle(const ZcRec& mine, bool ok) {
  // (the record of the exchange being settled, not the latest export: with gated launches the
  // caller may have exported later calls' buffers before this exchange ran)
  if (!mine.ok || !mine.fresh || mine.id == 0) return;
  std::lock_guard<std::mutex> zl(zc_mu_);
  auto it = std::find_if(zc_exports_.begin(), zc_exports_.end(), [&](const ZcExport& e) { return e.id == mine.id; });
  if (it != zc_exports_.end()) {
    if (ok) it->confirmed = true;
    else if (!it->pinned && !it->confirmed) zc_exports_.erase(it);  // announced fresh again next time
  }
}

void IpcComm::launch_zc(kern::IpcCall call, const std::vector<char*>& bufs, hipStream_t stream) {
  if ((int)bufs.size() != world_) throw std::runtime_error("pdcc: zero-copy IPC launch without every rank's buffer");
  call.zc = 1;
  prepare_staging(call, stream);  // (a rooted reduce stages its reduced tiles)
  if (log_ >= 3) fprintf(stderr, "[pdcc r%d] ipc: launch zc %zu B\n", rank_, call.bytes);
  launch_view(view(bufs), call, stream);
  // the mappings this launch reads through stay open until it has finished (eviction);
  // a captured launch reads exports pinned for the graph's lifetime (never evicted)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  zc_note_launch(new_launch_event(stream));
}

void IpcComm::zc_note_launch(const std::shared_ptr<LaunchEvent>& le) {
  std::lock_guard<std::mutex> il(imports_mu_);
  for (int r = 0; r < world_ && r < (int)zc_cur_ids_.size(); ++r) {
    if (r == rank_ || zc_cur_ids_[r] == 0) continue;
    for (auto& im : zc_imports_[r])
      if (im.id == zc_cur_ids_[r]) im.last = le;
  }
}

// ------------------------------------------------------------------ gated launches
uint64_t IpcComm::gate_reserve() {
  const uint64_t t = ++gate_next_;
  auto& prev = gate_last_[t % kern::kGateSlots];
  if (prev && prev->ev) {  // the launches of ticket t - kGateSlots read this slot
    DeviceScope ds(device_);
    if (hipEventQuery(prev->ev) == hipErrorNotReady) PDCC_HIP(hipEventSynchronize(prev->ev));
    (void)hipGetLastError();
  }
  prev.reset();
  kern::GateSlot* g = gates_host_ + (t % kern::kGateSlots);
  const uint32_t v = __atomic_exchange_n(&g->verdict, 0u, __ATOMIC_ACQ_REL);  // ticket t - kGateSlots's launch
  if (v == 0x101u) ++zx_fast_;
  else if (v == 0x102u) ++zx_host_;
  else if (v == 0x100u) ++zx_failed_;
  return t;
}

int IpcComm::tab_insert(int peer, uint64_t id, void* map) {
  if (!ztab_host_ || peer < 0 || peer >= kern::kMaxRanks) return -1;
  std::lock_guard<std::mutex> lk(closing_mu_);
  for (int j = 0; j < kern::kZcTab; ++j) {
    if (tab_busy_[peer][j]) continue;  // (a dropped slot stays busy until its mapping is closed)
    tab_busy_[peer][j] = true;
    __atomic_store_n(&ztab_host_->base[peer][j], reinterpret_cast<uint64_t>(map), __ATOMIC_RELAXED);
    __atomic_store_n(&ztab_host_->id[peer][j], id, __ATOMIC_RELEASE);  // last: the kernels match on it
    return j;
  }
  return -1;  // full: calls reading this buffer take the host gate
}

void IpcComm::tab_drop(int peer, int slot) {
  if (!ztab_host_ || slot < 0) return;
  __atomic_store_n(&ztab_host_->id[peer][slot], 0ull, __ATOMIC_RELEASE);
}

void IpcComm::tab_release(int peer, int slot) {
  if (!ztab_host_ || peer < 0 || slot < 0) return;
  __atomic_store_n(&ztab_host_->base[peer][slot], 0ull, __ATOMIC_RELEASE);
  tab_busy_[peer][slot] = false;
}

uint32_t IpcComm::zx_verdict(uint64_t tag) {
  DeviceScope ds(device_);
  kern::GateSlot r{};
  const char* slot = reinterpret_cast<const char*>(my_flags_) + kern::kZxResolvedOffset +
                     (tag % kern::kGateSlots) * sizeof(kern::GateSlot);
  PDCC_HIP(hipMemcpy(&r, slot, sizeof(r), hipMemcpyDeviceToHost));
  return (r.seq >> 2) == tag ? (uint32_t)(r.seq & 3u) : 0xffffffffu;  // (seq = tag << 2 | verdict)
}

std::vector<std::shared_ptr<IpcComm::LaunchEvent>> IpcComm::latest_gated() {
  std::lock_guard<std::mutex> lk(latest_mu_);
  std::vector<std::shared_ptr<LaunchEvent>> v;
  for (const auto& kv : latest_gated_) v.push_back(kv.second);
  return v;
}

void IpcComm::launch_gated(kern::IpcCall call, uint64_t t, size_t zoff, const ZcRec& mine, const void* self,
                           hipStream_t stream) {
  call.zc = 0;
  call.gate = gates_dev_ + (t % kern::kGateSlots);
  call.gate_seq = t;
  call.zoff = zoff;
  call.zx_tag = ++zx_tag_;  // gated launches run one after another (a group's collectives never overlap)
  call.zx_id = !mine.ok ? kern::kZxNoExport : mine.id;
  call.zx_off = mine.off;
  call.zx_self = static_cast<char*>(const_cast<void*>(self));
  call.ztab = zx_on_ ? ztab_dev_ : nullptr;
  prepare_staging(call, stream);  // (sized for either protocol, see ipc_staging_bytes)
  launch_view(view(peer_staging_), call, stream);
}

std::shared_ptr<IpcComm::LaunchEvent> IpcComm::gate_mark(uint64_t t, hipStream_t stream) {
  auto le = new_launch_event(stream);
  gate_last_[t % kern::kGateSlots] = le;
  {
    std::lock_guard<std::mutex> lk(latest_mu_);
    auto it = std::find_if(latest_gated_.begin(), latest_gated_.end(), [&](const auto& kv) { return kv.first == stream; });
    if (it == latest_gated_.end()) latest_gated_.emplace_back(stream, le);
    else it->second = le;
  }
  return le;
}

void IpcComm::gate_publish(uint64_t t, bool ok, const std::vector<char*>& ptrs) {
  kern::GateSlot* g = gates_host_ + (t % kern::kGateSlots);
  volatile uint64_t* vp = g->ptr;
  for (int r = 0; r < kern::kMaxRanks; ++r)
    vp[r] = (ok && r < (int)ptrs.size()) ? reinterpret_cast<uint64_t>(ptrs[r]) : 0;
  *reinterpret_cast<volatile uint32_t*>(&g->ok) = ok ? 1u : 0u;
  __atomic_store_n(&g->seq, t, __ATOMIC_RELEASE);  // last: the kernels poll it
}

void IpcComm::maintain() {
  DeviceScope ds(device_);
  reap_closing(true);
  if (graph_mode_) return;
  for (auto& r : retired_) {  // (own buffers wait for the group's teardown: a peer may map them still)
    for (void* m : r.maps)
      if (m) drop_map(m);
    if (r.mine) parked_.push_back(r.mine);
  }
  retired_.clear();
  for (void* q : deferred_free_) dev_free(q);
  deferred_free_.clear();
}

size_t IpcComm::zc_closing() const {
  std::lock_guard<std::mutex> lk(closing_mu_);
  return zc_closing_.size();
}

size_t IpcComm::zc_exports() const {
  std::lock_guard<std::mutex> zl(zc_mu_);
  return zc_exports_.size();
}

size_t IpcComm::zc_mappings() const {
  std::lock_guard<std::mutex> il(imports_mu_);
  size_t n = 0;
  for (const auto& p : zc_imports_) n += p.size();
  return n;
}

std::string IpcComm::describe_error(uint32_t w) {
  if (w == 0) return "none";
  if (w == kAbortWord) return "0x200: aborted by the host (watchdog / abort_group)";
  const char* what = "unknown";
  switch (w & ~0xffu & 0xffffu) {
    case 0x100u: what = "block-pairwise barrier"; break;
    case 0x300u: what = "LL flag poll"; break;
    case 0x400u: what = "zero-copy gate wait"; break;
    case 0x800u: what = "device-side record exchange"; break;
    case 0x900u: what = "dynamic protocol departure (done word)"; break;
    case 0xA00u: what = "dynamic protocol ready word"; break;
    case 0x1000u: what = "resolved zero-copy slot wait (block 0's exchange verdict)"; break;
    default: break;
  }
  char buf[128];
  std::snprintf(buf, sizeof(buf), "0x%x: %s timed out on rank %u", w, what, w & 0xffu);
  return buf;
}

uint32_t IpcComm::error_word() const { return err_host_ ? __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) : 0u; }
void IpcComm::clear_error() {
  if (err_host_) __atomic_store_n(err_host_, 0u, __ATOMIC_RELEASE);
}
std::vector<std::vector<uint64_t>> IpcComm::trace_records() const {
  std::vector<std::vector<uint64_t>> out;
  for (uint32_t i = 0; trace_host_ && i < trace_cap_; ++i) {
    const volatile uint64_t* r = trace_host_ + (size_t)i * kern::kTraceRecWords;
    if (r[1] == 0) continue;  // never written
    out.emplace_back(r, r + kern::kTraceRecWords);
  }
  std::sort(out.begin(), out.end(), [](const auto& a, const auto& b) { return a[1] < b[1]; });
  return out;
}

void IpcComm::abort() {
  if (!err_host_) return;
  uint32_t expect = 0;
  __atomic_compare_exchange_n(err_host_, &expect, kAbortWord, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
}

}  // namespace pdcc
