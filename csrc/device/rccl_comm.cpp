#include "rccl_comm.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "comm_util.h"

namespace pdcc {

namespace {

// restores the calling thread's current device, also when a call throws
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    PDCC_HIP(hipGetDevice(&prev));
    if (prev != d) PDCC_HIP(hipSetDevice(d));
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

ncclConfig_t make_config(const RcclOpts& o, bool for_split) {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = o.nonblocking ? 0 : 1;  // non-blocking: creation is polled against a deadline (wait_ready)
  if (o.min_ctas > 0) cfg.minCTAs = o.min_ctas;
  if (o.max_ctas > 0) cfg.maxCTAs = o.max_ctas;
  // RCCL validates the pair as given: a floor with the ceiling left undefined is rejected
  // ("Invalid config min/max channels attribute value 28/-2147483648", found by the world-1 RCCL
  // rehearsal of bench.py's CTA sweep). RCCL's channel maximum is not part of its public API, so a
  // floor alone (PDCC_RCCL_MIN_CTAS without _MAX_CTAS) means exactly that many channels; bench.py's
  // sweep sets both and reports exact counts
  if (o.min_ctas > 0 && cfg.maxCTAs < o.min_ctas) cfg.maxCTAs = o.min_ctas;
  if (for_split) cfg.splitShare = o.split_share ? 1 : 0;
  return cfg;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

std::mutex g_reg_mu;
std::map<std::string, std::weak_ptr<RcclComm>> g_reg;
std::atomic<int64_t> g_settle_ms{600000};

std::string nccl_msg(ncclResult_t r, const char* what, const char* file, int line) {
  const char* last = ncclGetLastError(nullptr);
  return std::string("pdcc: RCCL error '") + ncclGetErrorString(r) + "' (" + (last ? last : "") + ") in " + what +
         " at " + file + ":" + std::to_string(line);
}

}  // namespace

void set_rccl_settle_timeout_ms(int64_t ms) { g_settle_ms.store(std::max<int64_t>(1, ms)); }

void nccl_settle(ncclComm_t comm, ncclResult_t r, const char* what, const char* file, int line) {
  if (r == ncclInProgress && comm) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t lim = g_settle_ms.load();
    for (uint32_t it = 0;; ++it) {
      ncclResult_t st = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(comm, &st);
      if (q != ncclSuccess) {
        r = q;
        break;
      }
      if (st != ncclInProgress) {
        r = st;
        break;
      }
      if (ms_since(t0) > (double)lim)
        throw std::runtime_error("pdcc: RCCL operation still in progress after " + std::to_string(lim) + " ms (" +
                                 what + " at " + file + ":" + std::to_string(line) +
                                 "): a peer rank is not taking part");
      if (it > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  if (r != ncclSuccess) throw std::runtime_error(nccl_msg(r, what, file, line));
}

std::vector<std::string> forward_rccl_env() {
  static std::once_flag once;
  static std::vector<std::string> fwd;
  std::call_once(once, [] {
    static const char* kMap[][2] = {
        {"PDCC_RCCL_BUFFSIZE", "NCCL_BUFFSIZE"},           {"PDCC_RCCL_ALGO", "NCCL_ALGO"},
        {"PDCC_RCCL_PROTO", "NCCL_PROTO"},                 {"PDCC_RCCL_MIN_NCHANNELS", "NCCL_MIN_NCHANNELS"},
        {"PDCC_RCCL_MAX_NCHANNELS", "NCCL_MAX_NCHANNELS"}, {"PDCC_RCCL_NTHREADS", "NCCL_NTHREADS"},
        {"PDCC_RCCL_MSCCL", "RCCL_MSCCL_ENABLE"},          {"PDCC_RCCL_MSCCLPP", "RCCL_MSCCLPP_ENABLE"},
    };
    for (const auto& m : kMap) {
      const char* v = std::getenv(m[0]);
      if (!v || !*v) continue;
      const char* cur = std::getenv(m[1]);
      if (cur && *cur) continue;  // the user's own NCCL_* setting wins
      setenv(m[1], v, 0);
      fwd.push_back(std::string(m[1]) + "=" + v);
    }
  });
  return fwd;
}

RcclComm::RcclComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
                   int device, const RcclOpts& opts)
    : device_(device), world_(world) {
  forward_rccl_env();
  const auto t0 = std::chrono::steady_clock::now();
  const auto deadline = t0 + std::chrono::milliseconds(opts.init_timeout_ms);
  ncclUniqueId id;
  const std::string k = key + "/rccl_uid";
  if (rank == 0) {
    PDCC_NCCL(ncclGetUniqueId(&id));
    store->set(k, std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id)));
  } else {
    try {  // bounded: rank 0 may never get here
      store->wait({k}, std::chrono::milliseconds(std::max<int64_t>(1, opts.init_timeout_ms)));
    } catch (const std::exception& e) {
      throw std::runtime_error("pdcc: RCCL communicator creation: rank 0's unique id did not arrive within " +
                               std::to_string(opts.init_timeout_ms) + " ms (PDCC_RCCL_INIT_TIMEOUT_S): " + e.what());
    }
    const std::vector<uint8_t> v = store->get(k);
    if (v.size() != sizeof(id)) throw std::runtime_error("pdcc: malformed RCCL unique id in store");
    std::memcpy(&id, v.data(), sizeof(id));
  }
  DeviceGuard g(device);
  ncclConfig_t cfg = make_config(opts, false);
  const ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
    throw std::runtime_error(nccl_msg(r, "ncclCommInitRankConfig", __FILE__, __LINE__));
  }
  wait_ready(deadline, opts.init_timeout_ms, "ncclCommInitRankConfig");
  init_ms_ = ms_since(t0);
}

RcclComm::RcclComm(const RcclComm& parent, int rank, const RcclOpts& opts)
    : device_(parent.device_), world_(parent.world_), split_(true) {
  const auto t0 = std::chrono::steady_clock::now();
  DeviceGuard g(device_);
  ncclConfig_t cfg = make_config(opts, true);
  const auto deadline = t0 + std::chrono::milliseconds(opts.init_timeout_ms);
  // A non-blocking split hands the child back through `*slot` only when RCCL's own thread has
  // finished building it. The slot is heap memory that is deliberately leaked if we give up:
  // that thread may still write it after this constructor has thrown.
  auto* slot = new ncclComm_t(nullptr);
  const ncclResult_t r = ncclCommSplit(parent.comm_, /*color=*/0, /*key=*/rank, slot, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (*slot) ncclCommAbort(*slot);
    delete slot;
    throw std::runtime_error(nccl_msg(r, "ncclCommSplit", __FILE__, __LINE__));
  }
  for (uint32_t it = 0;; ++it) {
    ncclComm_t c = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
    if (c) {
      comm_ = c;
      delete slot;
      break;
    }
    // (RCCL returns ncclSuccess at once for a non-blocking split and sets the slot when its
    // job is done: "newcomm is NCCL_COMM_NULL until the split fully completes")
    ncclResult_t st = ncclSuccess;  // a failed split job reports on the parent
    if (ncclCommGetAsyncError(parent.comm_, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
      throw std::runtime_error(nccl_msg(st, "ncclCommSplit (async)", __FILE__, __LINE__));
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("pdcc: RCCL communicator creation (ncclCommSplit) did not complete within " +
                               std::to_string(opts.init_timeout_ms) + " ms (PDCC_RCCL_INIT_TIMEOUT_S): a peer rank "
                               "died or never joined the group");
    std::this_thread::sleep_for(std::chrono::microseconds(it < 200 ? 50 : 1000));
  }
  wait_ready(deadline, opts.init_timeout_ms, "ncclCommSplit");
  init_ms_ = ms_since(t0);
}

void RcclComm::wait_ready(std::chrono::steady_clock::time_point deadline, int64_t budget_ms, const char* what) {
  for (uint32_t it = 0;; ++it) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      throw std::runtime_error(nccl_msg(st, what, __FILE__, __LINE__));
    }
    if (std::chrono::steady_clock::now() > deadline) {
      ncclCommAbort(comm_);  // unblocks RCCL's bootstrap / connection threads
      comm_ = nullptr;
      throw std::runtime_error(std::string("pdcc: RCCL communicator creation (") + what + ") did not complete within " +
                               std::to_string(budget_ms) + " ms (PDCC_RCCL_INIT_TIMEOUT_S): a peer rank died or "
                               "never joined the group");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(it < 200 ? 50 : 1000));
  }
}

RcclComm::~RcclComm() {
  if (!comm_) return;
  if (aborted_.load()) return;  // ncclCommAbort already freed it
  // non-blocking communicator: finalize (flushes its work) may complete asynchronously; a
  // peer that is gone would keep it in progress forever -- abort after a bounded wait
  ncclResult_t r = ncclCommFinalize(comm_);
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress && ms_since(t0) < 10000.0) {
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    ncclResult_t st = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) break;
    r = st;
  }
  if (r == ncclSuccess) ncclCommDestroy(comm_);
  else ncclCommAbort(comm_);
}

void RcclComm::abort() {
  bool expected = false;
  if (comm_ && aborted_.compare_exchange_strong(expected, true)) ncclCommAbort(comm_);
}

ncclResult_t RcclComm::async_error() {
  if (!comm_ || aborted_.load()) return ncclSuccess;
  ncclResult_t r = ncclSuccess;
  ncclCommGetAsyncError(comm_, &r);
  return r;
}

void rccl_registry_put(const std::string& members_key, const std::shared_ptr<RcclComm>& c) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(members_key);
  if (it != g_reg.end() && !it->second.expired()) return;  // keep the first live one
  g_reg[members_key] = c;
}

std::shared_ptr<RcclComm> rccl_registry_get(const std::string& members_key) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(members_key);
  if (it == g_reg.end()) return nullptr;
  auto s = it->second.lock();
  if (!s || s->aborted()) {
    g_reg.erase(it);
    return nullptr;
  }
  return s;
}

}  // namespace pdcc
