#include "rccl_comm.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
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
  if (o.min_ctas > 0) cfg.minCTAs = o.min_ctas;
  if (o.max_ctas > 0) cfg.maxCTAs = o.max_ctas;
  if (for_split) cfg.splitShare = o.split_share ? 1 : 0;
  return cfg;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

std::mutex g_reg_mu;
std::map<std::string, std::weak_ptr<RcclComm>> g_reg;

}  // namespace

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
  ncclUniqueId id;
  const std::string k = key + "/rccl_uid";
  if (rank == 0) {
    PDCC_NCCL(ncclGetUniqueId(&id));
    store->set(k, std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id)));
  } else {
    const std::vector<uint8_t> v = store->get(k);
    if (v.size() != sizeof(id)) throw std::runtime_error("pdcc: malformed RCCL unique id in store");
    std::memcpy(&id, v.data(), sizeof(id));
  }
  DeviceGuard g(device);
  if (opts.any()) {
    ncclConfig_t cfg = make_config(opts, false);
    PDCC_NCCL(ncclCommInitRankConfig(&comm_, world, id, rank, &cfg));
  } else {
    PDCC_NCCL(ncclCommInitRank(&comm_, world, id, rank));
  }
  init_ms_ = ms_since(t0);
}

RcclComm::RcclComm(const RcclComm& parent, int rank, const RcclOpts& opts)
    : device_(parent.device_), world_(parent.world_), split_(true) {
  const auto t0 = std::chrono::steady_clock::now();
  DeviceGuard g(device_);
  ncclConfig_t cfg = make_config(opts, true);
  PDCC_NCCL(ncclCommSplit(parent.comm_, /*color=*/0, /*key=*/rank, &comm_, &cfg));
  if (!comm_) throw std::runtime_error("pdcc: ncclCommSplit returned no communicator");
  init_ms_ = ms_since(t0);
}

RcclComm::~RcclComm() {
  if (!comm_) return;
  if (aborted_.load()) return;  // ncclCommAbort already freed it
  ncclCommDestroy(comm_);
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
