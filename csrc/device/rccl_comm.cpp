#include "rccl_comm.h"

#include <cstring>
#include <vector>

#include "comm_util.h"

namespace pdcc {

RcclComm::RcclComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
                   int device, int min_ctas, int max_ctas)
    : device_(device) {
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
  int prev = 0;
  PDCC_HIP(hipGetDevice(&prev));
  PDCC_HIP(hipSetDevice(device));
  if (min_ctas > 0 || max_ctas > 0) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    if (min_ctas > 0) cfg.minCTAs = min_ctas;
    if (max_ctas > 0) cfg.maxCTAs = max_ctas;
    PDCC_NCCL(ncclCommInitRankConfig(&comm_, world, id, rank, &cfg));
  } else {
    PDCC_NCCL(ncclCommInitRank(&comm_, world, id, rank));
  }
  PDCC_HIP(hipSetDevice(prev));
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

}  // namespace pdcc
