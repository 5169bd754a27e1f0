// RCCL communicator for one process group on one device, bootstrapped through
// the group's c10d Store (the reference's env:// rendezvous, main.py:92-94, is
// reused as the control plane; no extra TCP code).
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <atomic>
#include <string>

namespace pdcc {

#define PDCC_NCCL(expr)                                                                             \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess)                                                                          \
      throw std::runtime_error(std::string("pdcc: RCCL error '") + ncclGetErrorString(_r) + "' (" + \
                               (ncclGetLastError(nullptr) ? ncclGetLastError(nullptr) : "") + ") at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                          \
  } while (0)

class RcclComm {
 public:
  // Collective over the group: rank 0 creates the unique id and publishes it.
  RcclComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world, int device,
           int min_ctas = -1, int max_ctas = -1);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  ncclComm_t get() const { return comm_; }
  int device() const { return device_; }
  // ncclCommAbort: unblocks kernels stuck on a dead peer (watchdog path)
  void abort();
  bool aborted() const { return aborted_.load(); }
  ncclResult_t async_error();

 private:
  ncclComm_t comm_ = nullptr;
  int device_;
  std::atomic<bool> aborted_{false};
};

}  // namespace pdcc
