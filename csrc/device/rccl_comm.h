// RCCL communicator for one process group on one device, bootstrapped through
// the group's c10d Store (the reference's env:// rendezvous, main.py:92-94, is
// reused as the control plane; no extra TCP code).
//
// Three ways to get one:
//   * fresh: rank 0 publishes a unique id in the store, every rank joins
//     (ncclCommInitRank, or ncclCommInitRankConfig when a config knob is set);
//   * split: a group whose member set equals that of a live communicator on the
//     same device (the reference builds `new_group(range(size))` in every demo,
//     main.py:11,21,31,46,63,75) derives its communicator with ncclCommSplit from
//     that one -- no unique-id round trip, and with splitShare the child reuses
//     the parent's channel buffers and proxy;
//   * pair: a 2-rank communicator for point-to-point between two ranks of a
//     larger group (send/recv must not need every rank of the group).
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "issue_order.h"

namespace pdcc {

#define PDCC_NCCL(expr)                                                                             \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess)                                                                          \
      throw std::runtime_error(std::string("pdcc: RCCL error '") + ncclGetErrorString(_r) + "' (" + \
                               (ncclGetLastError(nullptr) ? ncclGetLastError(nullptr) : "") + ") at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                          \
  } while (0)

// RCCL calls on a non-blocking communicator (every RcclComm is one, see below) may return
// ncclInProgress: RCCL's own thread is still connecting channels and enqueuing the op. Wait
// for it (bounded by the settle timeout) before returning, so the caller's stream order is
// exactly the one a blocking communicator gives; any other result throws like PDCC_NCCL.
// Not for calls between ncclGroupStart and ncclGroupEnd (settle the ncclGroupEnd instead).
void nccl_settle(ncclComm_t comm, ncclResult_t r, const char* what, const char* file, int line);
#define PDCC_NCCLC(comm, expr) ::pdcc::nccl_settle((comm), (expr), #expr, __FILE__, __LINE__)
// upper bound of one nccl_settle wait (process-wide; the groups set it from their config)
void set_rccl_settle_timeout_ms(int64_t ms);

// Per-communicator RCCL configuration (ncclConfig_t fields); -1 = RCCL's default.
struct RcclOpts {
  int min_ctas = -1;     // channels (one CTA each) at least / at most: 7 xGMI links per GPU
  int max_ctas = -1;
  int split_share = 1;   // ncclCommSplit children share the parent's resources
  // Deadline of the creation (unique-id wait + init / split): communicators are created
  // non-blocking (ncclConfig_t.blocking = 0) and polled; past the deadline the half-built
  // communicator is aborted and the constructor throws (a peer died or never joined)
  int64_t init_timeout_ms = 300000;
  bool nonblocking = true;  // PDCC_RCCL_NONBLOCKING=0: RCCL's blocking creation (no deadline), as before round 4
  bool any() const { return min_ctas > 0 || max_ctas > 0; }
};

// Forward PDCC_RCCL_{BUFFSIZE,ALGO,PROTO,NCHANNELS,...} to the NCCL_* variables RCCL
// reads once per process at its first communicator (only where the user did not
// set the NCCL_* variable itself). Returns "NAME=value" for every forwarded knob.
std::vector<std::string> forward_rccl_env();

class RcclComm {
 public:
  // Fresh communicator over the group: rank 0 creates the unique id and publishes it.
  RcclComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world, int device,
           const RcclOpts& opts = RcclOpts());
  // Child of `parent` (collective over the parent's ranks): ncclCommSplit(color 0, key = rank).
  RcclComm(const RcclComm& parent, int rank, const RcclOpts& opts);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  ncclComm_t get() const { return comm_; }
  int device() const { return device_; }
  int world() const { return world_; }
  bool is_split() const { return split_; }
  double init_ms() const { return init_ms_; }
  // ncclCommAbort: unblocks kernels stuck on a dead peer (watchdog path)
  void abort();
  bool aborted() const { return aborted_.load(); }
  ncclResult_t async_error();

  // identity of the group that created the communicator (identical on every rank):
  // the split vote compares it so all ranks derive their child from the same parent
  std::string tag;

  // Issue order (see IssueOrder): groups with the same members share one communicator
  // (PDCC_RCCL_GROUP_COMM=share) and enqueue on different streams; every RCCL enqueue is
  // bracketed by enter(s) / leave(s) so the ops of this communicator execute in issue order.
  IssueOrder& order() { return order_; }
  void add_user() { order_.add_user(); }

  // RAII enter/leave around the RCCL calls of one collective (skipped while capturing)
  struct Issue {
    IssueOrder* o;
    hipStream_t s;
    Issue(RcclComm& comm, hipStream_t st, bool capturing) : o(capturing ? nullptr : &comm.order_), s(st) {
      if (o) o->enter(s);
    }
    ~Issue() {
      if (o) o->leave(s);
    }
    Issue(const Issue&) = delete;
    Issue& operator=(const Issue&) = delete;
  };

 private:
  IssueOrder order_;

  // poll the non-blocking creation until it leaves ncclInProgress; abort + throw past `deadline`
  void wait_ready(std::chrono::steady_clock::time_point deadline, int64_t budget_ms, const char* what);

  ncclComm_t comm_ = nullptr;
  int device_;
  int world_;
  bool split_ = false;
  double init_ms_ = 0.0;
  std::atomic<bool> aborted_{false};
};

// Process-wide registry of live communicators by (device, member set): where a
// new group can split its communicator from. Weak references: a group that is
// destroyed takes its communicator with it.
void rccl_registry_put(const std::string& members_key, const std::shared_ptr<RcclComm>& c);
std::shared_ptr<RcclComm> rccl_registry_get(const std::string& members_key);

}  // namespace pdcc
