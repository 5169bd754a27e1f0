// POSIX shared-memory host transport: the CPU-tensor data path of the backend
// (replaces Gloo's TCP full mesh that the reference runs on, main.py:90-94).
//
// One segment per process group, created by group rank 0, name published through
// the group's c10d Store, attached by every rank and unlinked by rank 0 as soon as
// everybody is attached (so a crash never leaks /dev/shm). Layout:
//
//   [ header | set0: W slots + result | set1: W slots + result | W*W p2p channels ]
//
// Collectives move data in chunks of at most one slot; consecutive chunks
// alternate between the two slot sets, so each chunk needs a single barrier
// (two for the reductions) instead of the usual write/barrier/read/barrier.
// Every wait is a bounded spin + futex with peer-liveness checks, so a dead
// peer turns into an exception within milliseconds instead of a hang.
#pragma once
#include <c10/core/ScalarType.h>
#include <torch/csrc/distributed/c10d/Store.hpp>
#include <torch/csrc/distributed/c10d/Types.hpp>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace pdcc {
namespace host {

constexpr int kMaxShmRanks = 64;

struct ShmConfig {
  size_t slot_bytes = 8u << 20;   // per-rank staging slot per set
  size_t chan_bytes = 1u << 20;   // per directed pair p2p ring
  // busy-wait window before a waiter sleeps on the futex: must cover the usual
  // arrival skew between ranks (tens of us), or every op pays a ~100 us wake-up.
  // Shortened automatically when ranks outnumber the CPUs.
  int spin_us = 300;
  std::chrono::milliseconds timeout{std::chrono::minutes(30)};
};

class ShmComm {
 public:
  // Collective: every rank of the group must call it (lazily, on first CPU op).
  ShmComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
          const ShmConfig& cfg);
  ~ShmComm();
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }

  void barrier(std::chrono::milliseconds timeout);

  // All pointers are contiguous host buffers of `count` elements of `t`.
  void allreduce(void* buf, size_t count, at::ScalarType t, c10d::ReduceOp::RedOpType op,
                 std::chrono::milliseconds timeout);
  void reduce(void* buf, size_t count, at::ScalarType t, c10d::ReduceOp::RedOpType op, int root,
              std::chrono::milliseconds timeout);
  void broadcast(void* buf, size_t bytes, int root, std::chrono::milliseconds timeout);
  // outs[r] receives rank r's `bytes` (outs may be nullptr entries on non-roots for gather)
  void allgather(const void* in, const std::vector<void*>& outs, size_t bytes, std::chrono::milliseconds timeout);
  void gather(const void* in, const std::vector<void*>& outs, size_t bytes, int root,
              std::chrono::milliseconds timeout);
  void scatter(const std::vector<const void*>& ins, void* out, size_t bytes, int root,
               std::chrono::milliseconds timeout);
  // ins[r] is the chunk reduced onto rank r; out gets my chunk
  void reduce_scatter(const std::vector<const void*>& ins, void* out, size_t count, at::ScalarType t,
                      c10d::ReduceOp::RedOpType op, std::chrono::milliseconds timeout);
  // per-peer byte counts may differ (send_bytes[r] to r, recv_bytes[r] from r)
  void alltoall(const std::vector<const void*>& ins, const std::vector<size_t>& send_bytes,
                const std::vector<void*>& outs, const std::vector<size_t>& recv_bytes,
                std::chrono::milliseconds timeout);

  // point-to-point over the (me -> peer) SPSC ring; blocking until all bytes are
  // handed over (send) or received (recv)
  void send(const void* buf, size_t bytes, int peer, std::chrono::milliseconds timeout);
  void recv(void* buf, size_t bytes, int peer, std::chrono::milliseconds timeout);

  // mark the segment aborted (peers fail fast) -- used by the watchdog / abort()
  void abort();

 private:
  struct Header;
  Header* hdr() const;
  char* slot(int set, int r) const;
  char* result(int set) const;
  char* chan_data(int src, int dst) const;
  int next_set() { int s = set_; set_ ^= 1; return s; }
  template <class Pred>
  void wait_until(Pred pred, std::atomic<uint32_t>* futex_word, uint32_t futex_val,
                  std::chrono::milliseconds timeout, const char* what);
  void check_peers(const char* what);
  [[noreturn]] void fail(const std::string& msg);

  int rank_;
  int world_;
  int spin_us_ = 300;
  bool oversub_ = false;
  ShmConfig cfg_;
  std::string name_;
  void* base_ = nullptr;
  size_t size_ = 0;
  size_t data_off_ = 0;
  size_t chan_off_ = 0;
  int set_ = 0;
  std::vector<int32_t> peer_pids_;
  std::mutex send_mu_, recv_mu_;
};

}  // namespace host
}  // namespace pdcc
