// Issue order of one RCCL communicator across streams.
//
// The reference builds `new_group(range(size))` in every demo (main.py:11,21,31,
// 46,63,75); groups with the same members share one communicator here
// (PDCC_RCCL_GROUP_COMM=share), and each group enqueues on its own streams (an
// async op on the group's comm stream, a sync op on the caller's). RCCL requires
// the ops of one communicator to execute in the order every rank issued them;
// whether it orders ops it received on different streams is not something this
// library relies on. Instead every enqueue is bracketed by enter(s) / leave(s):
//
//   * enter(s): if the communicator's previous op went to another stream `p`,
//     `s` waits (hipStreamWaitValue64, no host block) until `p` has passed that
//     op: the tick is written on `p` right after the op (eagerly, when several
//     groups share the communicator), or lazily now (after whatever `p` holds);
//   * leave(s): remember `s`; when shared, append the tick write to `s`.
//
// The mutex is held from enter to leave: one thread enqueues on a communicator
// at a time. Without signal memory the hand-off falls back to an event.
//
// Dry mode (tests): no HIP call is made; every stream operation that would be
// issued is appended to log() as "write <stream> <tick>" / "wait <stream> <tick>".
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace pdcc {

class IssueOrder {
 public:
  explicit IssueOrder(bool dry = false) : dry_(dry) {}
  ~IssueOrder();
  IssueOrder(const IssueOrder&) = delete;
  IssueOrder& operator=(const IssueOrder&) = delete;

  void enter(hipStream_t s);
  void leave(hipStream_t s);
  // another group shares the communicator: ticks are written eagerly after each op
  void add_user() { users_.fetch_add(1); }
  int users() const { return users_.load(); }
  uint64_t ticks() const { return tick_; }
  uint64_t waits() const { return waits_; }
  const std::vector<std::string>& log() const { return log_; }

 private:
  bool ensure_word();  // mu_ held
  void write(hipStream_t s, uint64_t v);
  void wait(hipStream_t s, uint64_t v);

  const bool dry_;
  std::mutex mu_;
  uint64_t* word_ = nullptr;      // signal memory; null until the first cross-stream hand-off
  bool word_failed_ = false;      // signal memory unavailable: events instead
  hipEvent_t ev_ = nullptr;
  uint64_t tick_ = 0;             // last value written (or enqueued) to word_
  hipStream_t last_ = nullptr;    // stream of the previous op
  bool last_written_ = false;     // the previous op's tick is already enqueued after it
  uint64_t waits_ = 0;
  std::atomic<int> users_{1};
  std::vector<std::string> log_;
};

}  // namespace pdcc
