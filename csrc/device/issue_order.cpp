#include "issue_order.h"

#include <sstream>

#include "comm_util.h"

namespace pdcc {

namespace {
std::string sname(hipStream_t s) {
  std::ostringstream o;
  o << reinterpret_cast<uintptr_t>(s);
  return o.str();
}
}  // namespace

IssueOrder::~IssueOrder() {
  if (word_) (void)hipFree(word_);
  if (ev_) (void)hipEventDestroy(ev_);
}

bool IssueOrder::ensure_word() {
  if (word_ || (dry_ && !word_failed_)) return true;
  if (word_failed_) return false;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, sizeof(uint64_t), hipMallocSignalMemory) == hipSuccess && p) {
    *static_cast<volatile uint64_t*>(p) = 0;  // host-accessible: no null-stream memset
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    word_ = static_cast<uint64_t*>(p);
    return true;
  }
  (void)hipGetLastError();
  if (p) (void)hipFree(p);
  word_failed_ = true;
  return false;
}

void IssueOrder::write(hipStream_t s, uint64_t v) {
  if (dry_) log_.push_back("write " + sname(s) + " " + std::to_string(v));
  else PDCC_HIP(hipStreamWriteValue64(s, word_, v, 0));
}

void IssueOrder::wait(hipStream_t s, uint64_t v) {
  if (dry_) log_.push_back("wait " + sname(s) + " " + std::to_string(v));
  else PDCC_HIP(hipStreamWaitValue64(s, word_, v, hipStreamWaitValueGte, ~0ull));
}

void IssueOrder::enter(hipStream_t s) {
  mu_.lock();
  try {
    if (!last_ || last_ == s) return;  // first op, or the same stream: FIFO already
    if (ensure_word()) {
      if (!last_written_) {  // lazily: after everything enqueued on that stream so far
        ++tick_;
        write(last_, tick_);
      }
      wait(s, tick_);
    } else {
      if (!ev_) PDCC_HIP(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
      PDCC_HIP(hipEventRecord(ev_, last_));
      PDCC_HIP(hipStreamWaitEvent(s, ev_, 0));
    }
    ++waits_;
  } catch (...) {
    mu_.unlock();
    throw;
  }
}

void IssueOrder::leave(hipStream_t s) {
  last_ = s;
  last_written_ = false;
  // shared by several groups: tick right after the op, so a later switch waits for this
  // op only, not for whatever the caller enqueues on `s` afterwards
  if (users_.load() > 1 && ensure_word()) {
    try {
      write(s, tick_ + 1);
      ++tick_;
      last_written_ = true;
    } catch (...) {
      (void)hipGetLastError();  // the next switch falls back to a lazy tick
    }
  }
  mu_.unlock();
}

}  // namespace pdcc
