#include "shm_comm.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <immintrin.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>

#include "cpu_reduce.h"

namespace pdcc {
namespace host {

namespace {

constexpr uint64_t kMagic = 0x70646363'73686d31ull;  // "pdccshm1"

struct alignas(64) PadU32 {
  std::atomic<uint32_t> v;
  char pad[60];
};
struct alignas(64) PadU64 {
  std::atomic<uint64_t> v;
  char pad[56];
};
struct ChanCtl {
  PadU64 head;  // bytes produced (written by sender)
  PadU64 tail;  // bytes consumed (written by receiver)
};

long futex_wait(std::atomic<uint32_t>* w, uint32_t val, long ns) {
  struct timespec ts{ns / 1000000000L, ns % 1000000000L};
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, val, &ts, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// A peer is gone when the pid no longer exists OR is a zombie (exited but not yet
// reaped by its parent -- kill(pid, 0) still succeeds on a zombie).
bool pid_dead(int32_t pid) {
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0 && errno == ESRCH) return true;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = fopen(path, "r");
  if (!f) return true;
  char buf[512];
  size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');
  if (!rp || rp[1] == 0 || rp[2] == 0) return false;
  const char st = rp[2];
  return st == 'Z' || st == 'X';
}

// [lo, hi) of element range `count` owned by `r` when split `w` ways, 64-B aligned
void split_range(size_t count, size_t esz, int w, int r, size_t& lo, size_t& hi) {
  const size_t align = std::max<size_t>(1, 64 / esz);
  size_t per = (count + w - 1) / w;
  per = round_up(per, align);
  lo = std::min(count, per * r);
  hi = std::min(count, lo + per);
}

}  // namespace

struct ShmComm::Header {
  uint64_t magic;
  uint32_t world;
  uint32_t pad0;
  uint64_t slot_bytes;
  uint64_t chan_bytes;
  PadU32 arrive;
  PadU32 gen;
  PadU32 aborted;
  PadU32 attached;
  int32_t pids[kMaxShmRanks];
  ChanCtl chan[kMaxShmRanks * kMaxShmRanks];
};

ShmComm::Header* ShmComm::hdr() const { return static_cast<Header*>(base_); }
char* ShmComm::slot(int set, int r) const {
  return static_cast<char*>(base_) + data_off_ + ((size_t)set * (world_ + 1) + r) * cfg_.slot_bytes;
}
char* ShmComm::result(int set) const { return slot(set, world_); }
char* ShmComm::chan_data(int src, int dst) const {
  return static_cast<char*>(base_) + chan_off_ + ((size_t)src * world_ + dst) * cfg_.chan_bytes;
}

ShmComm::ShmComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
                 const ShmConfig& cfg)
    : rank_(rank), world_(world), cfg_(cfg) {
  if (world > kMaxShmRanks) throw std::runtime_error("pdcc: shm transport supports at most 64 ranks per group");
  cfg_.slot_bytes = round_up(std::max<size_t>(cfg_.slot_bytes, 4096), 4096);
  cfg_.chan_bytes = round_up(std::max<size_t>(cfg_.chan_bytes, 4096), 4096);
  data_off_ = round_up(sizeof(Header), 4096);
  chan_off_ = data_off_ + 2 * (size_t)(world + 1) * cfg_.slot_bytes;
  size_ = chan_off_ + (size_t)world * world * cfg_.chan_bytes;

  const std::string name_key = key + "/shm_name";
  if (rank == 0) {
    std::random_device rd;
    name_ = "/pdcc_" + std::to_string(getpid()) + "_" + std::to_string(rd()) + "_" + std::to_string(rd());
    int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("pdcc: shm_open(create) failed: " + std::string(strerror(errno)));
    if (ftruncate(fd, (off_t)size_) != 0) {
      close(fd);
      shm_unlink(name_.c_str());
      throw std::runtime_error("pdcc: ftruncate of shm segment failed: " + std::string(strerror(errno)));
    }
    base_ = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_NORESERVE, fd, 0);
    close(fd);
    if (base_ == MAP_FAILED) {
      shm_unlink(name_.c_str());
      throw std::runtime_error("pdcc: mmap of shm segment failed");
    }
    Header* h = hdr();
    h->world = world;
    h->slot_bytes = cfg_.slot_bytes;
    h->chan_bytes = cfg_.chan_bytes;
    h->arrive.v.store(0);
    h->gen.v.store(0);
    h->aborted.v.store(0);
    h->attached.v.store(0);
    h->pids[0] = getpid();
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->store(kMagic, std::memory_order_release);
    store->set(name_key, std::vector<uint8_t>(name_.begin(), name_.end()));
    // unlink once everybody mapped it
    const auto deadline = std::chrono::steady_clock::now() + cfg_.timeout;
    while ((int)h->attached.v.load(std::memory_order_acquire) < world - 1) {
      if (std::chrono::steady_clock::now() > deadline) {
        shm_unlink(name_.c_str());
        throw std::runtime_error("pdcc: timed out waiting for ranks to attach the shm segment");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    shm_unlink(name_.c_str());
  } else {
    const std::vector<uint8_t> nm = store->get(name_key);  // blocks (store timeout)
    name_.assign(nm.begin(), nm.end());
    int fd = shm_open(name_.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("pdcc: shm_open(attach) failed: " + std::string(strerror(errno)));
    base_ = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_NORESERVE, fd, 0);
    close(fd);
    if (base_ == MAP_FAILED) throw std::runtime_error("pdcc: mmap(attach) failed");
    Header* h = hdr();
    if (reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->load(std::memory_order_acquire) != kMagic ||
        (int)h->world != world || h->slot_bytes != cfg_.slot_bytes)
      throw std::runtime_error("pdcc: shm segment header mismatch (inconsistent PDCC_SHM_* config across ranks?)");
    h->pids[rank] = getpid();
    h->attached.v.fetch_add(1, std::memory_order_acq_rel);
  }
  // more ranks than CPUs on this host: spinning steals the CPU a peer needs
  const long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
  oversub_ = ncpu > 0 && world > ncpu;
  spin_us_ = oversub_ ? std::min(cfg_.spin_us, 20) : cfg_.spin_us;
  // everybody attached and published its pid
  barrier(cfg_.timeout);
  peer_pids_.assign(hdr()->pids, hdr()->pids + world);
}

ShmComm::~ShmComm() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, size_);
}

void ShmComm::abort() {
  if (!base_) return;
  hdr()->aborted.v.store(1, std::memory_order_release);
  futex_wake_all(&hdr()->gen.v);
}

void ShmComm::fail(const std::string& msg) {
  abort();
  throw std::runtime_error(msg);
}

void ShmComm::check_peers(const char* what) {
  if (hdr()->aborted.v.load(std::memory_order_acquire))
    throw std::runtime_error(std::string("pdcc: ") + what + ": group aborted by a peer rank");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_ || peer_pids_.empty()) continue;
    if (pid_dead(peer_pids_[r]))
      fail(std::string("pdcc: ") + what + ": peer rank " + std::to_string(r) + " (pid " +
           std::to_string(peer_pids_[r]) + ") exited");
  }
}

template <class Pred>
void ShmComm::wait_until(Pred pred, std::atomic<uint32_t>* fw, uint32_t fval, std::chrono::milliseconds timeout,
                         const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    if (pred()) return;
    _mm_pause();
    if ((i & 63) == 63) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
      if (oversub_) std::this_thread::yield();
    }
  }
  auto last_check = t0;
  while (!pred()) {
    if (fw) futex_wait(fw, fval, 200000);  // 200 us
    else std::this_thread::yield();
    const auto now = std::chrono::steady_clock::now();
    if (now - last_check > std::chrono::milliseconds(20)) {
      last_check = now;
      check_peers(what);
      if (now - t0 > timeout)
        fail(std::string("pdcc: ") + what + " timed out after " + std::to_string(timeout.count()) + " ms on rank " +
             std::to_string(rank_));
    }
  }
}

void ShmComm::barrier(std::chrono::milliseconds timeout) {
  Header* h = hdr();
  if (h->aborted.v.load(std::memory_order_acquire)) throw std::runtime_error("pdcc: shm group was aborted");
  const uint32_t g = h->gen.v.load(std::memory_order_acquire);
  if (h->arrive.v.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)world_ - 1) {
    h->arrive.v.store(0, std::memory_order_relaxed);
    h->gen.v.store(g + 1, std::memory_order_release);
    futex_wake_all(&h->gen.v);
    return;
  }
  wait_until([&] { return h->gen.v.load(std::memory_order_acquire) != g || h->aborted.v.load(); }, &h->gen.v, g,
             timeout, "barrier");
  if (h->aborted.v.load(std::memory_order_acquire) && h->gen.v.load() == g)
    throw std::runtime_error("pdcc: shm group was aborted");
}

// ----------------------------------------------------------------- reductions
void ShmComm::allreduce(void* buf, size_t count, at::ScalarType t, c10d::ReduceOp::RedOpType op,
                        std::chrono::milliseconds timeout) {
  reduce(buf, count, t, op, -1, timeout);
}

void ShmComm::reduce(void* buf, size_t count, at::ScalarType t, c10d::ReduceOp::RedOpType op, int root,
                     std::chrono::milliseconds timeout) {
  const size_t esz = c10::elementSize(t);
  const size_t chunk = cfg_.slot_bytes / esz;
  char* p = static_cast<char*>(buf);
  for (size_t off = 0; off < count; off += chunk) {
    const size_t c = std::min(chunk, count - off);
    const int s = next_set();
    std::memcpy(slot(s, rank_), p + off * esz, c * esz);
    barrier(timeout);
    size_t lo, hi;
    split_range(c, esz, world_, rank_, lo, hi);
    if (hi > lo) {
      const void* srcs[kMaxShmRanks];
      for (int r = 0; r < world_; ++r) srcs[r] = slot(s, r) + lo * esz;
      reduce_cpu(t, result(s) + lo * esz, srcs, world_, hi - lo, op, world_);
    }
    barrier(timeout);
    if (root < 0 || root == rank_) std::memcpy(p + off * esz, result(s), c * esz);
  }
}

void ShmComm::reduce_scatter(const std::vector<const void*>& ins, void* out, size_t count, at::ScalarType t,
                             c10d::ReduceOp::RedOpType op, std::chrono::milliseconds timeout) {
  const size_t esz = c10::elementSize(t);
  const size_t sub = (cfg_.slot_bytes / world_) / 64 * 64;  // bytes per destination per chunk
  const size_t chunk = std::max<size_t>(1, sub / esz);
  for (size_t off = 0; off < count; off += chunk) {
    const size_t c = std::min(chunk, count - off);
    const int s = next_set();
    for (int r = 0; r < world_; ++r)
      std::memcpy(slot(s, rank_) + r * sub, static_cast<const char*>(ins[r]) + off * esz, c * esz);
    barrier(timeout);
    const void* srcs[kMaxShmRanks];
    for (int q = 0; q < world_; ++q) srcs[q] = slot(s, q) + rank_ * sub;
    reduce_cpu(t, static_cast<char*>(out) + off * esz, srcs, world_, c, op, world_);
  }
}

// ----------------------------------------------------------------- copies
void ShmComm::broadcast(void* buf, size_t bytes, int root, std::chrono::milliseconds timeout) {
  char* p = static_cast<char*>(buf);
  for (size_t off = 0; off < bytes; off += cfg_.slot_bytes) {
    const size_t c = std::min(cfg_.slot_bytes, bytes - off);
    const int s = next_set();
    if (rank_ == root) std::memcpy(slot(s, root), p + off, c);
    barrier(timeout);
    if (rank_ != root) std::memcpy(p + off, slot(s, root), c);
  }
}

void ShmComm::allgather(const void* in, const std::vector<void*>& outs, size_t bytes,
                        std::chrono::milliseconds timeout) {
  gather(in, outs, bytes, -1, timeout);
}

void ShmComm::gather(const void* in, const std::vector<void*>& outs, size_t bytes, int root,
                     std::chrono::milliseconds timeout) {
  const char* p = static_cast<const char*>(in);
  for (size_t off = 0; off < bytes; off += cfg_.slot_bytes) {
    const size_t c = std::min(cfg_.slot_bytes, bytes - off);
    const int s = next_set();
    std::memcpy(slot(s, rank_), p + off, c);
    barrier(timeout);
    if (root < 0 || root == rank_)
      for (int j = 0; j < world_; ++j) {
        const int r = (rank_ + j) % world_;
        std::memcpy(static_cast<char*>(outs[r]) + off, slot(s, r), c);
      }
  }
}

void ShmComm::scatter(const std::vector<const void*>& ins, void* out, size_t bytes, int root,
                      std::chrono::milliseconds timeout) {
  char* p = static_cast<char*>(out);
  for (size_t off = 0; off < bytes; off += cfg_.slot_bytes) {
    const size_t c = std::min(cfg_.slot_bytes, bytes - off);
    const int s = next_set();
    if (rank_ == root)
      for (int r = 0; r < world_; ++r) std::memcpy(slot(s, r), static_cast<const char*>(ins[r]) + off, c);
    barrier(timeout);
    std::memcpy(p + off, slot(s, rank_), c);
  }
}

void ShmComm::alltoall(const std::vector<const void*>& ins, const std::vector<size_t>& send_bytes,
                       const std::vector<void*>& outs, const std::vector<size_t>& recv_bytes,
                       std::chrono::milliseconds timeout) {
  const size_t sub = (cfg_.slot_bytes / world_) / 64 * 64;
  // every rank must run the same number of rounds: agree on the max through the
  // shm itself (one tiny max-allreduce)
  uint64_t need = 0;
  for (int r = 0; r < world_; ++r) {
    need = std::max<uint64_t>(need, (send_bytes[r] + sub - 1) / sub);
    need = std::max<uint64_t>(need, (recv_bytes[r] + sub - 1) / sub);
  }
  int64_t rounds = (int64_t)need;
  allreduce(&rounds, 1, at::kLong, c10d::ReduceOp::MAX, timeout);
  for (int64_t k = 0; k < rounds; ++k) {
    const size_t off = (size_t)k * sub;
    const int s = next_set();
    for (int r = 0; r < world_; ++r)
      if (send_bytes[r] > off)
        std::memcpy(slot(s, rank_) + r * sub, static_cast<const char*>(ins[r]) + off,
                    std::min(sub, send_bytes[r] - off));
    barrier(timeout);
    for (int j = 0; j < world_; ++j) {
      const int q = (rank_ + j) % world_;
      if (recv_bytes[q] > off)
        std::memcpy(static_cast<char*>(outs[q]) + off, slot(s, q) + rank_ * sub, std::min(sub, recv_bytes[q] - off));
    }
  }
}

// ----------------------------------------------------------------- p2p
void ShmComm::send(const void* buf, size_t bytes, int peer, std::chrono::milliseconds timeout) {
  std::lock_guard<std::mutex> lk(send_mu_);
  ChanCtl& cc = hdr()->chan[rank_ * kMaxShmRanks + peer];
  char* data = chan_data(rank_, peer);
  const size_t cap = cfg_.chan_bytes;
  const char* p = static_cast<const char*>(buf);
  size_t done = 0;
  while (done < bytes) {
    const uint64_t head = cc.head.v.load(std::memory_order_relaxed);
    uint64_t tail = cc.tail.v.load(std::memory_order_acquire);
    if (head - tail == cap) {
      wait_until([&] { return cc.head.v.load(std::memory_order_relaxed) - cc.tail.v.load(std::memory_order_acquire) < cap; },
                 nullptr, 0, timeout, "send");
      tail = cc.tail.v.load(std::memory_order_acquire);
    }
    const size_t free_b = cap - (size_t)(head - tail);
    const size_t pos = (size_t)(head % cap);
    const size_t n = std::min({bytes - done, free_b, cap - pos});
    std::memcpy(data + pos, p + done, n);
    cc.head.v.store(head + n, std::memory_order_release);
    done += n;
  }
}

void ShmComm::recv(void* buf, size_t bytes, int peer, std::chrono::milliseconds timeout) {
  std::lock_guard<std::mutex> lk(recv_mu_);
  ChanCtl& cc = hdr()->chan[peer * kMaxShmRanks + rank_];
  const char* data = chan_data(peer, rank_);
  const size_t cap = cfg_.chan_bytes;
  char* p = static_cast<char*>(buf);
  size_t done = 0;
  while (done < bytes) {
    const uint64_t tail = cc.tail.v.load(std::memory_order_relaxed);
    uint64_t head = cc.head.v.load(std::memory_order_acquire);
    if (head == tail) {
      wait_until([&] { return cc.head.v.load(std::memory_order_acquire) != cc.tail.v.load(std::memory_order_relaxed); },
                 nullptr, 0, timeout, "recv");
      head = cc.head.v.load(std::memory_order_acquire);
    }
    const size_t avail = (size_t)(head - tail);
    const size_t pos = (size_t)(tail % cap);
    const size_t n = std::min({bytes - done, avail, cap - pos});
    std::memcpy(p + done, data + pos, n);
    cc.tail.v.store(tail + n, std::memory_order_release);
    done += n;
  }
}

}  // namespace host
}  // namespace pdcc
