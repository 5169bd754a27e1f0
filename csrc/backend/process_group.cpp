// ProcessGroupMI355X: construction, Work objects, CPU (shared-memory) paths,
// argument validation, debug fingerprinting, fault injection and the watchdog.
// GPU data paths live in gpu_ops.cpp.
#include "process_group.h"

#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <dlfcn.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <sstream>

#include "../device/comm_util.h"

namespace pdcc {

// =================================================================== Work
WorkMI355X::WorkMI355X(int rank, c10d::OpType type, uint64_t seq, std::vector<at::Tensor> outputs,
                       std::exception_ptr err)
    : c10d::Work(rank, type), seq_(seq), outputs_(std::move(outputs)), start_(std::chrono::steady_clock::now()) {
  if (err) finish(err);
  else finish();
}

WorkMI355X::WorkMI355X(int rank, c10d::OpType type, uint64_t seq, std::vector<at::Tensor> outputs)
    : c10d::Work(rank, type), seq_(seq), outputs_(std::move(outputs)), start_(std::chrono::steady_clock::now()) {}

WorkMI355X::WorkMI355X(int rank, c10d::OpType type, uint64_t seq, std::vector<at::Tensor> outputs, c10::Device dev,
                       hipEvent_t ev, c10::hip::HIPStreamMasqueradingAsCUDA comm, std::shared_ptr<Health> health,
                       bool blocking, std::chrono::milliseconds timeout, std::shared_ptr<IpcComm> ipc,
                       std::shared_ptr<EventPool> pool)
    : c10d::Work(rank, type),
      seq_(seq),
      gpu_(true),
      outputs_(std::move(outputs)),
      dev_(dev),
      ev_(ev),
      health_(std::move(health)),
      ipc_(std::move(ipc)),
      blocking_(blocking),
      timeout_(timeout),
      start_(std::chrono::steady_clock::now()),
      pool_(std::move(pool)),
      comm_(comm) {}

Gate::~Gate() {
  if (ev) (void)hipEventDestroy(ev);
}

WorkMI355X::~WorkMI355X() {
  if (!ev_ || gate_) return;  // a gated work's event belongs to its gate
  if (pool_) pool_->put(ev_);  // re-recording a pooled event later is fine: nobody waits on this one any more
  else hipEventDestroy(ev_);
}

void WorkMI355X::done(std::exception_ptr e) {
  c10::intrusive_ptr<c10::ivalue::Future> f;
  {
    std::lock_guard<std::mutex> lk(mutex_);
    f = fut_;
  }
  finish(e);
  if (f) {
    if (e) f->setError(e);
    else f->markCompleted(c10::IValue(outputs_));
  }
}

c10::intrusive_ptr<c10::ivalue::Future> WorkMI355X::getFuture() {
  std::unique_lock<std::mutex> lk(mutex_);
  if (fut_) return fut_;
  if (gpu_) {
    if (gate_) {  // the future's events go on the comm stream: the op must be there first
      lk.unlock();
      wait_gate(timeout_);
      lk.lock();
      if (fut_) return fut_;
    }
    fut_ = c10::make_intrusive<c10::ivalue::Future>(c10::ListType::create(c10::TensorType::get()),
                                                    std::vector<c10::Device>{dev_});
    auto f = fut_;
    lk.unlock();
    // the future's own events land on the comm stream after this collective
    c10::hip::HIPStreamGuardMasqueradingAsCUDA g(*comm_);
    f->markCompleted(c10::IValue(outputs_));
    return f;
  }
  fut_ = c10::make_intrusive<c10::ivalue::Future>(c10::ListType::create(c10::TensorType::get()));
  auto f = fut_;
  const bool done_now = completed_;
  const std::exception_ptr e = exception_;
  lk.unlock();
  if (done_now) {
    if (e) f->setError(e);
    else f->markCompleted(c10::IValue(outputs_));
  }
  return f;
}

// =================================================================== StreamSync
// Words are allocated kSlabWords at a time, the first batch when the device state is
// created: handing one out later makes no allocation and no memset -- both can
// synchronise with streams that wait on the IPC launcher's thread.
bool StreamSync::grow() {
  // (signal memory comes in 8-byte allocations)
  for (size_t i = 0; i < kSlabWords; ++i) {
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, sizeof(uint64_t), hipMallocSignalMemory) != hipSuccess || !p) {
      (void)hipGetLastError();
      return !spare.empty();
    }
    // signal memory is host-accessible: zero it from the host (no stream involved)
    *static_cast<volatile uint64_t*>(p) = 0;
    words.push_back(static_cast<uint64_t*>(p));
    spare.push_back(static_cast<uint64_t*>(p));
  }
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  return true;
}
uint64_t* StreamSync::alloc() {
  std::lock_guard<std::mutex> lk(slab_mu);
  if (!ok) return nullptr;
  if (spare.empty() && !grow()) {
    ok = false;
    return nullptr;
  }
  uint64_t* w = spare.back();
  spare.pop_back();
  return w;
}
StreamSync::~StreamSync() {
  for (uint64_t* p : words) (void)hipFree(p);
}

// =================================================================== EventPool
hipEvent_t EventPool::get() {
  {
    std::lock_guard<std::mutex> lk(mu);
    if (free.size() > 8) {  // FIFO with slack: re-record the least recently used event
      hipEvent_t e = free.front();
      free.pop_front();
      return e;
    }
  }
  hipEvent_t e;
  PDCC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}
void EventPool::put(hipEvent_t e) {
  std::lock_guard<std::mutex> lk(mu);
  free.push_back(e);
}
EventPool::~EventPool() {
  for (hipEvent_t e : free) hipEventDestroy(e);
}

void WorkMI355X::fail(const std::string& msg) {
  std::lock_guard<std::mutex> lk(mutex_);
  if (!exception_) exception_ = std::make_exception_ptr(std::runtime_error(msg));
}

bool WorkMI355X::gate_open() {
  if (!gate_) return true;
  const int st = gate_->state.load(std::memory_order_acquire);
  if (st == 0) return false;
  if (st < 0) {
    std::lock_guard<std::mutex> lk(gate_->mu);
    throw std::runtime_error("pdcc: " + gate_->error);
  }
  return true;
}

void WorkMI355X::wait_gate(std::chrono::milliseconds lim) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!gate_open()) {
    check_health();
    if (std::chrono::steady_clock::now() - t0 > lim)
      throw std::runtime_error("pdcc: Work.wait() timed out after " + std::to_string(lim.count()) +
                               " ms waiting for the point-to-point channel to be set up");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

bool WorkMI355X::gpu_event_done() {
  if (gate_) {
    const int st = gate_->state.load(std::memory_order_acquire);
    if (st == 0) return false;
    if (st < 0) return true;
  }
  if (done_word_) return __atomic_load_n(done_word_, __ATOMIC_ACQUIRE) >= done_value_;
  if (!ev_) return true;
  return hipEventQuery(ev_) == hipSuccess;
}

void WorkMI355X::check_health() {
  if (health_ && health_->poisoned.load())
    throw std::runtime_error("pdcc: process group is in an error state: " + health_->message());
  if (ipc_ && ipc_->error_word() != 0)
    throw std::runtime_error("pdcc: an IPC collective timed out waiting for a peer (error word " +
                             IpcComm::describe_error(ipc_->error_word()) + ")");
  std::lock_guard<std::mutex> lk(mutex_);
  if (exception_) std::rethrow_exception(exception_);
}

bool WorkMI355X::isCompleted() {
  if (!gpu_) return c10d::Work::isCompleted();
  if (health_ && health_->poisoned.load()) return true;
  return gpu_event_done();
}

bool WorkMI355X::isSuccess() const {
  if (!gpu_) return c10d::Work::isSuccess();
  if (health_ && health_->poisoned.load()) return false;
  if (gate_ && gate_->state.load() < 0) return false;
  std::lock_guard<std::mutex> lk(mutex_);
  return !exception_;
}

void WorkMI355X::synchronize() {
  if (!gpu_) return;
  wait_gate(timeout_);
  c10::hip::HIPGuardMasqueradingAsCUDA g(dev_);
  auto cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(dev_.index());
  if (comm_ && *comm_ == cur) return;  // enqueued on this very stream: already ordered
  if (done_word_) {
    PDCC_HIP(hipStreamWaitValue64(cur.stream(), const_cast<uint64_t*>(done_word_), done_value_,
                                  hipStreamWaitValueGte, ~0ull));
    return;
  }
  PDCC_HIP(hipStreamWaitEvent(cur.stream(), ev_, 0));
}

bool WorkMI355X::wait(std::chrono::milliseconds timeout) {
  if (!gpu_) return c10d::Work::wait(timeout);
  check_health();
  synchronize();  // current stream waits for the collective: host not blocked
  if (blocking_ || timeout != kNoTimeout) {
    const auto lim = (timeout == kNoTimeout) ? timeout_ : timeout;
    const auto t0 = std::chrono::steady_clock::now();
    while (!gpu_event_done()) {
      check_health();
      if (std::chrono::steady_clock::now() - t0 > lim)
        throw std::runtime_error("pdcc: Work.wait() timed out after " + std::to_string(lim.count()) + " ms");
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    check_health();
  }
  return true;
}

std::vector<at::Tensor> WorkMI355X::result() { return outputs_; }

// =================================================================== helpers
namespace {

c10d::OpType op_type_of(int c) {
  switch (c) {
    case 0: return c10d::OpType::ALLREDUCE;
    case 1: return c10d::OpType::REDUCE;
    case 2: return c10d::OpType::BROADCAST;
    case 3: return c10d::OpType::ALLGATHER;
    case 4: return c10d::OpType::GATHER;
    case 5: return c10d::OpType::SCATTER;
    case 6: return c10d::OpType::REDUCE_SCATTER;
    case 7: return c10d::OpType::ALLTOALL;
    case 8: return c10d::OpType::SEND;
    case 9: return c10d::OpType::RECV;
    default: return c10d::OpType::BARRIER;
  }
}

std::string shape_str(const at::Tensor& t) {
  std::ostringstream o;
  o << c10::toString(t.scalar_type()) << "[" << t.numel() << "]@" << t.device();
  return o.str();
}

void check_single(const std::vector<at::Tensor>& ts, const char* fn) {
  TORCH_CHECK(ts.size() == 1, "ProcessGroupMI355X::", fn, ": expects exactly one tensor per call, got ", ts.size());
}

void check_root(int64_t root, int size, const char* fn) {
  TORCH_CHECK(root >= 0 && root < size, "ProcessGroupMI355X::", fn, ": invalid root rank: ", root);
}

void check_list(const std::vector<at::Tensor>& list, const at::Tensor& like, int size, const char* fn,
                const char* what) {
  TORCH_CHECK((int)list.size() == size, "ProcessGroupMI355X::", fn, ": invalid ", what,
              " tensor list at index 0 (expected length ", size, ", got ", list.size(), ")");
  for (size_t i = 0; i < list.size(); ++i) {
    TORCH_CHECK(list[i].scalar_type() == like.scalar_type(), "ProcessGroupMI355X::", fn, ": ", what,
                " tensor ", i, " has dtype ", list[i].scalar_type(), ", expected ", like.scalar_type());
    TORCH_CHECK(list[i].numel() == like.numel(), "ProcessGroupMI355X::", fn, ": ", what, " tensor ", i, " has ",
                list[i].numel(), " elements, expected ", like.numel());
    TORCH_CHECK(list[i].device() == like.device(), "ProcessGroupMI355X::", fn, ": ", what, " tensor ", i,
                " is on ", list[i].device(), ", expected ", like.device());
  }
}

void check_cpu_dtype(at::ScalarType t, c10d::ReduceOp::RedOpType op, const char* fn) {
  const bool fl = at::isFloatingType(t);
  const bool integral = at::isIntegralType(t, /*includeBool=*/true);
  TORCH_CHECK(fl || integral, "ProcessGroupMI355X::", fn, ": unsupported dtype ", t);
  TORCH_CHECK(op != c10d::ReduceOp::PREMUL_SUM, "ProcessGroupMI355X::", fn, ": PREMUL_SUM is not supported");
  if (op == c10d::ReduceOp::BAND || op == c10d::ReduceOp::BOR || op == c10d::ReduceOp::BXOR)
    TORCH_CHECK(!fl, "ProcessGroupMI355X::", fn, ": bitwise reductions need an integer dtype, got ", t);
  if (op == c10d::ReduceOp::AVG) TORCH_CHECK(t != at::kBool, "ProcessGroupMI355X::", fn, ": AVG on bool");
}

// contiguous host staging copy (CPU tensors may be strided views)
struct Contig {
  at::Tensor orig, work;
  explicit Contig(const at::Tensor& t) : orig(t), work(t.is_contiguous() ? t : t.contiguous()) {}
  void* ptr() { return work.data_ptr(); }
  void write_back() {
    if (!work.is_same(orig)) orig.copy_(work);
  }
};

}  // namespace

const char* ProcessGroupMI355X::coll_name(Coll c) {
  switch (c) {
    case Coll::ALLREDUCE: return "allreduce";
    case Coll::REDUCE: return "reduce";
    case Coll::BROADCAST: return "broadcast";
    case Coll::ALLGATHER: return "allgather";
    case Coll::GATHER: return "gather";
    case Coll::SCATTER: return "scatter";
    case Coll::REDUCE_SCATTER: return "reduce_scatter";
    case Coll::ALLTOALL: return "alltoall";
    case Coll::SEND: return "send";
    case Coll::RECV: return "recv";
    case Coll::BARRIER: return "barrier";
  }
  return "?";
}

// roctx ranges (optional, resolved with dlopen so there is no link dependency)
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    for (const char* lib : {"librocprofiler-sdk-roctx.so", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (push && pop) break;
    }
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}
}  // namespace

// =================================================================== construction
ProcessGroupMI355X::ProcessGroupMI355X(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size,
                                       std::chrono::milliseconds timeout, std::vector<int64_t> global_ranks,
                                       std::string group_name)
    : c10d::Backend(rank, size),
      store_(store),
      timeout_(timeout),
      global_ranks_(std::move(global_ranks)),
      group_name_(std::move(group_name)),
      cfg_(Config::from_env()),
      health_(std::make_shared<Health>()) {
  members_key_ = make_members_key(global_ranks_, size);
  // an RCCL op left in progress by a non-blocking communicator is waited for at most this long
  set_rccl_settle_timeout_ms(timeout_.count());
  if (const char* hp = std::getenv("PDCC_HOST_PROF")) hp_.on = *hp && *hp != '0';
  if (!cfg_.fault.empty()) {
    unsigned long long s = 0;
    char kind[32] = {0};
    int r = -1;
    if (sscanf(cfg_.fault.c_str(), "%d:%llu:%31s", &r, &s, kind) == 3) {
      fault_rank_ = r;
      fault_seq_ = s;
      fault_kind_ = kind;
    }
  }
  // topology: all ranks of this group on one host? (shm host path + IPC need it)
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  const std::string h(host);
  const auto all = store_allgather(store_, "pdcc/topo", rank, size, std::vector<uint8_t>(h.begin(), h.end()));
  for (const auto& v : all) same_host_ = same_host_ && (std::string(v.begin(), v.end()) == h);
  // The store's server usually lives in rank 0's process: rank 0 leaves construction only once every rank
  // has read the records above, so a job without a single collective (the reference's hello_world,
  // main.py:86-87) cannot end rank 0 -- and the server with it -- under a peer still reading them
  // (seen as "Failed to recv ... Connection was likely closed" in a peer's constructor)
  if (size > 1) {
    store_->add("pdcc/topo_read", 1);
    if (rank == 0) {
      const auto deadline = std::chrono::steady_clock::now() + timeout_;
      while (store_->add("pdcc/topo_read", 0) < size && std::chrono::steady_clock::now() < deadline)
        std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  }
  if (cfg_.log_level >= 1 && rank == 0)
    fprintf(stderr, "[pdcc] group '%s' size=%d same_host=%d %s\n", group_name_.c_str(), size, (int)same_host_,
            cfg_.describe().c_str());
  if (cfg_.roctx) {
    roctx_push_ = roctx().push;
    roctx_pop_ = roctx().pop;
  }
  if (const char* fr = std::getenv("PDCC_FLIGHT_RECORDER")) fr_cap_ = (size_t)std::max(0, std::atoi(fr));
  if (cfg_.watchdog_ms > 0) wd_thr_ = std::thread([this] { watchdog_loop(); });
  if (cfg_.eager_init) {
    int n = 0, d = 0;
    if (hipGetDeviceCount(&n) == hipSuccess && n > 0 && hipGetDevice(&d) == hipSuccess) eager_init(d);
    else (void)hipGetLastError();
  }
}

ProcessGroupMI355X::~ProcessGroupMI355X() {
  stop_launchers();
  wd_stop_.store(true);
  if (wd_thr_.joinable()) wd_thr_.join();
  {
    std::lock_guard<std::mutex> lk(p2p_mu_);
    stop_ = true;
  }
  p2p_cv_.notify_all();
  if (send_thr_.joinable()) send_thr_.join();
  if (recv_thr_.joinable()) recv_thr_.join();
  for (auto& kv : devs_) {
    DeviceState& ds = *kv.second;
    if (!health_->poisoned.load()) continue;
    if (ds.rccl) ds.rccl->abort();
    if (ds.rccl_wide) ds.rccl_wide->abort();
    for (auto& p : ds.pairs) {
      std::lock_guard<std::mutex> lk(p.second->mu);
      if (p.second->comm) p.second->comm->abort();
    }
  }
}

std::chrono::milliseconds ProcessGroupMI355X::eff_timeout(std::chrono::milliseconds t) const {
  return t == c10d::kUnsetTimeout ? timeout_ : t;
}

// 2-rank shared-memory channel pair for point-to-point with `peer`: built by the
// two ranks alone (lazily, on the send/recv worker threads), so send/recv never
// wait for the other ranks of the group. One mutex per peer: the send and recv
// threads may both ask for the same pair, and different pairs never block each other.
host::ShmComm& ProcessGroupMI355X::shm_pair(int peer) {
  std::shared_ptr<std::mutex> m;
  {
    std::lock_guard<std::mutex> lk(pair_mu_);
    auto it = shm_pairs_.find(peer);
    if (it != shm_pairs_.end()) return *it->second;
    auto& pm = shm_pair_mu_[peer];
    if (!pm) pm = std::make_shared<std::mutex>();
    m = pm;
  }
  std::lock_guard<std::mutex> plk(*m);
  {
    std::lock_guard<std::mutex> lk(pair_mu_);
    auto it = shm_pairs_.find(peer);
    if (it != shm_pairs_.end()) return *it->second;
  }
  TORCH_CHECK(same_host_, "pdcc: the shared-memory host path needs every rank of the group on one host");
  host::ShmConfig sc;
  sc.slot_bytes = 4096;  // collectives never run on a pair channel
  sc.spin_us = cfg_.shm_spin_us;
  sc.chan_bytes = cfg_.shm_chan_bytes;
  sc.timeout = timeout_;
  const int lo = std::min(rank_, peer), hi = std::max(rank_, peer);
  auto c = std::make_unique<host::ShmComm>(store_, "pdcc/shmp2p/" + std::to_string(lo) + ":" + std::to_string(hi),
                                           rank_ == lo ? 0 : 1, 2, sc);
  std::lock_guard<std::mutex> lk(pair_mu_);
  host::ShmComm& ref = *c;
  shm_pairs_[peer] = std::move(c);
  return ref;
}

host::ShmComm& ProcessGroupMI355X::shm() {
  std::lock_guard<std::mutex> lk(init_mu_);
  if (!shm_) {
    TORCH_CHECK(same_host_, "pdcc: the shared-memory host path needs every rank of the group on one host");
    host::ShmConfig sc;
    sc.slot_bytes = cfg_.shm_slot_bytes;
    sc.spin_us = cfg_.shm_spin_us;
    sc.chan_bytes = size_ > 16 ? std::min<size_t>(cfg_.shm_chan_bytes, 256u << 10) : cfg_.shm_chan_bytes;
    sc.timeout = timeout_;
    shm_ = std::make_unique<host::ShmComm>(store_, "pdcc/shm", rank_, size_, sc);
  }
  return *shm_;
}

void ProcessGroupMI355X::maybe_inject_fault() {
  const uint64_t s = op_seq_.load();
  if (fault_rank_ != rank_ || fault_seq_ != s) return;
  fprintf(stderr, "[pdcc] rank %d: injecting fault '%s' at op %llu\n", rank_, fault_kind_.c_str(),
          (unsigned long long)s);
  fflush(stderr);
  if (fault_kind_ == "exit") _exit(13);
  if (fault_kind_ == "hang")
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
  throw std::runtime_error("pdcc: injected fault at op " + std::to_string(s));
}

void ProcessGroupMI355X::before_op(Coll c, const std::vector<at::Tensor>& ts, int root) {
  // (the stage profiler's clock: allreduce() starts it on entry; every other collective here, so its
  // first stage is not measured from the previous op)
  if (c != Coll::ALLREDUCE) hp_.start();
  if (health_->poisoned.load())
    throw std::runtime_error("pdcc: process group is in an error state: " + health_->message());
  ++op_seq_;
  maybe_inject_fault();
  if (cfg_.debug && c != Coll::SEND && c != Coll::RECV) debug_check(c, ts, root);
  if (cfg_.log_level >= 2)
    fprintf(stderr, "[pdcc r%d] #%llu %s %s root=%d\n", rank_, (unsigned long long)op_seq_.load(), coll_name(c),
            ts.empty() ? "-" : shape_str(ts[0]).c_str(), root);
}

// PDCC_DEBUG=1: every rank publishes a fingerprint of the op it is about to run
// and compares it with everyone else's -- catches the silent desync the survey
// found with Gloo (per-rank shape mismatch: rank 0 "OK", rank 1 error).
void ProcessGroupMI355X::debug_check(Coll c, const std::vector<at::Tensor>& ts, int root) {
  struct Fp {
    uint64_t seq;
    int32_t coll, dtype;
    int64_t numel;
    int32_t root, dev_type;
    int32_t async_op, pad;  // with PDCC_IPC_ASYNC_GRID set, async collectives run capped grids: ranks must agree
  };
  Fp mine{op_seq_.load(), (int32_t)c, ts.empty() ? -1 : (int32_t)ts[0].scalar_type(),
          ts.empty() ? 0 : ts[0].numel(), root, ts.empty() ? -1 : (int32_t)ts[0].device().type(),
          (int32_t)op_async_, 0};
  std::vector<Fp> all(size_);
  std::vector<void*> outs(size_);
  for (int r = 0; r < size_; ++r) outs[r] = &all[r];
  shm().allgather(&mine, outs, sizeof(Fp), timeout_);
  for (int r = 0; r < size_; ++r) {
    const Fp& f = all[r];
    if (f.seq != mine.seq || f.coll != mine.coll || f.dtype != mine.dtype || f.numel != mine.numel ||
        f.root != mine.root || f.dev_type != mine.dev_type ||
        (f.async_op != mine.async_op && cfg_.ipc_async_grid > 0 && mine.dev_type == (int32_t)c10::DeviceType::CUDA)) {
      std::ostringstream o;
      o << "pdcc DEBUG: collective mismatch at op #" << mine.seq << ": rank " << rank_ << " runs "
        << coll_name(c) << "(dtype=" << mine.dtype << ", numel=" << mine.numel << ", root=" << mine.root
        << ") but rank " << r << " runs " << coll_name((Coll)f.coll) << "(dtype=" << f.dtype
        << ", numel=" << f.numel << ", root=" << f.root << ", op #" << f.seq << ")"
        << (f.async_op != mine.async_op ? " (async_op differs)" : "");
      throw std::runtime_error(o.str());
    }
  }
}

void ProcessGroupMI355X::record_setup(const std::string& key, std::chrono::steady_clock::time_point t0) {
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> lk(stats_mu_);
  OpStats& s = stats_[key];
  s.calls++;
  s.host_ms += ms;
}

void ProcessGroupMI355X::record(Coll c, const char* algo, size_t bytes, std::chrono::steady_clock::time_point t0) {
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> lk(stats_mu_);
  if (sdma_ran_) algo = "ipc_sdma";  // (the engine job ran on the copy engines: sdma_run)
  sdma_ran_ = false;
  PendingRec p{++rec_id_, c, algo, bytes, ms, {}};
  // an IPC op whose zero-copy attempts all ran zero-copy is counted as "<algo>_zc" -- decided from
  // the outcome (a gated attempt's exchange may still be running: the record waits in pending_)
  if (std::strncmp(algo, "ipc", 3) == 0) p.parts = std::move(zc_parts_);
  zc_parts_.clear();
  if (fr_cap_ > 0) {
    FrEntry e{op_seq_.load(), std::string(coll_name(c)) + "/" + algo + (p.parts.empty() ? "" : "_zc?"), bytes,
              std::chrono::duration<double, std::milli>(t0 - created_).count(), (bool)fr_last_work_,
              fr_last_work_ ? c10::weak_intrusive_ptr<WorkMI355X>(fr_last_work_)
                            : c10::weak_intrusive_ptr<WorkMI355X>(c10::intrusive_ptr<WorkMI355X>()),
              p.id};
    fr_last_work_.reset();
    fr_.push_back(std::move(e));
    while (fr_.size() > fr_cap_) fr_.pop_front();
  }
  pending_.push_back(std::move(p));
  zc_resolve_locked(false);
}

void ProcessGroupMI355X::finalize_locked(PendingRec& p) {
  bool zc = !p.parts.empty();
  for (const auto& z : p.parts) zc = zc && z.state == 1;
  if (!p.parts.empty()) ++(zc ? zc_ran_calls_ : zc_staged_calls_);
  const std::string name = p.algo + (zc ? "_zc" : "");
  const std::string key = std::string(coll_name(p.coll)) + "/" + name;
  OpStats& s = stats_[key];
  s.calls++;
  s.bytes += p.bytes;
  s.host_ms += p.ms;
  if (p.id == rec_id_) last_algo_ = name;
  if (!p.parts.empty())
    for (auto it = fr_.rbegin(); it != fr_.rend(); ++it)
      if (it->rec_id == p.id) {
        it->what = key;
        break;
      }
}

void ProcessGroupMI355X::zc_resolve_locked(bool block) {
  const auto deadline = std::chrono::steady_clock::now() + timeout_;
  while (!pending_.empty()) {
    PendingRec& p = pending_.front();
    bool done = true;
    for (auto& z : p.parts) {
      if (z.state >= 0) continue;
      IpcLauncher& L = *z.launcher;
      std::unique_lock<std::mutex> lk(L.mu);
      for (;;) {
        auto it = L.outcome.find(z.ticket);
        if (it != L.outcome.end()) {
          z.state = it->second ? 1 : 0;
          L.outcome.erase(it);
          break;
        }
        // (its job has run but the entry is gone, or the exchange can no longer run: not zero-copy)
        if (L.done_hi >= z.ticket || L.stop || health_->poisoned.load() || !block ||
            std::chrono::steady_clock::now() >= deadline) {
          if (block || L.done_hi >= z.ticket || L.stop) z.state = 0;
          break;
        }
        L.outcome_cv.wait_for(lk, std::chrono::milliseconds(50));
      }
      done = done && z.state >= 0;
    }
    if (!done) break;  // (records settle in issue order: their jobs run in that order)
    finalize_locked(p);
    pending_.pop_front();
  }
}

std::string ProcessGroupMI355X::last_algo() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  zc_resolve_locked(true);
  return last_algo_;
}

std::map<std::string, uint64_t> ProcessGroupMI355X::zc_counters() {
  std::map<std::string, uint64_t> out;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    zc_resolve_locked(true);
    out["zc_calls"] = zc_ran_calls_;
    out["zc_fallbacks"] = zc_staged_calls_;
    out["zc_pending"] = pending_.size();
  }
  uint64_t size_ref = 0, full_ref = 0, xchg_fallbacks = 0, kept = 0, exp_fail = 0, map_fail = 0;
  std::lock_guard<std::mutex> lk(init_mu_);
  for (auto& kv : devs_) {
    if (kv.second->ipc) {
      kept += kv.second->ipc->kept_exports();
      exp_fail += kv.second->ipc->zc_export_failures();
      map_fail += kv.second->ipc->zc_map_failures();
      size_ref += kv.second->ipc->zc_size_refusals();
      full_ref += kv.second->ipc->zc_full_refusals();
    }
    if (kv.second->launcher) {
      std::lock_guard<std::mutex> l2(kv.second->launcher->mu);
      xchg_fallbacks += kv.second->launcher->fallbacks;
    }
  }
  out["zc_size_refusals"] = size_ref;
  out["zc_full_refusals"] = full_ref;
  out["zc_exchange_fallbacks"] = xchg_fallbacks;
  out["ipc_stale_maps"] = IpcComm::stale_mappings();
  out["ipc_kept_exports"] = kept;
  out["zc_export_failures"] = exp_fail;
  out["zc_map_failures"] = map_fail;
  return out;
}

std::vector<std::tuple<std::string, uint64_t, double>> ProcessGroupMI355X::host_profile() {
  static const char* kNames[] = {"before_op", "dev_state", "choose", "pre", "enqueue", "work", "record",
                                 "zc_export", "zc_reserve", "zc_launch", "zc_mark", "zc_job"};
  static_assert(sizeof(kNames) / sizeof(kNames[0]) == (size_t)HostStage::N, "stage names");
  std::vector<std::tuple<std::string, uint64_t, double>> out;
  for (int i = 0; i < (int)HostStage::N; ++i) out.emplace_back(kNames[i], hp_.calls[i], hp_.ns[i] / 1e3);
  return out;
}

std::vector<ProcessGroupMI355X::FrRecord> ProcessGroupMI355X::flight_recorder() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  zc_resolve_locked(false);  // (never waits: also read while a peer is stuck)
  std::vector<FrRecord> out;
  for (auto& e : fr_) {
    std::string st = "done";
    if (e.gpu) {
      auto w = e.work.lock();
      if (!w) st = "released";
      else if (!w->isCompleted()) st = "pending";
      else if (!w->isSuccess()) st = "failed";
    }
    out.push_back({e.seq, e.what, e.bytes, e.t_ms, st});
  }
  return out;
}

std::string ProcessGroupMI355X::flight_recorder_dump(size_t last) {
  auto recs = flight_recorder();
  std::ostringstream o;
  o << "[pdcc] flight recorder, rank " << rank_ << ", last " << std::min(last, recs.size()) << " of " << recs.size()
    << " ops:\n";
  for (size_t i = recs.size() > last ? recs.size() - last : 0; i < recs.size(); ++i)
    o << "  #" << recs[i].seq << " " << recs[i].what << " bytes=" << recs[i].bytes << " t=" << recs[i].t_ms
      << "ms state=" << recs[i].state << "\n";
  return o.str();
}

std::map<std::string, OpStats> ProcessGroupMI355X::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  zc_resolve_locked(true);
  return stats_;
}
void ProcessGroupMI355X::reset_stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  zc_resolve_locked(true);  // (a call issued before the reset is not counted after it)
  stats_.clear();
}

std::string ProcessGroupMI355X::describe() {
  std::ostringstream o;
  o << "ProcessGroupMI355X(group=" << group_name_ << ", rank=" << rank_ << ", size=" << size_
    << ", same_host=" << same_host_ << ", timeout_ms=" << timeout_.count() << ", " << cfg_.describe();
  std::lock_guard<std::mutex> lk(init_mu_);
  for (auto& kv : devs_) {
    o << ", dev" << kv.first << "{rccl_ok=" << kv.second->rccl_ok << ", ipc_ok=" << kv.second->ipc_ok
      << ", zc_ok=" << kv.second->zc_ok << ", zx_ok=" << (kv.second->ipc ? kv.second->ipc->zx_on() : kv.second->zx_ok)
      << ", zx_fast=" << (kv.second->ipc ? kv.second->ipc->zx_fast() : 0)
      << ", zx_host=" << (kv.second->ipc ? kv.second->ipc->zx_host() : 0)
      << ", ll_ok=" << kv.second->ll_ok << ", shared_device=" << kv.second->shared_device
      << ", rccl=" << (kv.second->rccl != nullptr) << ", ipc=" << (kv.second->ipc != nullptr)
      << ", rccl_users=" << (kv.second->rccl ? kv.second->rccl->order().users() : 0)
      << ", rccl_issue_waits=" << (kv.second->rccl ? kv.second->rccl->order().waits() : 0)
      << ", zc_exports=" << (kv.second->ipc ? kv.second->ipc->zc_exports() : 0)
      << ", zc_mappings=" << (kv.second->ipc ? kv.second->ipc->zc_mappings() : 0)
      << ", zc_closing=" << (kv.second->ipc ? kv.second->ipc->zc_closing() : 0)
      << ", zc_full_refusals=" << (kv.second->ipc ? kv.second->ipc->zc_full_refusals() : 0)
      << ", zc_size_refusals=" << (kv.second->ipc ? kv.second->ipc->zc_size_refusals() : 0)
      << ", ipc_stale_maps=" << IpcComm::stale_mappings()
      << ", async_capped=" << (kv.second->ipc ? kv.second->ipc->async_capped() : 0)
      << ", launcher_jobs=" << (kv.second->launcher ? kv.second->launcher->jobs : 0)
      << ", zc_fallbacks=" << (kv.second->launcher ? kv.second->launcher->fallbacks : 0);
    if (kv.second->launcher) {
      IpcLauncher& L = *kv.second->launcher;
      std::lock_guard<std::mutex> lk2(L.mu);
      if (L.jobs)
        o << ", xchg_wait_us=" << (int)(L.wait_ns / 1e3 / L.jobs) << ", xchg_us=" << (int)(L.run_ns / 1e3 / L.jobs)
          << ", xchg_gather_us=" << (int)(L.gather_ns / 1e3 / L.jobs)
          << ", xchg_depth_x10=" << (int)(10.0 * (double)L.depth_sum / (double)L.jobs);
    }
    o << "}";
  }
  o << ")";
  return o.str();
}

void ProcessGroupMI355X::abort_group(const std::string& why) {
  health_->poison(why);
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) {
      DeviceState& ds = *kv.second;
      if (ds.rccl) ds.rccl->abort();
      if (ds.rccl_wide) ds.rccl_wide->abort();
      for (auto& p : ds.pairs) {
        std::lock_guard<std::mutex> plk(p.second->mu);
        if (p.second->comm) p.second->comm->abort();
      }
      if (ds.ipc) ds.ipc->abort();  // kernels spinning in a cross-GPU barrier leave it
      if (ds.xchg) ds.xchg->abort();  // a launcher job (or an inline call) stuck in an exchange
    }
    if (shm_) shm_->abort();
  }
  std::lock_guard<std::mutex> lk(pair_mu_);
  for (auto& kv : shm_pairs_) kv.second->abort();
}

void ProcessGroupMI355X::abort() { abort_group("aborted by ProcessGroup.abort()"); }

std::vector<std::vector<uint64_t>> ProcessGroupMI355X::ipc_trace() {
  std::lock_guard<std::mutex> lk(init_mu_);
  for (auto& kv : devs_)
    if (kv.second->ipc) return kv.second->ipc->trace_records();
  return {};
}

// Orderly shutdown (destroy_process_group): let enqueued GPU work drain for up to the
// group timeout; a group that cannot drain (a peer is gone) is aborted instead of hanging.
void ProcessGroupMI355X::shutdown() {
  if (health_->poisoned.load()) return;
  std::vector<hipStream_t> streams;
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) {
      streams.push_back(kv.second->stream.stream());
      // (synchronous collectives ran on the caller's stream)
      streams.push_back(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)kv.first).stream());
      for (auto& p : kv.second->pairs) streams.push_back(p.second->stream.stream());
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (hipStream_t s : streams) {
    while (hipStreamQuery(s) == hipErrorNotReady) {
      if (health_->poisoned.load()) return;
      if (std::chrono::steady_clock::now() - t0 > timeout_) {
        abort_group("shutdown: GPU work did not drain within the group timeout");
        return;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    (void)hipGetLastError();
  }
  // Release the group's IPC memory now (collectively: every rank closes its mappings of the peers'
  // buffers before any rank frees its own, IpcComm::release), not whenever the last reference goes
  stop_launchers();
  for (hipStream_t s : streams) (void)hipStreamSynchronize(s);
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) {
      for (hipStream_t x : kv.second->sdma_side) (void)hipStreamSynchronize(x);
      if (kv.second->ipc)
        kv.second->ipc->release(std::min<std::chrono::milliseconds>(
            std::chrono::duration_cast<std::chrono::milliseconds>(timeout_), std::chrono::milliseconds(30000)));
    }
  }
  (void)hipGetLastError();
}

c10d::ErrorType ProcessGroupMI355X::getError() {
  if (!health_->poisoned.load()) return c10d::ErrorType::SUCCESS;
  const std::string m = health_->message();
  if (m.find("timeout") != std::string::npos || m.find("timed out") != std::string::npos)
    return c10d::ErrorType::TIMEOUT;
  return c10d::ErrorType::COMM_ERROR;
}

c10::intrusive_ptr<c10d::Backend> ProcessGroupMI355X::split(const c10::intrusive_ptr<c10d::Store>& store,
                                                            const std::vector<int>& ranks,
                                                            const c10::intrusive_ptr<c10d::Backend::Options>& opts) {
  const auto me = std::find(ranks.begin(), ranks.end(), rank_);
  if (me == ranks.end()) return nullptr;  // not a member of this split
  std::vector<int64_t> global;
  for (int r : ranks) {
    TORCH_CHECK(r >= 0 && r < size_, "ProcessGroupMI355X::split: rank ", r, " is not in this group");
    global.push_back(global_ranks_.empty() ? r : global_ranks_[r]);
  }
  const auto timeout = opts ? opts->timeout : timeout_;
  std::string name = opts && !opts->group_name.empty() ? opts->group_name : group_name_ + ":split";
  return c10::make_intrusive<ProcessGroupMI355X>(store, (int)(me - ranks.begin()), (int)ranks.size(), timeout,
                                                 std::move(global), std::move(name));
}

void ProcessGroupMI355X::set_algo(const std::string& a) {
  if (a == "auto") cfg_.force_algo = Algo::AUTO;
  else if (a == "rccl") cfg_.force_algo = Algo::RCCL;
  else if (a == "ipc") cfg_.force_algo = Algo::IPC;
  else if (a == "host") cfg_.force_algo = Algo::HOST;
  else if (a == "ipc_push") cfg_.force_algo = Algo::IPC_PUSH;
  else if (a == "rccl_wide") cfg_.force_algo = Algo::RCCL_WIDE;
  else if (a == "ipc_wide") cfg_.force_algo = Algo::IPC_WIDE;
  else if (a == "ipc_staged") cfg_.force_algo = Algo::IPC_STAGED;
  else if (a == "ipc_dyn") cfg_.force_algo = Algo::IPC_DYN;
  else if (a == "ipc_sdma") cfg_.force_algo = Algo::IPC_SDMA;
  else TORCH_CHECK(false, "set_algo: expected auto|rccl|rccl_wide|ipc|ipc_push|ipc_wide|ipc_staged|ipc_dyn|ipc_sdma|host, got ", a);
}

void ProcessGroupMI355X::set_ipc_thresholds(int64_t one_shot_max, int64_t two_shot_max, int64_t copy_max) {
  if (one_shot_max >= 0) cfg_.ipc_1shot_max = (size_t)one_shot_max;
  if (two_shot_max >= 0) cfg_.ipc_2shot_max = (size_t)two_shot_max;
  if (copy_max >= 0) cfg_.ipc_copy_max = (size_t)copy_max;
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::cpu_done(Coll c, std::vector<at::Tensor> outputs) {
  return c10::make_intrusive<WorkMI355X>(rank_, op_type_of((int)c), op_seq_.load(), std::move(outputs), nullptr);
}

// =================================================================== watchdog
void ProcessGroupMI355X::watchdog_loop() {
  // the caller's thread may capture collectives into a hipGraph while this one
  // polls events: relaxed capture mode keeps those queries from breaking the capture
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  while (!wd_stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.watchdog_ms));
    std::vector<c10::intrusive_ptr<WorkMI355X>> live;
    {
      std::lock_guard<std::mutex> lk(wd_mu_);
      std::vector<c10::weak_intrusive_ptr<WorkMI355X>> keep;
      for (auto& w : inflight_) {
        auto s = w.lock();
        if (!s) continue;
        live.push_back(s);
      }
      inflight_.clear();
      for (auto& s : live) inflight_.emplace_back(s);
    }
    std::vector<c10::intrusive_ptr<WorkMI355X>> still;
    const auto now = std::chrono::steady_clock::now();
    for (auto& w : live) {
      if (w->gpu_event_done()) continue;
      if (now - w->start() > w->timeout()) {
        const std::string msg = "watchdog: collective #" + std::to_string(w->getSequencenumber()) + " on rank " +
                                std::to_string(rank_) + " exceeded its timeout of " +
                                std::to_string(w->timeout().count()) + " ms; aborting the group";
        fprintf(stderr, "[pdcc] %s\n%s", msg.c_str(), flight_recorder_dump().c_str());
        w->fail(msg);
        abort_group(msg);
        continue;
      }
      still.push_back(w);
    }
    {
      std::lock_guard<std::mutex> lk(wd_mu_);
      std::vector<c10::weak_intrusive_ptr<WorkMI355X>> merged;
      for (auto& w : inflight_) {
        auto s = w.lock();
        if (s && !s->gpu_event_done()) merged.emplace_back(s);
      }
      inflight_.swap(merged);
    }
    // asynchronous RCCL errors and IPC spin timeouts poison the group
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) {
      DeviceState& ds = *kv.second;
      std::vector<std::shared_ptr<RcclComm>> comms;
      if (ds.rccl) comms.push_back(ds.rccl);
      if (ds.rccl_wide) comms.push_back(ds.rccl_wide);
      for (auto& p : ds.pairs) {
        std::lock_guard<std::mutex> plk(p.second->mu);
        if (p.second->comm) comms.push_back(p.second->comm);
      }
      for (auto& c : comms) {
        ncclResult_t r = c->async_error();
        if (r != ncclSuccess && r != ncclInProgress) {
          const std::string m = std::string("RCCL async error: ") + ncclGetErrorString(r);
          fprintf(stderr, "[pdcc] rank %d: %s\n", rank_, m.c_str());
          health_->poison(m);
          c->abort();
          if (ds.ipc) ds.ipc->abort();
        }
      }
      if (ds.ipc && ds.ipc->error_word() != 0 && !health_->poisoned.load() && !tuning_.load()) {
        const std::string m = "IPC collective timed out waiting for a peer (error word " +
                              IpcComm::describe_error(ds.ipc->error_word()) + ")";
        fprintf(stderr, "[pdcc] rank %d: %s\n", rank_, m.c_str());
        health_->poison(m);
      }
    }
  }
}

// =================================================================== p2p threads (CPU)
void ProcessGroupMI355X::p2p_loop(std::deque<Job>* q, bool* stop) {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(p2p_mu_);
      p2p_cv_.wait(lk, [&] { return *stop || !q->empty(); });
      if (q->empty()) return;
      j = std::move(q->front());
      q->pop_front();
    }
    std::exception_ptr e;
    try {
      j.fn();
    } catch (...) {
      e = std::current_exception();
    }
    j.work->done(e);
  }
}

void ProcessGroupMI355X::p2p_submit(bool is_send, Job j) {
  std::lock_guard<std::mutex> lk(p2p_mu_);
  if (is_send && !send_thr_.joinable()) send_thr_ = std::thread([this] { p2p_loop(&send_q_, &stop_); });
  if (!is_send && !recv_thr_.joinable()) recv_thr_ = std::thread([this] { p2p_loop(&recv_q_, &stop_); });
  (is_send ? send_q_ : recv_q_).push_back(std::move(j));
  p2p_cv_.notify_all();
}

// =================================================================== collectives
c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::allreduce(std::vector<at::Tensor>& tensors,
                                                             const c10d::AllreduceOptions& opts) {
  hp_.start();
  op_async_ = opts.asyncOp;
  check_single(tensors, "allreduce");
  at::Tensor& t = tensors[0];
  before_op(Coll::ALLREDUCE, tensors, -1);
  hp_.lap(HostStage::BEFORE_OP);
  if (t.is_cuda()) return gpu_allreduce(t, opts.reduceOp.op_, -1, false, eff_timeout(opts.timeout));
  check_cpu_dtype(t.scalar_type(), opts.reduceOp.op_, "allreduce");
  const auto t0 = std::chrono::steady_clock::now();
  if (size_ > 1) {
    Contig c(t);
    shm().allreduce(c.ptr(), t.numel(), t.scalar_type(), opts.reduceOp.op_, eff_timeout(opts.timeout));
    c.write_back();
  }
  record(Coll::ALLREDUCE, "shm", t.nbytes(), t0);
  return cpu_done(Coll::ALLREDUCE, tensors);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::reduce(std::vector<at::Tensor>& tensors,
                                                          const c10d::ReduceOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(tensors, "reduce");
  check_root(opts.rootRank, size_, "reduce");
  at::Tensor& t = tensors[0];
  before_op(Coll::REDUCE, tensors, (int)opts.rootRank);
  if (t.is_cuda()) return gpu_allreduce(t, opts.reduceOp.op_, (int)opts.rootRank, true, eff_timeout(opts.timeout));
  check_cpu_dtype(t.scalar_type(), opts.reduceOp.op_, "reduce");
  const auto t0 = std::chrono::steady_clock::now();
  if (size_ > 1) {
    Contig c(t);
    shm().reduce(c.ptr(), t.numel(), t.scalar_type(), opts.reduceOp.op_, (int)opts.rootRank,
                 eff_timeout(opts.timeout));
    if (rank_ == opts.rootRank) c.write_back();
  }
  record(Coll::REDUCE, "shm", t.nbytes(), t0);
  return cpu_done(Coll::REDUCE, tensors);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::broadcast(std::vector<at::Tensor>& tensors,
                                                             const c10d::BroadcastOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(tensors, "broadcast");
  check_root(opts.rootRank, size_, "broadcast");
  at::Tensor& t = tensors[0];
  before_op(Coll::BROADCAST, tensors, (int)opts.rootRank);
  if (t.is_cuda()) return gpu_broadcast(t, (int)opts.rootRank, eff_timeout(opts.timeout));
  const auto t0 = std::chrono::steady_clock::now();
  if (size_ > 1) {
    Contig c(t);
    shm().broadcast(c.ptr(), t.nbytes(), (int)opts.rootRank, eff_timeout(opts.timeout));
    c.write_back();
  }
  record(Coll::BROADCAST, "shm", t.nbytes(), t0);
  return cpu_done(Coll::BROADCAST, tensors);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::allgather(std::vector<std::vector<at::Tensor>>& outputs,
                                                             std::vector<at::Tensor>& inputs,
                                                             const c10d::AllgatherOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(inputs, "allgather");
  TORCH_CHECK(outputs.size() == 1, "ProcessGroupMI355X::allgather: expects one output list");
  at::Tensor& in = inputs[0];
  check_list(outputs[0], in, size_, "allgather", "output");
  before_op(Coll::ALLGATHER, inputs, -1);
  if (in.is_cuda()) return gpu_allgather(outputs[0], in, -1, false, eff_timeout(opts.timeout));
  const auto t0 = std::chrono::steady_clock::now();
  Contig ci(in);
  std::vector<Contig> co;
  std::vector<void*> ptrs;
  for (auto& o : outputs[0]) co.emplace_back(o);
  for (auto& c : co) ptrs.push_back(c.ptr());
  if (size_ > 1) shm().allgather(ci.ptr(), ptrs, in.nbytes(), eff_timeout(opts.timeout));
  else std::memcpy(ptrs[0], ci.ptr(), in.nbytes());
  for (auto& c : co) c.write_back();
  record(Coll::ALLGATHER, "shm", in.nbytes(), t0);
  return cpu_done(Coll::ALLGATHER, outputs[0]);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::_allgather_base(at::Tensor& output, at::Tensor& input,
                                                                   const c10d::AllgatherOptions& opts) {
  TORCH_CHECK(output.numel() == input.numel() * size_, "ProcessGroupMI355X::_allgather_base: output has ",
              output.numel(), " elements, expected ", input.numel() * size_);
  TORCH_CHECK(output.scalar_type() == input.scalar_type(), "ProcessGroupMI355X::_allgather_base: dtype mismatch");
  TORCH_CHECK(output.is_contiguous(), "ProcessGroupMI355X::_allgather_base: output must be contiguous");
  // one 1-D view per rank (only numel, dtype and device are checked; the engines need the pointers):
  // one split instead of a narrow + view per rank keeps a small call's host time down
  std::vector<std::vector<at::Tensor>> outs(1);
  outs[0] = input.numel() > 0 ? output.view({-1}).split(input.numel())
                              : std::vector<at::Tensor>((size_t)size_, output.view({-1}));
  std::vector<at::Tensor> ins{input};
  return allgather(outs, ins, opts);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::gather(std::vector<std::vector<at::Tensor>>& outputs,
                                                          std::vector<at::Tensor>& inputs,
                                                          const c10d::GatherOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(inputs, "gather");
  check_root(opts.rootRank, size_, "gather");
  at::Tensor& in = inputs[0];
  const int root = (int)opts.rootRank;
  if (rank_ == root) {
    TORCH_CHECK(outputs.size() == 1, "ProcessGroupMI355X::gather: root expects one output list");
    check_list(outputs[0], in, size_, "gather", "output");
  } else {
    TORCH_CHECK(outputs.empty() || outputs[0].empty(),
                "ProcessGroupMI355X::gather: output list must be empty on non-root ranks");
  }
  before_op(Coll::GATHER, inputs, root);
  std::vector<at::Tensor> empty;
  std::vector<at::Tensor>& outl = (rank_ == root) ? outputs[0] : empty;
  if (in.is_cuda()) return gpu_allgather(outl, in, root, true, eff_timeout(opts.timeout));
  const auto t0 = std::chrono::steady_clock::now();
  Contig ci(in);
  std::vector<Contig> co;
  std::vector<void*> ptrs(size_, nullptr);
  for (auto& o : outl) co.emplace_back(o);
  for (size_t i = 0; i < co.size(); ++i) ptrs[i] = co[i].ptr();
  if (size_ > 1) shm().gather(ci.ptr(), ptrs, in.nbytes(), root, eff_timeout(opts.timeout));
  else std::memcpy(ptrs[0], ci.ptr(), in.nbytes());
  for (auto& c : co) c.write_back();
  record(Coll::GATHER, "shm", in.nbytes(), t0);
  return cpu_done(Coll::GATHER, outl);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::scatter(std::vector<at::Tensor>& outputs,
                                                           std::vector<std::vector<at::Tensor>>& inputs,
                                                           const c10d::ScatterOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(outputs, "scatter");
  check_root(opts.rootRank, size_, "scatter");
  at::Tensor& out = outputs[0];
  const int root = (int)opts.rootRank;
  if (rank_ == root) {
    TORCH_CHECK(inputs.size() == 1, "ProcessGroupMI355X::scatter: root expects one input list");
    check_list(inputs[0], out, size_, "scatter", "input");
  } else {
    TORCH_CHECK(inputs.empty() || inputs[0].empty(),
                "ProcessGroupMI355X::scatter: input list must be empty on non-root ranks");
  }
  before_op(Coll::SCATTER, outputs, root);
  std::vector<at::Tensor> empty;
  std::vector<at::Tensor>& inl = (rank_ == root) ? inputs[0] : empty;
  if (out.is_cuda()) return gpu_scatter(out, inl, root, eff_timeout(opts.timeout));
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<at::Tensor> ci;
  std::vector<const void*> ptrs(size_, nullptr);
  for (auto& i : inl) ci.push_back(i.contiguous());
  for (size_t i = 0; i < ci.size(); ++i) ptrs[i] = ci[i].data_ptr();
  Contig co(out);
  if (size_ > 1) shm().scatter(ptrs, co.ptr(), out.nbytes(), root, eff_timeout(opts.timeout));
  else std::memcpy(co.ptr(), ptrs[0], out.nbytes());
  co.write_back();
  record(Coll::SCATTER, "shm", out.nbytes(), t0);
  return cpu_done(Coll::SCATTER, outputs);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::reduce_scatter(std::vector<at::Tensor>& outputs,
                                                                  std::vector<std::vector<at::Tensor>>& inputs,
                                                                  const c10d::ReduceScatterOptions& opts) {
  op_async_ = opts.asyncOp;
  check_single(outputs, "reduce_scatter");
  TORCH_CHECK(inputs.size() == 1, "ProcessGroupMI355X::reduce_scatter: expects one input list");
  at::Tensor& out = outputs[0];
  check_list(inputs[0], out, size_, "reduce_scatter", "input");
  before_op(Coll::REDUCE_SCATTER, outputs, -1);
  if (out.is_cuda()) return gpu_reduce_scatter(out, inputs[0], opts.reduceOp.op_, eff_timeout(opts.timeout));
  check_cpu_dtype(out.scalar_type(), opts.reduceOp.op_, "reduce_scatter");
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<at::Tensor> ci;
  std::vector<const void*> ptrs;
  for (auto& i : inputs[0]) ci.push_back(i.contiguous());
  for (auto& c : ci) ptrs.push_back(c.data_ptr());
  Contig co(out);
  if (size_ > 1)
    shm().reduce_scatter(ptrs, co.ptr(), out.numel(), out.scalar_type(), opts.reduceOp.op_,
                         eff_timeout(opts.timeout));
  else
    std::memcpy(co.ptr(), ptrs[0], out.nbytes());
  co.write_back();
  record(Coll::REDUCE_SCATTER, "shm", out.nbytes(), t0);
  return cpu_done(Coll::REDUCE_SCATTER, outputs);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::_reduce_scatter_base(at::Tensor& output, at::Tensor& input,
                                                                        const c10d::ReduceScatterOptions& opts) {
  TORCH_CHECK(input.numel() == output.numel() * size_, "ProcessGroupMI355X::_reduce_scatter_base: input has ",
              input.numel(), " elements, expected ", output.numel() * size_);
  TORCH_CHECK(input.is_contiguous(), "ProcessGroupMI355X::_reduce_scatter_base: input must be contiguous");
  std::vector<std::vector<at::Tensor>> ins(1);  // (one split, as in _allgather_base)
  ins[0] = output.numel() > 0 ? input.view({-1}).split(output.numel())
                              : std::vector<at::Tensor>((size_t)size_, input.view({-1}));
  std::vector<at::Tensor> outs{output};
  return reduce_scatter(outs, ins, opts);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::alltoall_base(at::Tensor& output, at::Tensor& input,
                                                                 std::vector<int64_t>& output_splits,
                                                                 std::vector<int64_t>& input_splits,
                                                                 const c10d::AllToAllOptions& opts) {
  op_async_ = opts.asyncOp;
  TORCH_CHECK(input.is_contiguous() && output.is_contiguous(), "ProcessGroupMI355X::alltoall_base: contiguous tensors only");
  TORCH_CHECK(input.scalar_type() == output.scalar_type(), "ProcessGroupMI355X::alltoall_base: dtype mismatch");
  const bool equal = output_splits.empty() && input_splits.empty();
  auto split = [&](const at::Tensor& t, const std::vector<int64_t>& sp) {
    std::vector<at::Tensor> v;
    const int64_t rows = t.dim() == 0 ? 1 : t.size(0);
    const int64_t row_el = rows == 0 ? 0 : t.numel() / rows;
    auto flat = t.view({-1});
    int64_t off = 0;
    for (int r = 0; r < size_; ++r) {
      const int64_t n = sp.empty() ? rows / size_ : sp[r];
      v.push_back(flat.narrow(0, off * row_el, n * row_el));
      off += n;
    }
    return v;
  };
  if (equal) {
    const int64_t rows = input.dim() == 0 ? 1 : input.size(0);
    TORCH_CHECK(rows % size_ == 0, "ProcessGroupMI355X::alltoall_base: dim 0 (", rows,
                ") must be divisible by the group size (", size_, ")");
    TORCH_CHECK(input.numel() == output.numel(), "ProcessGroupMI355X::alltoall_base: numel mismatch");
  } else {
    TORCH_CHECK((int)output_splits.size() == size_ && (int)input_splits.size() == size_,
                "ProcessGroupMI355X::alltoall_base: split lists must have one entry per rank");
  }
  auto outs = split(output, output_splits);
  auto ins = split(input, input_splits);
  std::vector<at::Tensor> one{input};
  before_op(Coll::ALLTOALL, one, -1);
  if (input.is_cuda()) return gpu_alltoall(outs, ins, equal, eff_timeout(opts.timeout));
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<const void*> ip;
  std::vector<void*> op;
  std::vector<size_t> sb, rb;
  for (auto& t : ins) { ip.push_back(t.data_ptr()); sb.push_back(t.nbytes()); }
  for (auto& t : outs) { op.push_back(t.data_ptr()); rb.push_back(t.nbytes()); }
  if (size_ > 1) shm().alltoall(ip, sb, op, rb, eff_timeout(opts.timeout));
  else std::memcpy(op[0], ip[0], sb[0]);
  record(Coll::ALLTOALL, "shm", input.nbytes(), t0);
  return cpu_done(Coll::ALLTOALL, {output});
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::alltoall(std::vector<at::Tensor>& outputs,
                                                            std::vector<at::Tensor>& inputs,
                                                            const c10d::AllToAllOptions& opts) {
  op_async_ = opts.asyncOp;
  TORCH_CHECK((int)outputs.size() == size_ && (int)inputs.size() == size_,
              "ProcessGroupMI355X::alltoall: expects one input and one output tensor per rank");
  before_op(Coll::ALLTOALL, inputs, -1);
  if (inputs[0].is_cuda()) {
    // equal chunks (every input and output of every rank the same byte count) take the
    // same engines as all_to_all_single with empty splits: IPC / LL / autotuned. Chunk
    // sizes are rank-local facts here, so the ranks agree first (one host-transport
    // round of two doubles): a rank with uneven chunks sends everyone to grouped p2p.
    bool equal = true;
    const size_t b0 = inputs[0].nbytes();
    for (int r = 0; r < size_; ++r)
      equal = equal && inputs[r].nbytes() == b0 && outputs[r].nbytes() == b0 &&
              inputs[r].scalar_type() == inputs[0].scalar_type() &&
              outputs[r].scalar_type() == inputs[0].scalar_type();
    if (size_ > 1 && same_host_ && cfg_.a2a_list_agree) {
      const double x = equal ? (double)b0 : -1.0;
      double v[2] = {x, -x};  // MIN -> {min over ranks, -max over ranks}
      shm().allreduce(v, 2, at::kDouble, c10d::ReduceOp::MIN, eff_timeout(opts.timeout));
      equal = v[0] >= 0.0 && v[0] == -v[1];
    } else if (size_ > 1) {
      equal = false;
    }
    return gpu_alltoall(outputs, inputs, equal, eff_timeout(opts.timeout));
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<at::Tensor> ci;
  std::vector<Contig> co;
  std::vector<const void*> ip;
  std::vector<void*> op;
  std::vector<size_t> sb, rb;
  size_t total = 0;
  for (auto& t : inputs) { ci.push_back(t.contiguous()); }
  for (auto& t : ci) { ip.push_back(t.data_ptr()); sb.push_back(t.nbytes()); total += t.nbytes(); }
  for (auto& t : outputs) co.emplace_back(t);
  for (size_t i = 0; i < co.size(); ++i) { op.push_back(co[i].ptr()); rb.push_back(outputs[i].nbytes()); }
  if (size_ > 1) shm().alltoall(ip, sb, op, rb, eff_timeout(opts.timeout));
  else std::memcpy(op[0], ip[0], sb[0]);
  for (auto& c : co) c.write_back();
  record(Coll::ALLTOALL, "shm", total, t0);
  return cpu_done(Coll::ALLTOALL, outputs);
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::send(std::vector<at::Tensor>& tensors, int dst, int tag) {
  op_async_ = true;  // p2p pairs must be able to overlap: comm stream
  check_single(tensors, "send");
  TORCH_CHECK(dst >= 0 && dst < size_ && dst != rank_, "ProcessGroupMI355X::send: invalid destination rank ", dst);
  before_op(Coll::SEND, tensors, dst);
  at::Tensor t = tensors[0];
  if (t.is_cuda()) return gpu_p2p(t, dst, true, timeout_);
  at::Tensor c = t.contiguous();
  auto work = c10::make_intrusive<WorkMI355X>(rank_, c10d::OpType::SEND, op_seq_.load(), std::vector<at::Tensor>{t});
  auto to = timeout_;
  const int pi = dst < rank_ ? 0 : 1;  // the peer's rank inside the pair channel
  // the pair channel is built on the worker thread: a ring of first isends cannot deadlock
  p2p_submit(true, Job{[this, c, dst, pi, to] { shm_pair(dst).send(c.data_ptr(), c.nbytes(), pi, to); }, work});
  if (coalescing_) coalesced_cpu_.push_back(work);
  return work;
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::recv(std::vector<at::Tensor>& tensors, int src, int tag) {
  op_async_ = true;  // p2p pairs must be able to overlap: comm stream
  check_single(tensors, "recv");
  TORCH_CHECK(src >= 0 && src < size_ && src != rank_, "ProcessGroupMI355X::recv: invalid source rank ", src);
  before_op(Coll::RECV, tensors, src);
  at::Tensor t = tensors[0];
  if (t.is_cuda()) return gpu_p2p(t, src, false, timeout_);
  auto work = c10::make_intrusive<WorkMI355X>(rank_, c10d::OpType::RECV, op_seq_.load(), std::vector<at::Tensor>{t});
  auto to = timeout_;
  const int pi = src < rank_ ? 0 : 1;
  p2p_submit(false, Job{[this, t, src, pi, to]() mutable {
                          at::Tensor c = t.is_contiguous() ? t : at::empty_like(t, at::MemoryFormat::Contiguous);
                          shm_pair(src).recv(c.data_ptr(), c.nbytes(), pi, to);
                          if (!c.is_same(t)) t.copy_(c);
                        },
                        work});
  if (coalescing_) coalesced_cpu_.push_back(work);
  return work;
}

c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::barrier(const c10d::BarrierOptions& opts) {
  before_op(Coll::BARRIER, {}, -1);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<DeviceState*> dss;
  {
    std::lock_guard<std::mutex> lk(init_mu_);
    for (auto& kv : devs_) dss.push_back(kv.second.get());
  }
  for (DeviceState* ds : dss) {
    const hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)ds->device).stream();
    launcher_quiesce(*ds);  // every zero-copy exchange published (gated kernels can finish)
    PDCC_HIP(hipStreamSynchronize(ds->stream.stream()));
    // synchronous collectives were enqueued on the caller's stream
    PDCC_HIP(hipStreamSynchronize(cur));
  }
  if (size_ > 1) {
    if (same_host_) shm().barrier(eff_timeout(opts.timeout));
    else store_barrier(store_, "pdcc/barrier/" + std::to_string(op_seq_.load()), rank_, size_);
  }
  // every rank's IPC kernels have finished: release what the launcher's thread only queued
  // (evicted mappings, outgrown staging)
  for (DeviceState* ds : dss)
    if (ds->ipc && ds->launcher) ds->ipc->maintain();
  record(Coll::BARRIER, same_host_ ? "shm" : "store", 0, t0);
  return cpu_done(Coll::BARRIER, {});
}

c10::intrusive_ptr<c10d::Backend> create_backend(const c10::intrusive_ptr<c10d::Store>& store, int rank, int size,
                                                 std::chrono::milliseconds timeout, std::vector<int64_t> global_ranks,
                                                 std::string group_name) {
  return c10::make_intrusive<ProcessGroupMI355X>(store, rank, size, timeout, std::move(global_ranks),
                                                 std::move(group_name));
}

}  // namespace pdcc
