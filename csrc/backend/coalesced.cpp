// Coalesced collectives of ProcessGroupMI355X: ONE collective per call.
//
// torch's _coalescing_manager fast path (torch/distributed/distributed_c10d.py:2690-2715)
// hands a backend the whole bucket at once -- allreduce_coalesced (also
// dist.all_reduce_coalesced), allgather_into_tensor_coalesced and
// reduce_scatter_tensor_coalesced -- which is how DDP-style gradient averaging
// (the reference's motivation, README.md:5; all_reduce at main.py:23) and ZeRO
// parameter gathers issue many small tensors. Instead of one collective per
// member (one launch, one autotune key and one zero-copy exchange each), the
// members are packed into one flat buffer by K2 (multi_copy: one launch per 64
// pieces, 16-B aligned slots), the collective runs ONCE on it through the normal
// engine choice (LL / IPC / RCCL / autotuned), and K2 unpacks the result on the
// collective's own stream (Coalesced::run inside the enqueue job), so async
// works and graph capture see a single operation.
//
// CPU tensors take the same packing through the host transport.
#include "gpu_util.h"

namespace pdcc {

using namespace gpu;

namespace {

// byte offsets of pieces of `bytes` packed into one buffer, each slot 16-B aligned (the K2
// vector path); returns the buffer size (a multiple of 16) and whether any slot is padded
size_t pack_layout(const std::vector<size_t>& bytes, std::vector<size_t>& off, bool& padded) {
  size_t total = 0;
  padded = false;
  off.clear();
  for (size_t b : bytes) {
    off.push_back(total);
    const size_t slot = (b + 15) / 16 * 16;
    padded = padded || slot != b;
    total += slot;
  }
  return total;
}

char* byte_ptr(const at::Tensor& t, size_t off = 0) { return static_cast<char*>(t.data_ptr()) + off; }

// copy `src` (any layout) into `dst_bytes` bytes of the flat buffer at `off` (bytes): K2
// descriptor when `src` is contiguous on the GPU, a torch copy into a view otherwise
void pack_piece(const at::Tensor& src, const at::Tensor& flat, size_t off, std::vector<kern::CopyDesc>& d) {
  if (src.numel() == 0) return;
  if (src.is_cuda() && src.is_contiguous()) {
    d.push_back({src.data_ptr(), byte_ptr(flat, off), src.nbytes()});
    return;
  }
  at::Tensor view = flat.narrow(0, (int64_t)off, (int64_t)src.nbytes()).view(src.scalar_type()).view(src.sizes());
  view.copy_(src);
}

// the way back: K2 descriptor for a contiguous GPU member, else a (member, flat view) pair
void unpack_piece(const at::Tensor& dst, const at::Tensor& flat, size_t off, Coalesced& co) {
  if (dst.numel() == 0) return;
  if (dst.is_cuda() && dst.is_contiguous()) {
    co.unpack.push_back({byte_ptr(flat, off), dst.data_ptr(), dst.nbytes()});
    return;
  }
  co.copies.emplace_back(dst,
                         flat.narrow(0, (int64_t)off, (int64_t)dst.nbytes()).view(dst.scalar_type()).view(dst.sizes()));
}

// torch's _coalescing_manager calls the coalesced entry points between start- and endCoalescing;
// the one collective they run is issued at once, so it may be autotuned like any other call
struct IssueNow {
  bool& flag;
  const bool saved;
  explicit IssueNow(bool& f) : flag(f), saved(f) { flag = false; }
  ~IssueNow() { flag = saved; }
};

void run_copies(const std::vector<kern::CopyDesc>& d, hipStream_t s) {
  if (!d.empty()) PDCC_HIP(kern::multi_copy(d.data(), (int)d.size(), s));
}

// flat byte buffer of `bytes` on `like`'s device (zeroed when slots are padded and the
// collective reduces: stale padding must not feed NaN/Inf into an autotuner comparison)
at::Tensor flat_bytes(const at::Tensor& like, size_t bytes, bool zero) {
  const auto o = like.options().dtype(at::kByte);
  return zero ? at::zeros({(int64_t)bytes}, o) : at::empty({(int64_t)bytes}, o);
}

void check_members(const std::vector<at::Tensor>& ts, const char* fn, bool same_dtype) {
  TORCH_CHECK(!ts.empty(), "ProcessGroupMI355X::", fn, ": empty tensor list");
  for (size_t i = 1; i < ts.size(); ++i) {
    TORCH_CHECK(ts[i].device() == ts[0].device(), "ProcessGroupMI355X::", fn, ": tensor ", i, " is on ",
                ts[i].device(), ", expected ", ts[0].device());
    TORCH_CHECK(!same_dtype || ts[i].scalar_type() == ts[0].scalar_type(), "ProcessGroupMI355X::", fn, ": tensor ",
                i, " has dtype ", ts[i].scalar_type(), ", expected ", ts[0].scalar_type(),
                " (a reduction is coalesced over one dtype)");
  }
}

}  // namespace

void Coalesced::run(hipStream_t s) const {
  run_copies(unpack, s);
  for (const auto& c : copies) const_cast<at::Tensor&>(c.first).copy_(c.second);
}

// ----------------------------------------------------------------- all-reduce
c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::allreduce_coalesced(std::vector<at::Tensor>& tensors,
                                                                       const c10d::AllreduceCoalescedOptions& opts) {
  check_members(tensors, "allreduce_coalesced", true);
  if (tensors.size() == 1) {
    c10d::AllreduceOptions o;
    o.reduceOp = opts.reduceOp;
    o.timeout = opts.timeout;
    o.asyncOp = opts.asyncOp;
    return allreduce(tensors, o);
  }
  const auto t0 = std::chrono::steady_clock::now();
  op_async_ = opts.asyncOp;
  std::vector<size_t> bytes, off;
  for (const auto& t : tensors) bytes.push_back(t.nbytes());
  bool padded = false;
  const size_t total = pack_layout(bytes, off, padded);
  const auto dt = tensors[0].scalar_type();
  if (tensors[0].is_cuda() && ((size_ == 1 && cfg_.world1_local) || total == 0)) {
    before_op(Coll::ALLREDUCE, tensors, -1);  // a no-op, like a single all_reduce at W = 1
    record(Coll::ALLREDUCE, "local", total, t0);
    return cpu_done(Coll::ALLREDUCE, tensors);
  }
  at::Tensor flat = flat_bytes(tensors[0], total, padded);
  std::vector<kern::CopyDesc> pk;
  {
    c10::OptionalDeviceGuard g(tensors[0].device());
    for (size_t i = 0; i < tensors.size(); ++i) pack_piece(tensors[i], flat, off[i], pk);
    if (tensors[0].is_cuda()) run_copies(pk, current_stream(tensors[0].device().index()));
  }
  at::Tensor typed = flat.view(dt);  // total is a multiple of 16 B: whole elements
  if (tensors[0].is_cuda()) {
    auto co = std::make_shared<Coalesced>();
    co->members = tensors;
    for (size_t i = 0; i < tensors.size(); ++i) unpack_piece(tensors[i], flat, off[i], *co);
    std::vector<at::Tensor> one{typed};
    before_op(Coll::ALLREDUCE, one, -1);
    IssueNow now(coalescing_);
    auto w = gpu_allreduce(typed, opts.reduceOp.op_, -1, false, eff_timeout(opts.timeout), co);
    record_setup("coalesced/allreduce x" + std::to_string(tensors.size()), t0);
    return w;
  }
  std::vector<at::Tensor> one{typed};
  c10d::AllreduceOptions o;
  o.reduceOp = opts.reduceOp;
  o.timeout = opts.timeout;
  allreduce(one, o);  // host transport: synchronous
  Coalesced co;
  for (size_t i = 0; i < tensors.size(); ++i) unpack_piece(tensors[i], flat, off[i], co);
  co.run(nullptr);
  return cpu_done(Coll::ALLREDUCE, tensors);
}

// ----------------------------------------------------------------- all-gather into tensors
c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::allgather_into_tensor_coalesced(std::vector<at::Tensor>& outputs,
                                                                                   std::vector<at::Tensor>& inputs,
                                                                                   const c10d::AllgatherOptions& opts) {
  TORCH_CHECK(outputs.size() == inputs.size(), "allgather_into_tensor_coalesced: list size mismatch");
  check_members(inputs, "allgather_into_tensor_coalesced", false);
  for (size_t i = 0; i < inputs.size(); ++i) {
    TORCH_CHECK(outputs[i].numel() == inputs[i].numel() * size_ && outputs[i].scalar_type() == inputs[i].scalar_type(),
                "ProcessGroupMI355X::allgather_into_tensor_coalesced: output ", i, " must hold ", size_,
                " x input ", i, " (", inputs[i].numel(), " x ", inputs[i].scalar_type(), ")");
    TORCH_CHECK(outputs[i].device() == inputs[0].device() && outputs[i].is_contiguous(),
                "ProcessGroupMI355X::allgather_into_tensor_coalesced: output ", i,
                " must be contiguous and on the inputs' device");
  }
  if (inputs.size() == 1) return _allgather_base(outputs[0], inputs[0], opts);
  const auto t0 = std::chrono::steady_clock::now();
  op_async_ = opts.asyncOp;
  std::vector<size_t> bytes, off;
  for (const auto& t : inputs) bytes.push_back(t.nbytes());
  bool padded = false;
  const size_t S = pack_layout(bytes, off, padded);  // one rank's block of the gathered buffer
  const bool gpu = inputs[0].is_cuda();
  if (size_ == 1 && (!gpu || cfg_.world1_local)) {
    before_op(Coll::ALLGATHER, inputs, -1);
    for (size_t i = 0; i < inputs.size(); ++i) outputs[i].view(-1).copy_(inputs[i].reshape(-1));
    record(Coll::ALLGATHER, "local", S, t0);
    return cpu_done(Coll::ALLGATHER, outputs);
  }
  at::Tensor fin = flat_bytes(inputs[0], S, false), fout = flat_bytes(inputs[0], S * size_, false);
  std::vector<kern::CopyDesc> pk;
  {
    c10::OptionalDeviceGuard g(inputs[0].device());
    for (size_t i = 0; i < inputs.size(); ++i) pack_piece(inputs[i], fin, off[i], pk);
    if (gpu) run_copies(pk, current_stream(inputs[0].device().index()));
  }
  // output i of rank r's block: bytes[i] at r * S + off[i] -> outputs[i][r * bytes[i]] (outputs are
  // contiguous: raw pointers, no per-piece tensor views -- 2 x 64 views cost more host time than the
  // whole collective)
  auto co = std::make_shared<Coalesced>();
  co->members = outputs;
  for (size_t i = 0; i < outputs.size(); ++i) {
    if (bytes[i] == 0) continue;
    for (int r = 0; r < size_; ++r) {
      if (gpu) {
        co->unpack.push_back({byte_ptr(fout, (size_t)r * S + off[i]), byte_ptr(outputs[i], (size_t)r * bytes[i]),
                              bytes[i]});
      } else {
        at::Tensor dst = outputs[i].view(-1).narrow(0, (int64_t)r * inputs[i].numel(), inputs[i].numel());
        unpack_piece(dst, fout, (size_t)r * S + off[i], *co);
      }
    }
  }
  std::vector<at::Tensor> outs;
  for (int r = 0; r < size_; ++r) outs.push_back(fout.narrow(0, (int64_t)r * S, (int64_t)S));
  std::vector<at::Tensor> one{fin};
  before_op(Coll::ALLGATHER, one, -1);
  if (gpu) {
    IssueNow now(coalescing_);
    auto w = gpu_allgather(outs, fin, -1, false, eff_timeout(opts.timeout), co);
    record_setup("coalesced/allgather x" + std::to_string(inputs.size()), t0);
    return w;
  }
  std::vector<void*> ptrs;
  for (auto& o : outs) ptrs.push_back(o.data_ptr());
  shm().allgather(fin.data_ptr(), ptrs, S, eff_timeout(opts.timeout));
  co->run(nullptr);
  record(Coll::ALLGATHER, "shm", S, t0);
  return cpu_done(Coll::ALLGATHER, outputs);
}

// ----------------------------------------------------------------- reduce-scatter of tensors
c10::intrusive_ptr<c10d::Work> ProcessGroupMI355X::reduce_scatter_tensor_coalesced(
    std::vector<at::Tensor>& outputs, std::vector<at::Tensor>& inputs, const c10d::ReduceScatterOptions& opts) {
  TORCH_CHECK(outputs.size() == inputs.size(), "reduce_scatter_tensor_coalesced: list size mismatch");
  check_members(outputs, "reduce_scatter_tensor_coalesced", true);
  for (size_t i = 0; i < inputs.size(); ++i)
    TORCH_CHECK(inputs[i].numel() == outputs[i].numel() * size_ && inputs[i].scalar_type() == outputs[i].scalar_type() &&
                    inputs[i].device() == outputs[0].device(),
                "ProcessGroupMI355X::reduce_scatter_tensor_coalesced: input ", i, " must hold ", size_,
                " x output ", i, " (", outputs[i].numel(), " x ", outputs[i].scalar_type(), ") on the same device");
  TORCH_CHECK(opts.reduceOp.op_ != c10d::ReduceOp::PREMUL_SUM,
              "ProcessGroupMI355X::reduce_scatter_tensor_coalesced: PREMUL_SUM is not supported");
  if (inputs.size() == 1) return _reduce_scatter_base(outputs[0], inputs[0], opts);
  const auto t0 = std::chrono::steady_clock::now();
  op_async_ = opts.asyncOp;
  std::vector<size_t> bytes, off;
  for (const auto& t : outputs) bytes.push_back(t.nbytes());
  bool padded = false;
  const size_t S = pack_layout(bytes, off, padded);  // one rank's chunk of the flat input
  const bool gpu = outputs[0].is_cuda();
  const auto dt = outputs[0].scalar_type();
  if (size_ == 1 && (!gpu || cfg_.world1_local)) {
    before_op(Coll::REDUCE_SCATTER, outputs, -1);
    for (size_t i = 0; i < inputs.size(); ++i) outputs[i].view(-1).copy_(inputs[i].reshape(-1));
    record(Coll::REDUCE_SCATTER, "local", S, t0);
    return cpu_done(Coll::REDUCE_SCATTER, outputs);
  }
  // chunk r of the flat input = chunk r of every input, at r * S + off[i]
  at::Tensor fin = flat_bytes(outputs[0], S * size_, padded), fout = flat_bytes(outputs[0], S, false);
  std::vector<kern::CopyDesc> pk;
  std::vector<at::Tensor> hold;  // contiguous copies of strided inputs (stream-ordered reuse)
  {
    c10::OptionalDeviceGuard g(outputs[0].device());
    for (size_t i = 0; i < inputs.size(); ++i) {
      if (bytes[i] == 0) continue;
      if (gpu && inputs[i].is_contiguous()) {  // raw pointers (no per-piece tensor views)
        for (int r = 0; r < size_; ++r)
          pk.push_back({byte_ptr(inputs[i], (size_t)r * bytes[i]), byte_ptr(fin, (size_t)r * S + off[i]), bytes[i]});
        continue;
      }
      hold.push_back(inputs[i].reshape(-1));
      for (int r = 0; r < size_; ++r)
        pack_piece(hold.back().narrow(0, (int64_t)r * outputs[i].numel(), outputs[i].numel()), fin,
                   (size_t)r * S + off[i], pk);
    }
    if (gpu) run_copies(pk, current_stream(outputs[0].device().index()));
  }
  auto co = std::make_shared<Coalesced>();
  co->members = outputs;
  for (size_t i = 0; i < outputs.size(); ++i) unpack_piece(outputs[i], fout, off[i], *co);
  at::Tensor tin = fin.view(dt), tout = fout.view(dt);
  const int64_t per = (int64_t)(S / c10::elementSize(dt));
  std::vector<at::Tensor> ins;
  for (int r = 0; r < size_; ++r) ins.push_back(tin.narrow(0, r * per, per));
  std::vector<at::Tensor> one{tout};
  before_op(Coll::REDUCE_SCATTER, one, -1);
  if (gpu) {
    IssueNow now(coalescing_);
    auto w = gpu_reduce_scatter(tout, ins, opts.reduceOp.op_, eff_timeout(opts.timeout), co);
    record_setup("coalesced/reduce_scatter x" + std::to_string(inputs.size()), t0);
    return w;
  }
  std::vector<const void*> ptrs;
  for (auto& i : ins) ptrs.push_back(i.data_ptr());
  shm().reduce_scatter(ptrs, tout.data_ptr(), tout.numel(), dt, opts.reduceOp.op_, eff_timeout(opts.timeout));
  co->run(nullptr);
  record(Coll::REDUCE_SCATTER, "shm", S, t0);
  return cpu_done(Coll::REDUCE_SCATTER, outputs);
}

}  // namespace pdcc
