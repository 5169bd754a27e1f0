// Helpers shared by the GPU translation units of ProcessGroupMI355X:
//   gpu_setup.cpp   device state, topology, communicators, IPC self-test
//   autotune.cpp    the online engine race and its persisted decisions
//   gpu_ops.cpp     the engines and the collectives built on them
#pragma once
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>
#include <thread>

#include "../device/comm_util.h"
#include "process_group.h"

namespace pdcc {
namespace gpu {


using RedOpType = c10d::ReduceOp::RedOpType;

inline bool kern_dtype(at::ScalarType t, kern::DType& d) {
  switch (t) {
    case at::kFloat: d = kern::DType::F32; return true;
    case at::kHalf: d = kern::DType::F16; return true;
    case at::kBFloat16: d = kern::DType::BF16; return true;
    case at::kDouble: d = kern::DType::F64; return true;
    case at::kChar: d = kern::DType::I8; return true;
    case at::kByte: d = kern::DType::U8; return true;
    case at::kInt: d = kern::DType::I32; return true;
    case at::kLong: d = kern::DType::I64; return true;
    case at::kBool: d = kern::DType::BOOL; return true;
    default: return false;
  }
}

inline bool kern_op(RedOpType op, kern::RedOp& o) {
  switch (op) {
    case RedOpType::SUM: o = kern::RedOp::SUM; return true;
    case RedOpType::AVG: o = kern::RedOp::AVG; return true;
    case RedOpType::PRODUCT: o = kern::RedOp::PROD; return true;
    case RedOpType::MIN: o = kern::RedOp::MIN; return true;
    case RedOpType::MAX: o = kern::RedOp::MAX; return true;
    case RedOpType::BAND: o = kern::RedOp::BAND; return true;
    case RedOpType::BOR: o = kern::RedOp::BOR; return true;
    case RedOpType::BXOR: o = kern::RedOp::BXOR; return true;
    default: return false;
  }
}

inline bool nccl_dtype(at::ScalarType t, ncclDataType_t& d) {
  switch (t) {
    case at::kFloat: d = ncclFloat32; return true;
    case at::kHalf: d = ncclFloat16; return true;
    case at::kBFloat16: d = ncclBfloat16; return true;
    case at::kDouble: d = ncclFloat64; return true;
    case at::kChar: d = ncclInt8; return true;
    case at::kByte: d = ncclUint8; return true;
    case at::kBool: d = ncclUint8; return true;
    case at::kInt: d = ncclInt32; return true;
    case at::kLong: d = ncclInt64; return true;
    default: return false;
  }
}

inline bool nccl_op(RedOpType op, at::ScalarType t, ncclRedOp_t& o) {
  const bool b = t == at::kBool;  // bool: SUM = OR = max, PRODUCT = AND = min
  switch (op) {
    case RedOpType::SUM: o = b ? ncclMax : ncclSum; return true;
    case RedOpType::PRODUCT: o = b ? ncclMin : ncclProd; return true;
    case RedOpType::MIN: o = ncclMin; return true;
    case RedOpType::MAX: o = ncclMax; return true;
    case RedOpType::AVG: o = ncclAvg; return !b;
    default: return false;  // BAND/BOR/BXOR: no RCCL op (IPC kernels or the host path)
  }
}

inline const char* op_name(int op) {
  switch (op) {
    case RedOpType::SUM: return "SUM";
    case RedOpType::AVG: return "AVG";
    case RedOpType::PRODUCT: return "PRODUCT";
    case RedOpType::MIN: return "MIN";
    case RedOpType::MAX: return "MAX";
    case RedOpType::BAND: return "BAND";
    case RedOpType::BOR: return "BOR";
    case RedOpType::BXOR: return "BXOR";
    default: return "?";
  }
}

// tune-key "op" slot of the copy collectives: the output/input list layout
constexpr int kLayoutFlat = 100, kLayoutList = 101;

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// input used in place: contiguous + 16-B aligned, else a copy (on the current stream). `any_align`:
// a call every engine of which takes any alignment -- the LL kernels (byte-wise where a line is not
// 8-B aligned), RCCL, the host path -- so a view of one flat tensor at a small offset (a 4 B chunk of
// all_gather_into_tensor's output) is used in place instead of costing a copy kernel per chunk
inline at::Tensor prep_in(const at::Tensor& t, bool any_align = false) {
  if (t.is_contiguous() && (any_align || aligned16(t.data_ptr()))) return t;
  at::Tensor c = at::empty_like(t, at::MemoryFormat::Contiguous);
  c.copy_(t);
  return c;
}
// pure output: contiguous + aligned (or `any_align`, as above), else fresh storage (copied back afterwards)
inline at::Tensor prep_out(const at::Tensor& t, bool any_align = false) {
  if (t.is_contiguous() && (any_align || aligned16(t.data_ptr()))) return t;
  return at::empty_like(t, at::MemoryFormat::Contiguous);
}

// consecutive views of one allocation, in rank order?
inline bool is_flat(const std::vector<at::Tensor>& v, size_t bytes) {
  if (v.empty()) return false;
  const char* base = static_cast<const char*>(v[0].data_ptr());
  for (size_t i = 0; i < v.size(); ++i) {
    if (!v[i].is_contiguous()) return false;
    if (static_cast<const char*>(v[i].data_ptr()) != base + i * bytes) return false;
  }
  return true;
}

// K2 (one launch) when every descriptor is 16-B aligned, hipMemcpyAsync otherwise
inline void multi_copy_or_memcpy(const std::vector<kern::CopyDesc>& d, hipStream_t s) {
  bool ok = true;
  for (const auto& x : d) ok = ok && aligned16(x.src) && aligned16(x.dst);
  if (ok) {
    PDCC_HIP(kern::multi_copy(d.data(), (int)d.size(), s));
  } else {
    for (const auto& x : d)
      if (x.bytes) PDCC_HIP(hipMemcpyAsync(x.dst, x.src, x.bytes, hipMemcpyDeviceToDevice, s));
  }
}

inline int size_bucket(size_t bytes) { return bytes ? 63 - __builtin_clzll((unsigned long long)bytes) : 0; }
// tune-key size slot of an async_op call whose IPC launches run the capped grid: bucket + this
constexpr int kAsyncBucket = 64;

// is `s` being captured into a graph (torch.cuda.graph / parallel.graphs)?
inline bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}
inline bool capturing_on(int device) {
  return capturing(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device).stream());
}
inline hipStream_t current_stream(int device) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device).stream();
}

// host path only competes for small messages, where its latency can beat a GPU protocol
constexpr size_t kHostTuneMax = 4u << 20;

// autotuner numerics check: candidate result vs the reference engine's result on the same data
inline bool results_match(const at::Tensor& ref, const at::Tensor& got, RedOpType op, int world) {
  if (!ref.is_floating_point() || op == RedOpType::MAX || op == RedOpType::MIN) return at::equal(ref, got);
  const at::Tensor r = ref.to(at::kFloat), g = got.to(at::kFloat);
  const bool wide = ref.scalar_type() == at::kFloat || ref.scalar_type() == at::kDouble;
  // engines differ only in summation order (and, for 16-bit types, in where they round):
  // allow a few ulps per rank relative to the largest magnitude; stale or misplaced data is far off
  const double amax = r.abs().max().item<double>();
  const double tol = (wide ? 4e-7 : 8e-3) * world;
  if (!std::isfinite(amax)) return at::equal(ref, got);
  return at::allclose(g, r, tol, tol * amax + 1e-30);
}

inline bool lists_equal(const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!at::equal(a[i], b[i])) return false;
  return true;
}

// Elements of a tuning sample: at most `budget` bytes (per `units` tensors), a whole
// number of 16-B vectors unless the full tensor fits.
inline int64_t sample_numel(int64_t numel, size_t esize, size_t budget, int units = 1) {
  const int64_t cap = (int64_t)(budget / std::max<size_t>(1, esize) / std::max(1, units));
  if (numel <= cap) return numel;
  const int64_t vec = std::max<int64_t>(1, 16 / (int64_t)esize);
  return std::max<int64_t>(vec, cap / vec * vec);
}

// Read-only inputs for a tuning run: the first n elements of each tensor; a flat list
// stays flat (copied into one allocation) so the timed path is the one the call takes.
inline std::vector<at::Tensor> sample_inputs(const std::vector<at::Tensor>& v, int64_t n, bool flat) {
  if (v.empty() || n >= v[0].numel()) return v;
  std::vector<at::Tensor> out;
  if (flat) {
    at::Tensor buf = at::empty({(int64_t)v.size() * n}, v[0].options());
    for (size_t i = 0; i < v.size(); ++i) {
      out.push_back(buf.narrow(0, (int64_t)i * n, n));
      out.back().copy_(v[i].reshape({-1}).narrow(0, 0, n));
    }
  } else {
    for (const auto& t : v) out.push_back(t.reshape({-1}).narrow(0, 0, n));
  }
  return out;
}
// Scratch outputs for a tuning run, laid out like the caller's (flat or separate tensors).
inline std::vector<at::Tensor> scratch_outputs(const at::TensorOptions& opt, size_t count, int64_t n, bool flat) {
  std::vector<at::Tensor> out;
  if (flat) {
    at::Tensor buf = at::empty({(int64_t)count * n}, opt);
    for (size_t i = 0; i < count; ++i) out.push_back(buf.narrow(0, (int64_t)i * n, n));
  } else {
    for (size_t i = 0; i < count; ++i) out.push_back(at::empty({n}, opt));
  }
  return out;
}

// Which groups may split from / share each other's RCCL communicator: same member set
inline std::string members_key(const std::vector<int64_t>& global_ranks, int size) {
  std::vector<int64_t> r = global_ranks;
  if (r.empty())
    for (int i = 0; i < size; ++i) r.push_back(i);
  std::sort(r.begin(), r.end());
  std::ostringstream o;
  for (size_t i = 0; i < r.size(); ++i) o << (i ? "," : "") << r[i];
  return o.str();
}

}  // namespace gpu
}  // namespace pdcc
