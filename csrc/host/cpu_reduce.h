// CPU element-wise reductions for the shared-memory host transport (the path
// the reference's CPU tensors take: main.py:12,22 build torch.ones(1) on CPU).
// bf16/f16 accumulate across all sources in f32 and round once, matching the
// device kernels so CPU and GPU results agree.
#pragma once
#include <c10/core/ScalarType.h>
#include <c10/util/BFloat16.h>
#include <c10/util/Half.h>
#include <torch/csrc/distributed/c10d/Types.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace pdcc {
namespace host {

using RedOpType = c10d::ReduceOp::RedOpType;

template <class T>
inline T op_apply(RedOpType op, T a, T b) {
  switch (op) {
    case RedOpType::SUM:
    case RedOpType::AVG:
      if constexpr (std::is_same_v<T, bool>) return a || b;
      else return a + b;
    case RedOpType::PRODUCT:
      if constexpr (std::is_same_v<T, bool>) return a && b;
      else return a * b;
    case RedOpType::MAX: return (a > b || a != a) ? a : b;
    case RedOpType::MIN: return (a < b || a != a) ? a : b;
    case RedOpType::BAND:
      if constexpr (std::is_integral_v<T>) return a & b;
      break;
    case RedOpType::BOR:
      if constexpr (std::is_integral_v<T>) return a | b;
      break;
    case RedOpType::BXOR:
      if constexpr (std::is_integral_v<T>) return a ^ b;
      break;
    default:
      break;
  }
  throw std::runtime_error("pdcc: unsupported reduce op for this dtype");
}

// dst[i] = op(srcs[0][i], ..., srcs[n-1][i]); dst may alias srcs[0].
template <class S, class C>
void reduce_typed(void* dst_v, const void* const* srcs_v, int n, size_t count, RedOpType op, int avg_div) {
  S* dst = static_cast<S*>(dst_v);
  constexpr size_t B = 1024;
  C acc[B];
  for (size_t base = 0; base < count; base += B) {
    const size_t m = std::min(B, count - base);
    const S* s0 = static_cast<const S*>(srcs_v[0]) + base;
    for (size_t i = 0; i < m; ++i) acc[i] = static_cast<C>(s0[i]);
    for (int k = 1; k < n; ++k) {
      const S* sk = static_cast<const S*>(srcs_v[k]) + base;
      switch (op) {  // hoisted per block so the inner loops vectorize
        case RedOpType::SUM:
        case RedOpType::AVG:
          if constexpr (std::is_same_v<C, bool>) { for (size_t i = 0; i < m; ++i) acc[i] = acc[i] || (bool)sk[i]; }
          else { for (size_t i = 0; i < m; ++i) acc[i] += static_cast<C>(sk[i]); }
          break;
        case RedOpType::PRODUCT:
          if constexpr (std::is_same_v<C, bool>) { for (size_t i = 0; i < m; ++i) acc[i] = acc[i] && (bool)sk[i]; }
          else { for (size_t i = 0; i < m; ++i) acc[i] *= static_cast<C>(sk[i]); }
          break;
        default:
          for (size_t i = 0; i < m; ++i) acc[i] = op_apply<C>(op, acc[i], static_cast<C>(sk[i]));
      }
    }
    if (op == RedOpType::AVG) {
      if constexpr (std::is_same_v<C, bool>) throw std::runtime_error("pdcc: AVG is not defined for bool");
      else for (size_t i = 0; i < m; ++i) acc[i] = acc[i] / static_cast<C>(avg_div);
    }
    S* d = dst + base;
    for (size_t i = 0; i < m; ++i) d[i] = static_cast<S>(acc[i]);
  }
}

inline void reduce_cpu(at::ScalarType t, void* dst, const void* const* srcs, int n, size_t count, RedOpType op,
                       int avg_div) {
  switch (t) {
    case at::kFloat: return reduce_typed<float, float>(dst, srcs, n, count, op, avg_div);
    case at::kDouble: return reduce_typed<double, double>(dst, srcs, n, count, op, avg_div);
    case at::kHalf: return reduce_typed<c10::Half, float>(dst, srcs, n, count, op, avg_div);
    case at::kBFloat16: return reduce_typed<c10::BFloat16, float>(dst, srcs, n, count, op, avg_div);
    case at::kChar: return reduce_typed<int8_t, int8_t>(dst, srcs, n, count, op, avg_div);
    case at::kByte: return reduce_typed<uint8_t, uint8_t>(dst, srcs, n, count, op, avg_div);
    case at::kShort: return reduce_typed<int16_t, int16_t>(dst, srcs, n, count, op, avg_div);
    case at::kInt: return reduce_typed<int32_t, int32_t>(dst, srcs, n, count, op, avg_div);
    case at::kLong: return reduce_typed<int64_t, int64_t>(dst, srcs, n, count, op, avg_div);
    case at::kBool: return reduce_typed<bool, bool>(dst, srcs, n, count, op, avg_div);
    default:
      throw std::runtime_error(std::string("pdcc: unsupported dtype for CPU reduction: ") + c10::toString(t));
  }
}

}  // namespace host
}  // namespace pdcc
