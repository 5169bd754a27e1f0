// Python bindings of the native library (module `_C` of the package).
//  * ProcessGroupMI355X  -- the c10d backend (subclass of torch's Backend type)
//  * kernel ops           -- K1 reduce_nway (LDS-DMA and register variants) and
//                            K2 multi_copy on torch tensors, on the current stream
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <pybind11/chrono.h>
#include <pybind11/stl.h>
#include <torch/csrc/utils/pybind.h>
#include <torch/python.h>

#include "backend/process_group.h"
#include "device/comm_util.h"
#include "kernels/kernel_api.h"

namespace py = pybind11;

namespace {

pdcc::kern::DType kdtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return pdcc::kern::DType::F32;
    case at::kHalf: return pdcc::kern::DType::F16;
    case at::kBFloat16: return pdcc::kern::DType::BF16;
    case at::kDouble: return pdcc::kern::DType::F64;
    case at::kChar: return pdcc::kern::DType::I8;
    case at::kByte: return pdcc::kern::DType::U8;
    case at::kInt: return pdcc::kern::DType::I32;
    case at::kLong: return pdcc::kern::DType::I64;
    case at::kBool: return pdcc::kern::DType::BOOL;
    default: TORCH_CHECK(false, "pdcc.ops: unsupported dtype ", t);
  }
}

pdcc::kern::RedOp kop(const std::string& s) {
  if (s == "sum") return pdcc::kern::RedOp::SUM;
  if (s == "avg") return pdcc::kern::RedOp::AVG;
  if (s == "prod" || s == "product") return pdcc::kern::RedOp::PROD;
  if (s == "min") return pdcc::kern::RedOp::MIN;
  if (s == "max") return pdcc::kern::RedOp::MAX;
  if (s == "band") return pdcc::kern::RedOp::BAND;
  if (s == "bor") return pdcc::kern::RedOp::BOR;
  if (s == "bxor") return pdcc::kern::RedOp::BXOR;
  TORCH_CHECK(false, "pdcc.ops: unknown reduce op '", s, "'");
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// mode: OR of kern::K1Mode bits (LDS-DMA engine, non-temporal stores, streaming kernel, non-temporal loads)
void reduce_nway(const std::vector<at::Tensor>& srcs, at::Tensor& out, const std::string& op, int mode,
                 int max_blocks) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= pdcc::kern::kMaxRanks, "reduce_nway: 1..8 sources");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && al16(out.data_ptr()), "reduce_nway: out must be a contiguous, "
              "16-byte aligned GPU tensor");
  std::vector<const void*> p;
  for (const auto& s : srcs) {
    TORCH_CHECK(s.device() == out.device() && s.scalar_type() == out.scalar_type() && s.numel() == out.numel() &&
                    s.is_contiguous() && al16(s.data_ptr()),
                "reduce_nway: sources must match out (device, dtype, numel) and be contiguous + 16-byte aligned");
    p.push_back(s.data_ptr());
  }
  const auto k = kop(op);
  const auto d = kdtype(out.scalar_type());
  TORCH_CHECK(pdcc::kern::supports(d, k), "reduce_nway: op '", op, "' unsupported for ", out.scalar_type());
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(out.device().index()).stream();
  hipError_t e = pdcc::kern::reduce_nway_mode(p.data(), (int)p.size(), out.data_ptr(), out.numel(), d, k,
                                               (int)srcs.size(), s, max_blocks, mode);
  TORCH_CHECK(e == hipSuccess, "reduce_nway launch failed: ", hipGetErrorString(e));
}

void multi_copy(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts, int max_blocks, int depth,
                int ntl) {
  TORCH_CHECK(srcs.size() == dsts.size(), "multi_copy: list length mismatch");
  if (srcs.empty()) return;
  std::vector<pdcc::kern::CopyDesc> d;
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& a = srcs[i];
    const auto& b = dsts[i];
    TORCH_CHECK(a.is_cuda() && b.device() == a.device(), "multi_copy: tensors must be on one GPU");
    TORCH_CHECK(a.nbytes() == b.nbytes(), "multi_copy: pair ", i, " size mismatch");
    TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "multi_copy: tensors must be contiguous");
    d.push_back({a.data_ptr(), b.data_ptr(), a.nbytes()});
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(srcs[0].device());
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(srcs[0].device().index()).stream();
  hipError_t e = pdcc::kern::multi_copy(d.data(), (int)d.size(), s, max_blocks, depth, ntl);
  TORCH_CHECK(e == hipSuccess, "multi_copy launch failed: ", hipGetErrorString(e));
}

// Peer links between every pair of visible GPUs, as the runtime reports them: HSA link
// type (xGMI on an MI355X node, PCIe otherwise), hop count, P2P access / atomics and
// the runtime's relative performance rank. Local queries only (no collective).
py::list device_links() {
  static const char* kLink[] = {"hypertransport", "qpi", "pcie", "infiniband", "xgmi"};
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  py::list out;
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      if (a == b) continue;
      py::dict d;
      d["src"] = a;
      d["dst"] = b;
      uint32_t type = 0, hops = 0;
      if (hipExtGetLinkTypeAndHopCount(a, b, &type, &hops) == hipSuccess) {
        d["link"] = type < 5 ? std::string(kLink[type]) : std::to_string(type);
        d["hops"] = hops;
      } else {
        (void)hipGetLastError();
        d["link"] = "unknown";
      }
      int v = 0;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrAccessSupported, a, b) == hipSuccess) d["p2p"] = v;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrNativeAtomicSupported, a, b) == hipSuccess) d["atomics"] = v;
      if (hipDeviceGetP2PAttribute(&v, hipDevP2PAttrPerformanceRank, a, b) == hipSuccess) d["perf_rank"] = v;
      (void)hipGetLastError();
      out.append(d);
    }
  return out;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native collective communication backend (c10d) and gfx950 kernels";
  py::module::import("torch.distributed");  // registers c10d::Backend / Store with pybind

  py::class_<pdcc::ProcessGroupMI355X, c10d::Backend, c10::intrusive_ptr<pdcc::ProcessGroupMI355X>>(
      m, "ProcessGroupMI355X")
      .def(py::init([](const c10::intrusive_ptr<c10d::Store>& store, int rank, int size,
                       std::chrono::milliseconds timeout, std::vector<int64_t> ranks, std::string name) {
             return c10::make_intrusive<pdcc::ProcessGroupMI355X>(store, rank, size, timeout, std::move(ranks),
                                                                  std::move(name));
           }),
           py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("timeout"),
           py::arg("global_ranks") = std::vector<int64_t>{}, py::arg("group_name") = std::string(""),
           py::call_guard<py::gil_scoped_release>())
      .def("stats",
           [](pdcc::ProcessGroupMI355X& pg) {
             std::map<std::string, pdcc::OpStats> st;
             {  // (may wait for pending zero-copy outcomes)
               py::gil_scoped_release nogil;
               st = pg.stats();
             }
             py::dict d;
             for (const auto& kv : st)
               d[py::str(kv.first)] = py::make_tuple(kv.second.calls, kv.second.bytes, kv.second.host_ms);
             return d;
           })
      .def("autotune_table",
           [](pdcc::ProcessGroupMI355X& pg) {
             py::list l;
             for (const auto& r : pg.autotune_table()) {
               py::dict d;
               d["coll"] = r.coll;
               d["dtype"] = r.dtype;
               d["op"] = r.op;
               d["lo"] = r.lo;
               d["hi"] = r.hi;
               d["ref"] = r.ref;
               d["ref_us"] = r.rccl_us;
               d["ipc_us"] = r.ipc_us;
               d["push_us"] = r.push_us;
               d["dyn_us"] = r.dyn_us;
               d["sdma_us"] = r.sdma_us;
               d["wide_us"] = r.wide_us;
               d["ipc_wide_us"] = r.ipc_wide_us;
               d["staged_us"] = r.staged_us;
               d["ipc_valid"] = r.valid;
               d["algo"] = r.algo;
               d["iters"] = r.iters;
               d["async_capped"] = r.async_capped;
               l.append(d);
             }
             return l;
           })
      .def("flight_recorder",
           [](pdcc::ProcessGroupMI355X& pg) {
             py::list l;
             for (const auto& r : pg.flight_recorder()) {
               py::dict d;
               d["seq"] = r.seq;
               d["op"] = r.what;
               d["bytes"] = r.bytes;
               d["t_ms"] = r.t_ms;
               d["state"] = r.state;
               l.append(d);
             }
             return l;
           })
      .def("flight_recorder_dump", &pdcc::ProcessGroupMI355X::flight_recorder_dump, py::arg("last") = 16)
      .def("reset_stats", &pdcc::ProcessGroupMI355X::reset_stats)
      .def("describe", &pdcc::ProcessGroupMI355X::describe)
      .def("timeout_ms", &pdcc::ProcessGroupMI355X::timeout_ms)
      .def("last_algo", &pdcc::ProcessGroupMI355X::last_algo, py::call_guard<py::gil_scoped_release>())
      .def("zc_counters", &pdcc::ProcessGroupMI355X::zc_counters, py::call_guard<py::gil_scoped_release>())
      .def("healthy", &pdcc::ProcessGroupMI355X::healthy)
      .def("health_message", &pdcc::ProcessGroupMI355X::health_message)
      .def("set_algo", &pdcc::ProcessGroupMI355X::set_algo)
      .def("host_profile",
           [](pdcc::ProcessGroupMI355X& pg) {
             py::dict d;
             for (const auto& r : pg.host_profile())
               d[py::str(std::get<0>(r))] = py::make_tuple(std::get<1>(r), std::get<2>(r));
             return d;
           },
           "PDCC_HOST_PROF / set_host_profile(True): {stage: (calls, total_us)} of the GPU all_reduce host path")
      .def("set_host_profile", &pdcc::ProcessGroupMI355X::set_host_profile, py::arg("on"))
      .def("set_ipc_thresholds", &pdcc::ProcessGroupMI355X::set_ipc_thresholds, py::arg("one_shot_max") = -1,
           py::arg("two_shot_max") = -1, py::arg("copy_max") = -1)
      .def("abort_group", &pdcc::ProcessGroupMI355X::abort_group, py::call_guard<py::gil_scoped_release>())
      .def("ipc_trace", &pdcc::ProcessGroupMI355X::ipc_trace,
           "PDCC_IPC_TRACE records: [seq, t_entry, t_seq, t_staged, t_barrier0, t_phase1, t_barrier1, t_exit] "
           "in 100 MHz device ticks, block 0 of each IPC kernel (words 8-11: zero-copy exchange, 12-15: call number "
           "and zero-copy arrival barrier), then per block b < 256: [16 + b] phase 1 done, [272 + b] exit")
      .def("eager_init", &pdcc::ProcessGroupMI355X::eager_init, py::arg("device"),
           py::call_guard<py::gil_scoped_release>())
      // torch calls this on non-member ranks of a new group when the default group is bound
      // to a device (see supportsSplitting in process_group.h): nothing to do here
      .def("perform_nocolor_split", [](pdcc::ProcessGroupMI355X&, const at::Device&) {});

  // the cross-stream issue order of one RCCL communicator (csrc/device/issue_order.h), exposed
  // for tests: dry=True logs the stream operations instead of issuing them (no GPU needed)
  py::class_<pdcc::IssueOrder>(m, "IssueOrder")
      .def(py::init<bool>(), py::arg("dry") = false)
      .def("enter", [](pdcc::IssueOrder& o, uintptr_t s) { o.enter(reinterpret_cast<hipStream_t>(s)); })
      .def("leave", [](pdcc::IssueOrder& o, uintptr_t s) { o.leave(reinterpret_cast<hipStream_t>(s)); })
      .def("add_user", &pdcc::IssueOrder::add_user)
      .def("users", &pdcc::IssueOrder::users)
      .def("ticks", &pdcc::IssueOrder::ticks)
      .def("waits", &pdcc::IssueOrder::waits)
      .def("log", &pdcc::IssueOrder::log);

  m.def("reduce_nway", &reduce_nway, py::arg("srcs"), py::arg("out"), py::arg("op") = "sum",
        py::arg("mode") = 1, py::arg("max_blocks") = 0,
        "K1: out = op(srcs...) on the current stream (mode: 1 LDS-DMA engine | 2 non-temporal stores | "
        "4 streaming kernel | 8 non-temporal loads)");
  m.def("multi_copy", &multi_copy, py::arg("srcs"), py::arg("dsts"), py::arg("max_blocks") = 0, py::arg("depth") = 0,
        py::arg("ntl") = -1,
        "K2: one-launch multi-tensor copy (max_blocks/depth 0 = defaults)");
  m.def("ipc_signal_bytes", &pdcc::kern::ipc_signal_bytes);
  m.def("device_links", &device_links,
        "peer links between every pair of visible GPUs: link type (xgmi/pcie), hops, p2p, atomics, perf_rank");
  m.def("forwarded_rccl_env", &pdcc::forward_rccl_env,
        "NCCL_* variables set from PDCC_RCCL_* before the first communicator (once per process)");
  m.attr("MAX_RANKS_IPC") = pdcc::kern::kMaxRanks;
  m.attr("TILE_BYTES") = pdcc::kern::kTileBytes;
}
