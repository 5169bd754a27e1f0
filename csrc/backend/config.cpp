#include "config.h"

#include "../kernels/kernel_api.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <stdexcept>

namespace pdcc {

namespace {
const char* env(const char* k) {
  const char* v = std::getenv(k);
  return (v && *v) ? v : nullptr;
}
size_t env_size(const char* k, size_t def) {
  const char* v = env(k);
  if (!v) return def;
  char* end = nullptr;
  double x = std::strtod(v, &end);
  std::string suf = end ? std::string(end) : "";
  if (suf == "k" || suf == "K" || suf == "KiB") x *= 1024.0;
  else if (suf == "m" || suf == "M" || suf == "MiB") x *= 1024.0 * 1024.0;
  else if (suf == "g" || suf == "G" || suf == "GiB") x *= 1024.0 * 1024.0 * 1024.0;
  return (size_t)x;
}
int env_int(const char* k, int def) {
  const char* v = env(k);
  return v ? std::atoi(v) : def;
}
bool env_bool(const char* k, bool def) {
  const char* v = env(k);
  if (!v) return def;
  std::string s(v);
  return !(s == "0" || s == "false" || s == "False" || s == "no" || s == "off");
}
}  // namespace

const char* algo_name(Algo a) {
  switch (a) {
    case Algo::AUTO: return "auto";
    case Algo::RCCL: return "rccl";
    case Algo::IPC: return "ipc";
    case Algo::HOST: return "host";
    case Algo::IPC_PUSH: return "ipc_push";
    case Algo::RCCL_WIDE: return "rccl_wide";
    case Algo::IPC_WIDE: return "ipc_wide";
    case Algo::IPC_STAGED: return "ipc_staged";
    case Algo::IPC_DYN: return "ipc_dyn";
    case Algo::IPC_SDMA: return "ipc_sdma";
  }
  return "?";
}

Algo algo_from_name(const std::string& n) {
  for (Algo a : {Algo::RCCL, Algo::IPC, Algo::HOST, Algo::IPC_PUSH, Algo::RCCL_WIDE, Algo::IPC_WIDE, Algo::IPC_STAGED,
                 Algo::IPC_DYN, Algo::IPC_SDMA})
    if (n == algo_name(a)) return a;
  return Algo::AUTO;
}

Config Config::from_env() {
  Config c;
  if (const char* a = env("PDCC_ALGO")) {
    std::string s(a);
    if (s == "auto") c.force_algo = Algo::AUTO;
    else if (s == "rccl") c.force_algo = Algo::RCCL;
    else if (s == "ipc") c.force_algo = Algo::IPC;
    else if (s == "host") c.force_algo = Algo::HOST;
    else if (s == "ipc_push") c.force_algo = Algo::IPC_PUSH;
    else if (s == "rccl_wide") c.force_algo = Algo::RCCL_WIDE;
    else if (s == "ipc_wide") c.force_algo = Algo::IPC_WIDE;
    else if (s == "ipc_staged") c.force_algo = Algo::IPC_STAGED;
    else if (s == "ipc_dyn") c.force_algo = Algo::IPC_DYN;
    else if (s == "ipc_sdma") c.force_algo = Algo::IPC_SDMA;
    else throw std::runtime_error("PDCC_ALGO must be auto|rccl|rccl_wide|ipc|ipc_push|ipc_wide|ipc_staged|ipc_dyn|ipc_sdma|host, got " + s);
  }
  c.ipc_1shot_max = env_size("PDCC_IPC_1SHOT_MAX", c.ipc_1shot_max);
  c.ipc_2shot_max = env_size("PDCC_IPC_2SHOT_MAX", c.ipc_2shot_max);
  c.ipc_copy_max = env_size("PDCC_IPC_COPY_MAX", c.ipc_copy_max);
  c.ipc_max_staging = env_size("PDCC_IPC_MAX_STAGING", c.ipc_max_staging);
  c.ipc_enable = env_bool("PDCC_IPC", c.ipc_enable);
  c.ipc_selftest = env_bool("PDCC_IPC_SELFTEST", c.ipc_selftest);
  c.ipc_selftest_ms = env_int("PDCC_IPC_SELFTEST_MS", c.ipc_selftest_ms);
  c.ipc_zc = env_bool("PDCC_IPC_ZC", c.ipc_zc);
  c.ipc_push = env_bool("PDCC_IPC_PUSH", c.ipc_push);
  c.ipc_dyn = std::min(64, std::max(0, env_int("PDCC_IPC_DYN", c.ipc_dyn)));
  c.ipc_sdma = env_bool("PDCC_IPC_SDMA", c.ipc_sdma);
  c.sdma_streams = std::min(6, std::max(0, env_int("PDCC_SDMA_STREAMS", c.sdma_streams)));
  c.ipc_dyn_min_rows = std::min(4096, std::max(0, env_int("PDCC_IPC_DYN_MIN_ROWS", c.ipc_dyn_min_rows)));
  c.ipc_zc_min = env_size("PDCC_IPC_ZC_MIN", c.ipc_zc_min);
  c.ipc_ll_max = env_size("PDCC_IPC_LL_MAX", c.ipc_ll_max);
  c.ipc_zc_cache = std::max<size_t>(1, env_size("PDCC_IPC_ZC_CACHE", c.ipc_zc_cache));
  if (c.ipc_zc_cache > (size_t)kern::kZcTab) {
    fprintf(stderr, "[pdcc] PDCC_IPC_ZC_CACHE=%zu exceeds the device mapping table (%d per peer): clamped\n",
            c.ipc_zc_cache, kern::kZcTab);
    c.ipc_zc_cache = (size_t)kern::kZcTab;
  }
  c.ipc_zx = env_bool("PDCC_IPC_ZX", c.ipc_zx);
  c.ipc_zc_size_guard = env_bool("PDCC_IPC_ZC_SIZE_GUARD", c.ipc_zc_size_guard);
  if (c.ipc_zc_size_guard && c.ipc_max_staging >= (size_t{1} << 31)) {
    // the staging buffer is exported and mapped like a zero-copy buffer: a 2 GiB+ window could take
    // a size with bit 31 set, whose mapping stalls (IpcComm::zc_export)
    fprintf(stderr, "[pdcc] PDCC_IPC_MAX_STAGING=%zu: staging stays below 2 GiB while PDCC_IPC_ZC_SIZE_GUARD=1: "
            "clamped to 1 GiB\n", c.ipc_max_staging);
    c.ipc_max_staging = size_t{1} << 30;
  }
  c.ipc_async_grid = std::min(1024, std::max(0, env_int("PDCC_IPC_ASYNC_GRID", c.ipc_async_grid)));
  c.ipc_zc_async = env_bool("PDCC_IPC_ZC_ASYNC", c.ipc_zc_async);
  c.autotune = env_bool("PDCC_AUTOTUNE", c.autotune);
  c.autotune_min = env_size("PDCC_AUTOTUNE_MIN", c.autotune_min);
  c.autotune_max = env_size("PDCC_AUTOTUNE_MAX", c.autotune_max);
  c.autotune_sample = std::max<size_t>(env_size("PDCC_AUTOTUNE_SAMPLE", c.autotune_sample), 64u << 10);
  if (const char* ac = env("PDCC_AUTOTUNE_COLLS")) {
    static const char* kNames[] = {"allreduce", "reduce", "broadcast", "allgather", "gather",
                                   "scatter", "reduce_scatter", "alltoall"};
    c.autotune_colls = 0;
    std::string s(ac);
    size_t pos = 0;
    while (pos <= s.size()) {
      const size_t e = std::min(s.find(',', pos), s.size());
      const std::string tok = s.substr(pos, e - pos);
      bool known = tok.empty() || tok == "none";
      if (tok == "all") {
        c.autotune_colls = 0xffffffffu;
        known = true;
      }
      for (int i = 0; i < 8; ++i)
        if (tok == kNames[i]) {
          c.autotune_colls |= 1u << i;
          known = true;
        }
      if (!known) throw std::runtime_error("PDCC_AUTOTUNE_COLLS: unknown collective '" + tok + "'");
      pos = e + 1;
    }
  }
  c.ipc_spin_ms = (int64_t)env_size("PDCC_IPC_SPIN_MS", (size_t)c.ipc_spin_ms);
  c.ipc_grid = std::min(1024, std::max(1, env_int("PDCC_IPC_GRID", c.ipc_grid)));
  c.ipc_wide_grid = std::min(1024, std::max(0, env_int("PDCC_IPC_WIDE_GRID", c.ipc_wide_grid)));
  c.autotune_spin_ms = (int64_t)env_size("PDCC_AUTOTUNE_SPIN_MS", (size_t)c.autotune_spin_ms);
  if (const char* f = env("PDCC_AUTOTUNE_FILE")) c.autotune_file = f;
  if (const char* gc = env("PDCC_RCCL_GROUP_COMM")) {
    std::string v(gc);
    if (v == "split") c.group_comm = 0;
    else if (v == "share") c.group_comm = 1;
    else if (v == "init") c.group_comm = 2;
    else throw std::runtime_error("PDCC_RCCL_GROUP_COMM must be split|share|init, got " + v);
  }
  c.rccl_split_share = env_bool("PDCC_RCCL_SPLIT_SHARE", c.rccl_split_share);
  if (const char* lg = env("PDCC_LIST_GATHER")) {
    std::string v(lg);
    if (v == "p2p") c.list_gather_p2p = true;
    else if (v == "staged") c.list_gather_p2p = false;
    else throw std::runtime_error("PDCC_LIST_GATHER must be p2p|staged, got " + v);
  }
  c.a2a_list_agree = env_bool("PDCC_A2A_LIST_AGREE", c.a2a_list_agree);
  if (const char* it = env("PDCC_RCCL_INIT_TIMEOUT_S")) c.rccl_init_timeout_ms = (int64_t)(std::atof(it) * 1000.0);
  c.rccl_init_timeout_ms = std::max<int64_t>(1, c.rccl_init_timeout_ms);
  c.rccl_nonblocking = env_bool("PDCC_RCCL_NONBLOCKING", c.rccl_nonblocking);
  c.rccl_min_ctas = env_int("PDCC_RCCL_MIN_CTAS", c.rccl_min_ctas);
  c.rccl_max_ctas = env_int("PDCC_RCCL_MAX_CTAS", c.rccl_max_ctas);
  c.rccl_wide_ctas = std::max(0, env_int("PDCC_RCCL_WIDE_CTAS", c.rccl_wide_ctas));
  c.rccl_wide_min = env_size("PDCC_RCCL_WIDE_MIN", c.rccl_wide_min);
  if (c.rccl_min_ctas > 0 && c.rccl_max_ctas > 0 && c.rccl_min_ctas > c.rccl_max_ctas)
    throw std::runtime_error("PDCC_RCCL_MIN_CTAS must not exceed PDCC_RCCL_MAX_CTAS");
  c.world1_local = env_bool("PDCC_WORLD1_LOCAL", c.world1_local);
  c.eager_init = env_bool("PDCC_EAGER_INIT", c.eager_init);
  if (const char* sm = env("PDCC_STREAM")) {
    std::string v(sm);
    if (v == "auto") c.stream_mode = 0;
    else if (v == "high") c.stream_mode = 1;
    else if (v == "comm") c.stream_mode = 2;
    else if (v == "current") c.stream_mode = 3;
    else throw std::runtime_error("PDCC_STREAM must be auto|high|comm|current, got " + v);
  }
  c.shm_slot_bytes = env_size("PDCC_SHM_SLOT_BYTES", c.shm_slot_bytes);
  c.shm_chan_bytes = env_size("PDCC_SHM_CHAN_BYTES", c.shm_chan_bytes);
  c.shm_spin_us = (int)env_int("PDCC_SHM_SPIN_US", c.shm_spin_us);
  c.xchg_spin_us = (int)env_int("PDCC_XCHG_SPIN_US", c.xchg_spin_us);
  c.debug = env_bool("PDCC_DEBUG", c.debug);
  c.log_level = env_int("PDCC_LOG_LEVEL", c.log_level);
  c.blocking_wait = env_bool("PDCC_BLOCKING_WAIT", c.blocking_wait);
  c.roctx = env_bool("PDCC_ROCTX", c.roctx);
  c.watchdog_ms = env_int("PDCC_WATCHDOG_MS", c.watchdog_ms);
  if (const char* f = env("PDCC_FAULT")) c.fault = f;
  return c;
}

std::string Config::describe() const {
  std::ostringstream o;
  o << "algo=" << algo_name(force_algo) << " ipc=" << ipc_enable << " ipc_selftest=" << ipc_selftest
    << " ipc_1shot_max=" << ipc_1shot_max
    << " ipc_2shot_max=" << ipc_2shot_max << " ipc_copy_max=" << ipc_copy_max
    << " ipc_max_staging=" << ipc_max_staging << " ipc_zc=" << ipc_zc << " ipc_zc_min=" << ipc_zc_min
    << " ipc_zc_cache=" << ipc_zc_cache << " ipc_zc_async=" << ipc_zc_async << " ipc_zx=" << ipc_zx << " ipc_zc_size_guard=" << ipc_zc_size_guard << " ipc_async_grid=" << ipc_async_grid << " ipc_ll_max=" << ipc_ll_max << " ipc_push=" << ipc_push << " ipc_dyn=" << ipc_dyn << " ipc_dyn_min_rows=" << ipc_dyn_min_rows << " ipc_sdma=" << ipc_sdma << " sdma_streams=" << sdma_streams << " ipc_spin_ms=" << ipc_spin_ms << " ipc_grid=" << ipc_grid << " ipc_wide_grid=" << ipc_wide_grid << " autotune=" << autotune
    << " autotune_sample=" << autotune_sample << " autotune_file=" << (autotune_file.empty() ? "-" : autotune_file) << " rccl_ctas=" << rccl_min_ctas << ".." << rccl_max_ctas << " rccl_wide_ctas=" << rccl_wide_ctas
    << " rccl_wide_min=" << rccl_wide_min << " rccl_init_timeout_ms=" << rccl_init_timeout_ms << " rccl_nonblocking=" << rccl_nonblocking
    << " group_comm=" << (group_comm == 0 ? "split" : group_comm == 1 ? "share" : "init")
    << " split_share=" << rccl_split_share << " list_gather=" << (list_gather_p2p ? "p2p" : "staged")
    << " a2a_list_agree=" << a2a_list_agree
    << " xchg_spin_us=" << xchg_spin_us << " shm_slot=" << shm_slot_bytes << " shm_chan=" << shm_chan_bytes
    << " debug=" << debug << " log=" << log_level << " blocking_wait=" << blocking_wait
    << " watchdog_ms=" << watchdog_ms << " stream=" << (stream_mode == 0 ? "auto" : stream_mode == 1 ? "high" : stream_mode == 2 ? "comm" : "current");
  return o.str();
}

}  // namespace pdcc
