// Backend configuration: every knob is a PDCC_* environment variable read once
// when a process group is constructed. The Python mirror is
// pytorch_distributed_collective_communication_amd/config.py.
#pragma once
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <string>

namespace pdcc {

// IPC_PUSH: the push all-reduce (zero-copy, every remote access a write), an autotuner
// candidate next to the pull protocols of IPC. RCCL_WIDE: RCCL on a child communicator
// with at least rccl_wide_ctas channels, an autotuner candidate next to the default one.
// IPC_WIDE: the pull all-reduce with ipc_wide_grid workgroups (more remote reads in flight
// per xGMI link), an autotuner candidate next to IPC for bulk all_reduce keys.
// IPC_STAGED: the IPC protocols with zero copy off for the call (inputs copied into the
// registered staging buffer): raced against IPC (zero copy) for keys from ipc_zc_min, so the
// zero-copy / staging crossover is measured per node instead of fixed.
// IPC_DYN: the zero-copy 2-shot all-reduce with work items claimed dynamically and per-chunk
// ready words instead of fixed tile ranges and a block-pairwise barrier (kern::kDynOffset),
// an autotuner candidate next to IPC for zero-copy all_reduce keys.
// IPC_SDMA: the copy collectives (broadcast, all_gather, gather, scatter, all_to_all) at zero-copy
// sizes as hipMemcpyAsync pulls between IPC-mapped user buffers -- the runtime's copy engines move
// the bytes instead of CU kernels (gpu_ops.cpp sdma_run); an autotuner candidate for those keys.
enum class Algo : int { AUTO = 0, RCCL, IPC, HOST, IPC_PUSH, RCCL_WIDE, IPC_WIDE, IPC_STAGED, IPC_DYN, IPC_SDMA };
inline bool is_ipc(Algo a) {
  return a == Algo::IPC || a == Algo::IPC_PUSH || a == Algo::IPC_WIDE || a == Algo::IPC_STAGED ||
         a == Algo::IPC_DYN || a == Algo::IPC_SDMA;
}
inline bool is_rccl(Algo a) { return a == Algo::RCCL || a == Algo::RCCL_WIDE; }

struct Config {
  // algorithm selection
  Algo force_algo = Algo::AUTO;            // PDCC_ALGO=auto|rccl|ipc|host
  size_t ipc_1shot_max = 512u << 10;       // PDCC_IPC_1SHOT_MAX   all-reduce/reduce <= this: 1-shot
  size_t ipc_2shot_max = 8u << 20;         // PDCC_IPC_2SHOT_MAX   <= this: 2-shot, else RCCL
  size_t ipc_copy_max = 1u << 20;          // PDCC_IPC_COPY_MAX    broadcast/gather/... <= this: IPC
  size_t ipc_max_staging = 1u << 30;       // PDCC_IPC_MAX_STAGING staging bytes; larger messages are chunked
  bool ipc_enable = true;                  // PDCC_IPC=0 disables the peer-memory path
  // Zero-copy IPC (all-reduce 2-shot, broadcast 2-shot, all-gather/gather, reduce-scatter and
  // all-to-all with flat inputs): from ipc_zc_min bytes the kernels read the peers' USER buffers
  // in place -- mapped per call after a host-side exchange of allocation handles -- instead of
  // a copy into the staging buffer (all-reduce: ~55% less HBM traffic per rank). Mappings are
  // cached per peer allocation (ipc_zc_cache exports per rank, LRU).
  bool ipc_zc = true;                      // PDCC_IPC_ZC
  // The autotuner also races the push all-reduce (owners receive their tiles by remote writes,
  // reduce locally and write the result into every rank's tensor) for zero-copy sizes.
  bool ipc_push = true;                    // PDCC_IPC_PUSH
  // PDCC_IPC_DYN: chunks per workgroup of the dynamic 2-shot all-reduce (IPC_DYN; fewer = less
  // per-item overhead, more = finer load balance); 0: the autotuner does not race it (0..64)
  int ipc_dyn = 3;
  // PDCC_IPC_SDMA: the autotuner races the copy-engine candidate (IPC_SDMA) for copy-collective keys
  // of zero-copy sizes; PDCC_SDMA_STREAMS: side streams a call's pulls fan out over (0..6; each
  // stream's copies run in order, several streams keep several copy engines busy)
  bool ipc_sdma = true;
  int sdma_streams = 2;
  // PDCC_IPC_DYN_MIN_ROWS: rows (W tiles each) per dynamic item, at least (0 = kern::kDynMinRows = 16;
  // 1..4096; voted group-wide like PDCC_IPC_DYN)
  int ipc_dyn_min_rows = 0;
  size_t ipc_zc_min = 1u << 20;            // PDCC_IPC_ZC_MIN
  // All-reduces up to this size (<= 256 KiB, kern::kLLMaxBytes) use the LL protocol: every
  // rank pushes flag-tagged 8-byte words into its peers' signal areas and polls its own --
  // no staging copy and no barrier (0 = off; gated by its own self-test).
  // (256 KiB: LL beats the staged protocols at 128-256 KiB on MI355X, 8.1 vs 14.9 us per 256 KiB
  // all_reduce at W = 2, 11.6 vs 23.7 at W = 4: profiles/r3/ll_bench_256k_r3.jsonl)
  size_t ipc_ll_max = 256u << 10;          // PDCC_IPC_LL_MAX
  // (at most kern::kZcTab: the device-side exchange looks mappings up in a table of that many
  // entries per peer; a larger cache would silently send calls to the host gate)
  size_t ipc_zc_cache = 16;                // PDCC_IPC_ZC_CACHE
  // Device-side record exchange of gated zero-copy calls (kern::ZcTable). Every rank's intent
  // is voted on at the group's first GPU use (AND), so ranks with different settings agree.
  bool ipc_zx = true;                      // PDCC_IPC_ZX
  // Zero-copy refuses buffers whose allocation size has bit 31 set: mapping them in a peer stalls
  // (IpcComm::zc_export); they run staged. 0 lifts the guard (a runtime that maps them).
  bool ipc_zc_size_guard = true;           // PDCC_IPC_ZC_SIZE_GUARD
  // Workgroup cap of IPC / LL launches issued on the comm stream (async_op=True collectives,
  // e.g. DDP / ZeRO buckets overlapped with backward): the kernels spin in cross-GPU
  // barriers while a peer lags, holding CU slots that the overlapped GEMMs need. 0 = no cap
  // (the synchronous cap PDCC_IPC_GRID applies). 64: scripts/zero_bench.py, 403 M-param bf16 step, two
  // ranks on one MI355X (profiles/r4/zero_bench_async_grid_r4.jsonl): replicated DP 36.4-36.7 ms at 64
  // vs 37.2-37.5 uncapped, ZeRO 30.8-31.2 either way, 32 worse; 64 workgroups still keep ~4 MiB of
  // remote loads in flight per GPU at W = 8 -- about RCCL's own CTA footprint for a collective.
  // OPT-IN (default 0): the grid then depends on each rank's own async_op, which torch treats as
  // rank-local; the block-pairwise protocol needs the same grid on every rank, so with a cap set
  // every rank must pass the same async_op to each collective (DDP / ZeRO buckets do). PDCC_DEBUG=1
  // checks that per call; the autotuner keys capped (async) calls separately from full-grid ones.
  int ipc_async_grid = 0;                  // PDCC_IPC_ASYNC_GRID
  // Zero-copy calls exchange their records on a per-device launcher thread (IpcLauncher in
  // process_group.h): the caller's host never waits for its peers (0 = inline exchange)
  bool ipc_zc_async = true;                // PDCC_IPC_ZC_ASYNC
  // Before a group first uses a device, every rank runs the IPC protocol once on known data (1-shot
  // and 2-shot all-reduce, all-gather) with a short spin timeout and checks the results; one failure
  // on any rank (handle open error, timeout, wrong data) disables IPC for the whole group, so a
  // topology the protocol does not work on falls back to RCCL instead of hanging or corrupting data.
  bool ipc_selftest = true;                // PDCC_IPC_SELFTEST
  int ipc_selftest_ms = 20000;             // PDCC_IPC_SELFTEST_MS spin timeout during the self-test
  // Upper bound on one cross-GPU barrier spin of the IPC kernels (the group timeout applies if
  // shorter); the watchdog's abort stops a spin at once.
  int64_t ipc_spin_ms = 600000;            // PDCC_IPC_SPIN_MS
  // Workgroup cap of the IPC kernels on distinct devices (1..1024; one workgroup pulls one
  // row of W tiles / one tile at a time, so more workgroups = more remote reads in flight
  // per xGMI link). Ranks sharing one device are capped at 256 / W for co-residency.
  int ipc_grid = 512;                      // PDCC_IPC_GRID
  // Workgroup cap of the IPC_WIDE autotuner candidate (all_reduce keys >= rccl_wide_min on
  // distinct GPUs); raced only when larger than ipc_grid (0 = off).
  int ipc_wide_grid = 1024;                // PDCC_IPC_WIDE_GRID
  // Online autotuner (GPU all_reduce, groups where both RCCL and IPC are feasible): the first call
  // in each power-of-two size bucket >= autotune_min runs both engines on scratch copies, checks
  // that the IPC result matches RCCL's, times both and adopts the faster one on every rank.
  // Every GPU collective with two feasible engines is tuned per (collective, dtype, op, size
  // bucket); the key's first call pays it, later calls look the decision up.
  bool autotune = true;                    // PDCC_AUTOTUNE=0 keeps the static thresholds above
  size_t autotune_min = 64u << 10;         // PDCC_AUTOTUNE_MIN
  size_t autotune_max = 1ull << 42;        // PDCC_AUTOTUNE_MAX
  // Tuning runs on scratch buffers of at most this many bytes per engine (a prefix of the
  // caller's data): above it both engines are bandwidth-bound, so the sample decides the bucket.
  size_t autotune_sample = 1ull << 30;     // PDCC_AUTOTUNE_SAMPLE
  uint32_t autotune_colls = 0xffffffffu;   // PDCC_AUTOTUNE_COLLS=allreduce,reduce,... (default all)
  // Cross-GPU barrier spin bound while tuning: an IPC run that cannot finish (a topology
  // the protocol fails on at this size) costs this much once, disqualifies IPC for the key
  // and leaves the group healthy, instead of hanging for the group timeout.
  int64_t autotune_spin_ms = 10000;        // PDCC_AUTOTUNE_SPIN_MS
  // Decisions persisted across runs: a key with a line in this file (same topology signature,
  // the same on every rank) takes the recorded engine without a race; every new race's
  // verdict is appended by rank 0 ("" = off). Offline tuning = a file written by an earlier run.
  std::string autotune_file;               // PDCC_AUTOTUNE_FILE
  // PDCC_STREAM: auto (default) = synchronous collectives (async_op=False) on the caller's stream,
  // async ones on a normal-priority comm stream; high = auto with a high-priority comm stream;
  // comm = always the comm stream; current = always the caller's stream.
  // (Measured on MI355X: a cross-stream event hand-off costs ~20 us per op on a normal
  // stream and ~150 us on a high-priority one; the caller's stream ~5 us end to end.)
  int stream_mode = 0;
  // RCCL channel tuning: each CTA drives one channel (ring/tree lane); on 8 GPUs one
  // channel per xGMI link needs >= 7. -1 leaves RCCL's own topology tuner in charge
  // (ncclCommInitRank); any value set goes through ncclCommInitRankConfig.
  // Deadline of one RCCL communicator creation (group comm, split / wide children, pair
  // channels; capped by the group timeout): communicators are created non-blocking and
  // polled, so a peer that dies or never arrives fails the group within this bound
  // instead of hanging every other rank (the reference's Gloo surfaces it in ~0.2 s).
  int64_t rccl_init_timeout_ms = 300000;   // PDCC_RCCL_INIT_TIMEOUT_S (seconds)
  bool rccl_nonblocking = true;            // PDCC_RCCL_NONBLOCKING=0: blocking creation, no deadline
  int rccl_min_ctas = -1;                  // PDCC_RCCL_MIN_CTAS
  int rccl_max_ctas = -1;                  // PDCC_RCCL_MAX_CTAS
  // Wide RCCL: a child communicator (ncclCommSplit, own resources) with at least this many
  // channels; the autotuner races it against the default communicator for all_reduce keys
  // from rccl_wide_min bytes, so a node whose 7 xGMI links want more channels than RCCL's
  // topology tuner picks gets them measured, not guessed (0 = off).
  int rccl_wide_ctas = 112;                // PDCC_RCCL_WIDE_CTAS
  size_t rccl_wide_min = 16u << 20;        // PDCC_RCCL_WIDE_MIN
  // Groups whose member set equals a live communicator's (new_group(range(size)) in every demo
  // of the reference): share = use that communicator (RCCL runs the ops of one communicator in
  // issue order on every stream, which is the order every rank issues them in), split =
  // ncclCommSplit from it, init = always a fresh ncclCommInitRank. Measured on MI355X
  // (profiles/group_churn.jsonl, 1-rank communicators): init 41-44 ms, split 40-44 ms,
  // share 0.1 ms per group.
  int group_comm = 1;                      // PDCC_RCCL_GROUP_COMM=split|share|init (0|1|2)
  bool rccl_split_share = true;            // PDCC_RCCL_SPLIT_SHARE: split children share parent resources
  // all_gather into a list of separate tensors on RCCL: p2p = grouped ncclSend/Recv straight
  // into the list (zero copy), staged = ncclAllGather into a staging buffer + K2 unpack
  bool list_gather_p2p = true;             // PDCC_LIST_GATHER=p2p|staged
  // all_to_all with tensor lists: chunk sizes are rank-local, so the ranks agree (one
  // host-transport round) whether every chunk is equal before taking the IPC/LL/autotuned
  // engines; 0 = lists always go to grouped point-to-point (no host round per call)
  bool a2a_list_agree = true;              // PDCC_A2A_LIST_AGREE
  bool world1_local = true;                // PDCC_WORLD1_LOCAL=0: run RCCL even for 1-rank groups (tests)
  bool eager_init = false;                 // PDCC_EAGER_INIT=1: GPU setup at group construction
  // host transport
  size_t shm_slot_bytes = 8u << 20;        // PDCC_SHM_SLOT_BYTES
  size_t shm_chan_bytes = 1u << 20;        // PDCC_SHM_CHAN_BYTES
  int shm_spin_us = 300;                   // PDCC_SHM_SPIN_US (busy-wait window before futex sleep)
  // the zero-copy exchange thread spins this long after its last job before it sleeps (0: at
  // once). Off by default: in steady state the kernels resolve zero-copy buffers on the device
  // and the thread is off the critical path; a spinning thread costs CPU quota (measured on a
  // 16-CPU box share: 500 us of spin made the host-gated exchange slower, profiles/r3/zx/)
  int xchg_spin_us = 0;                    // PDCC_XCHG_SPIN_US
  // robustness / observability
  bool debug = false;                      // PDCC_DEBUG=1: cross-rank op fingerprint check
  int log_level = 0;                       // PDCC_LOG_LEVEL 0 quiet, 1 info, 2 every collective
  bool blocking_wait = false;              // PDCC_BLOCKING_WAIT=1: Work.wait() blocks the host
  bool roctx = false;                      // PDCC_ROCTX=1: roctx ranges per collective
  int watchdog_ms = 100;                   // PDCC_WATCHDOG_MS poll period (0 disables)
  std::string fault;                       // PDCC_FAULT=rank:seq:kind (kind exit|raise|hang)

  static Config from_env();
  std::string describe() const;
};

const char* algo_name(Algo a);
// inverse of algo_name (AUTO for an unknown name)
Algo algo_from_name(const std::string& n);

}  // namespace pdcc
