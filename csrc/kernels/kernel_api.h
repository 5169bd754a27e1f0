// Host-visible launch API of the gfx950 HIP kernels (no torch headers here, so
// the .hip translation units stay small and compile in parallel).
//
// Kernel inventory:
//   K1  reduce_nway      out = Op(src_0 .. src_{k-1}), LDS-DMA staged tiles
//   K2  multi_copy       pack / unpack a list of tensors <-> one staging buffer
//   K3  peer pull        (inside the IPC collectives) xGMI reads of peer buffers
//   K4  cross-GPU flags  (inside the IPC collectives) system-scope signal words
//
// The reference (main.py:14,23,37,52,68,81) calls the six torch.distributed
// primitives on CPU/Gloo; these kernels are what the GPU path of this library
// runs underneath the same calls.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pdcc {
namespace kern {

constexpr int kMaxRanks = 8;        // one xGMI-connected MI355X node
constexpr int kMaxBlocks = 1024;    // per-block pairwise flags in the signal area
constexpr int kTileBytes = 4096;    // 256 lanes x 16 B: the unit every engine moves
constexpr int kBlockThreads = 256;  // 4 wave64s

enum class DType : int32_t { F32 = 0, F16, BF16, F64, I8, U8, I32, I64, BOOL, kCount };
enum class RedOp : int32_t { SUM = 0, AVG, PROD, MIN, MAX, BAND, BOR, BXOR, COPY, kCount };

inline size_t dtype_size(DType t) {
  switch (t) {
    case DType::F32: return 4;
    case DType::F16: return 2;
    case DType::BF16: return 2;
    case DType::F64: return 8;
    case DType::I8: return 1;
    case DType::U8: return 1;
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::BOOL: return 1;
    default: return 0;
  }
}

// true iff the (dtype, op) pair has a device kernel
bool supports(DType t, RedOp op);

// ---------------------------------------------------------------- K1
// out[i] = Op(srcs[0][i], ..., srcs[nsrc-1][i]), 1 <= nsrc <= kMaxRanks.
// AVG divides by `avg_div` (float types: multiply by 1/avg_div).
// All pointers must be 16-byte aligned; count is in elements.
hipError_t reduce_nway(const void* const* srcs, int nsrc, void* out, size_t count, DType t,
                       RedOp op, int avg_div, hipStream_t stream, int max_blocks = 0, bool nt = false);

// register-staged variant of K1 (same numerics) kept for A/B measurement
hipError_t reduce_nway_regs(const void* const* srcs, int nsrc, void* out, size_t count, DType t,
                            RedOp op, int avg_div, hipStream_t stream, int max_blocks = 0, bool nt = false);

// any K1 variant (`mode` = OR of K1Mode bits); the two calls above are LDS and REGS
enum K1Mode : int { K1_LDS = 1, K1_NT = 2, K1_STREAM = 4, K1_NT_LOADS = 8 };
hipError_t reduce_nway_mode(const void* const* srcs, int nsrc, void* out, size_t count, DType t, RedOp op,
                            int avg_div, hipStream_t stream, int max_blocks, int mode);

// ---------------------------------------------------------------- K2
struct CopyDesc {
  const void* src;
  void* dst;
  size_t bytes;
};
constexpr int kMaxCopyDescs = 64;  // per launch (kernarg); host splits longer lists
constexpr int kK2Depth = 4;        // K2 default LDS-DMA ring depth (tiles in flight per workgroup)
// One launch copies every descriptor (pack = many->one, unpack = one->many).
// max_blocks / depth: 0 = defaults (grid from the list's shape, see k2_grid in copy.hip;
// kK2Depth tiles in flight per workgroup)
// ntl_mode: non-temporal source loads (1 on, 0 off, -1 = by the list's shape)
hipError_t multi_copy(const CopyDesc* descs, int n, hipStream_t stream, int max_blocks = 0, int depth = 0,
                      int ntl_mode = -1);

// ---------------------------------------------------------------- IPC collectives
// Per-rank view of the group's registered (hipIpc) memory for ONE call.
//
// Sequencing is per workgroup and lives on the device: block b of every rank
// keeps a call counter in its own signal area (counters[b]), bumps it at entry
// and derives its flag epochs from it. Block b takes part in the same calls on
// every rank (the grid is a function of the call's arguments only), so the
// counters agree without any host-side number -- eager launches and graph
// replays (which repeat kernel arguments verbatim) run the same code.
constexpr int kCountWord = kMaxBlocks * kMaxRanks;  // u32 index of counters[0] in the signal area
constexpr int kEpochsPerCall = 4;                   // arrival, data, second data phase (+1 spare)

// LL ("low-latency") all-reduce for small payloads (IpcColl::ALLREDUCE_LL): every 8-byte
// word a rank pushes carries 4 data bytes and the call's epoch, so a receiver polls the
// data itself -- no staging copy, no barrier. Receive slots live in the (uncached)
// signal area after the flags and counters: [parity][source rank] slots of kLLSlotBytes.
// The epoch is per rank and per LL call: read by every block at entry, advanced by the
// block that finishes last (ctl[0] = epoch of the last finished call, ctl[1] = exit count).
constexpr int kLLCtlWord = kCountWord + kMaxBlocks;        // u32 index of ctl[0] in the signal area
constexpr size_t kLLOffset = 40960;                        // byte offset of the receive slots
constexpr size_t kLLMaxBytes = 256u << 10;                 // payload per rank of one LL call (cap of PDCC_IPC_LL_MAX)
constexpr size_t kLLSlotBytes = 2 * kLLMaxBytes;           // 8-byte words of 4 data bytes
static_assert(kLLOffset >= (size_t)(kLLCtlWord + 16) * 4, "LL slots overlap the signal words");
// The view and call structs are templates over the pointer type P<T>: the host (and the
// kernel arguments) use plain pointers (IpcView / IpcCall); the IPC kernels copy their
// arguments into LDS as dev::DView / dev::DCall, whose pointers are typed global
// (address space 1) -- a plain pointer read back from LDS is a generic one, and every
// access through it would be a flat instruction. Same layout either way.
template <class T>
using RawPtr = T*;

template <template <class> class P>
struct IpcViewT {
  P<char> buf[kMaxRanks];        // staging buffer per rank (own included), `cap` bytes; zero-copy: user buffers
  P<char> stg[kMaxRanks];        // staging buffer per rank (zero-copy calls that still stage results)
  P<uint32_t> flags[kMaxRanks];  // signal area (uncached device memory) per rank
  P<uint32_t> err;               // host-mapped error word (0 = ok), written on spin timeout
  P<uint32_t> counters;          // own signal area + kCountWord: per-block call counters
  size_t cap;                    // staging bytes
  int rank;
  int world;
  uint64_t timeout_ticks;        // s_memrealtime ticks (100 MHz) before a spin gives up
  P<uint64_t> trace;             // PDCC_IPC_TRACE: ring of kTraceWords-word records (host-mapped), or null
  uint32_t trace_cap;            // records in the ring
  uint32_t trace_slot;           // this launch's record (the host's launch counter % trace_cap)
  // this rank's control words of the dynamic protocols (claim / exit counters, epoch: word
  // indices kDynClaimWord / kDynExitWord / kDynEpochWord) in ordinary device memory -- only
  // this device's blocks touch them (agent-scope atomics), and an atomic on the uncached
  // signal area serialises at the memory controller
  P<uint32_t> dctl;
};
using IpcView = IpcViewT<RawPtr>;

// Device-side phase trace of an IPC call (block 0, s_memrealtime ticks at 100 MHz):
// [0] block 0's call number, [1] entry, [2] arrival barrier passed, [3] local data
// staged (a gated launch: its gate passed), [4] data barrier passed, [5] first pull / reduce done, [6] second data
// barrier passed (2-shot), [7] exit; a gated zero-copy launch's device-side exchange (block 0):
// [8] every rank's record in, [9] mapping lookup done, [10] every vote in, [11] verdict published.
// [12] after the block's call number was taken, and inside the zero-copy arrival barrier: [13] every
// wave drained (before the release), [14] flags stored to the peers, [15] every peer's flag seen.
// Dynamic protocols (block 0's totals, ticks): [16] waiting for claimed items, [17] publishing
// ready words (drain + release + store), [18] waiting for peers' ready words (+ acquire),
// [19] departure (exit count, and for the last block the done exchange), [20] items run,
// [21] of them phase-1 items, [22] 1 = block 0 departed last, [23] reading the call's epoch.
// Record `trace_slot` (one per launch, whatever the grid).
constexpr int kTraceWords = 24;
// After the header, per block b < kTraceBlocks: [kTraceWords + b] the block's first pull /
// reduce done ([5]), [kTraceWords + kTraceBlocks + b] its exit ([7]) -- how far the slowest
// block trails block 0.
constexpr int kTraceBlocks = 256;
constexpr int kTraceRecWords = kTraceWords + 2 * kTraceBlocks;

enum class IpcColl : int32_t {
  ALLREDUCE_1SHOT = 0,   // stage, barrier, every rank reduces everything from all peers
  ALLREDUCE_2SHOT,       // stage, barrier, reduce own 1/W, barrier, gather the other W-1
  REDUCE_1SHOT,          // stage, barrier, root reduces everything
  REDUCE_2SHOT,          // reduce-scatter, barrier, root gathers
  BROADCAST_1SHOT,       // root stages, barrier, everyone pulls from root
  BROADCAST_2SHOT,       // scatter from root, barrier, all-gather among all
  ALLGATHER,             // stage, barrier, pull W chunks
  GATHER,                // stage, barrier, root pulls W chunks
  SCATTER,               // root stages W chunks, barrier, rank r pulls chunk r
  REDUCE_SCATTER,        // stage W chunks, barrier, rank r reduces chunk r
  ALLTOALL,              // stage W chunks, barrier, rank r pulls chunk r of every peer
  BARRIER,               // flags only
  ALLREDUCE_PUSH,        // zero-copy only: push tiles to their owners' staging, owners reduce and
                         // push the result into every rank's tensor (remote writes, no remote reads)
  ALLREDUCE_LL,          // <= kLLMaxBytes: push flag-tagged words into every peer's LL slot, poll, reduce
  ALLGATHER_LL,          // <= kLLMaxBytes per rank: the same pushes, every peer's words into its output
  REDUCE_LL,             // <= kLLMaxBytes: peers push to the root only, the root reduces; tokens elsewhere
  BROADCAST_LL,          // <= kLLMaxBytes: the root pushes to every peer; tokens elsewhere
  GATHER_LL,             // <= kLLMaxBytes per rank: peers push to the root, the root writes out[q]
  SCATTER_LL,            // <= kLLMaxBytes per rank: the root pushes in[q] to rank q
  REDUCE_SCATTER_LL,     // <= kLLMaxBytes per chunk: in[q] pushed to rank q, reduced there
  ALLTOALL_LL,           // <= kLLMaxBytes per chunk: in[q] pushed to rank q, written to its out[src]
  kCount
};

// the flag-tagged push protocols (no staging, no barrier; payload <= kLLMaxBytes)
inline bool is_ll(IpcColl c) {
  return c == IpcColl::ALLREDUCE_LL || c == IpcColl::ALLGATHER_LL || c == IpcColl::REDUCE_LL ||
         c == IpcColl::BROADCAST_LL || c == IpcColl::GATHER_LL || c == IpcColl::SCATTER_LL ||
         c == IpcColl::REDUCE_SCATTER_LL || c == IpcColl::ALLTOALL_LL;
}

// Arguments of one IPC collective. `chunk_bytes` is the per-rank payload of one
// chunk (all-gather/scatter/... operate on W chunks of that size).
//
// Zero-copy calls (`zc` = 1): IpcView::buf[r] is rank r's USER buffer of this call
// (mapped for the call by IpcComm::zc_*), read in place -- no staging copy. Then
//   ALLREDUCE_2SHOT   buf[r] = rank r's tensor (in = out); bytes = whole rows of W tiles
//   ALLREDUCE_PUSH    buf[r] = rank r's tensor, stg[r] = its staging (W slots of bytes / W); whole rows
//   REDUCE_2SHOT      buf[r] = rank r's tensor, reduced tiles go to stg[r]; whole rows of W tiles
//   BROADCAST_2SHOT   buf[r] = rank r's tensor;             bytes = whole rows of W tiles
//   ALLGATHER/GATHER  buf[r] = rank r's input;              bytes = whole tiles
//   SCATTER           buf[root] = the root's flat list, chunk q at q * zstride; whole tiles
//   REDUCE_SCATTER    buf[r] = rank r's flat input, chunk q at q * zstride; bytes = whole tiles
//   ALLTOALL          buf[r] = rank r's flat input, chunk q at q * zstride; bytes = whole tiles
// and every call whose last phase reads user buffers ends with a departure barrier
// (no peer reads my buffer any more once my kernel is done, so the caller may
// overwrite or free it).
// Zero-copy gate. A gated launch (IpcCall::gate) is enqueued in stream order right away,
// before the host has exchanged the call's buffer records with the peers; the kernel's
// blocks wait (bounded spin) until the host's exchange thread publishes the slot: the
// peers' mapped buffers (ok = 1: the zero-copy protocol) or ok = 0 (some rank could not
// export or map: the same launch runs the staged protocol on its staging window).
// Slots live in pinned host memory, one per in-flight gated call (ring of kGateSlots).
struct GateSlot {
  uint64_t seq;              // == IpcCall::gate_seq once `ok` and `ptr` are valid (written last)
  uint32_t ok;
  uint32_t verdict;          // written by the kernel: how its device-side exchange ended (see ZcTable)
  uint64_t ptr[kMaxRanks];   // rank r's buffer of the call, mapped into this process (own: local)
};
constexpr int kGateSlots = 64;

// Device-side record exchange of a gated zero-copy launch (the steady state needs no host
// thread). Block 0's wave 0 pushes this rank's record {allocation id, offset} to every peer
// as flag-tagged 8-byte words (LL style, tag = a per-rank epoch of gated calls), looks the
// peers' ids up in this process's table of open mappings (ZcTable, pinned host memory the
// exchange thread maintains), votes (one more word per peer) and publishes the outcome
// for the kernel's other blocks in a resolved slot (same layout as GateSlot, in the
// uncached signal area): ok = 1 -> the peers' mapped buffers; ok = 2 -> some rank lacks a
// mapping: wait for the host gate as before (the exchange thread opens it).
constexpr int kZcTab = 32;  // mappings per peer the device can look up (>= PDCC_IPC_ZC_CACHE)
struct ZcTable {
  uint64_t id[kMaxRanks][kZcTab];    // allocation id (0 = free), written last
  uint64_t base[kMaxRanks][kZcTab];  // the mapping of that allocation in this process
};
constexpr uint64_t kZxNoExport = ~0ull;  // record id of a rank whose buffer could not be exported
// signal-area layout after the LL slots: per source rank 64 B (4 record words + 1 vote word),
// the epoch word, then the resolved slots
constexpr size_t kZxOffset = kLLOffset + 2 * (size_t)kMaxRanks * kLLSlotBytes;
constexpr size_t kZxSrcBytes = 64;
constexpr size_t kZxEpochOffset = kZxOffset + kMaxRanks * kZxSrcBytes;
constexpr size_t kZxResolvedOffset = kZxOffset + 1024;
constexpr size_t kZxBytes = 1024 + kGateSlots * sizeof(GateSlot);

// Dynamic zero-copy 2-shot all-reduce (IpcCall::dyn): instead of a fixed tile range per
// workgroup and a block-pairwise barrier between the phases, the workgroups of a rank claim
// work items from a counter in its signal area -- first "reduce my tiles of chunk i" (then
// publish chunk i's ready word), then "copy peer q's reduced tiles of chunk c" (after q's
// ready word for c) -- so fast workgroups take more items and a chunk's second phase starts
// as soon as its owner reduced it. The call ends when every rank's last workgroup has seen
// every peer's "done" word (no peer reads this rank's tensor any more).
// Own signal area after the exchange area: control words, per-source done words, then one
// ready word per chunk. Words hold a per-rank dyn-call epoch (never 0), compared for equality.
constexpr size_t kDynOffset = kZxOffset + kZxBytes;
// (u32 word indices from kDynOffset; the two counters every block hits sit 128 B apart)
constexpr size_t kDynCtlBytes = 512;  // IpcView::dctl
constexpr int kDynEpochWord = 0;   // epoch of this rank's last finished dyn call
constexpr int kDynClaimWord = 32;  // work-item counter of the running call (reset by its last block)
constexpr int kDynExitWord = 64;   // blocks of the running call that finished (reset by the last one)
constexpr size_t kDynDoneOffset = kDynOffset + 384;   // u32 per source rank: its last block's epoch
constexpr size_t kDynReadyOffset = kDynOffset + 512;  // u32 per chunk: the epoch its owner reduced it in
constexpr uint32_t kDynMaxChunks = 16384;
// rows (W tiles each) per chunk, at least (IpcCall::dyn_min_rows, PDCC_IPC_DYN_MIN_ROWS; 0 = this):
// every item is its own short pipeline (fill, drain, ready fence), so small items turn the dynamic
// protocol latency-bound -- 16 MiB at W = 2 on one GPU: 8-row items moved the data at half the static
// protocol's rate (profiles/r5/)
constexpr uint32_t kDynMinRows = 16;
constexpr size_t kDynBytes = 512 + (size_t)kDynMaxChunks * 4;
// rows per chunk of a dyn call: about `per` chunks per workgroup (IpcCall::dyn, PDCC_IPC_DYN), at least
// kDynMinRows rows, at most kDynMaxChunks chunks (a function of the call's shape and a group-wide
// setting only: identical on every rank)
__host__ __device__ inline uint32_t dyn_rows_per_chunk(size_t nrows, uint32_t grid, uint32_t per,
                                                      uint32_t min_rows = 0) {
  size_t k = nrows / ((size_t)(per ? per : 1) * (size_t)(grid ? grid : 1));
  const size_t lo_rows = min_rows ? min_rows : kDynMinRows;
  if (k < lo_rows) k = lo_rows;
  const size_t lo = (nrows + kDynMaxChunks - 1) / kDynMaxChunks;
  return (uint32_t)(k < lo ? lo : k);
}

template <template <class> class P>
struct IpcCallT {
  IpcColl coll;
  DType dtype;
  RedOp op;
  int root;
  int avg_div;
  int grid;                      // 0 = pick
  int grid_cap;                  // > 0: upper bound on the picked grid (PDCC_IPC_GRID; 256/W on shared devices)
  int zc;                        // 1 = zero-copy call (see above)
  size_t bytes;                  // payload bytes (per rank / per chunk, see above)
  size_t zstride;                // zero-copy chunked inputs: byte distance between chunks
  P<const void> in[kMaxRanks];   // local inputs: in[0] for single-tensor inputs, in[c] per chunk for lists
  P<void> out[kMaxRanks];        // local outputs: out[0] single, out[c] per chunk for lists
  // gated zero-copy launch (see GateSlot): the slot (device-mapped host memory), the value
  // its seq takes for this call, and this launch's byte offset inside every rank's buffer.
  // The view passed with a gated call is the staged one (buf = staging); ok = 1 swaps in
  // the slot's buffers (+ zoff) and runs the zero-copy protocol (zc = 1).
  P<const GateSlot> gate;
  uint64_t gate_seq;
  size_t zoff;
  // device-side exchange of a gated call (see ZcTable): this rank's record (allocation id,
  // or 0 = nothing to share, kZxNoExport = not exportable; offset in the allocation), its own
  // buffer, and the mapping table; ztab = null: wait for the host gate only
  uint64_t zx_tag;  // this launch's number (one ticket may take several launches): its resolved slot
  uint64_t zx_id;
  uint64_t zx_off;
  P<char> zx_self;
  P<const ZcTable> ztab;
  int dyn;  // > 0: a zero-copy ALLREDUCE_2SHOT runs the dynamic protocol with about `dyn` chunks per
            // workgroup (see kDynOffset); staged runs ignore it
  int dyn_min_rows;  // rows per dynamic-protocol item, at least (0 = kDynMinRows; group-wide setting)
};
using IpcCall = IpcCallT<RawPtr>;

// Bytes of staging needed for `call` (padded to tiles).
size_t ipc_staging_bytes(const IpcCall& call, int world);
// Bytes of the signal area every rank must allocate (uncached memory).
size_t ipc_signal_bytes();
hipError_t ipc_launch(const IpcView& view, const IpcCall& call, hipStream_t stream);

}  // namespace kern
}  // namespace pdcc
