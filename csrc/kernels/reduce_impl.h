// K1 (standalone N-way reduce) and the reduction family of the IPC collectives,
// templated on (dtype, op, #sources). Included once per dtype by reduce_<dt>.hip,
// which instantiates PDCC_REDUCE_DTYPE(<dt>) -- 8 small TUs that hipcc builds in
// parallel instead of one huge one.
#pragma once
#include <cstdlib>

#include "dev_common.h"

namespace pdcc {
namespace dev {

using kern::IpcCall;
using kern::IpcColl;
using kern::IpcView;

struct Ptrs8 {
  const char* p[kern::kMaxRanks];
  int chunked;  // K1 tile->block map: 0 = strided (block b: b, b+G, ...), 1 = contiguous run per block
  int nt;       // K1 destination stores non-temporal (global_store ... nt)
  int ntl;      // K1 source loads non-temporal
};

// LDS ring depth per source count: keeps DEPTH*NSRC*4KiB <= 64 KiB (2 blocks/CU). Two sources
// (W = 2) take 6 tiles (48 KiB): the bytes in flight per workgroup set the rate (Little's law),
// and at depth 4 the zero-copy all-reduce's reduce phase ran at 4.2-4.4 TB/s on one GPU where K1
// at the same workgroup budget and depth 6 reaches 6.3 (profiles/r4/ipc_phase_trace_w2.jsonl).
template <int NSRC>
struct DepthFor {
  static constexpr int value = NSRC <= 2 ? 6 : (NSRC <= 4 ? 3 : 2);
};

// --------------------------------------------------------------------------- K1
struct StridedMap {
  const char* const* s;
  char* d;
  size_t first, stride, ntiles;
  __device__ size_t count() const { return first < ntiles ? (ntiles - 1 - first) / stride + 1 : 0; }
  __device__ size_t tile(size_t i) const { return first + i * stride; }
  __device__ const char* src(int k, size_t i) const { return s[k] + tile(i) * kTile; }
  __device__ char* dst(size_t i) const { return d + tile(i) * kTile; }
  __device__ size_t valid(size_t) const { return kTile; }
};

// tail (< 4 KiB past the last full tile) with plain bounded loads
template <DType DT, RedOp OP, int NSRC>
__device__ __forceinline__ void reduce_tail(const char* const* s, char* d, size_t nbytes, int avg_div) {
  const size_t full = (nbytes / kTile) * kTile;
  const size_t off = full + (threadIdx.x >> 6) * kWaveBytes + (threadIdx.x & 63) * 16;
  if (off >= nbytes) return;
  const uint32_t lim = (uint32_t)(nbytes - off < 16 ? nbytes - off : 16);
  uint4 v[NSRC];
#pragma unroll
  for (int k = 0; k < NSRC; ++k)
    v[k] = lim == 16 ? *reinterpret_cast<const uint4*>(s[k] + off) : load_partial(s[k] + off, lim);
  const uint4 r = reduce_vec<DT, OP, NSRC>(v, avg_div);
  if (lim == 16) *reinterpret_cast<uint4*>(d + off) = r;
  else store_partial(d + off, r, lim);
}

__device__ __forceinline__ StridedMap k1_map(const Ptrs8& s, char* dst, size_t nbytes) {
  const size_t nt = nbytes / kTile;
  if (s.chunked) {
    const size_t per = (nt + gridDim.x - 1) / gridDim.x;
    const size_t b0 = blockIdx.x * per;
    return StridedMap{s.p, dst, b0, 1, b0 + per < nt ? b0 + per : nt};
  }
  return StridedMap{s.p, dst, blockIdx.x, gridDim.x, nt};
}

// K1 runs one 256-thread workgroup per CU (measured fastest for streaming), so
// it can afford a deeper LDS ring than the IPC kernels (which want 2 per CU).
template <int NSRC>
struct K1Deep {
  static constexpr int value = NSRC <= 2 ? 6 : (NSRC <= 4 ? 4 : 3);
};

template <DType DT, RedOp OP, int NSRC, int D>
__global__ void __launch_bounds__(256) k1_reduce_lds(Ptrs8 srcs, char* dst, size_t nbytes, int avg_div) {
  __shared__ __attribute__((aligned(16))) char lds[PipeLds<NSRC, D>::kBytes];
  const StridedMap m = k1_map(srcs, dst, nbytes);
  if (srcs.ntl) pipe_run<DT, OP, NSRC, D, StridedMap, 1, true, true>(lds, m, avg_div);
  else if (srcs.nt) pipe_run<DT, OP, NSRC, D, StridedMap, 1, true>(lds, m, avg_div);
  else pipe_run<DT, OP, NSRC, D>(lds, m, avg_div);
  if (blockIdx.x == gridDim.x - 1) reduce_tail<DT, OP, NSRC>(srcs.p, dst, nbytes, avg_div);
}

template <DType DT, RedOp OP, int NSRC>
__global__ void __launch_bounds__(256) k1_reduce_regs(Ptrs8 srcs, char* dst, size_t nbytes, int avg_div) {
  const StridedMap m = k1_map(srcs, dst, nbytes);
  if (srcs.ntl) pipe_run_regs<DT, OP, NSRC, (NSRC <= 2 ? 4 : 2), StridedMap, true, true>(m, avg_div);
  else if (srcs.nt) pipe_run_regs<DT, OP, NSRC, (NSRC <= 2 ? 4 : 2), StridedMap, true>(m, avg_div);
  else pipe_run_regs<DT, OP, NSRC, (NSRC <= 2 ? 4 : 2)>(m, avg_div);
  if (blockIdx.x == gridDim.x - 1) reduce_tail<DT, OP, NSRC>(srcs.p, dst, nbytes, avg_div);
}

// Streaming K1 (mode bit 2): no software pipeline and no loop -- each workgroup reduces one
// slab of V 4 KiB tiles per source, every load issued before the first reduce, and the grid
// covers the whole buffer (the shape of torch's elementwise kernels: the dispatcher keeps
// every CU full of short workgroups, so the bytes in flight come from occupancy). NTL:
// non-temporal source loads (read once), NT: non-temporal stores.
template <int NSRC>
struct StreamV {
  static constexpr int value = NSRC <= 2 ? 4 : (NSRC <= 4 ? 2 : 1);
};

template <DType DT, RedOp OP, int NSRC, bool NT, bool NTL>
__global__ void __launch_bounds__(256) k1_reduce_stream(Ptrs8 srcs, char* dst, size_t nbytes, int avg_div) {
  constexpr int V = StreamV<NSRC>::value;
  const size_t base = (size_t)blockIdx.x * (V * kTile) + threadIdx.x * 16;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  if ((size_t)(blockIdx.x + 1) * (V * kTile) <= nbytes) {
    uint4 v[V][NSRC];
#pragma unroll
    for (int u = 0; u < V; ++u)
#pragma unroll
      for (int k = 0; k < NSRC; ++k) {
        const char* p = srcs.p[k] + base + u * kTile;
        if constexpr (NTL) {
          const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
          v[u][k] = make_uint4(x[0], x[1], x[2], x[3]);
        } else {
          v[u][k] = *reinterpret_cast<const uint4*>(p);
        }
      }
#pragma unroll
    for (int u = 0; u < V; ++u) store16<NT>(dst + base + u * kTile, reduce_vec<DT, OP, NSRC>(v[u], avg_div));
    return;
  }
  // the last (partial) slab: bounded loads
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const size_t off = base + u * kTile;
    if (off >= nbytes) return;
    const uint32_t lim = (uint32_t)(nbytes - off < 16 ? nbytes - off : 16);
    uint4 v[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k)
      v[k] = lim == 16 ? *reinterpret_cast<const uint4*>(srcs.p[k] + off) : load_partial(srcs.p[k] + off, lim);
    const uint4 r = reduce_vec<DT, OP, NSRC>(v, avg_div);
    if (lim == 16) *reinterpret_cast<uint4*>(dst + off) = r;
    else store_partial(dst + off, r, lim);
  }
}

// ------------------------------------------------------------- IPC reductions
// Tile partitions (MUST be identical on every rank: a block only ever reads
// tiles that the same-index block of each peer staged, which is what makes the
// block-pairwise barrier sufficient):
//   1-shot / reduce-scatter: tile t (within a chunk) -> block t % G
//   2-shot: tile t -> owner t % W, row t / W -> block row % G
__device__ __forceinline__ size_t pad_tiles(size_t b) { return (b + kTile - 1) / kTile * kTile; }

template <int W>
struct AllSrcMap {  // reduce tile t of every rank's staging (+ chunk offset)
  const DView* v;
  size_t base;   // byte offset of the chunk inside each staging buffer
  char* d;       // destination (user output or own staging)
  size_t dlim;   // bytes writable at d (user: payload bytes; staging: padded)
  size_t first, stride, ntiles;
  __device__ size_t count() const { return first < ntiles ? (ntiles - 1 - first) / stride + 1 : 0; }
  __device__ size_t tile(size_t i) const { return first + i * stride; }
  __device__ const char* src(int k, size_t i) const { return v->buf[k] + base + tile(i) * kTile; }
  __device__ char* dst(size_t i) const { return d + tile(i) * kTile; }
  __device__ size_t valid(size_t i) const {
    const size_t o = tile(i) * kTile;
    return o >= dlim ? 0 : (dlim - o < (size_t)kTile ? dlim - o : (size_t)kTile);
  }
};

struct OneSrcMap {  // copy tile t from one buffer to another
  const char* s;
  char* d;
  size_t dlim;
  size_t first, stride, ntiles;
  __device__ size_t count() const { return first < ntiles ? (ntiles - 1 - first) / stride + 1 : 0; }
  __device__ size_t tile(size_t i) const { return first + i * stride; }
  __device__ const char* src(int, size_t i) const { return s + tile(i) * kTile; }
  __device__ char* dst(size_t i) const { return d + tile(i) * kTile; }
  __device__ size_t valid(size_t i) const {
    const size_t o = tile(i) * kTile;
    return o >= dlim ? 0 : (dlim - o < (size_t)kTile ? dlim - o : (size_t)kTile);
  }
};

constexpr int kCopyDepth = 4;

// The zero-copy all-reduce's pipes (non-temporal loads / stores in either phase measured as noise,
// profiles/r5/nt_and_dyn_items_ab.jsonl: plain cached pipes).
// The gather phase runs in the reduce kernels, whose LDS is sized for the reduce pipe (W x
// DepthFor<W> tiles, >= 32 KiB for every W): the copy keeps 8 tiles in flight instead of 4 there
// (Little's law: the bytes in flight per workgroup set a streaming copy's rate).
constexpr int kZcCopyDepth = 8;
static_assert(2 * DepthFor<2>::value >= kZcCopyDepth && 3 * DepthFor<3>::value >= kZcCopyDepth &&
                  5 * DepthFor<5>::value >= kZcCopyDepth,
              "the reduce kernels' LDS must hold the gather phase's ring");
template <class Map>
__device__ __forceinline__ void zc_copy_pipe(char* lds, const Map& m) {
  ipc_pipe<DType::U8, RedOp::COPY, 1, kZcCopyDepth>(lds, m, 1);
}
template <DType DT, RedOp OP, int NSRC, int DEPTH, class Map>
__device__ __forceinline__ void zc_reduce_pipe(char* lds, const Map& m, int avg_div) {
  ipc_pipe_once<DT, OP, NSRC, DEPTH>(lds, m, avg_div);
}

// Owner-interleaved maps. A block's pipeline keeps DEPTH tiles in flight; if all
// of them (and, with blocks in lockstep, all blocks of the rank) pull from the
// same peer, a rank drives ONE xGMI link at a time. These maps rotate the owner
// per item, per row and per block, so in-flight tiles spread over every peer.

// 2-shot phase 2: tiles q + W*r of rows r = first + stride*k (owner q = rank whose
// staging holds the reduced tile). A partial last row reads staging padding
// (staging is sized to whole rows, see kern::ipc_staging_bytes); valid() = 0 there.
template <int W>
struct OwnerRowMap {
  const gp<char>* bufs;  // the owners' buffers (IpcView::buf, or ::stg for a zero-copy reduce)
  size_t poff;  // offset of this call in the staging buffers (0: one buffer)
  char* d;
  size_t dlim;
  uint32_t rot;
  size_t first, stride, nrows;
  __device__ size_t count() const { return first < nrows ? ((nrows - 1 - first) / stride + 1) * W : 0; }
  __device__ size_t tile(size_t i, int& q) const {
    const uint32_t k = (uint32_t)i / W, j = (uint32_t)i - k * W;
    q = (int)((rot + j + k) % W);
    return (size_t)q + (size_t)W * (first + stride * k);
  }
  __device__ const char* src(int, size_t i) const {
    int q;
    const size_t t = tile(i, q);
    return bufs[q] + poff + t * kTile;
  }
  __device__ char* dst(size_t i) const {
    int q;
    return d + tile(i, q) * kTile;
  }
  __device__ size_t valid(size_t i) const {
    int q;
    const size_t o = tile(i, q) * kTile;
    return o >= dlim ? 0 : (dlim - o < (size_t)kTile ? dlim - o : (size_t)kTile);
  }
};

// Zero-copy 2-shot phase 2 (IpcCall::zc): the W-1 tiles of each row that OTHER ranks
// own -- the own tiles were reduced (or fetched) in place in phase 1. Rows first +
// stride*k, owners rotated per item, row and block like OwnerRowMap. Rows are whole.
template <int W>
struct PeerRowMap {
  const DView* v;
  char* d;
  uint32_t rot;
  size_t first, stride, nrows;
  __device__ size_t count() const { return first < nrows ? ((nrows - 1 - first) / stride + 1) * (W - 1) : 0; }
  __device__ size_t tile(size_t i, int& q) const {
    const uint32_t k = (uint32_t)i / (W - 1), j = (uint32_t)i - k * (W - 1);
    q = (v->rank + 1 + (int)((rot + j + k) % (W - 1))) % W;
    return (size_t)q + (size_t)W * (first + stride * k);
  }
  __device__ const char* src(int, size_t i) const {
    int q;
    const size_t t = tile(i, q);
    return v->buf[q] + t * kTile;
  }
  __device__ char* dst(size_t i) const {
    int q;
    return d + tile(i, q) * kTile;
  }
  __device__ size_t valid(size_t) const { return kTile; }
};

// Push all-reduce phase 1: my tile of every row that another rank q owns goes to
// slot `me` of q's staging (slot s, row r at (s * nrows + r) * kTile). Local reads,
// remote writes; owners rotated per item, row and block like PeerRowMap.
template <int W>
struct PushMap {
  const char* mine;   // my tensor
  const gp<char>* stgs;  // every rank's staging (IpcView::stg)
  int me;
  uint32_t rot;
  size_t first, stride, nrows;
  __device__ size_t count() const { return first < nrows ? ((nrows - 1 - first) / stride + 1) * (W - 1) : 0; }
  __device__ size_t row(size_t i, int& q) const {
    const uint32_t k = (uint32_t)i / (W - 1), j = (uint32_t)i - k * (W - 1);
    q = (me + 1 + (int)((rot + j + k) % (W - 1))) % W;
    return first + stride * k;
  }
  __device__ const char* src(int, size_t i) const {
    int q;
    const size_t r = row(i, q);
    return mine + ((size_t)q + (size_t)W * r) * kTile;
  }
  __device__ char* dst(size_t i) const {
    int q;
    const size_t r = row(i, q);
    return stgs[q] + ((size_t)me * nrows + r) * kTile;
  }
  __device__ size_t valid(size_t) const { return kTile; }
};

// Push all-reduce phase 2: my owned tile of row r reduced from the W-1 staged
// slots and my own tensor (sources in rank order: every rank's copy is the same
// owner's bits), stored into every rank's tensor (destination j = rank j).
template <int W>
struct PushReduceMap {
  const gp<char>* bufs;  // every rank's tensor (IpcView::buf)
  const char* stg;    // my staging (slot s, row r at (s * nrows + r) * kTile)
  int me;
  size_t first, stride, nrows;
  __device__ size_t count() const { return first < nrows ? (nrows - 1 - first) / stride + 1 : 0; }
  __device__ size_t row(size_t i) const { return first + stride * i; }
  __device__ const char* src(int k, size_t i) const {
    const size_t r = row(i);
    const size_t slot = ((size_t)k * nrows + r) * kTile, own = ((size_t)me + (size_t)W * r) * kTile;
    return k == me ? bufs[me] + own : stg + slot;
  }
  __device__ char* dst(int j, size_t i) const { return bufs[j] + ((size_t)me + (size_t)W * row(i)) * kTile; }
  __device__ size_t valid(size_t) const { return kTile; }
};

// all-gather / gather / all-to-all: (tile t of this block, source rank q) pairs;
// source q's tile lives at v->buf[q] + sbase + t*kTile and lands in out[q].
template <int W>
struct PeerTileMap {
  const DView* v;
  const DCall* c;
  size_t sbase;  // offset of the chunk inside each staging buffer
  size_t dlim;
  uint32_t rot;
  size_t first, stride, ntiles;
  __device__ size_t count() const { return first < ntiles ? ((ntiles - 1 - first) / stride + 1) * W : 0; }
  __device__ size_t tile(size_t i, int& q) const {
    const uint32_t k = (uint32_t)i / W, j = (uint32_t)i - k * W;
    q = (int)((rot + j + k) % W);
    return first + stride * k;
  }
  __device__ const char* src(int, size_t i) const {
    int q;
    const size_t t = tile(i, q);
    return v->buf[q] + sbase + t * kTile;
  }
  __device__ char* dst(size_t i) const {
    int q;
    const size_t t = tile(i, q);
    return (char*)c->out[q] + t * kTile;
  }
  __device__ size_t valid(size_t i) const {
    int q;
    const size_t o = tile(i, q) * kTile;
    return o >= dlim ? 0 : (dlim - o < (size_t)kTile ? dlim - o : (size_t)kTile);
  }
};

// ---- dynamic zero-copy 2-shot all-reduce (IpcCall::dyn, layout at kern::kDynOffset) --------
__device__ __forceinline__ uint32_t* dyn_words(const DView& v, int rank, size_t off) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>((uint32_t*)v.flags[rank]) + off);
}

// Thread 0: bounded poll until *w == want (system scope); false on timeout (error word set) or
// when the group was aborted / another block timed out, so the grid always drains.
__device__ __forceinline__ bool dyn_wait(const DView& v, const uint32_t* w, uint32_t want, uint32_t code) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 1;; ++it) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == want) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks) {
      __hip_atomic_store(static_cast<uint32_t*>(v.err), code | (uint32_t)v.rank, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    if ((it & 255u) == 0 &&
        __hip_atomic_load(static_cast<uint32_t*>(v.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
      return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// Rows of W tiles (tile q + W*r belongs to rank q), K rows per chunk, nc chunks. Work items,
// claimed in order from this rank's counter: [0, nc) reduce my tiles of chunk i from every
// rank's tensor, in place (read-once loads), then publish ready[i] = dep; [nc, W*nc) copy
// peer q's tiles of chunk c into my tensor once q's ready[c] == dep (peers rotated per chunk,
// so the items in flight spread over every xGMI link). Every phase-1 item of a rank is claimed
// before any of its phase-2 items and a phase-1 item waits for nothing, so every ready word a
// phase-2 item waits for is eventually published: no cycle. Overwrites are safe: the peer
// positions I write in phase 2 (tile q + W*r of MY tensor) were read by q in its phase 1 of
// chunk c, which q finished before publishing ready[c]; my own tiles are written in phase 1
// only, and peers read them after my ready word.
// This rank's control words (claim / exit counters, epoch): ordinary device memory (IpcView::dctl).
__device__ __forceinline__ uint32_t* dyn_ctl(const DView& v) { return (uint32_t*)v.dctl; }

// This call's epoch: the previous dyn call's last block stored its own (never 0).
__device__ __forceinline__ uint32_t dyn_epoch(const DView& v, const PhaseTrace* tr) {
  __shared__ uint32_t s_dep;
  if (threadIdx.x == 0) {
    const uint64_t t0 = tr->now();
    const uint32_t e =
        __hip_atomic_load(dyn_ctl(v) + kern::kDynEpochWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_dep = e ? e : 1u;
    tr->add(23, t0);
  }
  __syncthreads();
  return s_dep;
}

// Claim loop: item(it) for every item this block claims, it < total. Items [0, 2G) are static --
// block b runs b, then b + G -- and only later items are claimed, as 2G + the counter: every block
// hitting one word at launch serialises at the memory side (round 4 measured a fixed ~17 us per
// call on the uncached word at any size, round 5's trace: profiles/r5/), and a call with at most 2G
// items claims nothing at all. Thread 0 claims one item ahead (from its second item on), so the
// atomic's round trip overlaps the current item. Claims are monotonic (b < b + G < 2G <= 2G + k): a
// block never holds an earlier item behind a later one, and a block's earlier items are always
// smaller, so every phase-1 item (index < nc, waiting for nothing) is reached without a wait.
// (b, G: this data block's index and the number of data blocks, see xchg_blocks)
template <class Item>
__device__ __forceinline__ void dyn_claim_loop(const DView& v, uint32_t total, const PhaseTrace* tr, uint32_t b,
                                               uint32_t G, Item&& item) {
  __shared__ uint32_t s_item;
  uint32_t* const claim = dyn_ctl(v) + kern::kDynClaimWord;
  const uint32_t base = 2u * G;  // first claimed item
  uint32_t next = b;
  for (;;) {
    const uint64_t t0 = tr->now();
    if (threadIdx.x == 0) s_item = next;  // (waits for the claim's return)
    __syncthreads();
    const uint32_t it = s_item;
    __syncthreads();  // (s_item is rewritten by the next claim)
    if (threadIdx.x == 0) tr->add(16, t0);
    if (it >= total) break;
    if (threadIdx.x == 0) {
      if (it < G) next = it + G;  // the second static item
      else next = total > base ? base + __hip_atomic_fetch_add(claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : total;
      tr->count(20);
    }
    item(it);
  }
}

// Departure: once every block of mine is done (exit counter), the last one tells every peer, waits
// until every peer's blocks are done too (nobody reads my tensor any more), then resets the counters
// and publishes this call's epoch for the next dyn call.
__device__ __forceinline__ void dyn_depart(const DView& v, uint32_t dep, bool ok, const PhaseTrace* tr, uint32_t G) {
  const int me = v.rank, W = v.world;
  uint32_t* const ctl = dyn_ctl(v);
  const uint64_t t0 = tr->now();
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctl + kern::kDynExitWord, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == G - 1) {
      for (int q = 0; q < W; ++q)
        if (q != me)
          __hip_atomic_store(dyn_words(v, q, kern::kDynDoneOffset) + me, dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint32_t* const done = dyn_words(v, me, kern::kDynDoneOffset);
      for (int q = 0; q < W; ++q)
        if (q != me && ok) ok = dyn_wait(v, done + q, dep, 0x900u);
      __hip_atomic_store(ctl + kern::kDynClaimWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl + kern::kDynExitWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl + kern::kDynEpochWord, dep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      tr->count(22);
    }
    tr->add(19, t0);
  }
}

template <DType DT, RedOp OP, int W>
__device__ __forceinline__ void ipc_allreduce_dyn(const DView& v, const DCall& c, char* lds, const PhaseTrace* tr) {
  constexpr int D = DepthFor<W>::value;
  const int me = v.rank;
  const uint32_t xb = xchg_blocks(c), G = gridDim.x - xb, b = blockIdx.x - xb;
  const size_t nrows = c.bytes / kTile / W;
  const uint32_t K = kern::dyn_rows_per_chunk(nrows, G, (uint32_t)c.dyn, (uint32_t)c.dyn_min_rows);
  const uint32_t nc = (uint32_t)((nrows + K - 1) / K);
  uint32_t* const ready = dyn_words(v, me, kern::kDynReadyOffset);
  __shared__ uint32_t s_ok;
  const uint32_t dep = dyn_epoch(v, tr);
  bool ok = true;
  dyn_claim_loop(v, nc * W, tr, b, G, [&](uint32_t it) {
    if (it < nc) {
      const size_t r0 = (size_t)it * K, r1 = r0 + K < nrows ? r0 + K : nrows;
      const AllSrcMap<W> m{&v, 0, v.buf[me], c.bytes, (size_t)me + W * r0, W, W * r1};
      zc_reduce_pipe<DT, OP, W, D>(lds, m, c.avg_div);
      const uint64_t t0 = tr->now();
      drain_vm();  // every wave's stores and loads (a peer overwrites what I read once it sees ready)
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back L2 dirty lines
        drain_vm();
        __hip_atomic_store(ready + it, dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        tr->add(17, t0);
        tr->count(21);
      }
    } else {
      const uint32_t j = it - nc, cc = j / (W - 1), k = j - cc * (W - 1);
      const int q = (me + 1 + (int)((k + cc) % (W - 1))) % W;
      if (threadIdx.x == 0) {
        const uint64_t t0 = tr->now();
        s_ok = ok && dyn_wait(v, dyn_words(v, q, kern::kDynReadyOffset) + cc, dep, 0xA00u) ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale L1/L2 lines
        drain_vm();
        tr->add(18, t0);
      }
      __syncthreads();
      ok = s_ok != 0;
      __syncthreads();
      if (ok) {
        const size_t r0 = (size_t)cc * K, r1 = r0 + K < nrows ? r0 + K : nrows;
        const OneSrcMap m{v.buf[q], v.buf[me], c.bytes, (size_t)q + W * r0, W, W * r1};
        zc_copy_pipe(lds, m);
      }
    }
  });
  dyn_depart(v, dep, ok, tr, G);
}

// Dynamic zero-copy reduce-scatter (IpcCall::dyn): my output chunk in items of K tiles, each reduced
// from every rank's flat input (chunk `me` at me * zstride) -- one phase, no ready words; the
// departure keeps every peer's input alive until the last reader is done.
template <DType DT, RedOp OP, int W>
__device__ __forceinline__ void ipc_reduce_scatter_dyn(const DView& v, const DCall& c, char* lds,
                                                       const PhaseTrace* tr) {
  constexpr int D = DepthFor<W>::value;
  const uint32_t xb = xchg_blocks(c), G = gridDim.x - xb, b = blockIdx.x - xb;
  const size_t nt = c.bytes / kTile;
  const uint32_t K = kern::dyn_rows_per_chunk(nt, G, (uint32_t)c.dyn, (uint32_t)c.dyn_min_rows);
  const uint32_t nc = (uint32_t)((nt + K - 1) / K);
  const uint32_t dep = dyn_epoch(v, tr);
  dyn_claim_loop(v, nc, tr, b, G, [&](uint32_t it) {
    const size_t t0 = (size_t)it * K, t1 = t0 + K < nt ? t0 + K : nt;
    const AllSrcMap<W> m{&v, (size_t)v.rank * c.zstride, (char*)c.out[0], c.bytes, t0, 1, t1};
    ipc_pipe_once<DT, OP, W, D>(lds, m, c.avg_div);
  });
  dyn_depart(v, dep, true, tr, G);
}

// Zero-copy reductions (IpcCall::zc): every rank's user buffer is read in place.
// The arrival barrier is a data barrier here -- it hands over each rank's input,
// written by the kernels before this one -- and a departure barrier ends the call:
// once it passes, no peer reads this rank's buffer any more (the caller may reuse it).
// Phase 1 of the all-reduce writes the reduced own tiles in place: peers only ever
// read tiles they own there, and those are not written by this rank.
template <DType DT, RedOp OP, int W>
__device__ __forceinline__ void ipc_reduce_zc(const DView& v, const DCall& c, char* lds, const PhaseTrace tr,
                                              uint32_t ep) {
  constexpr int D = DepthFor<W>::value;
  const size_t G = gridDim.x - xchg_blocks(c), b = blockIdx.x - xchg_blocks(c);  // the data blocks
  const int me = v.rank;
  const size_t nt = c.bytes / kTile;
  block_barrier(v, ep, &tr);
  tr.mark(2);
  tr.mark(4);
  if (c.coll == IpcColl::ALLREDUCE_2SHOT && c.dyn) {
    ipc_allreduce_dyn<DT, OP, W>(v, c, lds, &tr);
    tr.mark(5);
    return;
  }
  if (c.coll == IpcColl::REDUCE_SCATTER && c.dyn) {
    ipc_reduce_scatter_dyn<DT, OP, W>(v, c, lds, &tr);
    tr.mark(5);
    return;
  }
  if (c.coll == IpcColl::ALLREDUCE_2SHOT) {
    {  // phase 1: my owned tiles (t % W == me) from every rank's buffer, reduced in place
      const AllSrcMap<W> m{&v, 0, v.buf[me], c.bytes, (size_t)me + W * b, W * G, nt};
      zc_reduce_pipe<DT, OP, W, D>(lds, m, c.avg_div);
    }
    tr.mark(5);
    block_barrier(v, ep + 2u);
    tr.mark(6);
    {  // phase 2: the other owners' reduced tiles
      const PeerRowMap<W> m{&v, v.buf[me], (uint32_t)b, b, G, nt / W};
      zc_copy_pipe(lds, m);
    }
  } else if (c.coll == IpcColl::ALLREDUCE_PUSH) {
    // every remote access is a write (xGMI writes are posted; reads wait a round trip)
    const size_t nrows = nt / W;
    {  // phase 1: my tiles to their owners' staging slots
      const PushMap<W> m{v.buf[me], v.stg, me, (uint32_t)b, b, G, nrows};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
    }
    tr.mark(5);
    block_barrier(v, ep + 2u);
    tr.mark(6);
    {  // phase 2: reduce my owned tiles, store the result into every rank's tensor
      const PushReduceMap<W> m{v.buf, v.stg[me], me, b, G, nrows};
      ipc_pipe<DT, OP, W, D, W>(lds, m, c.avg_div);
    }
    block_barrier(v, ep + 3u);  // departure with data: the peers' results are in my tensor
    return;
  } else if (c.coll == IpcColl::REDUCE_2SHOT) {
    // rooted: the owners reduce from every rank's tensor into their STAGING (non-root
    // tensors stay untouched), the root pulls every owner's tiles from there. After the
    // data barrier nobody reads a user tensor any more: no departure barrier (staging
    // reuse is guarded by the next call's arrival barrier).
    {
      const AllSrcMap<W> m{&v, 0, v.stg[me], c.bytes, (size_t)me + W * b, W * G, nt};
      ipc_pipe_once<DT, OP, W, D>(lds, m, c.avg_div);
    }
    tr.mark(5);
    block_barrier(v, ep + 2u);
    tr.mark(6);
    if (me == c.root) {
      const OwnerRowMap<W> m{v.stg, 0, v.buf[me], c.bytes, (uint32_t)(me + b), b, G, nt / W};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
    }
    return;
  } else if (c.coll == IpcColl::REDUCE_SCATTER) {
    const AllSrcMap<W> m{&v, (size_t)me * c.zstride, (char*)c.out[0], c.bytes, b, G, nt};
    ipc_pipe_once<DT, OP, W, D>(lds, m, c.avg_div);
    tr.mark(5);
  }
  block_barrier<false>(v, ep + 3u);  // departure
}

template <DType DT, RedOp OP, int W>
__device__ __forceinline__ void ipc_reduce_body(const DView& v, const DCall& c, char* lds, const PhaseTrace tr,
                                                uint32_t seq) {
  constexpr int D = DepthFor<W>::value;
  const size_t G = gridDim.x - xchg_blocks(c), b = blockIdx.x - xchg_blocks(c);  // the data blocks
  const int me = v.rank;
  tr.seq(seq);
  tr.mark(12);
  const uint32_t ep = seq * kern::kEpochsPerCall, ph0 = ep + 1u, ph1 = ep + 2u;
  if (c.zc) {
    ipc_reduce_zc<DT, OP, W>(v, c, lds, tr, ep);
    return;
  }
  block_barrier<false>(v, ep);  // arrival: every peer's previous call is over
  tr.mark(2);
  const size_t poff = 0;        // single staging buffer (the arrival barrier guards reuse)
  char* mine = v.buf[me];
  const size_t nt = pad_tiles(c.bytes) / kTile;

  switch (c.coll) {
    case IpcColl::ALLREDUCE_1SHOT:
    case IpcColl::REDUCE_1SHOT: {
      stage_tiles((const char*)c.in[0], mine, c.bytes, b, G, nt);
      tr.mark(3);
      block_barrier(v, ph0);
      tr.mark(4);
      if (c.coll == IpcColl::REDUCE_1SHOT && me != c.root) return;
      const AllSrcMap<W> m{&v, poff, (char*)c.out[0], c.bytes, b, G, nt};
      ipc_pipe<DT, OP, W, D>(lds, m, c.avg_div);
      tr.mark(5);
      return;
    }
    case IpcColl::ALLREDUCE_2SHOT:
    case IpcColl::REDUCE_2SHOT: {
      // stage the rows of this block: tiles q + W*(b + G*k) for every owner q
      for (int q = 0; q < W; ++q) stage_tiles((const char*)c.in[0], mine, c.bytes, q + W * b, W * G, nt);
      tr.mark(3);
      block_barrier(v, ph0);
      tr.mark(4);
      // phase 1: reduce my owned tiles from every rank, in place into my staging
      {
        const AllSrcMap<W> m{&v, poff, mine, nt * kTile, me + W * b, W * G, nt};
        ipc_pipe<DT, OP, W, D>(lds, m, c.avg_div);
      }
      tr.mark(5);
      block_barrier(v, ph1);
      tr.mark(6);
      if (c.coll == IpcColl::REDUCE_2SHOT && me != c.root) return;
      // phase 2: pull every owner's reduced tiles, owners interleaved (all links at once)
      {
        const OwnerRowMap<W> m{v.buf, poff, (char*)c.out[0], c.bytes, (uint32_t)(me + b), b, G, (nt + W - 1) / W};
        ipc_pipe<DT, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      return;
    }
    case IpcColl::REDUCE_SCATTER: {
      const size_t cpad = pad_tiles(c.bytes);
      for (int q = 0; q < W; ++q) stage_tiles((const char*)c.in[q], mine + q * cpad, c.bytes, b, G, nt);
      tr.mark(3);
      block_barrier(v, ph0);
      tr.mark(4);
      const AllSrcMap<W> m{&v, poff + me * cpad, (char*)c.out[0], c.bytes, b, G, nt};
      ipc_pipe<DT, OP, W, D>(lds, m, c.avg_div);
      tr.mark(5);
      return;
    }
    default:
      return;
  }
}

template <DType DT, RedOp OP, int W>
__global__ void __launch_bounds__(256) k_ipc_reduce(IpcView v, IpcCall c) {
  __shared__ __attribute__((aligned(16))) char lds[PipeLds<W, DepthFor<W>::value>::kBytes];
  __shared__ DView sv;
  __shared__ DCall sc;
  const uint32_t xb = xchg_blocks(c);
  PhaseTrace tr(v, xb);
  if (xb && blockIdx.x == 0) {  // the exchange block (see xchg_blocks)
    if (threadIdx.x < 64) zx_resolve(v, c, tr);
    tr.finish_exchange(v);
    zx_publish_verdict(c);
    return;
  }
  // The block's call number is taken at entry, before the arguments are staged.
  const uint32_t seq = block_seq(v, block_seq_load(v));
  stage_args(v, c, sv, sc, tr);  // (a gated zero-copy launch waits for its buffers here)
  if (c.gate) tr.mark(3);    // gate passed (zero-copy calls do not stage: [3] is free there)
  ipc_reduce_body<DT, OP, W>(sv, sc, lds, tr, seq);
  tr.finish(v);
}

// ----------------------------------------------------------------------------
// LL all-reduce (IpcColl::ALLREDUCE_LL, payload <= kLLMaxBytes): one 8-byte line of the
// payload per thread. The thread pushes its line to every peer as two 8-byte words
// {4 data bytes, epoch} (system-scope stores into the peer's uncached LL slot, single-copy
// atomic), then polls its own slots until every peer's two words carry this call's epoch,
// reduces the W lines in rank order (the same bits on every rank) and writes the result.
// No staging copy and no barrier: the slot parity alternates per call, and a rank can only
// be at call e after receiving every peer's words of call e-1, which peers push only after
// their call e-2 -- the last reader of this parity -- has finished.
__device__ __forceinline__ uint64_t* ll_slot(uint32_t* sig, uint32_t parity, int src) {
  return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(sig) + kern::kLLOffset +
                                     ((size_t)parity * kern::kMaxRanks + (size_t)src) * kern::kLLSlotBytes);
}

// (byte-wise where the line is short or not 8-B aligned: views of one flat tensor at 4 B offsets are
// used in place, prep_in's any_align)
__device__ __forceinline__ bool ll_whole(const char* p, size_t off, size_t nbytes) {
  return off + 8 <= nbytes && (reinterpret_cast<uintptr_t>(p + off) & 7u) == 0;
}

__device__ __forceinline__ uint2 ll_load(const char* p, size_t off, size_t nbytes) {
  if (ll_whole(p, off, nbytes)) return *reinterpret_cast<const uint2*>(p + off);
  uint32_t w[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (off + k < nbytes) w[k >> 2] |= (uint32_t)(uint8_t)p[off + k] << (8 * (k & 3));
  return make_uint2(w[0], w[1]);
}

__device__ __forceinline__ void ll_store(char* p, size_t off, size_t nbytes, uint32_t x, uint32_t y) {
  if (ll_whole(p, off, nbytes)) {
    *reinterpret_cast<uint2*>(p + off) = make_uint2(x, y);
    return;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (off + k < nbytes) p[off + k] = (char)(((k < 4 ? x : y) >> (8 * (k & 3))) & 0xffu);
}

// The call's epoch (every block reads the last finished LL call's + 1) and its end (the
// block that finishes last publishes the epoch for the next LL call on this rank).
__device__ __forceinline__ uint32_t ll_begin(const IpcView& v) {
  __shared__ uint32_t s_ep;
  if (threadIdx.x == 0)
    s_ep = __hip_atomic_load(v.counters + kern::kMaxBlocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  return s_ep;
}

__device__ __forceinline__ void ll_end(const IpcView& v, uint32_t ep) {
  uint32_t* const ctl = v.counters + kern::kMaxBlocks;  // == own signal area + kLLCtlWord
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = __hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// line i of this rank's payload -> slot (parity, me) of every peer, as two {data, epoch} words
template <int W>
__device__ __forceinline__ void ll_push(const IpcView& v, uint32_t par, uint64_t tag, size_t i, uint2 d) {
#pragma unroll
  for (int q = 0; q < W; ++q) {
    if (q == v.rank) continue;
    uint64_t* dst = ll_slot(v.flags[q], par, v.rank) + 2 * i;
    __hip_atomic_store(dst, tag | d.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1, tag | d.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// wait for line i of peer q in my slot (parity, q); bounded (error word), stops on abort
__device__ __forceinline__ uint2 ll_poll(const IpcView& v, uint32_t par, uint32_t ep, int q, size_t i, uint64_t t0,
                                         bool& live) {
  const uint64_t* p = ll_slot(v.flags[v.rank], par, q) + 2 * i;
  uint64_t a = 0, b = 0;
  for (uint32_t it = 1; live; ++it) {
    a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((uint32_t)(a >> 32) == ep && (uint32_t)(b >> 32) == ep) break;
    if ((it & 63u) == 0) {  // bounded spin; a host abort or another thread's timeout stops it too
      if (__builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks) {
        __hip_atomic_store(v.err, 0x300u | (uint32_t)v.rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        live = false;
      } else if (__hip_atomic_load(v.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        live = false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return make_uint2((uint32_t)a, (uint32_t)b);
}

template <DType DT, RedOp OP, int W>
__global__ void __launch_bounds__(256) k_ll_allreduce(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const size_t lines = (c.bytes + 7) / 8;
  const char* in = static_cast<const char*>(c.in[0]);
  char* out = static_cast<char*>(c.out[0]);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 d = ll_load(in, i * 8, c.bytes);
    ll_push<W>(v, par, tag, i, d);
    uint4 src[W];
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 x = q == v.rank ? d : ll_poll(v, par, ep, q, i, t0, live);
      src[q] = make_uint4(x.x, x.y, 0u, 0u);
    }
    const uint4 r = reduce_vec<DT, OP, W>(src, c.avg_div);  // rank order: the same bits on every rank
    ll_store(out, i * 8, c.bytes, r.x, r.y);
  }
  ll_end(v, ep);
}

// LL all-gather (IpcColl::ALLGATHER_LL, per-rank payload <= kLLMaxBytes): the same pushes,
// every peer's lines written straight into its output (list entry or flat slice).
template <int W>
__global__ void __launch_bounds__(256) k_ll_allgather(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const size_t lines = (c.bytes + 7) / 8;
  const char* in = static_cast<const char*>(c.in[0]);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 d = ll_load(in, i * 8, c.bytes);
    ll_push<W>(v, par, tag, i, d);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 x = q == v.rank ? d : ll_poll(v, par, ep, q, i, t0, live);
      ll_store(static_cast<char*>(c.out[q]), i * 8, c.bytes, x.x, x.y);
    }
  }
  ll_end(v, ep);
}

// ----------------------------------------------------------------------------
// Rooted LL collectives: REDUCE_LL and GATHER_LL move lines peers -> root, BROADCAST_LL and
// SCATTER_LL root -> peers (the reference's rooted call sites, main.py:14,37,52,81, at their
// one-element sizes). Data goes one way only, so every ordered pair of ranks that carries no
// data exchanges a token instead: one line {0, epoch} in the same slot. Each rank then still
// hears from every peer in every LL call, which keeps the parity argument above valid for any
// sequence of LL kinds. Block 0's thread 0 pushes the tokens at entry and polls the expected
// ones before it exits, so the call ends only once every peer has entered it.
__device__ __forceinline__ void ll_push_one(const IpcView& v, int q, uint32_t par, uint64_t tag, size_t i, uint2 d) {
  uint64_t* dst = ll_slot(v.flags[q], par, v.rank) + 2 * i;
  __hip_atomic_store(dst, tag | d.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(dst + 1, tag | d.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// up: data flows peers -> root (reduce, gather); otherwise root -> peers (broadcast, scatter)
__device__ __forceinline__ bool ll_sends_data(int me, int q, int root, bool up) { return up ? q == root : me == root; }

template <int W>
__device__ __forceinline__ void ll_tokens_push(const IpcView& v, uint32_t par, uint64_t tag, int root, bool up) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
#pragma unroll
  for (int q = 0; q < W; ++q)
    if (q != v.rank && !ll_sends_data(v.rank, q, root, up)) ll_push_one(v, q, par, tag, 0, make_uint2(0u, 0u));
}

template <int W>
__device__ __forceinline__ void ll_tokens_poll(const IpcView& v, uint32_t par, uint32_t ep, int root, bool up,
                                               uint64_t t0, bool& live) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
#pragma unroll
  for (int q = 0; q < W; ++q)
    if (q != v.rank && !ll_sends_data(q, v.rank, root, up)) (void)ll_poll(v, par, ep, q, 0, t0, live);
}

// REDUCE_LL: peers push their lines to the root only; the root reduces in rank order into
// out[0]. Non-root tensors are left untouched.
template <DType DT, RedOp OP, int W>
__global__ void __launch_bounds__(256) k_ll_reduce(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const bool am_root = v.rank == c.root;
  ll_tokens_push<W>(v, par, tag, c.root, true);
  const size_t lines = (c.bytes + 7) / 8;
  const char* in = static_cast<const char*>(c.in[0]);
  char* out = static_cast<char*>(c.out[0]);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 d = ll_load(in, i * 8, c.bytes);
    if (!am_root) {
#pragma unroll
      for (int q = 0; q < W; ++q)
        if (q == c.root) ll_push_one(v, q, par, tag, i, d);
      continue;
    }
    uint4 src[W];
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 x = q == v.rank ? d : ll_poll(v, par, ep, q, i, t0, live);
      src[q] = make_uint4(x.x, x.y, 0u, 0u);
    }
    const uint4 r = reduce_vec<DT, OP, W>(src, c.avg_div);
    ll_store(out, i * 8, c.bytes, r.x, r.y);
  }
  ll_tokens_poll<W>(v, par, ep, c.root, true, t0, live);
  ll_end(v, ep);
}

// BROADCAST_LL (root: in[0] = out[0] = the tensor), SCATTER_LL (root: in[q] = chunk for rank q),
// GATHER_LL (root: out[q] = slot for rank q's input); c.bytes = per-rank payload.
template <int W>
__global__ void __launch_bounds__(256) k_ll_rooted(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const int root = c.root;
  const bool am_root = v.rank == root, up = c.coll == IpcColl::GATHER_LL;
  ll_tokens_push<W>(v, par, tag, root, up);
  const size_t lines = (c.bytes + 7) / 8;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    if (up) {  // gather
      const uint2 d = ll_load(static_cast<const char*>(c.in[0]), i * 8, c.bytes);
#pragma unroll
      for (int q = 0; q < W; ++q) {
        if (!am_root) {
          if (q == root) ll_push_one(v, q, par, tag, i, d);
        } else {
          const uint2 x = q == v.rank ? d : ll_poll(v, par, ep, q, i, t0, live);
          ll_store(static_cast<char*>(c.out[q]), i * 8, c.bytes, x.x, x.y);
        }
      }
    } else if (am_root) {  // broadcast / scatter, root side
      const bool scatter = c.coll == IpcColl::SCATTER_LL;
      const uint2 d0 = ll_load(static_cast<const char*>(c.in[0]), i * 8, c.bytes);
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const uint2 d = scatter && q > 0 ? ll_load(static_cast<const char*>(c.in[q]), i * 8, c.bytes) : d0;
        if (q != v.rank) ll_push_one(v, q, par, tag, i, d);
        else if (scatter) ll_store(static_cast<char*>(c.out[0]), i * 8, c.bytes, d.x, d.y);
      }
    } else {  // broadcast / scatter, receiving side: only the root's slot carries data
      uint2 x = make_uint2(0u, 0u);
#pragma unroll
      for (int q = 0; q < W; ++q)
        if (q == root) x = ll_poll(v, par, ep, q, i, t0, live);
      ll_store(static_cast<char*>(c.out[0]), i * 8, c.bytes, x.x, x.y);
    }
  }
  ll_tokens_poll<W>(v, par, ep, root, up, t0, live);
  ll_end(v, ep);
}

// REDUCE_SCATTER_LL / ALLTOALL_LL (per-chunk payload <= kLLMaxBytes): chunk q of every rank
// (c.in[q]) is pushed to rank q only. Every ordered pair of ranks carries data, so the reuse
// argument of the all-reduce holds without tokens. Reduce-scatter reduces the W chunks
// addressed to this rank in rank order into out[0]; all-to-all writes chunk-from-q to out[q].
template <DType DT, RedOp OP, int W>
__global__ void __launch_bounds__(256) k_ll_reduce_scatter(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const size_t lines = (c.bytes + 7) / 8;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
    uint2 own = make_uint2(0u, 0u);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 d = ll_load(static_cast<const char*>(c.in[q]), i * 8, c.bytes);
      if (q == v.rank) own = d;
      else ll_push_one(v, q, par, tag, i, d);
    }
    uint4 src[W];
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 x = q == v.rank ? own : ll_poll(v, par, ep, q, i, t0, live);
      src[q] = make_uint4(x.x, x.y, 0u, 0u);
    }
    const uint4 r = reduce_vec<DT, OP, W>(src, c.avg_div);
    ll_store(static_cast<char*>(c.out[0]), i * 8, c.bytes, r.x, r.y);
  }
  ll_end(v, ep);
}

template <int W>
__global__ void __launch_bounds__(256) k_ll_alltoall(IpcView v, IpcCall c) {
  const uint32_t ep = ll_begin(v), par = ep & 1u;
  const uint64_t tag = (uint64_t)ep << 32;
  const size_t lines = (c.bytes + 7) / 8;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool live = true;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint2 d = ll_load(static_cast<const char*>(c.in[q]), i * 8, c.bytes);
      if (q == v.rank) ll_store(static_cast<char*>(c.out[q]), i * 8, c.bytes, d.x, d.y);
      else ll_push_one(v, q, par, tag, i, d);
    }
#pragma unroll
    for (int q = 0; q < W; ++q) {
      if (q == v.rank) continue;
      const uint2 x = ll_poll(v, par, ep, q, i, t0, live);
      ll_store(static_cast<char*>(c.out[q]), i * 8, c.bytes, x.x, x.y);
    }
  }
  ll_end(v, ep);
}

// host-side dispatch, one pair of functions per dtype (defined in reduce_<dt>.hip)
#define PDCC_DECL_DISPATCH(DTNAME)                                                                   \
  hipError_t k1_dispatch_##DTNAME(const void* const* srcs, int n, void* out, size_t nb, RedOp op,    \
                                  int avg_div, hipStream_t s, int grid, int lds);                    \
  hipError_t ipc_dispatch_##DTNAME(const IpcView& v, const IpcCall& c, hipStream_t s, int grid);
PDCC_DECL_DISPATCH(F32)
PDCC_DECL_DISPATCH(F16)
PDCC_DECL_DISPATCH(BF16)
PDCC_DECL_DISPATCH(F64)
PDCC_DECL_DISPATCH(I8)
PDCC_DECL_DISPATCH(U8)
PDCC_DECL_DISPATCH(I32)
PDCC_DECL_DISPATCH(I64)
#undef PDCC_DECL_DISPATCH

// `mode` (kern::K1Mode): bit 0 = LDS-DMA engine (else registers), bit 1 = non-temporal stores,
// bit 2 = the streaming kernel (one slab per workgroup, `grid` ignored), bit 3 = its loads
// non-temporal too
template <DType DT, RedOp OP, int NSRC>
hipError_t launch_k1(const void* const* srcs, void* out, size_t nbytes, int avg_div, hipStream_t s, int grid,
                     int mode) {
  Ptrs8 p{};
  for (int k = 0; k < NSRC; ++k) p.p[k] = (const char*)srcs[k];
  if (mode & 4) {
    const size_t slab = (size_t)StreamV<NSRC>::value * kTile;
    const dim3 g((unsigned)((nbytes + slab - 1) / slab));
    if (mode & 8)
      hipLaunchKernelGGL((k1_reduce_stream<DT, OP, NSRC, true, true>), g, dim3(256), 0, s, p, (char*)out, nbytes,
                         avg_div);
    else if (mode & 2)
      hipLaunchKernelGGL((k1_reduce_stream<DT, OP, NSRC, true, false>), g, dim3(256), 0, s, p, (char*)out, nbytes,
                         avg_div);
    else
      hipLaunchKernelGGL((k1_reduce_stream<DT, OP, NSRC, false, false>), g, dim3(256), 0, s, p, (char*)out, nbytes,
                         avg_div);
    return hipGetLastError();
  }
  static const int chunked = [] {
    const char* e = getenv("PDCC_K1_CHUNKED");
    return e && *e == '1' ? 1 : 0;
  }();
  p.chunked = chunked;
  p.nt = (mode & 2) ? 1 : 0;
  p.ntl = (mode & 8) ? 1 : 0;  // (non-temporal loads come with non-temporal stores)
  const bool lds = (mode & 1) != 0;
  if (lds)
    hipLaunchKernelGGL((k1_reduce_lds<DT, OP, NSRC, K1Deep<NSRC>::value>), dim3(grid), dim3(256), 0, s, p, (char*)out,
                       nbytes, avg_div);
  else
    hipLaunchKernelGGL((k1_reduce_regs<DT, OP, NSRC>), dim3(grid), dim3(256), 0, s, p, (char*)out, nbytes, avg_div);
  return hipGetLastError();
}

template <DType DT, RedOp OP>
hipError_t k1_by_n(const void* const* srcs, int n, void* out, size_t nbytes, int avg_div, hipStream_t s, int grid,
                   int lds) {
  switch (n) {
    case 1: return launch_k1<DT, OP, 1>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 2: return launch_k1<DT, OP, 2>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 3: return launch_k1<DT, OP, 3>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 4: return launch_k1<DT, OP, 4>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 5: return launch_k1<DT, OP, 5>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 6: return launch_k1<DT, OP, 6>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 7: return launch_k1<DT, OP, 7>(srcs, out, nbytes, avg_div, s, grid, lds);
    case 8: return launch_k1<DT, OP, 8>(srcs, out, nbytes, avg_div, s, grid, lds);
    default: return hipErrorInvalidValue;
  }
}

template <DType DT, RedOp OP>
hipError_t ipc_by_w(const IpcView& v, const IpcCall& c, hipStream_t s, int grid) {
  if (c.coll == IpcColl::ALLREDUCE_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL((k_ll_allreduce<DT, OP, WW>), dim3(grid), dim3(256), 0, s, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (c.coll == IpcColl::REDUCE_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL((k_ll_reduce<DT, OP, WW>), dim3(grid), dim3(256), 0, s, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (c.coll == IpcColl::REDUCE_SCATTER_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL((k_ll_reduce_scatter<DT, OP, WW>), dim3(grid), dim3(256), 0, s, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL((k_ipc_reduce<DT, OP, WW>), dim3(grid), dim3(256), 0, s, v, c); break;
    PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dev
}  // namespace pdcc

// Instantiate the dispatchers for one dtype. Float types get SUM/AVG/PROD/MIN/MAX,
// integer types additionally BAND/BOR/BXOR.
#define PDCC_OPS_FLOAT(F, ...) \
  case RedOp::SUM: return F<DT, RedOp::SUM>(__VA_ARGS__); \
  case RedOp::AVG: return F<DT, RedOp::AVG>(__VA_ARGS__); \
  case RedOp::PROD: return F<DT, RedOp::PROD>(__VA_ARGS__); \
  case RedOp::MIN: return F<DT, RedOp::MIN>(__VA_ARGS__); \
  case RedOp::MAX: return F<DT, RedOp::MAX>(__VA_ARGS__);
#define PDCC_OPS_INT(F, ...)              \
  PDCC_OPS_FLOAT(F, __VA_ARGS__)          \
  case RedOp::BAND: return F<DT, RedOp::BAND>(__VA_ARGS__); \
  case RedOp::BOR: return F<DT, RedOp::BOR>(__VA_ARGS__); \
  case RedOp::BXOR: return F<DT, RedOp::BXOR>(__VA_ARGS__);

#define PDCC_REDUCE_DTYPE(DTNAME, OPSET)                                                              \
  namespace pdcc {                                                                                    \
  namespace dev {                                                                                     \
  hipError_t k1_dispatch_##DTNAME(const void* const* srcs, int n, void* out, size_t nb, RedOp op,     \
                                  int avg_div, hipStream_t s, int grid, int lds) {                    \
    constexpr DType DT = DType::DTNAME;                                                               \
    switch (op) { OPSET(k1_by_n, srcs, n, out, nb, avg_div, s, grid, lds) default: return hipErrorInvalidValue; } \
  }                                                                                                   \
  hipError_t ipc_dispatch_##DTNAME(const IpcView& v, const IpcCall& c, hipStream_t s, int grid) {     \
    constexpr DType DT = DType::DTNAME;                                                               \
    switch (c.op) { OPSET(ipc_by_w, v, c, s, grid) default: return hipErrorInvalidValue; }            \
  }                                                                                                   \
  }                                                                                                   \
  }
