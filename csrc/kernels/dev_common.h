// Device-side building blocks shared by every gfx950 kernel in this library.
//
//  * element traits + reduction functors (SUM/AVG/PROD/MIN/MAX/BAND/BOR/BXOR),
//    bf16/f16 accumulate in f32 across ALL sources and round once;
//  * `pipe_run`: the LDS-DMA streaming engine. Each wave64 moves 1 KiB per source
//    per tile with `global_load_lds_dwordx4` into a DEPTH-deep ring in LDS, waits
//    with a counted `s_waitcnt vmcnt(N)` (never 0 in steady state), reads its own
//    lanes back with `ds_read_b128` (inline asm, so hipcc does not insert the
//    conservative vmcnt(0) it emits before a ds_read that may alias an in-flight
//    LDS-DMA) and stores 16 B per lane. Waves only read LDS they filled
//    themselves, so the ring needs no workgroup barrier.
//  * cross-GPU signalling (K4): system-scope release -> relaxed system-scope flag
//    store into the peer's uncached signal area -> bounded relaxed poll -> ONE
//    system-scope acquire (cdna_hip_programming.md §6 Guideline 16, lifted from
//    agent to system scope because the consumer is another GPU over xGMI).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "kernel_api.h"

namespace pdcc {
namespace dev {

using kern::DType;
using kern::RedOp;

constexpr int kWaveBytes = 1024;  // 64 lanes x 16 B
constexpr int kTile = kern::kTileBytes;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_cvoid_t;

// A pointer known to be global (address space 1) that converts to a plain one where it
// is used: the conversion is an addrspacecast the compiler sees through, so loads and
// stores through it stay global_* instructions even when the pointer itself was read
// from LDS (a plain pointer read from LDS is generic: flat_* accesses).
template <class T>
struct gp {
  __attribute__((address_space(1))) T* p;
  __device__ __forceinline__ operator T*() const { return (T*)p; }
  template <class U>
  __device__ __forceinline__ explicit operator U*() const { return (U*)(T*)p; }
  __device__ __forceinline__ gp& operator=(T* q) {
    p = (__attribute__((address_space(1))) T*)q;
    return *this;
  }
};
using DView = kern::IpcViewT<gp>;  // the IPC kernels' arguments, staged in LDS
using DCall = kern::IpcCallT<gp>;
static_assert(sizeof(DView) == sizeof(kern::IpcView) && sizeof(DCall) == sizeof(kern::IpcCall),
              "device and host argument layouts differ");

// ----------------------------------------------------------------------------
// waits
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx9");
  // gfx9 s_waitcnt simm16: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  constexpr int enc = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
  __builtin_amdgcn_s_waitcnt(enc);
}
__device__ __forceinline__ void wait_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(lds_void_t*)(p);
}

template <int IMM>
__device__ __forceinline__ uint4 ds_read16(uint32_t addr) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(IMM));
  return v;
}

// NTL: non-temporal load (cache policy NT: streamed data read once)
template <bool NTL = false>
__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_cvoid_t*)g, (lds_void_t*)lds_wave_base, 16, 0, NTL ? 2 : 0);
}

template <bool NTL>
__device__ __forceinline__ uint4 load16(const char* p) {
  if constexpr (NTL) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(x[0], x[1], x[2], x[3]);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}

// ----------------------------------------------------------------------------
// element traits
__device__ __forceinline__ float bf16_to_f32(uint16_t x) { return __uint_as_float((uint32_t)x << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // keep NaN a (quiet) NaN
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);                 // RNE
}

template <DType DT> struct Tr;
template <> struct Tr<DType::F32> {
  using S = float; using C = float; static constexpr bool kFloat = true;
  __device__ static C in(S x) { return x; } __device__ static S out(C x) { return x; }
};
template <> struct Tr<DType::F64> {
  using S = double; using C = double; static constexpr bool kFloat = true;
  __device__ static C in(S x) { return x; } __device__ static S out(C x) { return x; }
};
template <> struct Tr<DType::F16> {
  using S = _Float16; using C = float; static constexpr bool kFloat = true;
  __device__ static C in(S x) { return (float)x; } __device__ static S out(C x) { return (_Float16)x; }
};
template <> struct Tr<DType::BF16> {
  using S = uint16_t; using C = float; static constexpr bool kFloat = true;
  __device__ static C in(S x) { return bf16_to_f32(x); } __device__ static S out(C x) { return f32_to_bf16(x); }
};
#define PDCC_INT_TR(DT, TYPE)                                                     \
  template <> struct Tr<DT> {                                                     \
    using S = TYPE; using C = TYPE; static constexpr bool kFloat = false;          \
    __device__ static C in(S x) { return x; } __device__ static S out(C x) { return x; } \
  };
PDCC_INT_TR(DType::I8, int8_t)
PDCC_INT_TR(DType::U8, uint8_t)
PDCC_INT_TR(DType::I32, int32_t)
PDCC_INT_TR(DType::I64, int64_t)
#undef PDCC_INT_TR

template <RedOp OP, class C>
__device__ __forceinline__ C apply_op(C a, C b) {
  if constexpr (OP == RedOp::SUM || OP == RedOp::AVG) return a + b;
  else if constexpr (OP == RedOp::PROD) return a * b;
  else if constexpr (OP == RedOp::MAX) return (a > b || a != a) ? a : b;  // NaN propagates
  else if constexpr (OP == RedOp::MIN) return (a < b || a != a) ? a : b;
  else if constexpr (OP == RedOp::BAND) return a & b;
  else if constexpr (OP == RedOp::BOR) return a | b;
  else if constexpr (OP == RedOp::BXOR) return a ^ b;
  else return a;
}

// Reduce NSRC 16-byte vectors element-wise (sources combined in index order, so
// every rank that runs the same reduction gets bit-identical results).
template <DType DT, RedOp OP, int NSRC>
__device__ __forceinline__ uint4 reduce_vec(const uint4 (&v)[NSRC], int avg_div) {
  if constexpr (OP == RedOp::COPY) {
    return v[0];
  } else {
    using T = Tr<DT>;
    using S = typename T::S;
    using C = typename T::C;
    constexpr int N = 16 / sizeof(S);
    S s[N];
    C acc[N];
    __builtin_memcpy(s, &v[0], 16);
#pragma unroll
    for (int e = 0; e < N; ++e) acc[e] = T::in(s[e]);
#pragma unroll
    for (int k = 1; k < NSRC; ++k) {
      __builtin_memcpy(s, &v[k], 16);
#pragma unroll
      for (int e = 0; e < N; ++e) acc[e] = apply_op<OP, C>(acc[e], T::in(s[e]));
    }
    if constexpr (OP == RedOp::AVG) {
#pragma unroll
      for (int e = 0; e < N; ++e) acc[e] = acc[e] / (C)avg_div;
    }
#pragma unroll
    for (int e = 0; e < N; ++e) s[e] = T::out(acc[e]);
    uint4 r;
    __builtin_memcpy(&r, s, 16);
    return r;
  }
}

// Store / load `lim` (< 16) leading bytes of a 16-B vector (buffer tails). Fully
// unrolled on constant byte indices so nothing lands in scratch or LDS.
__device__ __forceinline__ void store_partial(char* d, const uint4& r, uint32_t lim) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if ((uint32_t)j < lim) d[j] = (char)(w[j >> 2] >> (8 * (j & 3)));
}
__device__ __forceinline__ uint4 load_partial(const char* s, uint32_t lim) {
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if ((uint32_t)j < lim) w[j >> 2] |= (uint32_t)(uint8_t)s[j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ----------------------------------------------------------------------------
// LDS-DMA streaming engine.
//
// Map (per block) must provide:
//   size_t count()                 tiles this block processes
//   const char* src(int s, size_t i)   base of tile i in source s (tile is 4 KiB, fully readable)
//   char* dst(size_t i)            base of tile i in the destination
//   size_t valid(size_t i)         bytes of tile i that may be written (<= 4096)
template <int NSRC, int DEPTH>
struct PipeLds {
  static constexpr int kBytes = DEPTH * NSRC * kTile;
};

// Wait for tile i (< DEPTH-1) of the prologue: BASE younger loads plus the
// i * ST stores of the consumes issued since that tile (vmcnt needs an immediate).
template <int BASE, int DEPTH, int ST = 1>
__device__ __forceinline__ void wait_prologue(int i) {
  switch (i) {
    case 0: wait_vmcnt<BASE>(); break;
    case 1: if constexpr (DEPTH > 2) wait_vmcnt<BASE + 1 * ST>(); break;
    case 2: if constexpr (DEPTH > 3) wait_vmcnt<BASE + 2 * ST>(); break;
    case 3: if constexpr (DEPTH > 4) wait_vmcnt<BASE + 3 * ST>(); break;
    case 4: if constexpr (DEPTH > 5) wait_vmcnt<BASE + 4 * ST>(); break;
    case 5: if constexpr (DEPTH > 6) wait_vmcnt<BASE + 5 * ST>(); break;
    default: if constexpr (DEPTH > 7) wait_vmcnt<BASE + 6 * ST>(); break;
  }
}

// NDST > 1: every reduced vector is stored to NDST destinations, m.dst(j, i) for
// j < NDST (whole tiles only: the push all-reduce writes each owner's result into
// every rank's tensor); the vmcnt accounting counts NDST stores per consume.
// 16-B store; NT = non-temporal (global_store ... nt: streamed past the caches, for
// destinations nobody re-reads soon)
template <bool NT>
__device__ __forceinline__ void store16(char* d, const uint4& r) {
  if constexpr (NT) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = {r.x, r.y, r.z, r.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(d));
  } else {
    *reinterpret_cast<uint4*>(d) = r;
  }
}

template <DType DT, RedOp OP, int NSRC, int DEPTH, class Map, int NDST = 1, bool NT = false, bool NTL = false>
__device__ __forceinline__ void pipe_run(char* lds, const Map& m, int avg_div) {
  static_assert((DEPTH - 1) * (NSRC + NDST) < 64, "pipeline too deep for vmcnt");
  static_assert(DEPTH >= 2 && DEPTH <= 8, "prologue wait counts are written out for DEPTH <= 8");
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t lane_off = wave * kWaveBytes + lane * 16;
  const size_t n = m.count();

  auto issue = [&](size_t i, int stage) {
#pragma unroll
    for (int s = 0; s < NSRC; ++s)
      glds16<NTL>(m.src(s, i) + lane_off, lds + (stage * NSRC + s) * kTile + wave * kWaveBytes);
  };
  auto consume = [&](size_t i, int stage) {
    const uint32_t a = lds_off(lds + stage * NSRC * kTile + lane_off);
    uint4 v[NSRC];
#pragma unroll
    for (int s = 0; s < NSRC; ++s) {
      // offsets are compile-time immediates (s * 4096 < 64 KiB)
      switch (s) {
        case 0: v[s] = ds_read16<0 * kTile>(a); break;
        case 1: v[s] = ds_read16<1 * kTile>(a); break;
        case 2: v[s] = ds_read16<2 * kTile>(a); break;
        case 3: v[s] = ds_read16<3 * kTile>(a); break;
        case 4: v[s] = ds_read16<4 * kTile>(a); break;
        case 5: v[s] = ds_read16<5 * kTile>(a); break;
        case 6: v[s] = ds_read16<6 * kTile>(a); break;
        default: v[s] = ds_read16<7 * kTile>(a); break;
      }
    }
    wait_lgkm0();
    const uint4 r = reduce_vec<DT, OP, NSRC>(v, avg_div);
    if constexpr (NDST == 1) {
      char* d = m.dst(i);
      const size_t lim = m.valid(i);
      if (lane_off + 16 <= lim) {
        store16<NT>(d + lane_off, r);
      } else if (lane_off < lim) {
        store_partial(d + lane_off, r, (uint32_t)(lim - lane_off));
      }
      // The counted waits assume one store per consume. A wave with nothing to store
      // here (its 1 KiB lies past `lim`: a padding tile of a partial last 2-shot row,
      // the tail of a ragged tile) issues none, which would leave every later wait one
      // op too loose -- a younger tile's LDS slot could be read while its DMA is still
      // in flight. Drain instead: the later waits are then exact or stricter.
      if ((size_t)wave * kWaveBytes >= lim) drain_vm();
    } else {
#pragma unroll
      for (int j = 0; j < NDST; ++j) *reinterpret_cast<uint4*>(m.dst(j, i) + lane_off) = r;
    }
  };

#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d)
    if ((size_t)d < n) issue(d, d);
  size_t i = 0;
  int stage = 0;
  for (; i + (DEPTH - 1) < n; ++i) {
    int ns = stage + DEPTH - 1;
    if (ns >= DEPTH) ns -= DEPTH;
    issue(i + DEPTH - 1, ns);
    // Ops younger than tile i's loads: the (DEPTH-1) tiles issued after it
    // (x NSRC loads) plus the stores of the consumes in between -- i of them
    // while tile i was a prologue tile, DEPTH-1 in steady state. vmcnt retires
    // in issue order, so the count must be exact (a looser one lets tile i's
    // last load still be in flight when its LDS slot is read).
    if (i >= (size_t)(DEPTH - 1)) {
      wait_vmcnt<(DEPTH - 1) * (NSRC + NDST)>();
    } else {
      wait_prologue<(DEPTH - 1) * NSRC, DEPTH, NDST>((int)i);
    }
    consume(i, stage);
    stage = (stage + 1 == DEPTH) ? 0 : stage + 1;
  }
  for (; i < n; ++i) {
    wait_vmcnt<0>();
    consume(i, stage);
    stage = (stage + 1 == DEPTH) ? 0 : stage + 1;
  }
}

// The IPC kernels' pipelines. PDCC_IPC_NTL=1 makes their loads non-temporal (every source
// tile is read once per call; K1 gains 8-11 % from it). Off: on one MI355X the A/B cost the
// staged collectives 6-31 % at 4-64 MiB (profiles/r3/ipc_ntl_ab.md) -- their staging is
// re-read in the next phase and otherwise stays in the 256 MiB Infinity Cache.
#ifndef PDCC_IPC_NTL
#define PDCC_IPC_NTL 0
#endif
template <DType DT, RedOp OP, int NSRC, int DEPTH, int NDST = 1, class Map>
__device__ __forceinline__ void ipc_pipe(char* lds, const Map& m, int avg_div) {
  pipe_run<DT, OP, NSRC, DEPTH, Map, NDST, false, PDCC_IPC_NTL != 0>(lds, m, avg_div);
}

// Zero-copy reductions read every rank's tensor exactly once per call (the reduce phase of the
// 2-shot all-reduce / rooted reduce, the reduce-scatter): those loads are non-temporal, so the
// read-once inputs do not push out of the caches the reduced tiles the next phase re-reads.
// (The staged protocols keep normal loads: their staging is written and re-read within a call.)
#ifndef PDCC_IPC_ZC_NTL
#define PDCC_IPC_ZC_NTL 1
#endif
template <DType DT, RedOp OP, int NSRC, int DEPTH, int NDST = 1, class Map>
__device__ __forceinline__ void ipc_pipe_once(char* lds, const Map& m, int avg_div) {
  pipe_run<DT, OP, NSRC, DEPTH, Map, NDST, false, PDCC_IPC_ZC_NTL != 0>(lds, m, avg_div);
}

// Register-staged engine (same Map contract): UNROLL tiles of NSRC vectors in
// VGPRs per lane, no LDS. Kept for the A/B measurement against pipe_run.
template <DType DT, RedOp OP, int NSRC, int UNROLL, class Map, bool NT = false, bool NTL = false>
__device__ __forceinline__ void pipe_run_regs(const Map& m, int avg_div) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t lane_off = wave * kWaveBytes + lane * 16;
  const size_t n = m.count();
  size_t i = 0;
  for (; i + UNROLL <= n; i += UNROLL) {
    uint4 v[UNROLL][NSRC];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int s = 0; s < NSRC; ++s)
        v[u][s] = load16<NTL>(m.src(s, i + u) + lane_off);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint4 r = reduce_vec<DT, OP, NSRC>(v[u], avg_div);
      char* d = m.dst(i + u);
      const size_t lim = m.valid(i + u);
      if (lane_off + 16 <= lim) store16<NT>(d + lane_off, r);
      else if (lane_off < lim) store_partial(d + lane_off, r, (uint32_t)(lim - lane_off));
    }
  }
  for (; i < n; ++i) {
    uint4 v[NSRC];
#pragma unroll
    for (int s = 0; s < NSRC; ++s) v[s] = load16<NTL>(m.src(s, i) + lane_off);
    const uint4 r = reduce_vec<DT, OP, NSRC>(v, avg_div);
    char* d = m.dst(i);
    const size_t lim = m.valid(i);
    if (lane_off + 16 <= lim) *reinterpret_cast<uint4*>(d + lane_off) = r;
    else if (lane_off < lim) store_partial(d + lane_off, r, (uint32_t)(lim - lane_off));
  }
}

// Bounded local copy of the tiles {first, first+stride, ...} < ntiles of a user
// buffer (nbytes long, 16-B aligned) into a padded staging buffer. Plain 16-B
// loads (never LDS-DMA: reading past the end of a user allocation could fault).
__device__ __forceinline__ void stage_tiles(const char* __restrict__ src, char* __restrict__ dst,
                                            size_t nbytes, size_t first, size_t stride,
                                            size_t ntiles) {
  const uint32_t lane_off = (threadIdx.x >> 6) * kWaveBytes + (threadIdx.x & 63) * 16;
  constexpr int U = 4;
  size_t t = first;
  for (; t + (U - 1) * stride < ntiles; t += U * stride) {
    uint4 v[U];
    size_t off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      off[u] = (t + u * stride) * kTile + lane_off;
      v[u] = (off[u] + 16 <= nbytes) ? *reinterpret_cast<const uint4*>(src + off[u])
             : (off[u] < nbytes ? load_partial(src + off[u], (uint32_t)(nbytes - off[u]))
                                : make_uint4(0, 0, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) *reinterpret_cast<uint4*>(dst + off[u]) = v[u];
  }
  for (; t < ntiles; t += stride) {
    const size_t off = t * kTile + lane_off;
    uint4 v = (off + 16 <= nbytes) ? *reinterpret_cast<const uint4*>(src + off)
              : (off < nbytes ? load_partial(src + off, (uint32_t)(nbytes - off)) : make_uint4(0, 0, 0, 0));
    *reinterpret_cast<uint4*>(dst + off) = v;
  }
}

// ----------------------------------------------------------------------------
// This block's call number (see kern::IpcView): thread 0 reads its own counter
// and writes it back incremented. Only block b of this rank ever touches
// counters[b], and consecutive launches on a stream run in order, so relaxed
// accesses suffice (uncached signal memory: no stale line on any XCD); the store
// is drained by the arrival barrier that follows.
// The IPC kernels issue the load at entry (block_seq_load) and finish it after staging their
// arguments (block_seq): an uncached load waits ~8 us behind the thread's older stores, and a
// gated zero-copy launch's buffer exchange hides that wait.
template <class V>
__device__ __forceinline__ uint32_t block_seq_load(const V& v) {
  return threadIdx.x == 0 ? __hip_atomic_load(v.counters + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : 0u;
}
template <class V>
__device__ __forceinline__ uint32_t block_seq(const V& v, uint32_t loaded) {
  __shared__ uint32_t s_seq;
  if (threadIdx.x == 0) {
    const uint32_t s = loaded + 1u;
    __hip_atomic_store(v.counters + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_seq = s;
  }
  __syncthreads();
  return s_seq;
}

// ----------------------------------------------------------------------------
// Phase trace (PDCC_IPC_TRACE): thread 0 of every block keeps timestamps and writes
// them once, when the kernel body returns (finish(); no extra memory traffic inside
// the protocol): block 0 the record header, every block its phase-1 and exit stamps.
// The stamps live in LDS (96 B per workgroup): a trace object in registers gets
// demoted to scratch memory once it crosses the kernel body's many exit paths.
struct PhaseTrace {
  const bool on;
  const uint32_t xb;  // 1: block 0 is a gated launch's exchange block (its words 8-11 only; the data
                      // blocks are 1..grid-1, numbered 0.. in the record, the header is data block 0's)
  __device__ __forceinline__ static uint64_t* slots() {
    __shared__ uint64_t s[kern::kTraceWords];
    return s;
  }
  __device__ __forceinline__ explicit PhaseTrace(const kern::IpcView& view, uint32_t xchg_blocks = 0)
      : on(view.trace != nullptr && threadIdx.x == 0), xb(xchg_blocks) {
    if (on) {
#pragma unroll
      for (int k = 0; k < kern::kTraceWords; ++k) slots()[k] = 0;
      slots()[1] = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void seq(uint32_t s) const {
    if (on) slots()[0] = s;
  }
  __device__ __forceinline__ void mark(int k) const {
    if (on) slots()[k] = __builtin_amdgcn_s_memrealtime();
  }
  // accumulating words (the dynamic protocols' totals): now() -> ... -> add(k, t0)
  __device__ __forceinline__ uint64_t now() const { return on ? __builtin_amdgcn_s_memrealtime() : 0; }
  __device__ __forceinline__ void add(int k, uint64_t t0) const {
    if (on) slots()[k] += __builtin_amdgcn_s_memrealtime() - t0;
  }
  __device__ __forceinline__ void count(int k, uint64_t n = 1) const {
    if (on) slots()[k] += n;
  }
  __device__ __forceinline__ void finish(const kern::IpcView& view) const {
    if (!on) return;
    uint64_t* t = slots();
    t[7] = __builtin_amdgcn_s_memrealtime();
    uint64_t* r = view.trace + (size_t)view.trace_slot * kern::kTraceRecWords;
    const uint32_t b = blockIdx.x - xb;  // data block index
    if (b == 0) {
#pragma unroll
      for (int k = 0; k < kern::kTraceWords; ++k)
        if (!xb || k < 8 || k > 11) r[k] = t[k];
    }
    if (b < (unsigned)kern::kTraceBlocks) {
      r[kern::kTraceWords + b] = t[5];
      r[kern::kTraceWords + kern::kTraceBlocks + b] = t[7];
    }
  }
  // the exchange block's part of the record: the device-side exchange's stamps (words 8-11)
  __device__ __forceinline__ void finish_exchange(const kern::IpcView& view) const {
    if (!on) return;
    uint64_t* r = view.trace + (size_t)view.trace_slot * kern::kTraceRecWords;
    for (int k = 8; k <= 11; ++k) r[k] = slots()[k];
  }
};

// A gated zero-copy launch with the device-side exchange (kern::ZcTable) runs one more workgroup,
// block 0, that only does the exchange: the data blocks 1..grid-1 (b = blockIdx - 1, G = grid - 1)
// never carry its remote record stores. Run in a data block, those flat stores stayed outstanding for
// ~8 us and held the block's next LDS access (the r4/r5 traces' "block_seq" gap), delaying that block's
// share of the call; block 0 is dispatched first, so the data blocks' wait for its verdict always ends.
template <class C>
__device__ __forceinline__ uint32_t xchg_blocks(const C& c) {
  return (c.gate && c.ztab) ? 1u : 0u;
}

// ----------------------------------------------------------------------------
// K4: cross-GPU block-pairwise barrier.
//
// flags layout (per rank, uncached device memory): flags[block * kMaxRanks + src].
// Values are monotonic epochs (kEpochsPerCall * seq + phase, seq = the block's
// call number), compared with a wrap-safe signed difference, so flags never need
// re-zeroing and a fast peer that already moved on never deadlocks a slow one.
__device__ __forceinline__ bool reached(uint32_t have, uint32_t want) {
  return (int32_t)(have - want) >= 0;
}

// Every wave of the block calls this after its last store of data that peers
// will read (DATA = true: system-scope release before the flag, acquire after the
// poll). DATA = false is the arrival barrier at the start of a call: nothing is
// handed over, so no cache maintenance -- it only proves that every peer's block
// of the same index has started this call, i.e. (same-stream kernels run in
// order) that every peer's previous kernel has finished and no longer reads the
// staging this call is about to overwrite. Returns false on timeout (error word
// set, block continues so the grid always drains).
template <bool DATA = true, class V>
__device__ __forceinline__ bool block_barrier(const V& v, uint32_t value, const PhaseTrace* tr = nullptr) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  drain_vm();       // every storing wave drains its stores
  __syncthreads();  // ... before wave 0 publishes for the whole block
  bool ok = true;
  if (wave == 0) {
    if (tr) tr->mark(13);
    if constexpr (DATA) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back L2 dirty lines
      drain_vm();                                     // keep the wait after the fence (G16 pitfall 12)
    }
    const int b = blockIdx.x;
    if (lane < v.world) {
      uint32_t* f = v.flags[lane] + b * kern::kMaxRanks + v.rank;
      __hip_atomic_store(f, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tr) tr->mark(14);
    const uint32_t* mine = v.flags[v.rank] + b * kern::kMaxRanks;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 1;; ++it) {
      bool me_ok = true;
      if (lane < v.world)
        me_ok = reached(__hip_atomic_load(mine + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), value);
      if (__all(me_ok)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks) {
        if (lane == 0)
          __hip_atomic_store(static_cast<uint32_t*>(v.err), 0x100u | (uint32_t)v.rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      // every 256 polls: has the host aborted the group (IpcComm::abort), or did
      // another block already time out? Either way stop waiting, so the grid drains.
      if ((it & 255u) == 0 && __hip_atomic_load(static_cast<uint32_t*>(v.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (tr) tr->mark(15);
    if constexpr (DATA) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale L1/L2 lines
      drain_vm();
    }
  }
  __syncthreads();
  return ok;
}

// ----------------------------------------------------------------------------
// Kernel arguments of the IPC kernels, staged once per block into LDS: a gated zero-copy
// launch (kern::GateSlot) waits here until the host published the call's buffers, then
// swaps them into the view (ok = 1) or falls back to the staged protocol (ok = 0, or the
// wait gave up: error word set, the barriers that follow leave at once). Every block's
// thread 0 polls the slot itself (no block waits for another block of the grid).
__device__ __forceinline__ bool gate_wait(const kern::IpcView& v, const kern::IpcCall& c, uint32_t& ok) {
  const kern::GateSlot* g = c.gate;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 1;; ++it) {
    if (__hip_atomic_load(&g->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == c.gate_seq) {
      ok = __hip_atomic_load(&g->ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return true;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks) {
      __hip_atomic_store(static_cast<uint32_t*>(v.err), 0x400u | (uint32_t)v.rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    if ((it & 15u) == 0 && __hip_atomic_load(static_cast<uint32_t*>(v.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return false;
    // the slot is host memory: back off (a poll is a PCIe round trip), longer once the wait is long
    if (it < 64) __builtin_amdgcn_s_sleep(4);
    else __builtin_amdgcn_s_sleep(127);
  }
}

// ---- device-side record exchange of a gated zero-copy launch (kern::ZcTable) ----------
__device__ __forceinline__ uint64_t* zx_src_words(const kern::IpcView& v, int owner, int src) {
  return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(v.flags[owner]) + kern::kZxOffset +
                                     (size_t)src * kern::kZxSrcBytes);
}
__device__ __forceinline__ kern::GateSlot* zx_resolved(const kern::IpcView& v, uint64_t seq) {
  return reinterpret_cast<kern::GateSlot*>(reinterpret_cast<char*>(v.flags[v.rank]) + kern::kZxResolvedOffset) +
         (seq % kern::kGateSlots);
}
__device__ __forceinline__ uint64_t zx_tagged(uint64_t tag, uint64_t ptr) {
  return ((tag & 0xffffull) << 48) | (ptr & 0xffffffffffffull);
}
__device__ __forceinline__ void zx_put(uint64_t* p, uint32_t data, uint32_t tag) {
  __hip_atomic_store(p, ((uint64_t)tag << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t& zx_verdict_note() {
  __shared__ uint32_t s;
  return s;
}

// Wave 0 of block 0: push {id, off} to every rank, collect every rank's, look the peers' ids
// up in this process's mapping table, vote, and publish the verdict in this call's resolved
// slot (ok = 1 with the buffers, 2 = wait for the host gate, 0 = a peer never came: staged,
// the error word is set). Returns nothing; every block reads the resolved slot.
__device__ __forceinline__ void zx_resolve(const kern::IpcView& v, const kern::IpcCall& c, const PhaseTrace& tr) {
  const int lane = threadIdx.x & 63, W = v.world, me = v.rank;
  uint32_t* epw = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(v.flags[me]) + kern::kZxEpochOffset);
  uint32_t ep = 0;
  if (lane == 0) {  // only block 0 of this rank's gated kernels touches it, in stream order
    ep = __hip_atomic_load(epw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    // never tag 0 (fresh signal memory is zero), and skip it BEFORE storing: on the wrap the
    // stored word must move on to 1 too, or the next call would compute tag 1 again and
    // could take the previous call's records (and vote) for its own
    if (ep == 0u) ep = 1u;
    __hip_atomic_store(epw, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ep = __shfl(ep, 0);
  // round 1: my record into slot [me] of every rank (4 single-copy-atomic words)
  if (lane < W) {
    uint64_t* d = zx_src_words(v, lane, me);
    zx_put(d + 0, (uint32_t)c.zx_id, ep);
    zx_put(d + 1, (uint32_t)(c.zx_id >> 32), ep);
    zx_put(d + 2, (uint32_t)c.zx_off, ep);
    zx_put(d + 3, (uint32_t)(c.zx_off >> 32), ep);
  }
  uint64_t id = 0, off = 0;
  bool got = lane >= W, alive = true, timed_out = false;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 1;; ++it) {
    if (!got) {
      const uint64_t* s = zx_src_words(v, me, lane);
      uint64_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = __hip_atomic_load(s + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((uint32_t)(w[0] >> 32) == ep && (uint32_t)(w[1] >> 32) == ep && (uint32_t)(w[2] >> 32) == ep &&
          (uint32_t)(w[3] >> 32) == ep) {
        got = true;
        id = (w[0] & 0xffffffffull) | (w[1] << 32);
        off = (w[2] & 0xffffffffull) | (w[3] << 32);
      }
    }
    if (__all(got)) break;
    timed_out = __builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks;
    if (timed_out || ((it & 255u) == 0 && __hip_atomic_load(v.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
      alive = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  tr.mark(8);
  // lookup: lanes 0-31 scan table row q = 2p, lanes 32-63 row 2p + 1; ids and bases loaded in
  // one pass (a slot's base stays put until its mapping is closed, after every launch that
  // could have read the entry: an id match never pairs with another mapping's base)
  const kern::ZcTable* tab = c.ztab;
  const int half = lane >> 5, j = lane & 31;
  uint64_t cand[4], cbase[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int q = 2 * p + half;
    const bool look = alive && q < W && q != me;
    cand[p] = look ? __hip_atomic_load(&tab->id[q][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
    cbase[p] = look ? __hip_atomic_load(&tab->base[q][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
  }
  uint64_t masks[4], bases[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint64_t want = __shfl(id, 2 * p + half);  // row q's record id (lane q holds it)
    const bool hit = want != 0ull && want != kern::kZxNoExport && cand[p] == want && cbase[p] != 0ull;
    masks[p] = __ballot(hit);
    // the matching lane's base, broadcast per half (lanes without a hit contribute 0)
    bases[p] = hit ? cbase[p] : 0ull;
  }
  uint64_t ptr = 0;
  bool found = true;
  uint64_t base_q = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    // lane q (= 2p + h) takes the base from the first matching lane of half h
    const uint64_t m0 = masks[p] & 0xffffffffull, m1 = masks[p] >> 32;
    const int src0 = m0 ? __builtin_ctzll(m0) : 0, src1 = m1 ? 32 + __builtin_ctzll(m1) : 32;
    const uint64_t b0 = __shfl(bases[p], src0), b1 = __shfl(bases[p], src1);
    if (lane == 2 * p) base_q = m0 ? b0 : 0ull;
    if (lane == 2 * p + 1) base_q = m1 ? b1 : 0ull;
  }
  if (lane < W) {
    if (lane == me) {
      ptr = (uint64_t)(uintptr_t)static_cast<char*>(c.zx_self);
    } else if (id == 0ull) {
      ptr = 0;  // this peer shares nothing in this call
    } else if (base_q != 0ull) {
      ptr = base_q + off;
    } else {
      found = false;
    }
  }
  const bool mine_ok = alive && __all(found);
  tr.mark(9);
  // round 2: the vote (word 4 of slot [me] at every rank)
  bool all_ok = mine_ok;
  if (alive) {
    if (lane < W) zx_put(zx_src_words(v, lane, me) + 4, mine_ok ? 1u : 0u, ep);
    bool have = lane >= W, yes = true;
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 1;; ++it) {
      if (!have) {
        const uint64_t w = __hip_atomic_load(zx_src_words(v, me, lane) + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)(w >> 32) == ep) {
          have = true;
          yes = (uint32_t)w == 1u;
        }
      }
      if (__all(have)) break;
      timed_out = __builtin_amdgcn_s_memrealtime() - t1 > v.timeout_ticks;
      if (timed_out ||
          ((it & 255u) == 0 && __hip_atomic_load(v.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        alive = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    all_ok = alive && __all(yes);
  }
  tr.mark(10);
  // (only this wait's own timeout is filed: a word another block or the host set first names the
  // cause, and overwriting it hid a stalled host exchange behind "record exchange timed out")
  if (timed_out && lane == 0) __hip_atomic_store(v.err, 0x800u | (uint32_t)me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // publish for the kernel's blocks: every word carries this launch's tag (ptr words in their
  // top 16 bits -- virtual addresses are 48-bit -- the verdict as seq = tag << 2 | verdict), so
  // readers check each word and no write ordering (no fence) is needed
  kern::GateSlot* res = zx_resolved(v, c.zx_tag);
  const uint32_t verdict = !alive ? 0u : (all_ok ? 1u : 2u);
  if (lane < kern::kMaxRanks)
    __hip_atomic_store(&res->ptr[lane], zx_tagged(c.zx_tag, (all_ok && lane < W) ? ptr : 0ull), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  tr.mark(11);
  if (lane == 0) {
    __hip_atomic_store(&res->seq, (c.zx_tag << 2) | verdict, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    zx_verdict_note() = 0x100u | verdict;  // for the host, written at the kernel's end (zx_publish_verdict)
  }
}

// The verdict for the host's statistics (read when the gate slot is reused), stored to pinned host
// memory by the exchange block when its exchange is done (a store over PCIe stays outstanding for
// ~15 us; the exchange block has nothing left to wait for).
__device__ __forceinline__ void zx_publish_verdict(const kern::IpcCall& c) {
  if (c.gate && c.ztab && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(const_cast<uint32_t*>(&c.gate->verdict), zx_verdict_note(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// Thread 0 of every block: the resolved slot of this call (block 0 publishes it). Returns the
// verdict (0 / 1 / 2, see zx_resolve) and the buffers; false if the wait gave up.
__device__ __forceinline__ bool zx_wait(const kern::IpcView& v, const kern::IpcCall& c, uint32_t& ok,
                                        uint64_t (&ptrs)[kern::kMaxRanks]) {
  kern::GateSlot* res = zx_resolved(v, c.zx_tag);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t want = (c.zx_tag & 0xffffull) << 48;
  for (uint32_t it = 1;; ++it) {
    const uint64_t sq = __hip_atomic_load(&res->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((sq >> 2) == c.zx_tag) {
      bool all = true;
      for (int r = 0; r < v.world; ++r) {
        const uint64_t w = __hip_atomic_load(&res->ptr[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        all = all && (w & ~0xffffffffffffull) == want;
        ptrs[r] = w & 0xffffffffffffull;
      }
      if (all) {
        ok = (uint32_t)(sq & 3u);
        return true;
      }
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks) {
      __hip_atomic_store(v.err, 0x1000u | (uint32_t)v.rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    if ((it & 255u) == 0 && __hip_atomic_load(v.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void stage_args(const kern::IpcView& v, const kern::IpcCall& c, DView& sv, DCall& sc,
                                           const PhaseTrace& tr) {
  // (the exchange itself runs in the launch's exchange block, see xchg_blocks)
  if (threadIdx.x == 0) {
    __builtin_memcpy(&sv, &v, sizeof(DView));  // same layout, pointers retyped global
    __builtin_memcpy(&sc, &c, sizeof(DCall));
    if (c.gate) {
      uint32_t ok = 0;
      bool live = true, fast = false;
      if (c.ztab) {
        uint64_t ptrs[kern::kMaxRanks];
        live = zx_wait(v, c, ok, ptrs);
        if (live && ok == 1u) {
          fast = true;
          for (int r = 0; r < v.world; ++r) sv.buf[r] = reinterpret_cast<char*>((uintptr_t)ptrs[r]) + c.zoff;
        }
      }
      if (live && !fast && (!c.ztab || ok == 2u)) live = gate_wait(v, c, ok);  // the host's verdict
      if (fast) {
        sc.zc = 1;
      } else if (live && ok) {
        for (int r = 0; r < v.world; ++r)
          sv.buf[r] = reinterpret_cast<char*>((uintptr_t)__hip_atomic_load(&c.gate->ptr[r], __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_SYSTEM)) + c.zoff;
        sc.zc = 1;
      } else {
        sc.zc = 0;  // staged: the view's buffers are the staging windows already
        if (sc.coll == kern::IpcColl::ALLREDUCE_PUSH) sc.coll = kern::IpcColl::ALLREDUCE_2SHOT;
      }
    }
  }
  __syncthreads();
}

}  // namespace dev
}  // namespace pdcc
