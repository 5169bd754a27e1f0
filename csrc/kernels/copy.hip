// K2 multi-tensor pack/unpack and the copy family of the IPC collectives
// (broadcast, all-gather, gather, scatter, all-to-all, barrier), plus the
// host-side entry points that dispatch on dtype into reduce_<dt>.hip.
#include <algorithm>

#include "reduce_impl.h"

namespace pdcc {
namespace dev {

// --------------------------------------------------------------------------- K2
struct CopyArgs {
  kern::CopyDesc d[kern::kMaxCopyDescs];
  uint64_t prefix[kern::kMaxCopyDescs + 1];  // prefix sums of FULL tiles per descriptor
  int n;
  int ntail;                                  // descriptors with a partial last tile
  int tail_idx[kern::kMaxCopyDescs];
};

// Tile g of the launch lives in descriptor j with prefix[j] <= g < prefix[j+1]. A
// block visits its tiles in increasing order (and pipe_run asks for sources and
// destinations in increasing order too), so each side keeps a monotonic cursor:
// amortised O(1) uniform scalar steps per tile instead of a binary search.
struct DescMap {
  const CopyArgs* a;
  size_t first, stride, total;
  mutable int js = 0, jd = 0;  // descriptor cursors of the source and destination sides
  __device__ size_t count() const { return first < total ? (total - 1 - first) / stride + 1 : 0; }
  __device__ size_t advance(int& j, size_t i) const {
    const size_t g = first + i * stride;
    while (a->prefix[j + 1] <= g) ++j;
    return g - a->prefix[j];
  }
  __device__ const char* src(int, size_t i) const {
    const size_t lt = advance(js, i);
    return (const char*)a->d[js].src + lt * kTile;
  }
  __device__ char* dst(size_t i) const {
    const size_t lt = advance(jd, i);
    return (char*)a->d[jd].dst + lt * kTile;
  }
  __device__ size_t valid(size_t) const { return kTile; }
};

// NTL: non-temporal source loads (a pack / unpack reads each source once)
template <int D, bool NTL>
__global__ void __launch_bounds__(256) k2_multi_copy(CopyArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[PipeLds<1, D>::kBytes];
  const DescMap m{&a, blockIdx.x, gridDim.x, a.prefix[a.n]};
  pipe_run<DType::U8, RedOp::COPY, 1, D, DescMap, 1, false, NTL>(lds, m, 1);
  // partial last tiles: one block each, bounded plain loads
  for (int k = blockIdx.x; k < a.ntail; k += gridDim.x) {
    const kern::CopyDesc& d = a.d[a.tail_idx[k]];
    const size_t full = d.bytes / kTile * kTile;
    const size_t off = full + (threadIdx.x >> 6) * kWaveBytes + (threadIdx.x & 63) * 16;
    if (off < d.bytes) {
      const uint32_t lim = (uint32_t)(d.bytes - off < 16 ? d.bytes - off : 16);
      const char* s = (const char*)d.src + off;
      char* o = (char*)d.dst + off;
      if (lim == 16) *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(s);
      else store_partial(o, load_partial(s, lim), lim);
    }
  }
}

// ----------------------------------------------------------- IPC copy family
// Dynamic zero-copy all-gather (IpcCall::dyn): items of K tiles, each pulled from every rank's
// input (owners rotated per item) into out[q]; the claim loop and departure of the dynamic
// all-reduce (reduce_impl.h).
template <int W>
__device__ __forceinline__ void ipc_allgather_dyn(const DView& v, const DCall& c, char* lds, const PhaseTrace* tr) {
  const uint32_t xb = xchg_blocks(c), G = gridDim.x - xb, b = blockIdx.x - xb;
  const size_t nt = c.bytes / kTile;
  const uint32_t K = kern::dyn_rows_per_chunk(nt, G, (uint32_t)c.dyn, (uint32_t)c.dyn_min_rows);
  const uint32_t nc = (uint32_t)((nt + K - 1) / K);
  const uint32_t dep = dyn_epoch(v, tr);
  dyn_claim_loop(v, nc, tr, b, G, [&](uint32_t it) {
    const size_t t0 = (size_t)it * K, t1 = t0 + K < nt ? t0 + K : nt;
    const PeerTileMap<W> m{&v, &c, 0, c.bytes, (uint32_t)(v.rank + it), t0, 1, t1};
    ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
  });
  dyn_depart(v, dep, true, tr, G);
}

// Zero-copy copies (IpcCall::zc): peers' user buffers are read in place; data
// arrival barrier first, departure barrier last (see ipc_reduce_zc).
template <int W>
__device__ __forceinline__ void ipc_copy_zc(const DView& v, const DCall& c, char* lds, const PhaseTrace tr,
                                            uint32_t ep) {
  const size_t G = gridDim.x - xchg_blocks(c), b = blockIdx.x - xchg_blocks(c);  // the data blocks
  const int me = v.rank;
  const size_t nt = c.bytes / kTile;
  block_barrier(v, ep);
  tr.mark(2);
  tr.mark(4);
  if (c.coll == IpcColl::ALLGATHER && c.dyn) {
    ipc_allgather_dyn<W>(v, c, lds, &tr);
    tr.mark(5);
    return;
  }
  switch (c.coll) {
    case IpcColl::BROADCAST_2SHOT: {
      if (me != c.root) {  // phase 1: my owned tiles straight from the root's buffer into mine
        const OneSrcMap m{v.buf[c.root], v.buf[me], c.bytes, (size_t)me + W * b, W * G, nt};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      tr.mark(5);
      block_barrier(v, ep + 2u);
      tr.mark(6);
      if (me != c.root) {  // phase 2: the other owners' tiles (the root's own straight from the root)
        const PeerRowMap<W> m{&v, v.buf[me], (uint32_t)b, b, G, nt / W};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      break;
    }
    case IpcColl::ALLGATHER:
    case IpcColl::GATHER:
      if (c.coll == IpcColl::ALLGATHER || me == c.root) {
        const PeerTileMap<W> m{&v, &c, 0, c.bytes, (uint32_t)(me + b), b, G, nt};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      tr.mark(5);
      break;
    case IpcColl::ALLTOALL: {
      const PeerTileMap<W> m{&v, &c, (size_t)me * c.zstride, c.bytes, (uint32_t)(me + b), b, G, nt};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      tr.mark(5);
      break;
    }
    case IpcColl::SCATTER: {  // my chunk straight out of the root's flat list
      const OneSrcMap m{v.buf[c.root] + (size_t)me * c.zstride, (char*)c.out[0], c.bytes, b, G, nt};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      tr.mark(5);
      break;
    }
    default:
      break;
  }
  block_barrier<false>(v, ep + 3u);  // departure
}

template <int W>
__device__ __forceinline__ void ipc_copy_body(const DView& v, const DCall& c, char* lds, const PhaseTrace tr,
                                              uint32_t seq) {
  const size_t G = gridDim.x - xchg_blocks(c), b = blockIdx.x - xchg_blocks(c);  // the data blocks
  const int me = v.rank;
  tr.seq(seq);
  const uint32_t ep = seq * kern::kEpochsPerCall, ph0 = ep + 1u, ph1 = ep + 2u;
  if (c.coll == IpcColl::BARRIER) {  // the arrival barrier is the whole collective
    block_barrier<false>(v, ep);
    return;
  }
  if (c.zc) {
    ipc_copy_zc<W>(v, c, lds, tr, ep);
    return;
  }
  block_barrier<false>(v, ep);  // arrival: every peer's previous call is over
  tr.mark(2);
  const size_t poff = 0;        // single staging buffer (the arrival barrier guards reuse)
  char* mine = v.buf[me];
  const size_t nt = pad_tiles(c.bytes) / kTile;
  const size_t cpad = nt * kTile;

  switch (c.coll) {
    case IpcColl::BROADCAST_1SHOT: {
      if (me == c.root) stage_tiles((const char*)c.in[0], mine, c.bytes, b, G, nt);
      tr.mark(3);
      block_barrier(v, ph0);
      tr.mark(4);
      if (me == c.root) return;
      const OneSrcMap m{v.buf[c.root] + poff, (char*)c.out[0], c.bytes, b, G, nt};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      return;
    }
    case IpcColl::BROADCAST_2SHOT: {
      // rows (t / W) belong to block row % G; tile t is owned by rank t % W
      if (me == c.root)
        for (int q = 0; q < W; ++q) stage_tiles((const char*)c.in[0], mine, c.bytes, q + W * b, W * G, nt);
      block_barrier(v, ph0);
      if (me != c.root) {  // phase 1: fetch my owned tiles from the root (one link each)
        const OneSrcMap m{v.buf[c.root] + poff, mine, cpad, me + W * b, W * G, nt};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      block_barrier(v, ph1);
      if (me == c.root) return;
      {  // phase 2: every owner's tiles, owners interleaved (all links at once)
        const OwnerRowMap<W> m{v.buf, poff, (char*)c.out[0], c.bytes, (uint32_t)(me + b), b, G, (nt + W - 1) / W};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      return;
    }
    case IpcColl::ALLGATHER:
    case IpcColl::GATHER: {
      stage_tiles((const char*)c.in[0], mine, c.bytes, b, G, nt);
      tr.mark(3);
      block_barrier(v, ph0);
      tr.mark(4);
      if (c.coll == IpcColl::GATHER && me != c.root) return;
      {
        const PeerTileMap<W> m{&v, &c, poff, c.bytes, (uint32_t)(me + b), b, G, nt};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      return;
    }
    case IpcColl::SCATTER: {
      if (me == c.root)
        for (int q = 0; q < W; ++q) stage_tiles((const char*)c.in[q], mine + q * cpad, c.bytes, b, G, nt);
      block_barrier(v, ph0);
      const OneSrcMap m{v.buf[c.root] + poff + me * cpad, (char*)c.out[0], c.bytes, b, G, nt};
      ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      return;
    }
    case IpcColl::ALLTOALL: {
      for (int q = 0; q < W; ++q) stage_tiles((const char*)c.in[q], mine + q * cpad, c.bytes, b, G, nt);
      block_barrier(v, ph0);
      {
        const PeerTileMap<W> m{&v, &c, poff + me * cpad, c.bytes, (uint32_t)(me + b), b, G, nt};
        ipc_pipe<DType::U8, RedOp::COPY, 1, kCopyDepth>(lds, m, 1);
      }
      return;
    }
    default:
      return;
  }
}

template <int W>
__global__ void __launch_bounds__(256) k_ipc_copy(IpcView v, IpcCall c) {
  __shared__ __attribute__((aligned(16))) char lds[PipeLds<1, kCopyDepth>::kBytes];
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
  const uint32_t seq = block_seq(v, block_seq_load(v));  // (see k_ipc_reduce)
  stage_args(v, c, sv, sc, tr);  // (a gated zero-copy launch waits for its buffers here)
  if (c.gate) tr.mark(3);    // gate passed (zero-copy calls do not stage: [3] is free there)
  ipc_copy_body<W>(sv, sc, lds, tr, seq);
  tr.finish(v);
}

}  // namespace dev

// =============================================================== host entry points
namespace kern {

bool supports(DType t, RedOp op) {
  if (op == RedOp::COPY) return true;
  const bool is_float = t == DType::F32 || t == DType::F16 || t == DType::BF16 || t == DType::F64;
  const bool is_int = t == DType::I8 || t == DType::U8 || t == DType::I32 || t == DType::I64;
  if (t == DType::BOOL) return op == RedOp::MAX || op == RedOp::MIN || op == RedOp::BAND || op == RedOp::BOR ||
                               op == RedOp::BXOR || op == RedOp::SUM || op == RedOp::PROD;
  if (is_float) return op == RedOp::SUM || op == RedOp::AVG || op == RedOp::PROD || op == RedOp::MIN ||
                       op == RedOp::MAX;
  return is_int;
}

// bool: SUM == logical OR == MAX, PROD == logical AND == MIN (ProcessGroupNCCL semantics)
static void canon(DType& t, RedOp& op) {
  if (t == DType::BOOL) {
    t = DType::U8;
    if (op == RedOp::SUM) op = RedOp::MAX;
    if (op == RedOp::PROD) op = RedOp::MIN;
  }
}

static hipError_t k1_dispatch(const void* const* srcs, int nsrc, void* out, size_t count, DType t, RedOp op,
                              int avg_div, hipStream_t stream, int max_blocks, int lds) {
  if (nsrc < 1 || nsrc > kMaxRanks || op == RedOp::COPY || !supports(t, op)) return hipErrorInvalidValue;
  canon(t, op);
  const size_t nbytes = count * dtype_size(t);
  if (nbytes == 0) return hipSuccess;
  const size_t tiles = nbytes / kTileBytes;
  // one workgroup per CU streams fastest with the strided tile map (measured: 256 > 512 > 1024)
  int grid = (int)std::min<size_t>(std::max<size_t>(tiles, 1), max_blocks > 0 ? (size_t)max_blocks : 256);
  using namespace dev;
  switch (t) {
    case DType::F32: return k1_dispatch_F32(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::F16: return k1_dispatch_F16(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::BF16: return k1_dispatch_BF16(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::F64: return k1_dispatch_F64(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::I8: return k1_dispatch_I8(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::U8: return k1_dispatch_U8(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::I32: return k1_dispatch_I32(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    case DType::I64: return k1_dispatch_I64(srcs, nsrc, out, nbytes, op, avg_div, stream, grid, lds);
    default: return hipErrorInvalidValue;
  }
}

hipError_t reduce_nway(const void* const* srcs, int nsrc, void* out, size_t count, DType t, RedOp op, int avg_div,
                       hipStream_t stream, int max_blocks, bool nt) {
  return k1_dispatch(srcs, nsrc, out, count, t, op, avg_div, stream, max_blocks, 1 | (nt ? 2 : 0));
}
hipError_t reduce_nway_regs(const void* const* srcs, int nsrc, void* out, size_t count, DType t, RedOp op,
                            int avg_div, hipStream_t stream, int max_blocks, bool nt) {
  return k1_dispatch(srcs, nsrc, out, count, t, op, avg_div, stream, max_blocks, nt ? 2 : 0);
}
hipError_t reduce_nway_mode(const void* const* srcs, int nsrc, void* out, size_t count, DType t, RedOp op,
                            int avg_div, hipStream_t stream, int max_blocks, int mode) {
  if (mode < 0 || mode > 15) return hipErrorInvalidValue;
  return k1_dispatch(srcs, nsrc, out, count, t, op, avg_div, stream, max_blocks, mode);
}

// Default K2 grid from the launch's shape (scripts/k2_sweep.py on MI355X, profiles/README.md):
// small lists are latency-bound and want one tile per workgroup; big streams want few,
// long-running workgroups, and the fewer the larger the descriptors (each workgroup's
// strided tiles then stay within one DRAM-friendly window): 256 workgroups from 16 MiB
// per descriptor (8 x 32 MiB: 5.9 TB/s vs 4.9 at 1024), 512 below (64 x 4 MiB: 5.6 vs 5.1).
static int k2_grid(uint64_t tiles, int ndesc, size_t bytes) {
  if (tiles <= 4096) return (int)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 2048));
  const size_t avg = bytes / (size_t)std::max(1, ndesc);
  return avg >= (16u << 20) ? 256 : 512;
}

// Non-temporal source loads by default for big lists of mid-size tensors (scripts/k2_sweep.py on
// MI355X, profiles/r3/k2_sweep_ntl_r3.json: 64 x 4 MiB 5.90 vs 5.45 TB/s, 8 x 32 MiB 5.85 vs 5.80);
// a wash or slightly worse for 128-256 MiB descriptors and for small lists.
static bool k2_ntl(size_t bytes, int ndesc) {
  return bytes >= (64u << 20) && bytes / (size_t)std::max(1, ndesc) <= (32u << 20);
}

hipError_t multi_copy(const CopyDesc* descs, int n, hipStream_t stream, int max_blocks, int depth, int ntl_mode) {
  if (depth <= 0) depth = kK2Depth;
  auto aligned = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  for (int base = 0; base < n; base += kMaxCopyDescs) {
    dev::CopyArgs a{};
    const int m = std::min(kMaxCopyDescs, n - base);
    uint64_t acc = 0;
    size_t bytes = 0;
    for (int k = 0; k < m; ++k) {
      a.d[a.n] = descs[base + k];
      if (a.d[a.n].bytes == 0) continue;
      if (!aligned(a.d[a.n].src) || !aligned(a.d[a.n].dst)) {
        // the 16-B vector / LDS-DMA path needs aligned endpoints: DMA engine copy instead
        hipError_t e = hipMemcpyAsync(a.d[a.n].dst, a.d[a.n].src, a.d[a.n].bytes, hipMemcpyDeviceToDevice, stream);
        if (e != hipSuccess) return e;
        continue;
      }
      a.prefix[a.n] = acc;
      acc += a.d[a.n].bytes / kTileBytes;
      if (a.d[a.n].bytes % kTileBytes) a.tail_idx[a.ntail++] = a.n;
      bytes += a.d[a.n].bytes;
      ++a.n;
    }
    if (a.n == 0) continue;
    a.prefix[a.n] = acc;
    const int cap = max_blocks > 0 ? max_blocks : k2_grid(acc, a.n, bytes);
    const bool ntl = ntl_mode < 0 ? k2_ntl(bytes, a.n) : ntl_mode > 0;
    const int grid =
        (int)std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint64_t>(acc, (uint64_t)a.ntail), (uint64_t)cap));
    if (depth >= 8) {
      if (ntl) hipLaunchKernelGGL((dev::k2_multi_copy<8, true>), dim3(grid), dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((dev::k2_multi_copy<8, false>), dim3(grid), dim3(256), 0, stream, a);
    } else {
      if (ntl) hipLaunchKernelGGL((dev::k2_multi_copy<4, true>), dim3(grid), dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((dev::k2_multi_copy<4, false>), dim3(grid), dim3(256), 0, stream, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// block-pairwise flags, the per-block call counters, the LL control words and LL slots
size_t ipc_signal_bytes() { return kDynOffset + kDynBytes; }

size_t ipc_staging_bytes(const IpcCall& c, int world) {
  if (c.gate) {  // either protocol may run: the larger need
    IpcCall z = c, st = c;
    z.gate = st.gate = nullptr;
    z.ztab = st.ztab = nullptr;
    z.zc = 1;
    st.zc = 0;
    if (st.coll == IpcColl::ALLREDUCE_PUSH) st.coll = IpcColl::ALLREDUCE_2SHOT;
    return std::max(ipc_staging_bytes(z, world), ipc_staging_bytes(st, world));
  }
  if (c.zc)  // peers read the user buffers in place; a rooted reduce stages its reduced tiles,
             // the push all-reduce receives W slots of bytes / W
    return c.coll == IpcColl::REDUCE_2SHOT || c.coll == IpcColl::ALLREDUCE_PUSH
               ? (c.bytes + kTileBytes - 1) / kTileBytes * kTileBytes : 0;
  if (c.coll == IpcColl::ALLREDUCE_PUSH) return 0;  // (zero-copy only; rejected by ipc_launch)
  if (is_ll(c.coll)) return 0;  // straight into LL slots
  const size_t cpad = (c.bytes + kTileBytes - 1) / kTileBytes * kTileBytes;
  switch (c.coll) {
    case IpcColl::SCATTER:
    case IpcColl::REDUCE_SCATTER:
    case IpcColl::ALLTOALL:
      return cpad * world;
    case IpcColl::BARRIER:
      return 0;
    case IpcColl::ALLREDUCE_2SHOT:
    case IpcColl::REDUCE_2SHOT:
    case IpcColl::BROADCAST_2SHOT: {
      // whole rows of W tiles: phase 2 (dev::OwnerRowMap) reads a partial last row's padding
      const size_t row = (size_t)world * kTileBytes;
      return (cpad + row - 1) / row * row;
    }
    default:
      return cpad;
  }
}

hipError_t ipc_launch(const IpcView& v, const IpcCall& call, hipStream_t stream) {
  IpcCall c = call;
  if (v.world < 2 || v.world > kMaxRanks) return hipErrorInvalidValue;
  if (c.gate && (c.zc || is_ll(c.coll))) return hipErrorInvalidValue;  // the kernel picks zc for a gated call
  if (c.zc || c.gate) {  // in-place reads of user buffers: whole tiles (2-shot: whole rows of W tiles), no over-read
    const bool rows = c.coll == IpcColl::ALLREDUCE_2SHOT || c.coll == IpcColl::BROADCAST_2SHOT ||
                      c.coll == IpcColl::REDUCE_2SHOT || c.coll == IpcColl::ALLREDUCE_PUSH;
    const bool known = rows || c.coll == IpcColl::ALLGATHER || c.coll == IpcColl::GATHER ||
                       c.coll == IpcColl::SCATTER || c.coll == IpcColl::REDUCE_SCATTER ||
                       c.coll == IpcColl::ALLTOALL;
    const size_t unit = (size_t)kTileBytes * (rows ? v.world : 1);
    if (!known || c.bytes == 0 || c.bytes % unit != 0) return hipErrorInvalidValue;
  }
  const size_t nt = (c.bytes + kTileBytes - 1) / kTileBytes;
  int grid = c.grid;
  if (grid <= 0) {
    size_t g;
    switch (c.coll) {
      case IpcColl::ALLREDUCE_2SHOT:
      case IpcColl::ALLREDUCE_PUSH:
      case IpcColl::REDUCE_2SHOT:
      case IpcColl::BROADCAST_2SHOT:
        g = (nt + v.world - 1) / v.world;  // rows
        break;
      case IpcColl::BARRIER:
        g = 1;
        break;
      case IpcColl::ALLREDUCE_LL:
      case IpcColl::ALLGATHER_LL:
      case IpcColl::REDUCE_LL:
      case IpcColl::BROADCAST_LL:
      case IpcColl::GATHER_LL:
      case IpcColl::SCATTER_LL:
      case IpcColl::REDUCE_SCATTER_LL:
      case IpcColl::ALLTOALL_LL:
        g = ((c.bytes + 7) / 8 + kBlockThreads - 1) / kBlockThreads;  // one 8-byte line per thread
        break;
      default:
        g = nt;
    }
    grid = (int)std::max<size_t>(1, std::min<size_t>(g, c.grid_cap > 0 ? (size_t)c.grid_cap : 512));
  }
  if (c.grid_cap > 0) grid = std::min(grid, c.grid_cap);
  grid = std::min(grid, kMaxBlocks);
  // a gated zero-copy launch with the device-side exchange: one more workgroup, block 0, does only
  // the exchange (dev::xchg_blocks); the data blocks keep the grid every rank computes the same way
  if (c.gate && c.ztab && !is_ll(c.coll)) grid = std::min(grid, kMaxBlocks - 1) + 1;
  if (c.coll == IpcColl::ALLREDUCE_PUSH && !c.zc && !c.gate) return hipErrorInvalidValue;
  if (is_ll(c.coll) && (c.zc || c.bytes == 0 || c.bytes > kLLMaxBytes))
    return hipErrorInvalidValue;
  const bool ll_rooted = c.coll == IpcColl::REDUCE_LL || c.coll == IpcColl::BROADCAST_LL ||
                         c.coll == IpcColl::GATHER_LL || c.coll == IpcColl::SCATTER_LL;
  if (ll_rooted && (c.root < 0 || c.root >= v.world)) return hipErrorInvalidValue;
  const bool reducing = c.coll == IpcColl::ALLREDUCE_1SHOT || c.coll == IpcColl::ALLREDUCE_2SHOT ||
                        c.coll == IpcColl::ALLREDUCE_PUSH || c.coll == IpcColl::ALLREDUCE_LL ||
                        c.coll == IpcColl::REDUCE_LL || c.coll == IpcColl::REDUCE_SCATTER_LL ||
                        c.coll == IpcColl::REDUCE_1SHOT || c.coll == IpcColl::REDUCE_2SHOT ||
                        c.coll == IpcColl::REDUCE_SCATTER;
  if (c.coll == IpcColl::ALLGATHER_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL(dev::k_ll_allgather<WW>, dim3(grid), dim3(256), 0, stream, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (c.coll == IpcColl::ALLTOALL_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL(dev::k_ll_alltoall<WW>, dim3(grid), dim3(256), 0, stream, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (c.coll == IpcColl::BROADCAST_LL || c.coll == IpcColl::GATHER_LL || c.coll == IpcColl::SCATTER_LL) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL(dev::k_ll_rooted<WW>, dim3(grid), dim3(256), 0, stream, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (!reducing) {
    switch (v.world) {
#define PDCC_W(WW) \
  case WW: hipLaunchKernelGGL(dev::k_ipc_copy<WW>, dim3(grid), dim3(256), 0, stream, v, c); break;
      PDCC_W(2) PDCC_W(3) PDCC_W(4) PDCC_W(5) PDCC_W(6) PDCC_W(7) PDCC_W(8)
#undef PDCC_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (!supports(c.dtype, c.op)) return hipErrorInvalidValue;
  canon(c.dtype, c.op);
  using namespace dev;
  switch (c.dtype) {
    case DType::F32: return ipc_dispatch_F32(v, c, stream, grid);
    case DType::F16: return ipc_dispatch_F16(v, c, stream, grid);
    case DType::BF16: return ipc_dispatch_BF16(v, c, stream, grid);
    case DType::F64: return ipc_dispatch_F64(v, c, stream, grid);
    case DType::I8: return ipc_dispatch_I8(v, c, stream, grid);
    case DType::U8: return ipc_dispatch_U8(v, c, stream, grid);
    case DType::I32: return ipc_dispatch_I32(v, c, stream, grid);
    case DType::I64: return ipc_dispatch_I64(v, c, stream, grid);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace kern
}  // namespace pdcc
