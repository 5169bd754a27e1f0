// Peer-memory (hipIpc over xGMI) communicator: every rank owns
//   * a staging buffer of `cap` bytes (coarse-grained HBM), and
//   * a signal area (uncached device memory) holding the block-pairwise flags
//     and the per-block call counters,
// and maps every peer's staging + signal area into its own address space. The
// IPC collective kernels (csrc/kernels) stage local data into the own buffer,
// flag the peers, and pull/reduce straight out of the peers' buffers -- all 7
// xGMI links of a node busy at once instead of one ring neighbour.
//
// Every call starts with an arrival barrier (block b waits until block b of
// every peer has started the same call): since kernels on a stream run in order,
// that proves every peer's previous call has finished reading the staging this
// call is about to overwrite, whatever grids the two calls had. One staging
// buffer suffices, and no host-side sequence number is involved.
//
// Launches may be captured into a hipGraph (parallel/graphs.py) and replayed
// freely (the kernels' per-block counters live on the device); staging a graph
// may reference is retired, not freed, when it grows.
#pragma once
#include <hip/hip_runtime_api.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../kernels/kernel_api.h"

namespace pdcc {

class IpcComm {
 public:
  // Collective: allocate own signal area + error word and exchange handles.
  IpcComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world, int device,
          size_t max_staging, uint64_t timeout_ms, bool shared_device, size_t zc_cache = 16);
  ~IpcComm();
  // Close every peer mapping and free every buffer now (idempotent; the destructor does it
  // otherwise). Collective: this rank's mappings of the peers' memory are closed first, then the
  // ranks meet through the store (within `deadline`), then each frees what it exported -- never
  // while a peer may still map it. No deadline (the destructor) or a rank that does not arrive:
  // the exported buffers stay allocated. The group's shutdown calls it once its streams are
  // drained. Only the host error word stays (Works read it).
  void release(std::chrono::milliseconds deadline);
  IpcComm(const IpcComm&) = delete;
  IpcComm& operator=(const IpcComm&) = delete;

  // Collective (all ranks pass the same value): grow the staging so one call of
  // `bytes` fits. `stream` is drained before buffers are swapped.
  void ensure_staging(size_t bytes, hipStream_t stream);
  size_t max_staging() const { return max_staging_; }
  size_t cap() const { return cap_; }
  // Largest payload one launch may stage: on the IPC launcher's thread the staging it has
  // (never grown there: growth frees and maps buffers, which synchronises the device while
  // callers' streams wait on that thread -- the submitter primes it instead), else the cap.
  size_t chunk_cap() const { return tls_defer_frees_ && cap_ > 0 ? std::min(max_staging_, cap_) : max_staging_; }

  // Launch one collective call (consumes one sequence number). May be captured
  // into a hipGraph once the staging is large enough for the call.
  void launch(kern::IpcCall call, hipStream_t stream);

  // spin timeout of the cross-GPU barriers of later launches
  void set_timeout_ms(uint64_t ms) { timeout_ticks_ = ms * 100000ull; }
  // workgroup cap of every launch on distinct devices (PDCC_IPC_GRID); same on every rank
  void set_grid_max(int g) { grid_max_ = g; }
  // workgroup cap of the launches issued inside an AsyncScope (PDCC_IPC_ASYNC_GRID: collectives
  // on the comm stream, overlapped with compute); same on every rank (0 = none)
  void set_async_grid(int g) { async_grid_ = g; }
  int async_grid() const { return async_grid_; }
  // the calling thread's launches of one async collective (RAII; the issuing thread only)
  struct AsyncScope {
    IpcComm* c;
    bool saved;
    AsyncScope(IpcComm* comm, bool on) : c(comm), saved(comm ? comm->async_now_ : false) {
      if (c) c->async_now_ = on;
    }
    ~AsyncScope() {
      if (c) c->async_now_ = saved;
    }
    AsyncScope(const AsyncScope&) = delete;
    AsyncScope& operator=(const AsyncScope&) = delete;
  };
  uint64_t async_capped() const { return async_capped_; }
  uint64_t timeout_ms() const { return timeout_ticks_ / 100000ull; }
  // a launch was captured into a graph: sequence numbers live on the device from now on
  bool graph_mode() const { return graph_mode_; }

  // Error word written by a kernel whose spin timed out (0 = healthy).
  uint32_t error_word() const;
  void clear_error();
  // Host-side abort (watchdog / abort_group): sets the error word to kAbortWord;
  // kernels spinning in a cross-GPU barrier see it within ~256 polls and leave.
  static constexpr uint32_t kAbortWord = 0x200u;
  void abort();
  // The error word's meaning: high bits = what timed out, low byte = the rank whose kernel wrote it
  //   0x100|r block-pairwise barrier   0x200 host abort          0x300|r LL flag poll
  //   0x400|r zero-copy gate wait      0x800|r device-side record exchange
  //   0x900|r dyn departure (done)     0xA00|r dyn ready word    0x1000|r resolved-slot wait
  static std::string describe_error(uint32_t w);

  // PDCC_IPC_TRACE=N: kernels record per-phase device timestamps of block 0 into a
  // host-mapped ring of N records (kern::kTraceRecWords u64 each: header + per-block stamps); copies of the valid ones
  std::vector<std::vector<uint64_t>> trace_records() const;
  bool shared_device() const { return shared_device_; }
  int world() const { return world_; }
  uint64_t calls() const { return seq_; }

  // ---- zero-copy calls: the peers read this call's USER buffers in place ----------
  // One rank's buffer, exchanged over the host transport before the launch (the
  // caller drives the exchange; every rank runs the same steps):
  //   rec = zc_export(p, len)  ->  all-gather recs  ->  zc_import(all, ...)  ->
  //   [fresh anywhere: agree on the import result]  ->  zc_settle(mine, ok)  ->  launch_zc.
  // `id` is the exporter's allocation id (HIP BUFFER_ID): an allocation freed and
  // re-made at the same address gets a new one, so nobody reads through a stale
  // mapping. Importers keep a mapping until its exporter evicts it (`evict`, LRU
  // over PDCC_IPC_ZC_CACHE exports), so all caches stay in step without extra
  // messages; exports made while capturing a graph are pinned (the graph keeps
  // the pointers) and never evicted.
  struct ZcRec {
    uint8_t ok;     // 1 = exportable: 16-B aligned, inside one allocation, handle obtained
    uint8_t fresh;  // 1 = the peers have not confirmed a mapping of `id` yet
    uint8_t full;   // 1 = this rank's list of evicted-but-open mappings is at its limit (no fresh imports)
    uint8_t pad[5];
    uint64_t id;
    uint64_t evict;  // allocation id the exporter dropped (0 = none): importers unmap it
    uint64_t off;    // byte offset of the buffer in its allocation
    uint64_t len;    // readable bytes at the buffer
    hipIpcMemHandle_t handle;
  };
  // (p, len) = (nullptr, 0): this rank shares nothing (ok = 1, id = 0)
  ZcRec zc_export(const void* p, size_t len, bool capturing);
  // Apply every peer's eviction, then (all_ok) map every rank's buffer: ptrs[r]
  // (own = `mine`). False if a mapping failed on this rank.
  bool zc_import(const std::vector<ZcRec>& all, const void* mine, bool all_ok, std::vector<char*>& ptrs);
  // group-wide outcome of this exchange: this rank's fresh export is confirmed or dropped
  void zc_settle(const ZcRec& mine, bool ok);
  // one zero-copy launch (call.zc is set here); bufs[r] = rank r's mapped buffer
  void launch_zc(kern::IpcCall call, const std::vector<char*>& bufs, hipStream_t stream);

  // ---- gated zero-copy launches (kern::GateSlot): launched before the exchange -------
  // Next gate ticket (its slot is free: the launches that read the slot kGateSlots tickets
  // ago have finished -- waits for them on the host in the rare case they have not).
  uint64_t gate_reserve();
  // One launch of `call` (the staged view; whole units), gated on ticket `t`; `zoff` = its
  // byte offset inside every rank's buffer. Staging grows here (caller's thread) so the
  // staged fallback fits.
  // `mine` / `self`: this rank's record and buffer for the device-side exchange (the kernel
  // resolves the peers' buffers itself when every rank has them mapped already)
  void launch_gated(kern::IpcCall call, uint64_t t, size_t zoff, const ZcRec& mine, const void* self,
                    hipStream_t stream);
  // device-side exchange (kern::ZcTable): on / off for this group (the self-test turns it
  // off when it fails), the last gated launch's tag and, once it finished, its verdict
  // (1 = resolved on the device, 2 = waited for the host gate, 0 = exchange gave up)
  bool zx_on() const { return zx_on_; }
  void set_zx(bool on) { zx_on_ = on; }
  uint64_t zx_last_tag() const { return zx_tag_; }
  // verdicts of the gated launches whose slots were reused so far (device / host gate / gave up)
  uint64_t zx_fast() const { return zx_fast_; }
  uint64_t zx_host() const { return zx_host_; }
  uint64_t zx_failed() const { return zx_failed_; }
  uint32_t zx_verdict(uint64_t tag);
  // after the launches of ticket `t`: their completion (slot reuse, mapping lifetime)
  struct LaunchEvent;
  struct EventPool;
  std::shared_ptr<LaunchEvent> gate_mark(uint64_t t, hipStream_t stream);
  // exchange thread: the mappings just imported are read by the launches of `ev`
  void zc_note_launch(const std::shared_ptr<LaunchEvent>& ev);
  // exchange thread: open ticket `t`'s gate (ok: ptrs[r] = rank r's mapped buffer)
  void gate_publish(uint64_t t, bool ok, const std::vector<char*>& ptrs);
  size_t zc_exports() const;
  size_t zc_mappings() const;
  // evicted mappings not closed yet (their last launch may still run, or no safe point came)
  size_t zc_closing() const;

  // The IPC launcher's thread (ProcessGroupMI355X) sets this: hipFree and hipIpcCloseMemHandle
  // synchronise the whole device, and the callers' streams wait on that thread's launches --
  // there, evicted mappings and outgrown staging are only queued, never released.
  static void set_thread_defers_frees(bool v) { tls_defer_frees_ = v; }
  // Release what was queued: close evicted mappings whose last launch finished (waits for
  // it), free retired staging. Call only with no IPC work of this communicator in flight
  // and no stream waiting on the launcher (barrier, shutdown).
  void maintain();
  // close the evicted mappings whose last launch has finished (wait_all: wait for all);
  // synchronises the device like any hipIpcCloseMemHandle -- not on the launcher's thread
  void reap_closing(bool wait_all);
  // fresh exports refused / not made because some rank's closing list was full (describe())
  uint64_t zc_full_refusals() const { return full_refusals_.load(); }
  // exports refused because the allocation's size has bit 31 set (see zc_export)
  uint64_t zc_size_refusals() const { return size_refusals_.load(); }
  // exports the runtime refused (hipIpcGetMemHandle) / peer buffers this rank could not map
  uint64_t zc_export_failures() const { return export_failures_.load(); }
  uint64_t zc_map_failures() const { return map_failures_.load(); }
  // stale peer mappings the runtime handed back for fresh exports and that were re-opened
  // (process-wide; see open_handle in ipc_comm.cpp)
  static uint64_t stale_mappings();
  // exported buffers kept instead of freed (ranks sharing one GPU, see keep_exports_)
  uint64_t kept_exports() const { return kept_exports_.load(); }
  void set_zc_size_guard(bool on) { size_guard_ = on; }
  size_t zc_closing_limit() const { return closing_limit_; }

 private:
  void map_staging(size_t cap);
  kern::IpcView view(const std::vector<char*>& bufs) const;
  // grow the staging for `call` if needed (refused while the stream is being captured)
  void prepare_staging(const kern::IpcCall& call, hipStream_t stream);
  void launch_view(const kern::IpcView& v, kern::IpcCall call, hipStream_t stream);

  struct ZcExport {
    uint64_t id;
    char* base;
    hipIpcMemHandle_t handle;
    bool confirmed;
    bool pinned;
    uint64_t last;  // LRU tick
  };
  kern::GateSlot* gates_host_ = nullptr;  // pinned, device-mapped ring of kGateSlots
  kern::GateSlot* gates_dev_ = nullptr;
  uint64_t gate_next_ = 0;
  std::vector<std::shared_ptr<LaunchEvent>> gate_last_;  // per slot: the launches that read it
  std::shared_ptr<EventPool> ev_pool_ = std::make_shared<EventPool>();
  mutable std::mutex zc_mu_;  // zc_exports_ (the caller exports, the exchange thread settles)

 public:
  // completion of one zero-copy launch (recorded on its stream right after it)
  // Recycled completion events of zero-copy launches (one per call: creating a hipEvent on
  // every call costs host time the enqueue path does not need to spend). A LaunchEvent hands
  // its event back to the pool when the last reference to it goes (any thread).
  struct EventPool {
    std::mutex mu;
    std::vector<hipEvent_t> free;
    ~EventPool();
  };
  struct LaunchEvent {
    hipEvent_t ev = nullptr;
    std::shared_ptr<EventPool> pool;
    ~LaunchEvent();
  };
  std::shared_ptr<LaunchEvent> new_launch_event(hipStream_t stream);  // recorded on `stream`

 private:
  struct ZcImport {
    uint64_t id;
    void* map;  // hipIpcOpenMemHandle result (allocation base on this side)
    std::shared_ptr<LaunchEvent> last;  // the latest launch that read through this mapping
    int tab = -1;  // its entry in the device-visible table (kern::ZcTable), -1 = none
  };
  // Device-visible table of open mappings (pinned host memory; gated kernels look the peers'
  // records up there, see kern::ZcTable). An entry is dropped (id = 0) before its mapping is
  // queued for closing, and the close then also waits for the latest gated launch of every
  // stream at that moment (any kernel that could have read the entry was launched by then).
  bool zx_on_ = true;  // set by the group (Config::ipc_zx, voted): off = gated kernels wait for the host gate
  uint64_t zx_tag_ = 0;  // gated launches so far (resolved slot = tag % kGateSlots)
  std::atomic<uint64_t> zx_fast_{0}, zx_host_{0}, zx_failed_{0};
  kern::ZcTable* ztab_host_ = nullptr;
  kern::ZcTable* ztab_dev_ = nullptr;
  std::mutex latest_mu_;
  std::vector<std::pair<hipStream_t, std::shared_ptr<LaunchEvent>>> latest_gated_;
  bool tab_busy_[kern::kMaxRanks][kern::kZcTab] = {};  // guarded by closing_mu_
  int tab_insert(int peer, uint64_t id, void* map);
  void tab_drop(int peer, int slot);     // id = 0 (the base stays until the slot is released)
  void tab_release(int peer, int slot);  // after the mapping closed (closing_mu_ held)
  std::vector<std::shared_ptr<LaunchEvent>> latest_gated();
  // Evicted mappings are closed once the last launch that used them has finished (polled
  // at every exchange; the destructor waits): no device-wide synchronisation, so compute
  // streams and point-to-point pair streams are never drained by an eviction.
  struct Closing {
    void* map;
    std::vector<std::shared_ptr<LaunchEvent>> last;  // every launch that may still read through it
    int tab_peer = -1, tab_slot = -1;  // its mapping-table slot, reusable once the mapping is closed
  };
  mutable std::mutex closing_mu_;
  std::vector<Closing> zc_closing_;
  // Bound on that list. Evictions made while gated launches may be in flight are only queued:
  // closing a mapping synchronises the device, and the gated kernels wait for the exchange
  // thread (a close from any thread while they run can deadlock in the runtime -- measured:
  // a background closer thread hung the eviction churn test). Safe points (barrier /
  // maintain(), inline exchanges) drain the list. Between them it is bounded instead: a rank
  // whose list is full says so in its record (ZcRec::full); from then on no rank makes a
  // fresh export (nothing new to map, nothing evicted) and fresh imports are refused -- such
  // calls run staged -- while buffers every rank has mapped keep running zero-copy and
  // resolving on the device. limit = kZcTab - cache: live + closing mappings always fit the
  // device-side mapping table.
  size_t closing_limit_ = 16;
  std::atomic<bool> peer_full_{false};      // some rank reported `full` in the last exchange
  std::atomic<uint64_t> full_refusals_{0};
  std::atomic<uint64_t> size_refusals_{0};
  std::atomic<uint64_t> export_failures_{0};
  std::atomic<uint64_t> map_failures_{0};
  bool size_guard_ = true;
  bool released_ = false;
  // Ranks sharing one GPU: a buffer this rank exported is never freed (outgrown staging, the group's
  // signal area and staging at release). A buffer a peer had mapped, unmapped there and then freed here
  // -- in either order, also with a group-wide barrier between -- came back to both processes at once:
  // the next group's fresh tensors were zeroed in place by a peer's memset and a later zero-copy import
  // read the importer's own tensor. Never freeing avoided it, and so did never unmapping, but kept
  // mappings of freed buffers later hung an LL poll (tests/_workers.py regroup_probe / bulk_pre_diag /
  // zc_reuse_diag, profiles/r6/regroup/README.md). The memory stays with the process; distinct GPUs
  // (another device's memory imported) free as usual.
  bool keep_exports_ = false;
  std::atomic<uint64_t> kept_exports_{0};
  void drop_map(void* m);
  mutable std::mutex imports_mu_;  // zc_imports_ (launcher thread imports, describe() counts)
  static thread_local bool tls_defer_frees_;
  std::vector<void*> deferred_free_;  // refused exportable blocks allocated on the launcher's thread
  std::vector<char*> parked_;         // exported buffers a peer may still map: freed by release()
  std::vector<uint64_t> zc_cur_ids_;  // per peer: the allocation id mapped by the last zc_import
  std::vector<ZcExport> zc_exports_;
  std::vector<std::vector<ZcImport>> zc_imports_;  // per peer
  size_t zc_cache_ = 16;
  uint64_t zc_tick_ = 0;

  c10::intrusive_ptr<c10d::Store> store_;
  std::string key_;
  int rank_, world_, device_;
  int log_ = 0;  // PDCC_LOG_LEVEL >= 3: staging growth, mapping opens / closes
  size_t max_staging_;
  uint64_t timeout_ticks_;
  bool shared_device_;
  int grid_max_ = 0;  // 0: the kernel library's default cap
  int async_grid_ = 0;
  // workgroup caps of the launches when ranks share a device: 256 / W, and kSharedWideSlots / W - 1 per
  // rank from kSharedWideMin bytes (see launch_view)
  static constexpr int kSharedWideSlots = 448;
  static constexpr size_t kSharedWideMin = size_t{32} << 20;
  int shared_grid_ = 128;
  int shared_wide_grid_ = 223;
  bool async_now_ = false;     // inside an AsyncScope (the group's issuing thread)
  uint64_t async_capped_ = 0;  // launches the async cap applied to

  uint32_t* my_flags_ = nullptr;          // uncached device memory
  uint32_t* dyn_ctl_ = nullptr;           // the dynamic protocols' control words (kern::IpcView::dctl)
  std::vector<uint32_t*> peer_flags_;     // mapped (own entry = my_flags_)
  std::vector<void*> flags_maps_;         // hipIpcOpenMemHandle results to close (may precede the pointer)
  uint32_t* err_host_ = nullptr;          // pinned, device-visible
  uint32_t* err_dev_ = nullptr;
  uint64_t* trace_host_ = nullptr;        // PDCC_IPC_TRACE ring (pinned, device-visible), or null
  uint64_t* trace_dev_ = nullptr;
  uint32_t trace_cap_ = 0;

  char* my_staging_ = nullptr;
  size_t cap_ = 0;                         // staging bytes
  std::vector<char*> peer_staging_;
  std::vector<void*> staging_maps_;
  int staging_gen_ = 0;
  uint32_t seq_ = 0;
  bool graph_mode_ = false;
  struct Retired {
    char* mine;
    std::vector<void*> maps;
  };
  std::vector<Retired> retired_;  // staging a captured graph may still use (freed with the group)
};

}  // namespace pdcc
