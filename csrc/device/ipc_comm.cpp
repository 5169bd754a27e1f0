#include "ipc_comm.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>

#include "comm_util.h"

namespace pdcc {

namespace {

std::vector<uint8_t> handle_bytes(void* p) {
  hipIpcMemHandle_t h;
  PDCC_HIP(hipIpcGetMemHandle(&h, p));
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&h), reinterpret_cast<uint8_t*>(&h) + sizeof(h));
}

void* open_handle(const std::vector<uint8_t>& b) {
  if (b.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("pdcc: malformed hipIpc handle in store");
  hipIpcMemHandle_t h;
  std::memcpy(&h, b.data(), sizeof(h));
  void* p = nullptr;
  PDCC_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return p;
}

struct DeviceScope {
  int prev = 0;
  explicit DeviceScope(int d) {
    PDCC_HIP(hipGetDevice(&prev));
    if (prev != d) PDCC_HIP(hipSetDevice(d));
  }
  ~DeviceScope() { hipSetDevice(prev); }
};

}  // namespace

IpcComm::IpcComm(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank, int world,
                 int device, size_t max_staging, uint64_t timeout_ms, bool shared_device)
    : store_(store),
      key_(key),
      rank_(rank),
      world_(world),
      device_(device),
      max_staging_(std::max<size_t>(max_staging, 1u << 20)),
      timeout_ticks_(timeout_ms * 100000ull),  // s_memrealtime runs at 100 MHz
      shared_device_(shared_device) {
  if (world < 2 || world > kern::kMaxRanks)
    throw std::runtime_error("pdcc: the IPC path supports 2..8 ranks per group");
  DeviceScope ds(device);
  const size_t sig = kern::ipc_signal_bytes();
  PDCC_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&my_flags_), sig, hipDeviceMallocUncached));
  PDCC_HIP(hipMemset(my_flags_, 0, sig));
  PDCC_HIP(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 64, hipHostMallocMapped | hipHostMallocCoherent));
  *err_host_ = 0;
  PDCC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0));
  PDCC_HIP(hipDeviceSynchronize());

  const auto all = store_allgather(store_, key_ + "/ipc_sig", rank_, world_, handle_bytes(my_flags_));
  peer_flags_.assign(world_, nullptr);
  for (int r = 0; r < world_; ++r)
    peer_flags_[r] = (r == rank_) ? my_flags_ : static_cast<uint32_t*>(open_handle(all[r]));
}

IpcComm::~IpcComm() {
  try {
    DeviceScope ds(device_);
    unmap_staging();
    for (int r = 0; r < (int)peer_flags_.size(); ++r)
      if (r != rank_ && peer_flags_[r]) hipIpcCloseMemHandle(peer_flags_[r]);
    if (my_flags_) hipFree(my_flags_);
    if (err_host_) hipHostFree(err_host_);
  } catch (...) {
  }
}

void IpcComm::unmap_staging() {
  for (int r = 0; r < (int)peer_staging_.size(); ++r)
    if (r != rank_ && peer_staging_[r]) hipIpcCloseMemHandle(peer_staging_[r]);
  peer_staging_.clear();
  if (my_staging_) hipFree(my_staging_);
  my_staging_ = nullptr;
  cap_ = 0;
}

void IpcComm::map_staging(size_t cap) {
  PDCC_HIP(hipMalloc(reinterpret_cast<void**>(&my_staging_), 2 * cap));
  cap_ = cap;
  const auto all = store_allgather(store_, key_ + "/ipc_stg/" + std::to_string(staging_gen_), rank_, world_,
                                   handle_bytes(my_staging_));
  peer_staging_.assign(world_, nullptr);
  for (int r = 0; r < world_; ++r)
    peer_staging_[r] = (r == rank_) ? my_staging_ : static_cast<char*>(open_handle(all[r]));
}

void IpcComm::ensure_staging(size_t bytes, hipStream_t stream) {
  bytes = (bytes + kern::kTileBytes - 1) / kern::kTileBytes * kern::kTileBytes;
  if (bytes <= cap_) return;
  if (bytes > max_staging_) throw std::runtime_error("pdcc: IPC call larger than PDCC_IPC_MAX_STAGING");
  DeviceScope ds(device_);
  size_t cap = std::max<size_t>(bytes, 4u << 20);
  cap = std::max(cap, std::min(max_staging_, cap_ * 2));
  // nobody may still read the old buffers: drain locally, then agree globally
  PDCC_HIP(hipStreamSynchronize(stream));
  ++staging_gen_;
  store_barrier(store_, key_ + "/ipc_grow/" + std::to_string(staging_gen_), rank_, world_);
  unmap_staging();
  map_staging(cap);
}

void IpcComm::launch(kern::IpcCall call, hipStream_t stream) {
  const size_t need = kern::ipc_staging_bytes(call, world_);
  if (need > 0) ensure_staging(need, stream);
  kern::IpcView v{};
  ++seq_;  // flags compare with a wrap-safe signed difference, so uint32 wrap is harmless
  const size_t parity = seq_ & 1u;
  for (int r = 0; r < world_; ++r) {
    v.buf[r] = peer_staging_.empty() ? nullptr : peer_staging_[r] + parity * cap_;
    v.flags[r] = peer_flags_[r];
  }
  v.err = err_dev_;
  v.rank = rank_;
  v.world = world_;
  v.seq = seq_;
  v.timeout_ticks = timeout_ticks_;
  if (shared_device_) {
    // all ranks' grids must be co-resident on ONE device (test setups): keep them small
    call.grid_cap = std::max(1, 64 / world_);
  }
  DeviceScope ds(device_);
  PDCC_HIP(kern::ipc_launch(v, call, stream));
}

uint32_t IpcComm::error_word() const { return err_host_ ? __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) : 0u; }
void IpcComm::clear_error() {
  if (err_host_) __atomic_store_n(err_host_, 0u, __ATOMIC_RELEASE);
}

}  // namespace pdcc
