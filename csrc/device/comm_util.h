// Small helpers shared by the device communicators: HIP error checks and a
// Store-based all-gather of opaque blobs (used to bootstrap RCCL unique ids,
// hipIpc handles and topology records).
#pragma once
#include <hip/hip_runtime_api.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

namespace pdcc {

#define PDCC_HIP(expr)                                                                          \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      throw std::runtime_error(std::string("pdcc: HIP error '") + hipGetErrorString(_e) + "' at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);          \
  } while (0)

inline std::vector<std::vector<uint8_t>> store_allgather(const c10::intrusive_ptr<c10d::Store>& store,
                                                         const std::string& key, int rank, int world,
                                                         const std::vector<uint8_t>& mine) {
  store->set(key + "/" + std::to_string(rank), mine);
  std::vector<std::vector<uint8_t>> all(world);
  for (int r = 0; r < world; ++r) all[r] = (r == rank) ? mine : store->get(key + "/" + std::to_string(r));
  return all;
}

// Host barrier through the store (only used on rare control paths: buffer growth).
inline void store_barrier(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank,
                          int world) {
  store->set(key + "/" + std::to_string(rank), std::vector<uint8_t>{1});
  std::vector<std::string> keys;
  for (int r = 0; r < world; ++r) keys.push_back(key + "/" + std::to_string(r));
  store->wait(keys);
}

// The same with a deadline: false when some rank did not arrive in time (a peer that is gone).
inline bool store_barrier_for(const c10::intrusive_ptr<c10d::Store>& store, const std::string& key, int rank,
                              int world, std::chrono::milliseconds deadline) {
  try {
    store->set(key + "/" + std::to_string(rank), std::vector<uint8_t>{1});
    std::vector<std::string> keys;
    for (int r = 0; r < world; ++r) keys.push_back(key + "/" + std::to_string(r));
    store->wait(keys, deadline);
    return true;
  } catch (...) {
    return false;
  }
}

}  // namespace pdcc
