// build: hipcc --offload-arch=gfx950 -O2 scripts/probes/gate_latency.hip -o scripts/probes/gate_latency
// Probe: device-side cost of the zero-copy gate poll (dev_common.h gate_wait) on MI355X.
// Times, with s_memrealtime (100 MHz), (a) one system-scope acquire load of pinned coherent
// host memory, (b) the same of device memory, (c) s_sleep(4) and s_sleep(127), and (d) how
// long a kernel takes to see a host store into pinned memory (the host publishes while the
// kernel polls). One block of 64 threads; every spin is bounded.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_lat(const uint64_t* host, const uint64_t* dev, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint64_t acc = 0;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 100; ++i) acc += __hip_atomic_load(host, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 100; ++i) acc += __hip_atomic_load(dev, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t t2 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 100; ++i) __builtin_amdgcn_s_sleep(4);
  uint64_t t3 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 10; ++i) __builtin_amdgcn_s_sleep(127);
  uint64_t t4 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 100; ++i) acc += __hip_atomic_load(host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t t5 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; out[5] = acc;
}

// polls *flag until it equals want (bounded by ~2 s), records the ticks it took
__global__ void k_wait(const uint64_t* flag, uint64_t want, uint64_t* out, int sleep_mode) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t n = 0;
  for (;;) {
    ++n;
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == want) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
    if (sleep_mode == 1) __builtin_amdgcn_s_sleep(4);
    if (sleep_mode == 2) __builtin_amdgcn_s_sleep(127);
  }
  out[0] = __builtin_amdgcn_s_memrealtime() - t0;
  out[1] = n;
}

int main() {
  uint64_t *host = nullptr, *dev = nullptr, *out = nullptr, *hout = nullptr;
  CK(hipHostMalloc((void**)&host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipMalloc((void**)&dev, 4096));
  CK(hipMalloc((void**)&out, 4096));
  CK(hipHostMalloc((void**)&hout, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  uint64_t* host_d = nullptr;
  CK(hipHostGetDevicePointer((void**)&host_d, host, 0));
  uint64_t* hout_d = nullptr;
  CK(hipHostGetDevicePointer((void**)&hout_d, hout, 0));
  host[0] = 1;
  CK(hipMemset(dev, 0, 4096));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, host_d, dev, out);
    CK(hipDeviceSynchronize());
    uint64_t r[6];
    CK(hipMemcpy(r, out, sizeof(r), hipMemcpyDeviceToHost));
    printf("{\"probe\": \"latency\", \"host_acquire_load_us\": %.3f, \"dev_acquire_load_us\": %.3f, \"s_sleep4_us\": %.3f, "
           "\"s_sleep127_us\": %.3f, \"host_relaxed_load_us\": %.3f}\n",
           r[0] / 100.0 / 100.0, r[1] / 100.0 / 100.0, r[2] / 100.0 / 100.0, r[3] / 10.0 / 100.0, r[4] / 100.0 / 100.0);
  }
  // host publishes 200 us after the launch; the kernel polls with each sleep mode
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      const uint64_t want = 100 + mode * 10 + rep;
      hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, 0, host_d, want, hout_d, mode);
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {}
      __atomic_store_n(&host[0], want, __ATOMIC_RELEASE);
      CK(hipDeviceSynchronize());
      printf("{\"probe\": \"publish_after_200us\", \"sleep_mode\": %d, \"kernel_wait_us\": %.1f, \"polls\": %llu}\n",
             mode, hout[0] / 100.0, (unsigned long long)hout[1]);
    }
    // already published before the launch: the first poll must see it
    const uint64_t want = 200 + mode;
    __atomic_store_n(&host[0], want, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, 0, host_d, want, hout_d, mode);
    CK(hipDeviceSynchronize());
    printf("{\"probe\": \"published_before\", \"sleep_mode\": %d, \"kernel_wait_us\": %.2f, \"polls\": %llu}\n", mode,
           hout[0] / 100.0, (unsigned long long)hout[1]);
  }
  return 0;
}
