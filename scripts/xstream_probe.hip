// Cross-stream dependency cost on MI355X: stream A -> stream B -> A ping-pong
// with (1) hipEventRecord/hipStreamWaitEvent and (2) stream memory operations
// (hipStreamWriteValue64 / hipStreamWaitValue64 on signal memory), with a tiny
// kernel on each side. Prints host enqueue and end-to-end microseconds per hop.
//   hipcc --offload-arch=gfx950 -O2 scripts/xstream_probe.hip -o /tmp/xstream_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void tiny(int* p) { if (threadIdx.x == 0) p[0] += 1; }

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int* d;
  CK(hipMalloc(&d, 64));
  const int N = 2000;
  using clk = std::chrono::steady_clock;
  // 1) events
  hipEvent_t ea[16], eb[16];
  for (int i = 0; i < 16; ++i) {
    CK(hipEventCreateWithFlags(&ea[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb[i], hipEventDisableTiming));
  }
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, d);
      CK(hipEventRecord(ea[i & 15], a));
      CK(hipStreamWaitEvent(b, ea[i & 15], 0));
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, b, d);
      CK(hipEventRecord(eb[i & 15], b));
      CK(hipStreamWaitEvent(a, eb[i & 15], 0));
    }
    auto t1 = clk::now();
    CK(hipDeviceSynchronize());
    auto t2 = clk::now();
    if (rep) printf("events:       enqueue %.2f us/iter, e2e %.2f us/iter\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  }
  // 2) stream memory ops on signal memory
  uint64_t* sig = nullptr;
  uint64_t* sig2 = nullptr;
  if (hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory) != hipSuccess ||
      hipExtMallocWithFlags((void**)&sig2, 8, hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    printf("signal memory unavailable, using fine-grained host memory\n");
    CK(hipHostMalloc((void**)&sig, 4096, hipHostMallocCoherent));
    sig2 = sig + 8;
  }
  CK(hipMemset(sig, 0, 8));
  CK(hipMemset(sig2, 0, 8));
  CK(hipDeviceSynchronize());
  uint64_t ta = 0, tb = 0;
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, d);
      CK(hipStreamWriteValue64(a, sig, ++ta, 0));
      CK(hipStreamWaitValue64(b, sig, ta, hipStreamWaitValueGte, ~0ull));
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, b, d);
      CK(hipStreamWriteValue64(b, sig2, ++tb, 0));
      CK(hipStreamWaitValue64(a, sig2, tb, hipStreamWaitValueGte, ~0ull));
    }
    auto t1 = clk::now();
    CK(hipDeviceSynchronize());
    auto t2 = clk::now();
    if (rep) printf("stream-mem:   enqueue %.2f us/iter, e2e %.2f us/iter\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  }
  printf("host reads signal words: %llu %llu (expected %llu %llu)\n", (unsigned long long)__atomic_load_n(sig, __ATOMIC_ACQUIRE),
         (unsigned long long)__atomic_load_n(sig2, __ATOMIC_ACQUIRE), (unsigned long long)ta, (unsigned long long)tb);
  // 3) baseline: both kernels on one stream
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, d);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, d);
    }
    auto t1 = clk::now();
    CK(hipDeviceSynchronize());
    auto t2 = clk::now();
    if (rep) printf("same stream:  enqueue %.2f us/iter, e2e %.2f us/iter\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  }
  return 0;
}
