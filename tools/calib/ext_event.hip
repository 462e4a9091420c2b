// Events recorded by the kernel dispatch itself (hipExtLaunchKernelGGL's
// start / stop events) against separate hipEventRecord markers, on this image
// (ROCm 7.2, MI355X):
//  1. correctness: stream B waits for a stop event of a kernel on stream A that
//     writes a value late (a timed spin), then checks it; the host waits for the
//     same event and reads a value the kernel wrote to pinned host memory;
//  2. cost: a chain of N short dependent kernels on one stream with a marker
//     event after each, with the event attached to each kernel, and with none;
//     device time of the chain (hipEvents around it, median of 9).
//   hipcc --offload-arch=gfx950 -O2 -o tools/calib/ext_event tools/calib/ext_event.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void k_late_write(int *d, volatile int *h, int v, long long spin) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    d[0] = v;
    h[0] = v;
    __threadfence_system();
  }
}
__global__ void k_check(const int *d, int v, int *bad) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && d[0] != v) bad[0] += 1;
}
__global__ void k_short(int *d) {
  if (threadIdx.x == 0) d[blockIdx.x] += 1;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int *d = nullptr, *bad = nullptr, *h = nullptr;
  CK(hipMalloc(&d, 4096));
  CK(hipMalloc(&bad, 4));
  CK(hipHostMalloc((void **)&h, 64, hipHostMallocCoherent | hipHostMallocMapped));
  int *hd = nullptr;
  CK(hipHostGetDevicePointer((void **)&hd, h, 0));
  CK(hipMemset(d, 0, 4096));
  CK(hipMemset(bad, 0, 4));
  hipEvent_t e, t0, t1;
  CK(hipEventCreate(&e));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  // 1. correctness over 200 rounds
  int host_bad = 0;
  for (int r = 1; r <= 200; r++) {
    hipExtLaunchKernelGGL(k_late_write, dim3(1), dim3(64), 0, a, nullptr, e, 0, d, hd, r, 200000LL);
    CK(hipStreamWaitEvent(b, e, 0));
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, b, (const int *)d, r, bad);
    CK(hipEventSynchronize(e));
    if (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) != r) host_bad++;
  }
  CK(hipDeviceSynchronize());
  int dbad = -1;
  CK(hipMemcpy(&dbad, bad, 4, hipMemcpyDeviceToHost));
  printf("stop-event waits: device mismatches %d / 200, host mismatches %d / 200\n", dbad, host_bad);
  // 2. chain cost
  const int N = 16;
  std::vector<hipEvent_t> ev(N);
  for (auto &x : ev) CK(hipEventCreate(&x));
  const char *names[] = {"no events", "marker after each", "stop event on each"};
  for (int mode = 0; mode < 3; mode++) {
    std::vector<float> t;
    for (int r = 0; r < 9; r++) {
      CK(hipEventRecord(t0, a));
      for (int i = 0; i < N; i++) {
        if (mode == 2) hipExtLaunchKernelGGL(k_short, dim3(64), dim3(64), 0, a, nullptr, ev[i], 0, d);
        else hipLaunchKernelGGL(k_short, dim3(64), dim3(64), 0, a, d);
        if (mode == 1) CK(hipEventRecord(ev[i], a));
      }
      CK(hipEventRecord(t1, a));
      CK(hipEventSynchronize(t1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    float el = 0.f;
    (void)hipEventElapsedTime(&el, ev[0], ev[N - 1]);
    printf("%-22s %d kernels: %7.1f us (%5.2f us per kernel); ev[0]->ev[N-1] %7.1f us\n", names[mode], N,
           1e3f * t[4], 1e3f * t[4] / N, mode ? 1e3f * el : 0.f);
  }
  return 0;
}
