// Host cost of a kernel launch on this image (ROCm 7.2, MI355X): N launches
// of an empty kernel with a small / a ~400-byte argument block, on one
// stream, and with an event record between launches.  Prints us per launch
// (host enqueue time) and the device time of the whole sequence.  Modes 7-8:
// the same kernels as a hipGraph of 16 dependent launches, replayed N / 16
// times (one host call per 16 kernels: what graph replay of a group's chain
// would leave of the launch cost).
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/launch_rate tools/calib/launch_rate.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big {
  double a[48];
};
__global__ void k_small(int *p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}
__global__ void k_big(Big b, int *p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0 && b.a[0] < 0) p[0] = 1;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1, ev, evn, evo;
  hipStream_t s2;
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&ev);
  (void)hipEventCreateWithFlags(&evn, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&evo, hipEventDisableTiming);
  (void)hipEventRecord(evo, s2);
  int *p = nullptr;
  (void)hipMalloc(&p, 16);
  Big b{};
  const int N = 2000, G = 16;
  hipGraphExec_t gx[2] = {nullptr, nullptr};
  for (int v = 0; v < 2; v++) {
    hipGraph_t gr;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < G; i++) hipLaunchKernelGGL(k_small, dim3(v ? 4096 : 1), dim3(v ? 256 : 64), 0, s, p);
    (void)hipStreamEndCapture(s, &gr);
    (void)hipGraphInstantiate(&gx[v], gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
  }
  for (int mode = 0; mode < 9; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, s);
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; i++) {
        if (mode == 0) hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, p);
        if (mode == 1) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, p);
        if (mode == 2) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, p);
          (void)hipEventRecord(ev, s);
        }
        if (mode == 3) hipLaunchKernelGGL(k_small, dim3(4096), dim3(256), 0, s, p);
        if (mode == 4) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, p);
          (void)hipEventRecord(evn, s);
        }
        if (mode == 5) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, p);
          (void)hipStreamWaitEvent(s, evo, 0);
        }
        if (mode == 6) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, p);
          (void)hipEventRecord(evn, s);
          (void)hipStreamWaitEvent(s2, evn, 0);
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s2, p);
        }
        if (mode >= 7 && i % G == 0) (void)hipGraphLaunch(gx[mode - 7], s);
      }
      auto t1 = std::chrono::steady_clock::now();
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
      if (rep)
        printf("mode %d (%s): host %.2f us per launch, device %.2f us per launch\n", mode,
               mode == 0   ? "small args"
               : mode == 1 ? "400 B args"
               : mode == 2 ? "small + timing event record"
               : mode == 3 ? "4096 blocks"
               : mode == 4 ? "small + no-timing event record"
               : mode == 5 ? "small + wait on a completed event"
               : mode == 6 ? "launch, record, other stream waits and launches"
               : mode == 7 ? "graph of 16 small launches, per kernel"
                           : "graph of 16 launches of 4096 blocks, per kernel",
               us / N, 1e3 * ms / N);
    }
  }
  return 0;
}
