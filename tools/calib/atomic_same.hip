// Cost of per-block atomics on ONE address (a last-block ticket, a global
// minimum) against the same grid without them, on this image (ROCm 7.2,
// MI355X): N blocks of 64 or 256 threads; thread 0 of each block issues one
// atomic on one device address (returning atomicAdd = a ticket; no-return
// 64-bit atomicMin = seed_any), or one on its own address (spread), or none.
// Prints the device time per kernel (hipEvents, median of 9).
//   hipcc --offload-arch=gfx950 -O2 -o tools/calib/atomic_same tools/calib/atomic_same.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void k_none(unsigned *p) {
  if (threadIdx.x == 0 && p[0] == 0xFFFFFFFFu) p[1] = 1u;
}
__global__ void k_ticket(unsigned *p) { // returning, one address; the result used (as last_block does)
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(p, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) p[1] = 1u;
}
__global__ void k_min_same(unsigned long long *q) { // no-return 64-bit min, one address
  if (threadIdx.x == 0) atomicMin(q, (unsigned long long)blockIdx.x + 5ULL);
}
__global__ void k_min_spread(unsigned long long *q) { // no-return 64-bit min, one address per block
  if (threadIdx.x == 0) atomicMin(q + 16 * (size_t)blockIdx.x, (unsigned long long)blockIdx.x + 5ULL);
}
__global__ void k_ticket_spread(unsigned *p) { // returning, one address per block
  __shared__ unsigned r;
  if (threadIdx.x == 0) r = atomicAdd(p + 32 * (size_t)blockIdx.x, 1u);
  __syncthreads();
  if (r == 0xFFFFFFFFu && threadIdx.x == 0) p[1] = 1u;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int maxb = 65536;
  unsigned *p = nullptr;
  unsigned long long *q = nullptr;
  (void)hipMalloc(&p, 4ull * 32 * maxb + 64);
  (void)hipMalloc(&q, 8ull * 16 * maxb + 64);
  (void)hipMemsetAsync(p, 0, 4ull * 32 * maxb + 64, s);
  (void)hipMemsetAsync(q, 0xFF, 8ull * 16 * maxb + 64, s);
  (void)hipStreamSynchronize(s);
  const char *names[] = {"none", "ticket(1 addr, returning)", "min64(1 addr, no-return)", "min64(spread)",
                         "ticket(spread)"};
  printf("%-28s %6s %8s %10s %12s\n", "kernel", "block", "blocks", "us", "ns/block");
  for (int bs : {64, 256}) {
    for (int nb : {1024, 4096, 16384, 65536}) {
      for (int k = 0; k < 5; k++) {
        std::vector<float> t;
        for (int r = 0; r < 9; r++) {
          (void)hipMemsetAsync(p, 0, 8, s);
          (void)hipEventRecord(e0, s);
          if (k == 0) hipLaunchKernelGGL(k_none, dim3(nb), dim3(bs), 0, s, p);
          if (k == 1) hipLaunchKernelGGL(k_ticket, dim3(nb), dim3(bs), 0, s, p);
          if (k == 2) hipLaunchKernelGGL(k_min_same, dim3(nb), dim3(bs), 0, s, q);
          if (k == 3) hipLaunchKernelGGL(k_min_spread, dim3(nb), dim3(bs), 0, s, q);
          if (k == 4) hipLaunchKernelGGL(k_ticket_spread, dim3(nb), dim3(bs), 0, s, p);
          (void)hipEventRecord(e1, s);
          (void)hipEventSynchronize(e1);
          float ms = 0.f;
          (void)hipEventElapsedTime(&ms, e0, e1);
          t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const float us = 1e3f * t[t.size() / 2];
        printf("%-28s %6d %8d %10.1f %12.2f\n", names[k], bs, nb, us, 1e3f * us / nb);
      }
    }
  }
  (void)hipFree(p);
  (void)hipFree(q);
  return 0;
}
