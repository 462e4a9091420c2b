// Cost of pinning pageable host memory in place (hipHostRegister) against
// staging it through pinned buffers: one 2 GiB array, first touched, then
// (a) registered, copied to the device by the DMA engine, unregistered, and
// (b) copied host->device and device->host by hipMemcpy from pageable memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  for (size_t gib : {1, 2}) {
    const size_t n = gib << 30;
    char *h = (char *)aligned_alloc(4096, n);
    memset(h, 1, n);
    void *d;
    CK(hipMalloc(&d, n));
    for (int rep = 0; rep < 2; rep++) {
      double t0 = now();
      CK(hipHostRegister(h, n, hipHostRegisterDefault));
      double t1 = now();
      CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
      double t2 = now();
      CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
      double t3 = now();
      CK(hipHostUnregister(h));
      double t4 = now();
      CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
      double t5 = now();
      CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
      double t6 = now();
      printf("%zu GiB: register %.1f ms, H2D pinned-in-place %.1f ms (%.1f GB/s), D2H %.1f ms (%.1f GB/s), "
             "unregister %.1f ms | pageable H2D %.1f ms (%.1f GB/s), D2H %.1f ms (%.1f GB/s)\n",
             gib, 1e3 * (t1 - t0), 1e3 * (t2 - t1), n / (t2 - t1) / 1e9, 1e3 * (t3 - t2), n / (t3 - t2) / 1e9,
             1e3 * (t4 - t3), 1e3 * (t5 - t4), n / (t5 - t4) / 1e9, 1e3 * (t6 - t5), n / (t6 - t5) / 1e9);
    }
    CK(hipFree(d));
    free(h);
  }
  return 0;
}
