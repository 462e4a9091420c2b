// fetch_calib.hip — known-byte read patterns for calibrating rocprofv3's
// FETCH_SIZE on gfx950 against the access shapes of the transfer kernels
// (MI355X_MICROARCH.md: FETCH_SIZE reads exactly half of a 16 B/lane
// streaming read; other widths are uncalibrated).  Each pattern reads a
// 2 GiB table (far beyond the 256 MiB Infinity Cache) with a known number of
// compulsory bytes; rocprofv3 --pmc FETCH_SIZE over this program then gives
// reported/compulsory per pattern.  The kernel names say the pattern:
//
//   k_stream16   16 B per lane, coalesced, every byte once
//   k_lines<W>   one random 128 B line per lane, read in W-byte pieces by
//                consecutive instructions (W = 4, 8, 12, 16; for W = 12 the
//                first 120 B), so every line is read whole while 64 lanes of
//                an instruction touch 64 different lines (the gather shape)
//   k_rec32      one random 32 B record per lane as two 16 B loads, every
//                record once, records of a line at unrelated times (the
//                walk's tetra-record gather)
//   k_row12      one random 12 B row per lane (dwordx3), every row once
//                (the walk's fixed-point vertex rows)
//   k_word8      one 8 B word per random line, the rest of the line unused
//                (fetch granularity of an isolated gather)
//
// Random order: index t -> (t * odd) mod 2^k, a bijection.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib/fetch_calib tools/calib/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr unsigned kMul = 0x9E3779B1u;

__device__ __forceinline__ unsigned scramble(unsigned long long t, unsigned long long mask) {
  return (unsigned)((t * kMul) & mask);
}

__global__ __launch_bounds__(256) void k_stream16(const int4 *a, long long n, int *sink) {
  int acc = 0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    int4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void k_lines(const char *table, long long nlines, int *sink) {
  const long long t = blockIdx.x * 256LL + threadIdx.x;
  if (t >= nlines) return;
  const char *line = table + 128ULL * scramble(t, nlines - 1);
  int acc = 0;
  if constexpr (W == 4) {
#pragma unroll
    for (int p = 0; p < 32; p++) acc ^= *reinterpret_cast<const int *>(line + 4 * p);
  } else if constexpr (W == 8) {
#pragma unroll
    for (int p = 0; p < 16; p++) {
      int2 v = *reinterpret_cast<const int2 *>(line + 8 * p);
      acc ^= v.x ^ v.y;
    }
  } else if constexpr (W == 12) {
#pragma unroll
    for (int p = 0; p < 10; p++) {
      const int *q = reinterpret_cast<const int *>(line + 12 * p);
      acc ^= q[0] ^ q[1] ^ q[2];
    }
  } else {
#pragma unroll
    for (int p = 0; p < 8; p++) {
      int4 v = *reinterpret_cast<const int4 *>(line + 16 * p);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_rec32(const int4 *table, long long nrec, int *sink) {
  const long long t = blockIdx.x * 256LL + threadIdx.x;
  if (t >= nrec) return;
  const unsigned r = scramble(t, nrec - 1);
  int4 a = table[2ULL * r], b = table[2ULL * r + 1];
  int acc = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_row12(const int *table, long long nrow, int *sink) {
  const long long t = blockIdx.x * 256LL + threadIdx.x;
  if (t >= nrow) return;
  const int *q = table + 3ULL * scramble(t, nrow - 1);
  int acc = q[0] ^ q[1] ^ q[2];
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_word8(const long long *table, long long nlines, int *sink) {
  const long long t = blockIdx.x * 256LL + threadIdx.x;
  if (t >= nlines) return;
  long long v = table[16ULL * scramble(t, nlines - 1)];
  if ((int)v == 0x7fffffff) sink[0] = (int)v;
}

__global__ void k_fill(int *a, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) a[i] = (int)(i * 2654435761u);
}

int main() {
  const long long bytes = 1LL << 31; // 2 GiB
  char *table;
  int *sink;
  CK(hipMalloc(&table, bytes + 4096));
  CK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (int *)table, bytes / 4);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long long nlines = bytes / 128, nrec = bytes / 32;
  const long long nrow = 1LL << 27; // 1.5 GiB of 12 B rows
  auto run = [&](const char *name, double compulsory, auto launch) {
    launch(); // warm (page tables), then timed
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"compulsory_bytes\": %.0f, \"ms\": %.4f, \"gbps\": %.1f}\n", name, compulsory, ms,
           compulsory / (ms * 1e-3) / 1e9);
  };
  auto blocks = [](long long n) { return dim3((unsigned)((n + 255) / 256)); };
  run("k_stream16", (double)bytes, [&] {
    hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, (const int4 *)table, bytes / 16, sink);
  });
  run("k_lines<4>", (double)bytes,
      [&] { hipLaunchKernelGGL(k_lines<4>, blocks(nlines), dim3(256), 0, 0, table, nlines, sink); });
  run("k_lines<8>", (double)bytes,
      [&] { hipLaunchKernelGGL(k_lines<8>, blocks(nlines), dim3(256), 0, 0, table, nlines, sink); });
  run("k_lines<12>", (double)bytes * 120.0 / 128.0,
      [&] { hipLaunchKernelGGL(k_lines<12>, blocks(nlines), dim3(256), 0, 0, table, nlines, sink); });
  run("k_lines<16>", (double)bytes,
      [&] { hipLaunchKernelGGL(k_lines<16>, blocks(nlines), dim3(256), 0, 0, table, nlines, sink); });
  run("k_rec32", (double)bytes,
      [&] { hipLaunchKernelGGL(k_rec32, blocks(nrec), dim3(256), 0, 0, (const int4 *)table, nrec, sink); });
  run("k_row12", 12.0 * nrow,
      [&] { hipLaunchKernelGGL(k_row12, blocks(nrow), dim3(256), 0, 0, (const int *)table, nrow, sink); });
  run("k_word8", 8.0 * nlines,
      [&] { hipLaunchKernelGGL(k_word8, blocks(nlines), dim3(256), 0, 0, (const long long *)table, nlines, sink); });
  CK(hipFree(table));
  CK(hipFree(sink));
  return 0;
}
