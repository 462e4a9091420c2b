// gather_rate.hip — issue cost of one gather wave-instruction on gfx950 by
// access shape, from a table that stays in L2 (1 MiB) or in the Infinity
// Cache (64 MiB): how many CU cycles does a wave-instruction cost when its 64
// lanes touch D distinct 128-byte lines with W bytes per lane?  The transfer
// kernels' gathers (walk records, vertex rows, solution rows) are all of
// this kind; the answer decides between per-lane and cooperative loads.
//
// Each lane issues kLoads independent loads (addresses from a per-lane hash,
// so nothing is waited on between them except at the end); the XOR of the
// loaded words goes to a sink.  Printed: ns per kernel and CU-cycles per
// wave-instruction at 2.4 GHz.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib/gather_rate tools/calib/gather_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                                      \
  do {                                                                                                             \
    hipError_t e_ = (x);                                                                                           \
    if (e_ != hipSuccess) {                                                                                        \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                                               \
      exit(1);                                                                                                     \
    }                                                                                                              \
  } while (0)

constexpr int kLoads = 64;

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// W bytes per lane; lanes of a group of G consecutive lanes share one line
// (G = 1: 64 distinct lines per instruction; G = 8 with W = 16: 8 full lines)
template <int W, int G>
__global__ __launch_bounds__(256) void k_gather(const char *table, unsigned nlines, int *sink) {
  const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const unsigned grp = lane / G, sub = lane % G;
  int acc = 0;
#pragma unroll 8
  for (int t = 0; t < kLoads; t++) {
    const unsigned line = hash(wave * 977u + t * 131u + grp * 7919u) & (nlines - 1);
    const char *p = table + 128ull * line + (W * sub) % 128;
    if constexpr (W == 4) {
      acc ^= *reinterpret_cast<const int *>(p);
    } else if constexpr (W == 8) {
      int2 v = *reinterpret_cast<const int2 *>(p);
      acc ^= v.x ^ v.y;
    } else if constexpr (W == 12) {
      const int *q = reinterpret_cast<const int *>(p);
      acc ^= q[0] ^ q[1] ^ q[2];
    } else {
      int4 v = *reinterpret_cast<const int4 *>(p);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

// coalesced: the wave reads 64 * W consecutive bytes per instruction
template <int W>
__global__ __launch_bounds__(256) void k_coalesced(const char *table, unsigned nlines, int *sink) {
  const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const unsigned span = 64 * W / 128; // lines per instruction
  int acc = 0;
#pragma unroll 8
  for (int t = 0; t < kLoads; t++) {
    const unsigned base = (hash(wave * 977u + t * 131u) & (nlines - 1)) & ~(span - 1);
    const char *p = table + 128ull * base + W * lane;
    int4 v = *reinterpret_cast<const int4 *>(p);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

int main() {
  char *table;
  int *sink;
  const size_t big = 64ull << 20;
  CK(hipMalloc(&table, big + 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(table, 1, big + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 256 * 32; // 32 blocks of 4 waves per CU
  const double winstr = (double)blocks * 4 * kLoads;
  auto run = [&](const char *name, size_t bytes, auto kern) {
    const unsigned nlines = (unsigned)(bytes / 128);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, (const char *)table, nlines, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; r++)
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, (const char *)table, nlines, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double s = ms * 1e-3 / 5;
    printf("{\"kernel\": \"%s\", \"table_mib\": %zu, \"us\": %.1f, \"cu_cycles_per_wave_instr\": %.1f}\n", name,
           bytes >> 20, s * 1e6, s * 2.4e9 * 256 / winstr);
  };
  for (size_t bytes : {(size_t)1 << 20, big}) {
    run("d64 w4", bytes, k_gather<4, 1>);
    run("d64 w8", bytes, k_gather<8, 1>);
    run("d64 w12", bytes, k_gather<12, 1>);
    run("d64 w16", bytes, k_gather<16, 1>);
    run("d32 w16 (2 lanes/line)", bytes, k_gather<16, 2>);
    run("d16 w16 (4 lanes/line)", bytes, k_gather<16, 4>);
    run("d8 w16 (8 lanes/line, whole lines)", bytes, k_gather<16, 8>);
    run("d16 w8 (4 lanes/line)", bytes, k_gather<8, 4>);
    run("coalesced w16", bytes, k_coalesced<16>);
  }
  CK(hipFree(table));
  return 0;
}
