// pmmg_sort.hpp — the Morton binning's sort as device-gated kernels
// (included by pmmg_hip.hip only).
//
// A stable LSD radix sort of (32-bit key, 32-bit value) pairs, 8 bits per
// pass, whose every kernel returns at once unless *gate == want: the query
// order of a call is chosen on the device (the coherence test in k_bbox) and both orders'
// kernels are enqueued, so the call never waits for the flag on the host
// (rocPRIM's sort, used up to r03, takes its work from host arguments and
// cannot be skipped from the device).
//
// Per pass: k_rs_hist counts the digits of each tile of kRsTile keys (LDS
// histogram, digit-major table hist[digit][tile]; the first pass's table
// comes from the key kernel, k_bin_keys), k_rs_scan_* turns the table into
// each (digit, tile)'s first output position, and k_rs_scatter sorts each
// tile stably by digit in LDS and writes the digits' runs there.
#pragma once

#include "pmmg_prep.hpp"

namespace pmmg {

constexpr int kRsItems = 16, kRsTile = kBlock * kRsItems; // keys per tile (one block)

// The tile kernels loop over tiles (grid <= kRsGrid blocks): gated off, a
// launch is then a few hundred empty blocks instead of one per tile (r04o:
// 5000 empty blocks of the 38 KB-LDS scatter took 0.22 ms of CU slots beside
// the seed grid)
constexpr int kRsGrid = 1024;

__global__ __launch_bounds__(kBlock) void k_rs_hist(const unsigned *keys, int n, int shift, int ntile, int *hist,
                                                    const int *gate, int want) {
  if (gate_off(gate, want)) return;
  __shared__ int h[256];
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    h[threadIdx.x] = 0;
    __syncthreads();
    const long long base = (long long)tile * kRsTile;
    unsigned k[kRsItems]; // the tile's keys in flight together (r04: 4 at a time, 50 us per pass of 20M keys)
#pragma unroll
    for (int j = 0; j < kRsItems; j++) {
      const long long idx = base + j * kBlock + threadIdx.x;
      k[j] = idx < n ? keys[idx] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kRsItems; j++)
      if (base + j * kBlock + threadIdx.x < n) atomicAdd(&h[(k[j] >> shift) & 255u], 1);
    __syncthreads();
    hist[(size_t)threadIdx.x * ntile + tile] = h[threadIdx.x];
    __syncthreads();
  }
}

// exclusive scan of a[0..n) in place: per-chunk scans (chunk sums to
// csum), the scan of the chunk sums (k_scan_top), their addition
__global__ __launch_bounds__(kBlock) void k_rs_scan_local(int *a, int n, int *csum, const int *gate, int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  int v[kScanItems], s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; j++) {
    v[j] = i0 + j < n ? a[i0 + j] : 0;
    s += v[j];
  }
  int tot;
  int run = block_excl_scan(s, &tot);
#pragma unroll
  for (int j = 0; j < kScanItems; j++) {
    if (i0 + j < n) a[i0 + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 0) csum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_rs_scan_add(int *a, int n, const int *coff, const int *gate, int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  const int o = coff[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; j++)
    if (i0 + j < n) a[i0 + j] += o;
}

// One tile per block: the tile's keys are ranked stably by digit into LDS,
// then written out in that order, so consecutive threads store consecutive
// positions of one digit's run (r04g: ranking straight to global memory
// wrote every key as an isolated 4-byte store, 0.44 ms per pass of 20M
// random keys).  r04: each wave ranks its own 1024 consecutive keys (16
// chunks of 64, held in registers: one global read) with per-wave digit
// counters in LDS that only the wave itself touches, so the ranking needs
// no barrier; one block scan over {digit, wave} then gives every key its
// place — 4 barriers per tile instead of ~50 (the tile's keys were read
// twice and each chunk of 256 ranked between three barriers: 160-180 µs per
// pass of 20M keys, 366 beside the seed grid, r04v2 trace).
__global__ __launch_bounds__(kBlock) void k_rs_scatter(const unsigned *kin, const int *vin, int n, int shift, int ntile,
                                                       const int *off, unsigned *kout, int *vout, const int *gate,
                                                       int want) {
  static_assert(kBlock == 256, "one thread per digit");
  if (gate_off(gate, want)) return;
  constexpr int kWaveKeys = kRsTile / (kBlock / 64); // consecutive keys ranked by one wave
  __shared__ unsigned lk[kRsTile]; // the tile, sorted by digit (stable)
  __shared__ int lv[kRsTile];
  __shared__ int wdig[kBlock / 64][256]; // a wave's digit counts, then its keys' first local position per digit
  __shared__ int gdelta[256];            // global position - local position of each digit's keys
  const int t = threadIdx.x, w = t >> 6, lane = __lane_id();
  const unsigned long long below = (1ULL << lane) - 1ULL;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long long base = (long long)tile * kRsTile;
    const int cnt = (int)(n - base < kRsTile ? n - base : kRsTile);
#pragma unroll
    for (int q = 0; q < kBlock / 64; q++) wdig[q][t] = 0;
    __syncthreads();
    unsigned key[kRsItems];
    int val[kRsItems], rk[kRsItems];
#pragma unroll
    for (int j = 0; j < kRsItems; j++) {
      const int e = w * kWaveKeys + j * 64 + lane;
      key[j] = e < cnt ? kin[base + e] : 0u;
      val[j] = e < cnt ? vin[base + e] : 0;
    }
#pragma unroll
    for (int j = 0; j < kRsItems; j++) {
      const bool ok = w * kWaveKeys + j * 64 + lane < cnt;
      const unsigned d = (key[j] >> shift) & 255u;
      unsigned long long same = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const unsigned long long bb = __ballot((d >> b) & 1u);
        same &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const int r = __popcll(same & below);
      const int prior = wdig[w][d]; // (this wave's counter: read by every lane before its first lane writes it)
      rk[j] = prior + r;
      if (ok && r == 0) wdig[w][d] = prior + __popcll(same);
    }
    __syncthreads();
    int c[kBlock / 64], tot_d = 0;
#pragma unroll
    for (int q = 0; q < kBlock / 64; q++) {
      c[q] = wdig[q][t];
      tot_d += c[q];
    }
    int tot;
    const int dstart = block_excl_scan(tot_d, &tot);
    int acc = dstart;
#pragma unroll
    for (int q = 0; q < kBlock / 64; q++) {
      wdig[q][t] = acc;
      acc += c[q];
    }
    gdelta[t] = off[(size_t)t * ntile + tile] - dstart;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRsItems; j++) {
      if (w * kWaveKeys + j * 64 + lane < cnt) {
        const int pos = wdig[w][(key[j] >> shift) & 255u] + rk[j];
        lk[pos] = key[j];
        lv[pos] = val[j];
      }
    }
    __syncthreads();
    for (int e = t; e < cnt; e += kBlock) {
      const unsigned k = lk[e];
      const int pos = gdelta[(k >> shift) & 255u] + e;
      kout[pos] = k;
      vout[pos] = lv[e];
    }
    __syncthreads(); // the tile's LDS is free for the next tile
  }
}

} // namespace pmmg
