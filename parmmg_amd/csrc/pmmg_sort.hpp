// pmmg_sort.hpp — the Morton binning's sort as device-gated kernels
// (included by pmmg_hip.hip only).
//
// A stable LSD radix sort of (32-bit key, 32-bit value) pairs, 8 bits per
// pass, whose every kernel returns at once unless *gate == want: the query
// order of a call is chosen on the device (k_coherence) and both orders'
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
#pragma unroll 4
    for (int j = 0; j < kRsItems; j++) {
      const long long idx = base + j * kBlock + threadIdx.x;
      if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 255u], 1);
    }
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

// One tile per block: the tile's keys are first ranked stably by digit into
// LDS (sub-tiles of 256 keys in input order; a wave's lanes with equal digits
// found by 8 ballots), then written out in that order, so consecutive threads
// store consecutive positions of one digit's run (r04g: ranking straight to
// global memory wrote every key as an isolated 4-byte store, 0.44 ms per pass
// of 20M random keys).
__global__ __launch_bounds__(kBlock) void k_rs_scatter(const unsigned *kin, const int *vin, int n, int shift, int ntile,
                                                       const int *off, unsigned *kout, int *vout, const int *gate,
                                                       int want) {
  if (gate_off(gate, want)) return;
  __shared__ unsigned lk[kRsTile]; // the tile, sorted by digit (stable)
  __shared__ int lv[kRsTile];
  __shared__ int run[256];         // next local position of each digit
  __shared__ int gdelta[256];      // global position - local position of each digit's keys
  __shared__ int wcnt[4][256];     // keys of each digit in each wave of the current sub-tile
  const int t = threadIdx.x, w = t >> 6, lane = __lane_id();
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
  const long long base = (long long)tile * kRsTile;
  const int cnt = (int)(n - base < kRsTile ? n - base : kRsTile);
  // the tile's digit counts, their exclusive scan
  run[t] = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) wcnt[q][t] = 0;
  __syncthreads();
  for (int j = 0; j < kRsItems; j++) {
    const int e = j * kBlock + t;
    if (e < cnt) atomicAdd(&run[(kin[base + e] >> shift) & 255u], 1);
  }
  __syncthreads();
  int tot;
  const int lstart = block_excl_scan(run[t], &tot);
  __syncthreads();
  run[t] = lstart;
  gdelta[t] = off[(size_t)t * ntile + tile] - lstart;
  __syncthreads();
  for (int j = 0; j < kRsItems; j++) {
    const int e = j * kBlock + t;
    const bool ok = e < cnt;
    const unsigned key = ok ? kin[base + e] : 0u;
    const int val = ok ? vin[base + e] : 0;
    const unsigned d = (key >> shift) & 255u;
    unsigned long long same = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const unsigned long long bb = __ballot((d >> b) & 1u);
      same &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const int rank = __popcll(same & ((1ULL << lane) - 1ULL));
    if (ok && rank == 0) wcnt[w][d] = __popcll(same);
    __syncthreads();
    if (ok) {
      int pos = run[d] + rank;
      for (int w2 = 0; w2 < w; w2++) pos += wcnt[w2][d];
      lk[pos] = key;
      lv[pos] = val;
    }
    __syncthreads();
    run[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
    wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
    __syncthreads();
  }
  for (int e = t; e < cnt; e += kBlock) {
    const unsigned key = lk[e];
    const int pos = gdelta[(key >> shift) & 255u] + e;
    kout[pos] = key;
    vout[pos] = lv[e];
  }
  __syncthreads(); // the tile's LDS is free for the next tile
  }
}

} // namespace pmmg
