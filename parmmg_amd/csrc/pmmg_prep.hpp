// pmmg_prep.hpp — per-call preparation kernels of the transfer step
// (included by pmmg_hip.hip only): state reset, background frame, volume and
// surface seed grids, and the query order.
//
// The input-order coherence test runs on the device (in k_bbox: coherence_final's flag); in
// auto mode both the Morton binning (pmmg_sort.hpp) and the class compaction
// of the surface list are enqueued, each gated on that flag, and the volume
// kernel reads it: nothing is read back inside a call.
#pragma once

#include "pmmg_device.hpp"

namespace pmmg {

// Counters of one call.  The per-kind hit counts and the walk statistics are
// accumulated into kStatParts partial records (block b -> part b % kStatParts,
// summed on the host at pmmg_hip_sync): one counter address hit by every
// workgroup serialises the atomics at one L2 channel (a returning per-wave
// atomic on one address cost +4 ms on cfg4).
struct DevStats {
  int nvol, nbdy;       // query counts (nvol: Morton path only; the input-order walk counts its own)
  int nfb_vol, nfb_bdy; // fallback lists (exhaustive searches)
  int ncont;            // walks continued in exact arithmetic (k_vol_walk_exact)
  int sorted;           // 1: queries Morton-binned, 0: input order (coherent numbering)
  int bin_bits;         // Morton bits per axis of the binning keys (read back with `sorted`)
  int pad;
  int bdy_next[8];      // k_bdy: per-XCD work counters (the next unclaimed surface query of each eighth)
  int nac_vol, nac_bdy; // fallback queries no element accepted (the closest searches' lists)
  // uniform grids over each fallback list's queries (fb_grid_build): origin,
  // inverse cell size, cells per axis (0: not built)
  double fbg_lo[2][3], fbg_inv[2][3];
  int fbg_n[2];
  unsigned walk_done;   // k_vol_walk_exact blocks done (its last block builds the volume list's grid)
  unsigned bdy_done;    // k_bdy blocks done (the surface list's grid)
  unsigned fb_done[4];  // blocks done with an exhaustive kernel (volume accept / closest, surface accept /
                        // closest): the last one finishes
};

// the exhaustive searches' per-query state, initialised where a query joins
// a fallback list (no separate init launch): the lowest accepting element
struct FbInit {
  int *best;
  __device__ __forceinline__ void at(int slot) const { best[slot] = INT_MAX; }
};

constexpr int kStatParts = 256;
// extra counter slots next to the PMMG_HIT_* codes (1..11)
constexpr int kCntVolQueries = 12; // volume queries seen by the walk
constexpr int kCntWaveIters = 13;  // sum over waves of the longest walk in the wave (lockstep cost)
constexpr int kCntExact = 14;      // queries handed to the exact continuation (stuck, over-long, or rejected
                                   // by the exact test at the filter's candidate)
constexpr int kCntNoSeed = 15;     // volume queries without a seed (empty seed neighbourhood)
constexpr int kCntStuck = 16;      // exact walks stuck (no eligible neighbour)
constexpr int kCntLimit = 17;      // exact walks stopped at maxstep
constexpr int kCntFanScan = 18;    // surface queries whose cone test scanned every tria (tri_cone_scan)
constexpr int kNumCnt = 20;
struct StatPart {
  unsigned long long cnt[kNumCnt];
  unsigned long long steps;
  unsigned long long stepmax;
};
__device__ __forceinline__ StatPart *stat_part(DevStats *st) {
  return reinterpret_cast<StatPart *>(st + 1) + (blockIdx.x & (kStatParts - 1));
}

// per-wave aggregation into the block's partial record (one LDS atomic per
// wave and counter), flushed once per block
struct BlockStats {
  unsigned int cnt[kNumCnt];
  unsigned long long steps;
  unsigned int stepmax;
};

__device__ __forceinline__ void bstats_init(BlockStats *b) {
  if (threadIdx.x < kNumCnt) b->cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    b->steps = 0;
    b->stepmax = 0;
  }
}

__device__ __forceinline__ void bstats_flush(BlockStats *b, DevStats *st) {
  StatPart *pt = stat_part(st);
  if (threadIdx.x < kNumCnt && b->cnt[threadIdx.x]) atomicAdd(&pt->cnt[threadIdx.x], (unsigned long long)b->cnt[threadIdx.x]);
  if (threadIdx.x == 0) {
    if (b->steps) atomicAdd(&pt->steps, b->steps);
    if (b->stepmax) atomicMax(&pt->stepmax, (unsigned long long)b->stepmax);
  }
}

// steps of the active lanes, the wave's longest walk (kCntWaveIters) and one
// hit code per lane
__device__ __forceinline__ void wave_stats(BlockStats *bs, bool active, int hit, int steps) {
  unsigned int s = active ? (unsigned)steps : 0u, mx = s;
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_down(s, off);
    unsigned o = __shfl_down(mx, off);
    mx = o > mx ? o : mx;
  }
  if (__lane_id() == 0) {
    if (s) atomicAdd(&bs->steps, (unsigned long long)s);
    if (mx) {
      atomicMax(&bs->stepmax, mx);
      atomicAdd(&bs->cnt[kCntWaveIters], mx);
    }
  }
  int h = active ? hit : 0;
  unsigned long long any = __ballot(h > 0);
  while (any) {
    int first = __shfl(h, __ffsll((long long)any) - 1);
    unsigned long long same = __ballot(h == first);
    if (__lane_id() == 0) atomicAdd(&bs->cnt[first], (unsigned)__popcll(same));
    any &= ~same;
  }
}

__device__ __forceinline__ void wave_count(BlockStats *bs, int slot, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (__lane_id() == 0 && m) atomicAdd(&bs->cnt[slot], (unsigned)__popcll(m));
}

// Per-axis map of the volume seed grid (r03): on a strongly graded mesh (a
// boundary layer, a shock: elements 1000x smaller near a plane) a uniform
// grid puts hundreds of element layers into one cell next to the plane and
// the walks from its seed grow long (cfgG: 14.8 steps per point, stepmax
// 382).  Cell boundaries along axis d then follow the quantiles of the
// background vertices' coordinates (a sampled histogram of kMapBins bins,
// linear inside a bin): each slab of cells holds the same share of the
// vertices, which for a grading separable by axis makes every cell hold the
// same number of tetra.  An axis whose heaviest uniform-cell slab holds less
// than kMapRatio x the mean slab keeps the uniform cells (its bit of
// `adaptive` clear): the shell and cube lattices are not remapped.
constexpr int kMapBins = 2048;
constexpr int kMapRatio = 4;
constexpr int kHistBlocks = 32;

constexpr int kSeedAnyParts = 64;
struct Frame {
  unsigned long long key_lo[3], key_hi[3];
  double lo[3], ext[3];
  double inv_vol[3], inv_srf[3], inv_bin[3];
  double qc[3], qs; // fixed-point frame of the walk's vertex copy
  int adaptive;     // bit d: axis d of the volume seed grid follows map[d]
  // the lowest in-use tetra the seed grid sampled (INT_MAX: none), the last-resort seed: the minimum of
  // kSeedAnyParts partial minima (block b -> part b % kSeedAnyParts).  r06: one address took every block's
  // atomic, and atomics on one address serialise at ~11.4 ns each (tools/calib/atomic_same, profiles/r06j):
  // k_seed_vol's 8192 blocks held ~93 us of them
  int seed_any[kSeedAnyParts];
  unsigned bbox_done; // blocks done (the last block of k_bbox finalises the frame)
  float map[3][kMapBins + 1]; // map[d][b] = share of the vertices below bin b's lower edge
};

// position along axis d in cells of the volume seed grid (g cells), in [0, g]
__device__ __forceinline__ double seed_pos(const Frame *fr, int d, double x, int g) {
  const double u = (x - fr->lo[d]) * fr->inv_vol[d]; // uniform cells
  if (!((fr->adaptive >> d) & 1)) return u;
  double b = u * ((double)kMapBins / (double)g);
  b = b > 0.0 ? (b < (double)kMapBins ? b : (double)kMapBins - 1e-9) : 0.0;
  const int i = (int)b;
  const double m0 = fr->map[d][i], m1 = fr->map[d][i + 1];
  return (m0 + (b - (double)i) * (m1 - m0)) * (double)g;
}
__device__ __forceinline__ int seed_cell(double t, int g) {
  const int c = t > 0.0 ? (int)t : 0;
  return c < g ? c : g - 1;
}

// Fixed-point coordinates for the filter walk and the seed grid: int32
// (x - qc) * qs with |x - qc| <= 0.625 * (largest bbox side) mapped into
// +-2^29, so the difference of two vertices in range is exact in int32 and
// its rounding to fp32 costs the same relative precision as the fp64
// difference rounded to fp32.  12 bytes per vertex (one dwordx3 load)
// instead of 24.  A vertex outside the range (the bbox is sampled) clamps;
// that can only misdirect the filter walk, never an accepted result (the
// exact test uses the fp64 coordinates).
constexpr double kQuantHalf = 536870912.0; // 2^29
__device__ __forceinline__ int quant(double x, const Frame *fr, int d) {
  double t = (x - fr->qc[d]) * fr->qs;
  t = t > 2.0 * kQuantHalf ? 2.0 * kQuantHalf : (t < -2.0 * kQuantHalf ? -2.0 * kQuantHalf : t);
  return __double2int_rn(t);
}

// the seed grid axis maps' input: the per-axis histogram of np / stride
// background vertices at pseudo-random positions (splitmix64 of the sample
// index: a strided sample aliases with a lattice numbering's row length —
// cfg5's halo shard put 14 % of an every-256th sample on its x = 0 plane and
// mapped a uniform axis); vertices outside the (sampled) frame are left out,
// not clamped into the edge bins.  Block b < kHistBlocks's share, counted in
// its LDS histogram h and flushed to H[b][d][bin] (no atomics outside LDS)
__device__ __forceinline__ void axis_hist_block(int (*h)[kMapBins], const double *xyz, long long np, const Frame *fr,
                                                int stride, int *H) {
  for (int j = threadIdx.x; j < 3 * kMapBins; j += kBlock) (&h[0][0])[j] = 0;
  __syncthreads();
  const long long ns = (np + stride - 1) / stride;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < ns; j += (long long)kHistBlocks * blockDim.x) {
    unsigned long long z = (unsigned long long)j * 0x9E3779B97F4A7C15ULL + 0x5EED2025ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    const long long i = (long long)(z % (unsigned long long)np);
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const double e = fr->ext[d];
      const double b = e > 0.0 ? (xyz[3 * i + d] - fr->lo[d]) * ((double)kMapBins / e) : 0.0;
      if (b >= 0.0 && b < (double)kMapBins) atomicAdd(&h[d][(int)b], 1);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * kMapBins; j += kBlock) H[(size_t)blockIdx.x * 3 * kMapBins + j] = (&h[0][0])[j];
}

// The fixed-point copy is an elementwise map of the coordinate stream: with
// 3 ints per row, xq[e] = quant(xyz[e], axis e % 3) for every double e, so
// the kernel streams pairs of doubles in (one 16-byte load per lane, every
// wave-instruction one contiguous KiB) and pairs of ints out (8 bytes per
// lane, 512 contiguous bytes), kQuantU pairs in flight per lane.  (r04: two
// whole vertices per lane, 48-byte strided pieces: 175 us at cfg4, 3.5 TB/s.)
// The seed grid's axis histograms (one sample of np / hstride vertices, see
// axis_hist_block) are taken by the first kHistBlocks blocks of the same
// launch: both need only the frame (r05: one launch and its gap less per call;
// the grid is at least kHistBlocks blocks).
constexpr int kQuantU = 4;
// The axis histograms alone (kHistBlocks blocks): a large call's seed grid
// then needs only them and the frame, while the fixed-point copy runs on a
// stream of its own beside it (r06, run_device: quant_side)
__global__ __launch_bounds__(kBlock) void k_axis_hist(const double *xyz, long long np, const Frame *fr, int hstride,
                                                      int *H) {
  __shared__ int h[3][kMapBins];
  axis_hist_block(h, xyz, np, fr, hstride, H);
}

__global__ __launch_bounds__(kBlock) void k_quantize(const double *xyz, long long np, const Frame *fr, int *xq,
                                                     int hstride, int *H) {
  __shared__ int h[3][kMapBins];
  if (H && blockIdx.x < kHistBlocks) axis_hist_block(h, xyz, np, fr, hstride, H); // (block-uniform)
  const long long nth = (long long)gridDim.x * blockDim.x;
  if (kXqStride == 3 && ((uintptr_t)xyz & 15) == 0 && ((uintptr_t)xq & 7) == 0) {
    const double qs = fr->qs, qc0 = fr->qc[0], qc1 = fr->qc[1], qc2 = fr->qc[2];
    const double lim = 2.0 * kQuantHalf;
    auto q = [&](double x, unsigned d) {
      double t = (x - (d == 0 ? qc0 : (d == 1 ? qc1 : qc2))) * qs;
      t = t > lim ? lim : (t < -lim ? -lim : t);
      return __double2int_rn(t);
    };
    const long long n = 3 * np, npair = n / 2;
    const ntd2 *src = reinterpret_cast<const ntd2 *>(xyz);
    nti2 *dst = reinterpret_cast<nti2 *>(xq);
    for (long long p0 = blockIdx.x * (long long)blockDim.x * kQuantU + threadIdx.x; p0 < npair;
         p0 += nth * kQuantU) {
      ntd2 v[kQuantU];
#pragma unroll
      for (int u = 0; u < kQuantU; u++) {
        const long long p = p0 + (long long)u * blockDim.x;
        if (p < npair) v[u] = __builtin_nontemporal_load(src + p);
      }
#pragma unroll
      for (int u = 0; u < kQuantU; u++) {
        const long long p = p0 + (long long)u * blockDim.x;
        if (p < npair) {
          const unsigned d0 = (unsigned)((2 * p) % 3); // 64-bit: 3 * np doubles may pass 2^31
          const unsigned d1 = d0 == 2u ? 0u : d0 + 1u;
          const nti2 w = {q(v[u].x, d0), q(v[u].y, d1)};
          __builtin_nontemporal_store(w, dst + p); // (cached stores: ±0 for the seed grid and the walk, r05ac)
        }
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1))
      xq[n - 1] = q(xyz[n - 1], (unsigned)((n - 1) % 3));
    return;
  }
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < 3 * np; j += nth)
    xq[kXqStride * (j / 3) + j % 3] = quant(__builtin_nontemporal_load(xyz + j), fr, (int)(j % 3));
}

// one launch initialises the per-call state: frame accumulators, counters,
// seed grids
// (and writes the order flag of a forced order, when the coherence test is not
// launched: force >= 0)
__global__ __launch_bounds__(kBlock) void k_reset(Frame *fr, DevStats *st, unsigned long long *grid, long long ng,
                                                  unsigned long long *sgrid, long long nsg, int *flag, int force,
                                                  int force_bits) {
  const long long tid = blockIdx.x * (long long)blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  if (tid < kSeedAnyParts) fr->seed_any[tid] = INT_MAX;
  if (tid == 0) {
    for (int d = 0; d < 3; d++) {
      fr->key_lo[d] = ~0ULL;
      fr->key_hi[d] = 0ULL;
    }
    fr->adaptive = 0;
    fr->bbox_done = 0u;
    if (force >= 0) {
      flag[0] = force;
      flag[1] = force_bits;
    }
    unsigned int *w = reinterpret_cast<unsigned int *>(st);
    for (size_t j = 0; j < sizeof(DevStats) / 4; j++) w[j] = 0u;
  }
  {
    unsigned long long *pw = reinterpret_cast<unsigned long long *>(st + 1);
    for (long long j = tid; j < (long long)(kStatParts * sizeof(StatPart) / 8); j += nth) pw[j] = 0ULL;
  }
  for (long long j = tid; j < ng; j += nth) grid[j] = ~0ULL;
  for (long long j = tid; j < nsg; j += nth) sgrid[j] = ~0ULL;
}

// bbox of np / stride vertices at pseudo-random positions (a strided sample
// can alias with a lattice numbering's row length and collapse an axis) and
// of the first and last vertex: the frame only sizes the seed / bin grids,
// whose cell lookups clamp, so a sampled bbox costs at most slightly longer
// walks for the few points outside it
__device__ void frame_final(Frame *fr, int g, int gs, int gb);

// the last block to finish also finalises the frame (one launch less per
// call; the other blocks' atomics are read back atomically)
// flag != null (auto order): the queries' coherence test rides along — the
// first kCohBlocks blocks each also measure 512 of its 4096 consecutive-point
// distances (2 per thread) into cohd, and the last block, after finalising
// the frame, counts them (coherence_final) — so the order flag is on the main
// stream after k_bbox.  (r05: a one-block kernel on the second stream, every
// kernel of the other streams that reads the flag waited on it across
// queues; then one block of k_bbox running the whole test, ~30 us on the
// main stream's critical path, r05ag)
constexpr int kCohBlocks = 8, kCohSamples = 4096; // 2 samples per thread of each test block
__device__ void coherence_final(const Frame *fr, const double *cohd, int nq, int *flag, int *flag_host);
__device__ __forceinline__ double coh_sample(const double *xyz, int np, int smp) {
  // pseudo-random positions (splitmix64 of the sample index): an evenly
  // strided sample can alias with the row length of a lattice numbering
  unsigned long long z = (unsigned long long)smp * 0x9E3779B97F4A7C15ULL + 0x5EED2025ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  const long long i = (long long)(z % (unsigned long long)(np - 1));
  double d2 = 0.0;
  for (int d = 0; d < 3; d++) {
    const double t = xyz[3 * (size_t)(i + 1) + d] - xyz[3 * (size_t)i + d];
    d2 += t * t;
  }
  return sqrt(d2);
}
__global__ __launch_bounds__(kBlock) void k_bbox(const double *xyz, int np, Frame *fr, int stride, int g, int gs,
                                                 int gb, const double *qxyz, int nq, int *flag, double *cohd,
                                                 int *flag_host) {
  __shared__ unsigned long long slo[3][kBlock / 64], shi[3][kBlock / 64];
  unsigned long long lo[3] = {~0ULL, ~0ULL, ~0ULL}, hi[3] = {0ULL, 0ULL, 0ULL};
  const long long ns = ((long long)np + stride - 1) / stride + 2;
  if (flag && blockIdx.x < kCohBlocks && nq >= 2) {
#pragma unroll
    for (int s = 0; s < kCohSamples / (kCohBlocks * kBlock); s++) {
      const int smp = (blockIdx.x * (kCohSamples / (kCohBlocks * kBlock)) + s) * kBlock + threadIdx.x;
      cohd[smp] = coh_sample(qxyz, nq, smp);
    }
  }
  // kBboxBatch samples per thread and trip, their rows in flight together
  // (r06: one sample per trip was a chain of ~4 dependent HBM round trips)
  constexpr int kBboxBatch = 4;
  const long long gs_ = (long long)gridDim.x * blockDim.x;
  for (long long j0 = blockIdx.x * blockDim.x + threadIdx.x; j0 < ns; j0 += kBboxBatch * gs_) {
    double r[kBboxBatch][3];
    bool ok[kBboxBatch];
#pragma unroll
    for (int b = 0; b < kBboxBatch; b++) {
      const long long j = j0 + b * gs_;
      ok[b] = j < ns;
      unsigned long long z = (unsigned long long)j * 0x9E3779B97F4A7C15ULL + 0xB0B0B0B0ULL;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      z ^= z >> 31;
      const long long i = !ok[b] || j == 0 ? 0 : (j == 1 ? np - 1 : (long long)(z % (unsigned long long)np));
#pragma unroll
      for (int d = 0; d < 3; d++) r[b][d] = xyz[3 * i + d];
    }
#pragma unroll
    for (int b = 0; b < kBboxBatch; b++)
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const unsigned long long k = dkey(r[b][d]);
        lo[d] = ok[b] && k < lo[d] ? k : lo[d];
        hi[d] = ok[b] && k > hi[d] ? k : hi[d];
      }
  }
#pragma unroll
  for (int d = 0; d < 3; d++) {
    for (int off = 32; off > 0; off >>= 1) {
      unsigned long long a = __shfl_down(lo[d], off), b = __shfl_down(hi[d], off);
      lo[d] = a < lo[d] ? a : lo[d];
      hi[d] = b > hi[d] ? b : hi[d];
    }
  }
  int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
    for (int d = 0; d < 3; d++) {
      slo[d][w] = lo[d];
      shi[d][w] = hi[d];
    }
  __syncthreads();
  if (threadIdx.x < 3) {
    int d = threadIdx.x;
    unsigned long long a = ~0ULL, b = 0ULL;
    for (int j = 0; j < kBlock / 64; j++) {
      a = slo[d][j] < a ? slo[d][j] : a;
      b = shi[d][j] > b ? shi[d][j] : b;
    }
    atomicMin(&fr->key_lo[d], a);
    atomicMax(&fr->key_hi[d], b);
  }
  __threadfence();
  __syncthreads(); // every wave's atomics issued before the ticket
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(&fr->bbox_done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return; // (block-uniform)
  if (threadIdx.x == 0) {
    __threadfence();
    frame_final(fr, g, gs, gb);
  }
  __syncthreads();
  if (flag) coherence_final(fr, cohd, nq, flag, flag_host);
}

__device__ void frame_final(Frame *fr, int g, int gs, int gb) {
  double emax = 0.0;
  for (int d = 0; d < 3; d++) {
    // (atomic reads: the other blocks' atomicMin / atomicMax results)
    double lo = dunkey(atomicOr(&fr->key_lo[d], 0ULL)), hi = dunkey(atomicOr(&fr->key_hi[d], 0ULL));
    double ext = hi - lo;
    fr->lo[d] = lo;
    fr->ext[d] = ext;
    fr->inv_vol[d] = ext > 0.0 ? (double)g / ext : 0.0;
    fr->inv_srf[d] = ext > 0.0 ? (double)gs / ext : 0.0;
    fr->inv_bin[d] = ext > 0.0 ? (double)gb / ext : 0.0;
    fr->qc[d] = lo + 0.5 * ext;
    emax = ext > emax ? ext : emax;
  }
  fr->qs = emax > 0.0 ? kQuantHalf / (0.625 * emax) : 1.0;
}

// ---------------------------------------------------------------- volume seed grid
//
// A g^3 grid; every cell holds the sampled tetra whose centroid is nearest to
// the cell centre, as one 64-bit key {8-bit squared distance to the centre
// (cell units), 9-bit centroid offset per axis, 29-bit id} reduced with
// atomicMin (deterministic).  Samples are runs of 4 consecutive tetra (one
// 128-byte line of packed records), nsamp / 4 runs evenly spaced over the
// tetra; lanes of a run that land in the same cell combine their keys first.
// A query decodes the seeds' centroids from the keys of the 2x2x2 cells
// around its position and starts from the nearest.
constexpr int kSeedRun = 4;
constexpr unsigned long long kSeedIdMask = (1ULL << 29) - 1; // ids below 2^29 (the adja encoding's limit)

// One lane per sample, the 4 lanes of a run on consecutive records (their
// record and vertex loads share sectors: r04e, one thread per run read twice
// the sectors and took 0.72 ms against 0.25).  The grid-stride loop is
// unrolled by kSeedBatch: the records of kSeedBatch trips, then their vertex
// rows, are in flight together before the first key is computed.  The cell
// position comes from the fixed-point vertex sum in one multiply-add per
// axis (the uniform map folded with the fixed-point frame); an axis with a
// quantile map (Frame::adaptive) goes through seed_pos.
constexpr int kSeedBatch = 3;
__global__ __launch_bounds__(kBlock) void k_seed_vol(Bg bg, Frame *fr, unsigned long long *cell, int g,
                                                     long long nsamp, int lanes, int v0only, const double *xyzc) {
  constexpr int R = kSeedRun, B = kSeedBatch;
  __shared__ int smin;
  if (threadIdx.x == 0) smin = INT_MAX;
  __syncthreads();
  int kmin = INT_MAX;
  const long long nruns = (nsamp + R - 1) / R;
  const long long quads = bg.ne / 4;
  const long long nthreads = nruns * R;
  // XCD-aware: the blocks of XCD x (blockIdx % 8; gridDim is a multiple of
  // 8) sweep one contiguous eighth of the samples, so the vertex rows shared
  // by neighbouring tetra are fetched into one L2, not eight
  const long long per = (nthreads + 8LL * kBlock - 1) / (8LL * kBlock) * kBlock;
  const long long lo = (blockIdx.x & 7) * per, hi = lo + per < nthreads ? lo + per : nthreads;
  const long long bstride = (long long)(gridDim.x >> 3) * blockDim.x;
  const int adaptive = fr->adaptive;
  double sa[3], sb[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    sa[d] = (fr->qc[d] - fr->lo[d]) * fr->inv_vol[d];
    sb[d] = 0.25 * fr->inv_vol[d] / fr->qs;
  }
  const int lane = __lane_id(), r = lane % R, g0 = lane - r;
  for (long long s0 = lo + (blockIdx.x >> 3) * (long long)blockDim.x; s0 < hi; s0 += B * bstride) {
    int k[B];
    int4 tv[B];
    bool ok[B];
#pragma unroll
    for (int b = 0; b < B; b++) {
      const long long s = s0 + b * bstride + threadIdx.x;
      const long long run = s / R;
      const long long base = 4 * ((run * quads) / (nruns > 0 ? nruns : 1)); // a cache line of tet8 records
      k[b] = (int)(1 + base + r);
      ok[b] = s < hi && k[b] <= bg.ne && r < lanes; // `lanes` of the run's 4 records are sampled
      tv[b] = make_int4(0, 0, 0, 0);
      if (ok[b]) {
        const nti4 rr =
            __builtin_nontemporal_load(reinterpret_cast<const nti4 *>(bg.tetv + (size_t)(k[b] - 1) * bg.tstride));
        tv[b] = make_int4(rr.x, rr.y, rr.z, rr.w);
      }
    }
    long long sq[B][3]; // 64-bit: clamped coordinates (+-2^30) of vertices outside the sampled frame
    double cc[B][3];    // (xyzc: the centroids in fp64)
#pragma unroll
    for (int b = 0; b < B; b++) {
      ok[b] = ok[b] && tv[b].x > 0;
#pragma unroll
      for (int d = 0; d < 3; d++) {
        cc[b][d] = 0.0;
        sq[b][d] = 0;
      }
      if (xyzc) {
        if (ok[b]) {
          double p0[3], p1[3], p2[3], p3[3];
          load_pt(xyzc, tv[b].x, p0);
          load_pt(xyzc, tv[b].y, p1);
          load_pt(xyzc, tv[b].z, p2);
          load_pt(xyzc, tv[b].w, p3);
#pragma unroll
          for (int d = 0; d < 3; d++) cc[b][d] = 0.25 * ((p0[d] + p1[d]) + (p2[d] + p3[d]));
        }
        continue;
      }
      if (ok[b] && (v0only & 1)) { // measurement build (PMMG_HIP_SEEDV0=1): the first vertex stands for the centroid
        const int *q0 = bg.xq + kXqStride * (size_t)(tv[b].x - 1);
#pragma unroll
        for (int d = 0; d < 3; d++) sq[b][d] = 4LL * q0[d];
      } else if (ok[b]) {
        const int *q0 = bg.xq + kXqStride * (size_t)(tv[b].x - 1), *q1 = bg.xq + kXqStride * (size_t)(tv[b].y - 1);
        const int *q2 = bg.xq + kXqStride * (size_t)(tv[b].z - 1), *q3 = bg.xq + kXqStride * (size_t)(tv[b].w - 1);
        int a0[3], a1[3], a2[3], a3[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
          a0[d] = q0[d];
          a1[d] = q1[d];
          a2[d] = q2[d];
          a3[d] = q3[d];
        }
#pragma unroll
        for (int d = 0; d < 3; d++) sq[b][d] = ((long long)a0[d] + a1[d]) + ((long long)a2[d] + a3[d]);
      }
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
      unsigned long long key = ~0ULL;
      long long ci = -1;
      if (ok[b]) {
        int c[3];
        unsigned long long off = 0;
        float d2 = 0.f;
#pragma unroll
        for (int d = 0; d < 3; d++) {
          double t = xyzc ? (cc[b][d] - fr->lo[d]) * fr->inv_vol[d] : sa[d] + sb[d] * (double)sq[b][d];
          if ((adaptive >> d) & 1)
            t = seed_pos(fr, d, xyzc ? cc[b][d] : fr->qc[d] + 0.25 * (double)sq[b][d] / fr->qs, g);
          c[d] = seed_cell(t, g);
          float f = (float)(t - c[d]);
          f = f < 0.f ? 0.f : (f > 0.999f ? 0.999f : f);
          off |= (unsigned long long)(unsigned)(f * 512.f) << (9 * d);
          d2 += (f - 0.5f) * (f - 0.5f);
        }
        const unsigned q8 = d2 * 340.f < 255.f ? (unsigned)(d2 * 340.f) : 255u;
        key = ((unsigned long long)q8 << 56) | (off << 29) | (unsigned)k[b];
        ci = c[0] + (long long)g * (c[1] + (long long)g * c[2]);
        kmin = k[b] < kmin ? k[b] : kmin;
      }
      // combine within the run: the first lane of each distinct cell issues
      // the atomic with the run's minimum for that cell
      bool leader = ci >= 0;
      unsigned long long best = key;
#pragma unroll
      for (int o = 0; o < R; o++) {
        const long long co = __shfl(ci, g0 + o);
        const unsigned long long ko = __shfl(key, g0 + o);
        if (co == ci && ci >= 0) {
          best = ko < best ? ko : best;
          if (o < r) leader = false;
        }
      }
      if (leader) {
        if (v0only & 2) cell[ci] = best; // measurement build (PMMG_HIP_SEEDNOATOM=1): the atomics' price
        else atomicMin(&cell[ci], best);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int u = __shfl_down(kmin, o);
    kmin = u < kmin ? u : kmin;
  }
  if (__lane_id() == 0 && kmin != INT_MAX) atomicMin(&smin, kmin);
  __syncthreads();
  if (threadIdx.x == 0 && smin != INT_MAX) atomicMin(&fr->seed_any[blockIdx.x % kSeedAnyParts], smin);
}

// rare path of seed_vol (the 8 cells are empty): lowest seed id in the shells
// of radius 1, 2, ... kSeedRing around the cell; 0 when there is none
constexpr int kSeedRing = 6;
__device__ __noinline__ int seed_vol_ring(const unsigned long long *cell, int g, int ci, int cj, int ck) {
#pragma unroll 1
  for (int r = 1; r <= kSeedRing; r++) {
    unsigned long long best = ~0ULL;
#pragma unroll 1
    for (int dk = -r; dk <= r; dk++)
#pragma unroll 1
      for (int dj = -r; dj <= r; dj++)
#pragma unroll 1
        for (int di = -r; di <= r; di++) {
          if (max(abs(di), max(abs(dj), abs(dk))) != r) continue;
          int a = ci + di, b = cj + dj, c = ck + dk;
          if (a < 0 || b < 0 || c < 0 || a >= g || b >= g || c >= g) continue;
          unsigned long long v = cell[a + (size_t)g * (b + (size_t)g * c)];
          unsigned long long id = v & kSeedIdMask;
          if (v != ~0ULL && id < best) best = id;
        }
    if (best != ~0ULL) return (int)best;
  }
  return 0;
}

__device__ __forceinline__ int seed_vol(const unsigned long long *cell, int g, const Frame *fr, const double *x,
                                        bool &noseed) {
  // the query's position in cell units; candidate cells: its own and the 7
  // neighbours of the octant it lies in; the seed whose (quantised) centroid
  // is nearest wins (ties: lower id)
  double t[3];
  int c[3], o[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    t[d] = seed_pos(fr, d, x[d], g);
    c[d] = seed_cell(t[d], g);
    const double f = t[d] - c[d];
    o[d] = f < 0.5 ? (c[d] > 0 ? -1 : 0) : (c[d] < g - 1 ? 1 : 0);
  }
  unsigned long long v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int a = c[0] + ((j & 1) ? o[0] : 0), b = c[1] + ((j & 2) ? o[1] : 0), e = c[2] + ((j & 4) ? o[2] : 0);
    v[j] = cell[a + (size_t)g * (b + (size_t)g * e)];
  }
  float best = 3.4e38f;
  unsigned bid = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (v[j] == ~0ULL) continue;
    const int a = c[0] + ((j & 1) ? o[0] : 0), b = c[1] + ((j & 2) ? o[1] : 0), e = c[2] + ((j & 4) ? o[2] : 0);
    const unsigned q = (unsigned)((v[j] >> 29) & 0x7FFFFFFULL), id = (unsigned)(v[j] & kSeedIdMask);
    const float dx = (float)(t[0] - a) - ((q & 511u) + 0.5f) * (1.0f / 512.0f);
    const float dy = (float)(t[1] - b) - (((q >> 9) & 511u) + 0.5f) * (1.0f / 512.0f);
    const float dz = (float)(t[2] - e) - (((q >> 18) & 511u) + 0.5f) * (1.0f / 512.0f);
    const float d2 = dx * dx + dy * dy + dz * dz;
    if (d2 < best || (d2 == best && id < bid)) {
      best = d2;
      bid = id;
    }
  }
  noseed = false;
  if (bid != 0xFFFFFFFFu) return (int)bid;
  // rare: the 8 cells are empty; the lowest seed of the shells around them
  const int r = seed_vol_ring(cell, g, c[0], c[1], c[2]);
  if (r) return r;
  // no seed within kSeedRing cells (counted as nvol_noseed): the walk starts
  // from the lowest in-use tetra the grid sampled (a long walk, or the
  // exhaustive search if it gets stuck, costs less than sending the query
  // straight to the O(ne) search); 0 (the exhaustive search) when the grid
  // sampled no tetra in use
  noseed = true;
  int any = INT_MAX;
  for (int j = 0; j < kSeedAnyParts; j++) any = min(any, fr->seed_any[j]);
  return any != INT_MAX ? any : 0;
}

// ---------------------------------------------------------------- surface seeds and node -> tria CSR

// surface seeds (r06): per cell the tria whose centroid is nearest the cell
// centre, one 64-bit key {8-bit squared distance to the centre (cell units),
// 9-bit centroid offset per axis, 29-bit id} reduced with atomicMin
// (deterministic), the volume seed grid's scheme; a query takes the nearest
// centroid among the 8 cells of its octant.  (Up to r05 the cell held its
// lowest tria id and a query took its own cell's: 3.90 walk steps per
// surface point at cfg4, the wave's longest walk 8 at the median.)
__device__ __forceinline__ unsigned long long srf_key(const double *p, const Frame *fr, int g, long long &ci) {
  int c[3];
  unsigned long long off = 0;
  float d2 = 0.f;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const double t = (p[d] - fr->lo[d]) * fr->inv_srf[d];
    c[d] = cell_coord(p[d], fr->lo[d], fr->inv_srf[d], g);
    float f = (float)(t - c[d]);
    f = f < 0.f ? 0.f : (f > 0.999f ? 0.999f : f);
    off |= (unsigned long long)(unsigned)(f * 512.f) << (9 * d);
    d2 += (f - 0.5f) * (f - 0.5f);
  }
  const unsigned q8 = d2 * 340.f < 255.f ? (unsigned)(d2 * 340.f) : 255u;
  ci = c[0] + (long long)g * (c[1] + (long long)g * c[2]);
  return ((unsigned long long)q8 << 56) | (off << 29);
}

__global__ __launch_bounds__(kBlock) void k_seed_srf(Bg bg, const Frame *fr, unsigned long long *cell, int g) {
  for (int k = 1 + blockIdx.x * blockDim.x + threadIdx.x; k <= bg.nt; k += gridDim.x * blockDim.x) {
    const int *tv = bg.triv + 3 * (size_t)(k - 1);
    if (tv[0] <= 0) continue;
    double p0[3], p1[3], p2[3], m[3];
    load_pt(bg.xyz, tv[0], p0);
    load_pt(bg.xyz, tv[1], p1);
    load_pt(bg.xyz, tv[2], p2);
    for (int d = 0; d < 3; d++) m[d] = (p0[d] + p1[d] + p2[d]) * (1.0 / 3.0);
    long long ci;
    const unsigned long long key = srf_key(m, fr, g, ci) | (unsigned)k;
    atomicMin(&cell[ci], key);
  }
}

// squared distance (cell units) from a query at t (cell units) to the
// centroid a key of cell (a, b, e) records
__device__ __forceinline__ float srf_d2(unsigned long long v, const double *t, int a, int b, int e) {
  const unsigned q = (unsigned)((v >> 29) & 0x7FFFFFFULL);
  const float dx = (float)(t[0] - a) - ((q & 511u) + 0.5f) * (1.0f / 512.0f);
  const float dy = (float)(t[1] - b) - (((q >> 9) & 511u) + 0.5f) * (1.0f / 512.0f);
  const float dz = (float)(t[2] - e) - (((q >> 18) & 511u) + 0.5f) * (1.0f / 512.0f);
  return dx * dx + dy * dy + dz * dz;
}

// a query's surface seed: the nearest recorded centroid among the 8 cells of
// its octant; when all 8 are empty, among the cells of the shells of radius
// 1, 2 around its cell; 0 when none (-> exhaustive search)
__device__ int seed_srf(const unsigned long long *cell, int g, const Frame *fr, const double *x) {
  double t[3];
  int c[3], o[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    t[d] = (x[d] - fr->lo[d]) * fr->inv_srf[d];
    c[d] = cell_coord(x[d], fr->lo[d], fr->inv_srf[d], g);
    const double f = t[d] - c[d];
    o[d] = f < 0.5 ? (c[d] > 0 ? -1 : 0) : (c[d] < g - 1 ? 1 : 0);
  }
  unsigned long long v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int a = c[0] + ((j & 1) ? o[0] : 0), b = c[1] + ((j & 2) ? o[1] : 0), e = c[2] + ((j & 4) ? o[2] : 0);
    v[j] = cell[a + (size_t)g * (b + (size_t)g * e)];
  }
  float best = 3.4e38f;
  unsigned bid = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (v[j] == ~0ULL) continue;
    const int a = c[0] + ((j & 1) ? o[0] : 0), b = c[1] + ((j & 2) ? o[1] : 0), e = c[2] + ((j & 4) ? o[2] : 0);
    const float d2 = srf_d2(v[j], t, a, b, e);
    const unsigned id = (unsigned)(v[j] & kSeedIdMask);
    if (d2 < best || (d2 == best && id < bid)) {
      best = d2;
      bid = id;
    }
  }
  if (bid != 0xFFFFFFFFu) return (int)bid;
  for (int r = 1; r <= 2; r++) {
    for (int dk = -r; dk <= r; dk++)
      for (int dj = -r; dj <= r; dj++)
        for (int di = -r; di <= r; di++) {
          if (max(abs(di), max(abs(dj), abs(dk))) != r) continue;
          const int a = c[0] + di, b = c[1] + dj, e = c[2] + dk;
          if (a < 0 || b < 0 || e < 0 || a >= g || b >= g || e >= g) continue;
          const unsigned long long w = cell[a + (size_t)g * (b + (size_t)g * e)];
          if (w == ~0ULL) continue;
          const float d2 = srf_d2(w, t, a, b, e);
          const unsigned id = (unsigned)(w & kSeedIdMask);
          if (d2 < best || (d2 == best && id < bid)) {
            best = d2;
            bid = id;
          }
        }
    if (bid != 0xFFFFFFFFu) return (int)bid;
  }
  return 0;
}

// ---------------------------------------------------------------- block scans
//
// block-level exclusive scans, and k_scan_top (one block: the exclusive scan
// of a short array, e.g. per-block counts).  When `gate` is non-null the
// kernel runs only if *gate == want.
constexpr int kScanItems = 16, kScanChunk = kBlock * kScanItems;

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// exclusive scan of one int per thread over the block; the block total in *tot
__device__ __forceinline__ int block_excl_scan(int v, int *tot) {
  __shared__ int wsum[kBlock / 64];
  const int inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6;
  if (__lane_id() == 63) wsum[w] = inc;
  __syncthreads();
  int pre = 0, all = 0;
#pragma unroll
  for (int j = 0; j < kBlock / 64; j++) {
    pre += j < w ? wsum[j] : 0;
    all += wsum[j];
  }
  __syncthreads();
  *tot = all;
  return pre + inc - v;
}

__device__ __forceinline__ bool gate_off(const int *gate, int want) { return gate && *gate != want; }

// one block: bsum[0..nb) -> exclusive offsets in place; the total -> *total
__global__ __launch_bounds__(kBlock) void k_scan_top(int *bsum, int nb, int *total, const int *gate, int want) {
  if (gate_off(gate, want)) return;
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += kBlock) {
    const int b = b0 + threadIdx.x;
    const int v = b < nb ? bsum[b] : 0;
    int tot;
    const int pre = block_excl_scan(v, &tot);
    if (b < nb) bsum[b] = carry + pre;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

// ---------------------------------------------------------------- seed grid axis maps

// (the histograms: axis_hist_block, inside k_quantize)
// one block per axis: counts -> quantile map, adaptive bit.  The test is on
// the scale of the grid's cells: the heaviest window of kMapBins / g bins
// (one uniform cell's slab) against the mean slab, g * max / total.  Bins
// finer than a cell cannot decide it (a lattice's coordinates fill only the
// bins its planes fall into).
// (r04k: the map built by the histogram kernel's last block, one launch
// less, took the three axes in turn: preparation +0.08 ms at cfg4)
__global__ __launch_bounds__(kBlock) void k_axis_map(const int *H, Frame *fr, int g) {
  constexpr int R = kMapBins / kBlock; // bins per thread
  const int d = blockIdx.x;
  __shared__ int cum[kMapBins + 1]; // cum[b] = vertices in bins [0, b)
  int cnt[R], s = 0;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int b = R * threadIdx.x + q;
    int v = 0;
#pragma unroll 16
    for (int k = 0; k < kHistBlocks; k++) v += H[(size_t)k * 3 * kMapBins + d * kMapBins + b];
    cnt[q] = v;
    s += v;
  }
  int tot;
  const int pre = block_excl_scan(s, &tot);
  {
    int run = pre;
#pragma unroll
    for (int q = 0; q < R; q++) {
      cum[R * threadIdx.x + q] = run;
      run += cnt[q];
    }
    if (threadIdx.x == kBlock - 1) cum[kMapBins] = run;
  }
  __syncthreads();
  const int W = (kMapBins + g - 1) / (g > 0 ? g : 1); // bins per uniform cell
  int mx = 0;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int b = R * threadIdx.x + q, e = b + W < kMapBins ? b + W : kMapBins;
    const int w = cum[e] - cum[b];
    mx = w > mx ? w : mx;
  }
  __shared__ int smx[kBlock];
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) smx[threadIdx.x] = smx[threadIdx.x + o] > smx[threadIdx.x] ? smx[threadIdx.x + o] : smx[threadIdx.x];
    __syncthreads();
  }
  const bool adapt = tot > 0 && (long long)smx[0] * g > (long long)kMapRatio * tot;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int b = R * threadIdx.x + q;
    fr->map[d][b] = adapt ? (float)((double)cum[b] / (double)tot) : (float)b / (float)kMapBins;
  }
  if (threadIdx.x == kBlock - 1) fr->map[d][kMapBins] = 1.0f;
  if (threadIdx.x == 0 && adapt) atomicOr(&fr->adaptive, 1 << d);
}

// ---------------------------------------------------------------- query order

constexpr int kBinBitsAxis = 7;     // Morton binning: at most 128^3 cells (Frame::inv_bin); the sort keys use the top
                                    // `bits` of every axis
constexpr int kBinBitsCoherent = 5; // 32^3 cells for a mostly coherent numbering (r03: forced bins on the lattice
                                    // numbering, volume stage 4.71 ms at 7 bits, 3.85 at 5; a shuffled one 7.98 at 7,
                                    // 8.83 at 5)

// Is the input numbering spatially coherent?  Distances between consecutive
// points at 4096 pseudo-random positions against the mean spacing h of np
// points in the bbox of the sample: coherent when at least half of them are
// below 4h (a median test: the jumps at the ends of lattice rows or of Mmg's
// local numbering runs do not count; a shuffled numbering has almost every
// distance at the scale of the bbox).  One block of k_quantize runs it (r05:
// on a stream of its own, as a one-block kernel, every other stream's kernels
// that read the flag waited on it across queues); writes flag[0] (1: Morton
// bins) and flag[1] (their bits per axis), read on the device by the order
// kernels and the volume / surface kernels.
__device__ __noinline__ void coherence_final(const Frame *fr, const double *cohd, int nq, int *flag,
                                             int *flag_host) {
  constexpr int nw = kBlock / 64;
  __shared__ int s_near[nw];
  // the mean spacing of nq points in the (sampled) background box
  __threadfence(); // (the test blocks' distances, released before their tickets)
  const double vol = fmax(fr->ext[0], 1e-300) * fmax(fr->ext[1], 1e-300) * fmax(fr->ext[2], 1e-300);
  const double h = cbrt(vol / (double)(nq > 1 ? nq : 1));
  int near = 0;
  for (int j = threadIdx.x; nq >= 2 && j < kCohSamples; j += kBlock) near += cohd[j] < 4.0 * h ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) near += __shfl_xor(near, o);
  if (__lane_id() == 0) s_near[threadIdx.x >> 6] = near;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int j = 0; j < nw; j++) tot += s_near[j];
    // input order when 3 in 4 steps are short; else Morton bins, with
    // coarse cells (kBinBitsCoherent bits per axis: the input order inside a
    // cell is kept and mostly coherent) when at least half are short, fine
    // cells (kBinBitsAxis) for a numbering without coherence.  (r04h: an
    // Mmg-like numbering — 83 % short steps, the inserted sixth appended —
    // takes 4.96 ms per cfg4 call in input order, 5.96 binned; r03's 95 %
    // threshold binned it.)
    const bool coherent = nq > 1 && 4 * tot >= 3 * kCohSamples;
    flag[0] = coherent ? 0 : 1;
    flag[1] = 2 * tot >= kCohSamples ? kBinBitsCoherent : kBinBitsAxis;
    if (flag_host) { // (a large call's host reads the decision after this kernel: run_device)
      flag_host[0] = flag[0];
      flag_host[1] = flag[1];
      __threadfence_system();
    }
  }
}

// ---------------------------------------------------------------- Morton binning (sorted order only)
//
// Queries of a numbering without spatial coherence are processed in Morton
// order of a 128^3 grid over the frame: k_bin_keys writes one 32-bit key per
// query {class: 0 volume, 1 surface, 2 neither | 21-bit Morton code} and its
// id, rocPRIM's radix sort (stable, 3 passes of 8 bits) orders them (r03: the
// earlier per-query atomicAdd on 2M bins took 1.9 ms at cfg4 on a shuffled
// numbering; a hand-written two-level counting sort without global atomics
// still 2.5 ms, its scattered partial-line writes across XCDs dominating),
// and k_bin_split cuts the sorted ids into the volume list (plus a copy of
// the volume queries' coordinates in processing order, so that the walk loads
// them coalesced) and the surface list.  The radix sort is stable: the order
// is a deterministic function of the input.

// flag: the order decision {sorted, bits per axis} (coherence_final); the kernel
// runs only when flag[0] == 1.  Blocks loop over the radix sort's tiles
// (tile_keys keys, pmmg_sort.hpp): besides the keys it writes each tile's
// histogram of the first 8-bit digit (hist[digit * ntile + tile]), the first
// pass's table.
__global__ __launch_bounds__(kBlock) void k_bin_keys(const double *xyz, const uint8_t *pclass, int np, const Frame *fr,
                                                     const int *flag, unsigned *keys, int *vals, DevStats *st,
                                                     int tile_keys, int ntile, int *hist) {
  if (flag[0] != 1) return;
  const int bits = flag[1];
  __shared__ int h[kBlock];
  __shared__ int sv, sb;
  h[threadIdx.x] = 0;
  if (threadIdx.x == 0) sv = sb = 0;
  __syncthreads();
  int nv = 0, nb = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
  const long long base = (long long)tile * tile_keys;
  // batches of 8 points with their class and coordinates loaded together
  // (r04: one point at a time, a class load then its coordinates, 363 us for
  // 20M points beside the seed grid)
  constexpr int kBatch = 8;
  for (int e0 = 0; e0 < tile_keys; e0 += kBatch * kBlock) {
    int c[kBatch];
    double x[kBatch][3];
#pragma unroll
    for (int u = 0; u < kBatch; u++) {
      const long long i = base + e0 + u * kBlock + threadIdx.x;
      const bool in = e0 + u * kBlock + (int)threadIdx.x < tile_keys && i < np;
      c[u] = in ? (int)pclass[i] : -1;
#pragma unroll
      for (int d = 0; d < 3; d++) x[u][d] = in ? xyz[3 * i + d] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kBatch; u++) {
      if (c[u] < 0) continue;
      const long long i = base + e0 + u * kBlock + threadIdx.x;
      unsigned cls = 2u;
      uint32_t q[3] = {0u, 0u, 0u};
      if (c[u] == PMMG_PT_VOL || c[u] == PMMG_PT_BDY) {
        cls = c[u] == PMMG_PT_VOL ? 0u : 1u;
        nv += c[u] == PMMG_PT_VOL;
        nb += c[u] == PMMG_PT_BDY;
#pragma unroll
        for (int d = 0; d < 3; d++)
          q[d] = (uint32_t)cell_coord(x[u][d], fr->lo[d], fr->inv_bin[d], 1 << kBinBitsAxis) >> (kBinBitsAxis - bits);
      }
      const unsigned key = (cls << (3 * bits)) | (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
      keys[i] = key;
      vals[i] = (int)(i + 1);
      atomicAdd(&h[key & 255u], 1);
    }
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * ntile + tile] = h[threadIdx.x];
  h[threadIdx.x] = 0;
  __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) {
    nv += __shfl_down(nv, o);
    nb += __shfl_down(nb, o);
  }
  if (__lane_id() == 0) {
    atomicAdd(&sv, nv);
    atomicAdd(&sb, nb);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (sv) atomicAdd(&st->nvol, sv);
    if (sb) atomicAdd(&st->nbdy, sb);
  }
}

// sorted ids -> volume list (order_v, in place) + the volume queries'
// coordinates in that order (qs, when non-null), surface list (order_b)
__global__ __launch_bounds__(kBlock) void k_bin_split(const int *sorted_ids, const double *xyz, int np, int *order_b,
                                                      double *qs, const DevStats *st, const int *flag) {
  if (flag[0] != 1) return;
  const int nvol = st->nvol, nbdy = st->nbdy;
  for (long long j = (qs ? 0 : nvol) + blockIdx.x * (long long)blockDim.x + threadIdx.x; j < nvol + nbdy;
       j += (long long)gridDim.x * blockDim.x) {
    const int ip = sorted_ids[j];
    if (j < nvol) {
      if (qs) {
        qs[3 * j] = xyz[3 * (size_t)(ip - 1)];
        qs[3 * j + 1] = xyz[3 * (size_t)(ip - 1) + 1];
        qs[3 * j + 2] = xyz[3 * (size_t)(ip - 1) + 2];
      }
    } else {
      order_b[j - nvol] = ip;
    }
  }
}

// Stable class compaction (the surface list, input-order path only): out =
// the ids ip (1-based) with pclass[ip-1] == cls, in input order; *count =
// their number.  Three passes over the 1-byte classes (count per block, scan
// of the block counts, scatter).  Each block owns kScanChunk points.
// bit j = (pclass[i0 + j] == cls); the 16 classes of a thread come in one
// 16-byte load when the array is 16-byte aligned and the run is complete
__device__ __forceinline__ unsigned cls_bits(const uint8_t *pclass, long long np, long long i0, int cls) {
  unsigned m = 0;
  if (i0 + kScanItems <= np && ((uintptr_t)pclass & 15) == 0) {
    const uint4 w = *reinterpret_cast<const uint4 *>(pclass + i0);
    const unsigned words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < kScanItems; j++)
      m |= (((words[j >> 2] >> (8 * (j & 3))) & 0xFFu) == (unsigned)cls) ? (1u << j) : 0u;
    return m;
  }
#pragma unroll
  for (int j = 0; j < kScanItems; j++) {
    const long long i = i0 + j;
    m |= (i < np && pclass[i] == cls) ? (1u << j) : 0u;
  }
  return m;
}

__global__ __launch_bounds__(kBlock) void k_cls_count(const uint8_t *pclass, long long np, int cls, int *bcnt,
                                                      const int *gate, int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  int tot;
  block_excl_scan(__popc(cls_bits(pclass, np, i0, cls)), &tot);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_cls_scatter(const uint8_t *pclass, long long np, int cls,
                                                        const int *boff, int *out, const int *gate, int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  unsigned m = cls_bits(pclass, np, i0, cls);
  int tot;
  int pos = boff[blockIdx.x] + block_excl_scan(__popc(m), &tot);
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    out[pos++] = (int)(i0 + j + 1);
  }
}

// ---------------------------------------------------------------- exhaustive-search helpers
// (pmmg_fallback.hpp; the grids are built by the last blocks of k_vol_walk_exact and k_bdy)

// the last block of a grid to pass this point (after its device-scope
// atomics) gets true: the other blocks' results are then visible to it.  The
// barrier before the ticket: every wave of the block has issued its atomics
// (r04l: without it a block's later waves could still be scanning when the
// last block read the results — 4 surface points left unprocessed, once)
// The last block of a grid to get here returns true.  wrote: this thread
// stored data the last block reads; a block any of whose threads did
// releases it first (__threadfence).  The release is an L2 write-back on
// gfx950 (the XCDs' L2s are not coherent with each other): taken in every
// block of k_bdy (808 blocks for a 205k-point group) it took the kernel 17 ->
// 87 us and slowed the volume kernel beside it (r05h trace) — only the blocks
// that appended to a fallback list pay it.
__device__ __forceinline__ bool last_block(unsigned *done, bool wrote) {
  if (__syncthreads_or(wrote)) __threadfence();
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last) __threadfence();
  return last;
}

__device__ __forceinline__ int load_agent(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The bounding box of an element inflated so that every point its
// acceptance test can pass lies inside.  Volume: every barycentric
// coordinate > -EPS puts x within 3 EPS of the extent outside the vertices'
// box (x_c = sum_i b_i p_ic, sum_i b_i = 1); the pad is 1e-4 of the extent
// (33x that, room for the coordinates' rounding on any element with an
// aspect ratio below ~1e10) plus 1e-12 of the coordinates' magnitude.
// Surface: the projection is inside the tria within the same margin and
// |dist| <= hausd along the unit normal.  A degenerate element (zero or
// non-finite volume / area) gets an infinite box: every query takes the
// reference's test there, as in the oracle.
constexpr double kBoxRel = 1e-4, kBoxAbs = 1e-12;
struct Box {
  double lo[3], hi[3];
};
__device__ __forceinline__ bool in_box(const Box &b, const double *x) {
  // NaN coordinates compare false everywhere and fall through to the test
  return !(x[0] < b.lo[0] || x[0] > b.hi[0] || x[1] < b.lo[1] || x[1] > b.hi[1] || x[2] < b.lo[2] ||
           x[2] > b.hi[2]);
}
template <int NV>
__device__ __forceinline__ Box elem_box(const double (*p)[3], double extra, bool degenerate) {
  Box b;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    double lo = p[0][c], hi = p[0][c];
#pragma unroll
    for (int v = 1; v < NV; v++) {
      lo = fmin(lo, p[v][c]);
      hi = fmax(hi, p[v][c]);
    }
    const double pad = kBoxRel * (hi - lo) + kBoxAbs * fmax(fabs(lo), fabs(hi)) + extra + 1e-300;
    b.lo[c] = degenerate ? -INFINITY : lo - pad;
    b.hi[c] = degenerate ? INFINITY : hi + pad;
  }
  return b;
}

// ---------------------------------------------------------------- query grids
//
// The accept scans test an element only against the fallback queries in the
// grid cells its inflated box covers (r05: against every query of the list,
// the scan cost ne x nfb box tests — 92 ms for 2644 queries over 120M tetra
// in a carried iteration).  The grid is built by the last block of the kernel
// that finishes the list (k_vol_walk_exact, k_bdy): G^3 cells over the
// queries' box, G = cbrt(nfb / 4) + 1 <= kFbGridMax; cells[c] .. cells[c + 1]
// index items[], the list positions of cell c's queries.  A query inside an
// element's box is in a cell of the box's (clamped) cell range, so the pairs
// tested are a superset of the accepting pairs: the same results as the full
// scan.
constexpr int kFbGridMax = 16;
constexpr int kFbCells = kFbGridMax * kFbGridMax * kFbGridMax;
struct FbGridBufs {
  int *cells; // kFbCells + 1 starts
  int *cur;   // kFbCells scratch
  int *items; // one per list entry
};

__device__ __forceinline__ int fb_cell1(double x, double lo, double inv, int G) {
  const double t = (x - lo) * inv;
  return t > 0.0 ? (t < (double)G ? (int)t : G - 1) : 0; // NaN -> 0, +inf -> G - 1
}

// one block: the grid of the list fb[0, nfb) (cls 0 volume, 1 surface);
// cells[kFbCells + 1] starts, cur[kFbCells] scratch, items[nfb]
__device__ __noinline__ void fb_grid_build(const double *qxyz, const int *fb, int nfb, DevStats *st, int cls,
                                           int *cells, int *cur, int *items) {
  __shared__ double rlo[3][kBlock / 64], rhi[3][kBlock / 64]; // per-wave partial boxes
  __shared__ int sG;
  const int t = threadIdx.x, nt = blockDim.x, w = t >> 6, nw = (nt + 63) >> 6;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int j = t; j < nfb; j += nt) {
    double x[3];
    load_pt(qxyz, fb[j], x);
    for (int d = 0; d < 3; d++) {
      lo[d] = fmin(lo[d], x[d]);
      hi[d] = fmax(hi[d], x[d]);
    }
  }
  for (int d = 0; d < 3; d++)
    for (int o = 32; o > 0; o >>= 1) {
      lo[d] = fmin(lo[d], __shfl_xor(lo[d], o));
      hi[d] = fmax(hi[d], __shfl_xor(hi[d], o));
    }
  if (__lane_id() == 0)
    for (int d = 0; d < 3; d++) {
      rlo[d][w] = lo[d];
      rhi[d][w] = hi[d];
    }
  __syncthreads();
  if (t == 0) {
    for (int d = 0; d < 3; d++) {
      double a = INFINITY, b = -INFINITY;
      for (int i = 0; i < nw; i++) {
        a = fmin(a, rlo[d][i]);
        b = fmax(b, rhi[d][i]);
      }
      rlo[d][0] = a;
      rhi[d][0] = b;
    }
    int G = (int)cbrt((double)nfb / 4.0) + 1;
    G = G < 1 ? 1 : (G > kFbGridMax ? kFbGridMax : G);
    for (int d = 0; d < 3; d++) {
      const double e = rhi[d][0] - rlo[d][0];
      st->fbg_lo[cls][d] = rlo[d][0];
      st->fbg_inv[cls][d] = e > 0.0 ? (double)G / e : 0.0;
    }
    st->fbg_n[cls] = G;
    sG = G;
  }
  __syncthreads();
  const int G = sG, nc = G * G * G;
  const double l0 = st->fbg_lo[cls][0], l1 = st->fbg_lo[cls][1], l2 = st->fbg_lo[cls][2];
  const double i0 = st->fbg_inv[cls][0], i1 = st->fbg_inv[cls][1], i2 = st->fbg_inv[cls][2];
  for (int c = t; c < nc; c += nt) cur[c] = 0;
  __syncthreads();
  for (int j = t; j < nfb; j += nt) {
    double x[3];
    load_pt(qxyz, fb[j], x);
    const int c = fb_cell1(x[0], l0, i0, G) + G * (fb_cell1(x[1], l1, i1, G) + G * fb_cell1(x[2], l2, i2, G));
    atomicAdd(&cur[c], 1);
  }
  __threadfence_block();
  __syncthreads();
  if (t == 0) { // exclusive scan (at most kFbCells entries, once per call with fallbacks)
    int acc = 0;
    for (int c = 0; c < nc; c++) {
      const int v = cur[c];
      cells[c] = acc;
      cur[c] = acc;
      acc += v;
    }
    cells[nc] = acc;
  }
  __threadfence_block();
  __syncthreads();
  for (int j = t; j < nfb; j += nt) {
    double x[3];
    load_pt(qxyz, fb[j], x);
    const int c = fb_cell1(x[0], l0, i0, G) + G * (fb_cell1(x[1], l1, i1, G) + G * fb_cell1(x[2], l2, i2, G));
    items[atomicAdd(&cur[c], 1)] = j;
  }
}

// The query grid of a completed fallback list (cls 0: volume, 1: surface), one
// block, launched after the kernel that completes the list (r06: before, the
// last block of that kernel built it after a per-block ticket on one counter
// — k_bdy's 4096 tickets alone serialised ~47 us of atomics at the end of
// the surface branch, profiles/r06j); returns at once for an empty list
__global__ __launch_bounds__(kBlock) void k_fb_grid(const double *qxyz, const int *fb, DevStats *st, int cls,
                                                   FbGridBufs gb) {
  const int nfb = cls == 0 ? st->nfb_vol : st->nfb_bdy;
  if (nfb > 0) fb_grid_build(qxyz, fb, nfb, st, cls, gb.cells, gb.cur, gb.items);
}

// the queries of the cells an element's (inflated) box covers: visit(j) for
// each list position j (the accept test itself); nothing when the box misses
// the grid's box
template <class F>
__device__ __forceinline__ void fb_grid_visit(const DevStats *st, int cls, const int *cells, const int *items,
                                              const Box &b, F &&visit) {
  const int G = st->fbg_n[cls];
  int a[3], e[3];
  for (int d = 0; d < 3; d++) {
    const double lo = st->fbg_lo[cls][d], inv = st->fbg_inv[cls][d];
    const double hi = inv > 0.0 ? lo + (double)G / inv : lo;
    if (b.hi[d] < lo || b.lo[d] > hi) return; // (NaN boxes: degenerate elements have infinite ones)
    a[d] = fb_cell1(b.lo[d], lo, inv, G);
    e[d] = fb_cell1(b.hi[d], lo, inv, G);
  }
  for (int z = a[2]; z <= e[2]; z++)
    for (int y = a[1]; y <= e[1]; y++)
      for (int x = a[0]; x <= e[0]; x++) {
        const int c = x + G * (y + G * z);
        for (int q = cells[c]; q < cells[c + 1]; q++) visit(items[q]);
      }
}

// ---------------------------------------------------------------- accept scans

} // namespace pmmg
