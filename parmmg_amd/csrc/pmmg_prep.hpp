// pmmg_prep.hpp — per-call preparation kernels of the transfer step
// (included by pmmg_hip.hip only): state reset, background frame, volume and
// surface seed grids, and the query order.
//
// Every decision is taken on the device: the input-order coherence test
// writes DevStats::sorted, and the Morton-binning kernels and the class
// compaction of the surface list are both enqueued and return at once when
// the flag does not select them.  No kernel result is read back by the host
// inside a call.
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
  int pad[2];
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
// same number of tetra.  An axis whose densest bin is below kMapRatio x the
// mean of its occupied bins keeps the uniform cells (bit 0 of `adaptive`
// per axis clear): the shell and cube lattices are not remapped.
constexpr int kMapBins = 2048;
constexpr int kMapRatio = 16;
constexpr int kHistBlocks = 128;

struct Frame {
  unsigned long long key_lo[3], key_hi[3];
  double lo[3], ext[3];
  double inv_vol[3], inv_srf[3], inv_bin[3];
  double qc[3], qs; // fixed-point frame of the walk's vertex copy
  int adaptive;     // bit d: axis d of the volume seed grid follows map[d]
  int pad;
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

__global__ __launch_bounds__(kBlock) void k_quantize(const double *xyz, long long np, const Frame *fr, int *xq) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < 3 * np; j += (long long)gridDim.x * blockDim.x)
    xq[kXqStride * (j / 3) + j % 3] = quant(__builtin_nontemporal_load(xyz + j), fr, (int)(j % 3));
}

// one launch initialises the per-call state: frame accumulators, counters,
// seed grids
__global__ __launch_bounds__(kBlock) void k_reset(Frame *fr, DevStats *st, unsigned long long *grid, long long ng,
                                                  int *sgrid, long long nsg) {
  const long long tid = blockIdx.x * (long long)blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  if (tid == 0) {
    for (int d = 0; d < 3; d++) {
      fr->key_lo[d] = ~0ULL;
      fr->key_hi[d] = 0ULL;
    }
    fr->adaptive = 0;
    unsigned int *w = reinterpret_cast<unsigned int *>(st);
    for (size_t j = 0; j < sizeof(DevStats) / 4; j++) w[j] = 0u;
  }
  {
    unsigned long long *pw = reinterpret_cast<unsigned long long *>(st + 1);
    for (long long j = tid; j < (long long)(kStatParts * sizeof(StatPart) / 8); j += nth) pw[j] = 0ULL;
  }
  for (long long j = tid; j < ng; j += nth) grid[j] = ~0ULL;
  for (long long j = tid; j < nsg; j += nth) sgrid[j] = INT_MAX;
}

// bbox of every `stride`-th vertex (and the last one): the frame only sizes
// the seed / bin grids, whose cell lookups clamp, so a sampled bbox costs at
// most slightly longer walks for the few points outside it
__global__ __launch_bounds__(kBlock) void k_bbox(const double *xyz, int np, Frame *fr, int stride) {
  __shared__ unsigned long long slo[3][kBlock / 64], shi[3][kBlock / 64];
  unsigned long long lo[3] = {~0ULL, ~0ULL, ~0ULL}, hi[3] = {0ULL, 0ULL, 0ULL};
  const long long ns = ((long long)np + stride - 1) / stride + 1;
  for (long long j = blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += gridDim.x * blockDim.x) {
    const long long i = j * stride < np ? j * stride : np - 1;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      unsigned long long k = dkey(xyz[3 * i + d]);
      lo[d] = k < lo[d] ? k : lo[d];
      hi[d] = k > hi[d] ? k : hi[d];
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
}

__global__ void k_frame_final(Frame *fr, int g, int gs, int gb) {
  double emax = 0.0;
  for (int d = 0; d < 3; d++) {
    double lo = dunkey(fr->key_lo[d]), hi = dunkey(fr->key_hi[d]);
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

__global__ __launch_bounds__(kBlock) void k_seed_vol(Bg bg, const Frame *fr, unsigned long long *cell, int g,
                                                     long long nsamp, int lanes) {
  constexpr int R = kSeedRun;
  const long long nruns = (nsamp + R - 1) / R;
  const long long quads = bg.ne / 4;
  const long long nthreads = nruns * R;
  // XCD-aware: the blocks of XCD x (blockIdx % 8; gridDim is a multiple of
  // 8) sweep one contiguous eighth of the samples, so the vertex rows shared
  // by neighbouring tetra are fetched into one L2, not eight
  const long long per = (nthreads + 8LL * kBlock - 1) / (8LL * kBlock) * kBlock;
  const long long lo = (blockIdx.x & 7) * per, hi = lo + per < nthreads ? lo + per : nthreads;
  const long long bstride = (long long)(gridDim.x >> 3) * blockDim.x;
  for (long long s0 = lo + (blockIdx.x >> 3) * (long long)blockDim.x; s0 < hi; s0 += bstride) {
    const long long s = s0 + threadIdx.x;
    const long long run = s / R;
    const int r = (int)(s % R);
    const long long base = 4 * ((run * quads) / (nruns > 0 ? nruns : 1)); // a cache line of tet8 records
    const int k = (int)(1 + base + r);
    bool ok = s < hi && k <= bg.ne && r < lanes; // `lanes` of the run's 4 records are sampled
    int4 tv = make_int4(0, 0, 0, 0);
    if (ok) {
      const nti4 rr =
          __builtin_nontemporal_load(reinterpret_cast<const nti4 *>(bg.tetv + (size_t)(k - 1) * bg.tstride));
      tv = make_int4(rr.x, rr.y, rr.z, rr.w);
      ok = tv.x > 0;
    }
    unsigned long long key = ~0ULL;
    long long ci = -1;
    if (ok) {
      // centroid from the fixed-point copy (12-byte rows)
      const int *q0 = bg.xq + kXqStride * (size_t)(tv.x - 1), *q1 = bg.xq + kXqStride * (size_t)(tv.y - 1);
      const int *q2 = bg.xq + kXqStride * (size_t)(tv.z - 1), *q3 = bg.xq + kXqStride * (size_t)(tv.w - 1);
      double p[3];
      for (int d = 0; d < 3; d++)
        p[d] = fr->qc[d] + 0.25 * ((double)q0[d] + (double)q1[d] + (double)q2[d] + (double)q3[d]) / fr->qs;
      int c[3];
      unsigned long long off = 0;
      float d2 = 0.f;
      for (int d = 0; d < 3; d++) {
        const double t = seed_pos(fr, d, p[d], g);
        c[d] = seed_cell(t, g);
        float f = (float)(t - c[d]);
        f = f < 0.f ? 0.f : (f > 0.999f ? 0.999f : f);
        off |= (unsigned long long)(unsigned)(f * 512.f) << (9 * d);
        d2 += (f - 0.5f) * (f - 0.5f);
      }
      const unsigned q8 = d2 * 340.f < 255.f ? (unsigned)(d2 * 340.f) : 255u;
      key = ((unsigned long long)q8 << 56) | (off << 29) | (unsigned)k;
      ci = c[0] + (long long)g * (c[1] + (long long)g * c[2]);
    }
    // combine within the run: the first lane of each distinct cell issues
    // the atomic with the run's minimum for that cell
    const int lane = __lane_id(), g0 = lane - r;
    bool leader = ci >= 0;
    unsigned long long best = key;
    for (int o = 0; o < R; o++) {
      const long long co = __shfl(ci, g0 + o);
      const unsigned long long ko = __shfl(key, g0 + o);
      if (co == ci && ci >= 0) {
        best = ko < best ? ko : best;
        if (o < r) leader = false;
      }
    }
    if (leader) atomicMin(&cell[ci], best);
  }
}

// rare path of seed_vol (the 8 cells are empty): lowest seed id in the shells
// of radius 1 then 2 around the cell; 0 when there is none (the query then
// goes to the exact continuation, which hands it to the exhaustive search)
__device__ __noinline__ int seed_vol_ring(const unsigned long long *cell, int g, int ci, int cj, int ck) {
#pragma unroll 1
  for (int r = 1; r <= 2; r++) {
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

__device__ __forceinline__ int seed_vol(const unsigned long long *cell, int g, const Frame *fr, const double *x) {
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
  if (bid != 0xFFFFFFFFu) return (int)bid;
  return seed_vol_ring(cell, g, c[0], c[1], c[2]);
}

// ---------------------------------------------------------------- surface seeds and node -> tria CSR

// surface seeds: cell of each tria centroid -> min id
__global__ __launch_bounds__(kBlock) void k_seed_srf(Bg bg, const Frame *fr, int *cell, int g) {
  for (int k = 1 + blockIdx.x * blockDim.x + threadIdx.x; k <= bg.nt; k += gridDim.x * blockDim.x) {
    const int *tv = bg.triv + 3 * (size_t)(k - 1);
    if (tv[0] <= 0) continue;
    double p0[3], p1[3], p2[3];
    load_pt(bg.xyz, tv[0], p0);
    load_pt(bg.xyz, tv[1], p1);
    load_pt(bg.xyz, tv[2], p2);
    int c[3];
    for (int d = 0; d < 3; d++) c[d] = cell_coord((p0[d] + p1[d] + p2[d]) * (1.0 / 3.0), fr->lo[d], fr->inv_srf[d], g);
    atomicMin(&cell[c[0] + (size_t)g * (c[1] + (size_t)g * c[2])], k);
  }
}

// a tria's surface seed cell; empty cell -> lowest id of the shells of
// radius 1, 2; 0 when none (-> exhaustive search)
__device__ int seed_srf(const int *cell, int g, const Frame *fr, const double *x) {
  int ci = cell_coord(x[0], fr->lo[0], fr->inv_srf[0], g);
  int cj = cell_coord(x[1], fr->lo[1], fr->inv_srf[1], g);
  int ck = cell_coord(x[2], fr->lo[2], fr->inv_srf[2], g);
  int s = cell[ci + (size_t)g * (cj + (size_t)g * ck)];
  if (s != INT_MAX) return s;
  for (int r = 1; r <= 2; r++) {
    int best = INT_MAX;
    for (int dk = -r; dk <= r; dk++)
      for (int dj = -r; dj <= r; dj++)
        for (int di = -r; di <= r; di++) {
          if (max(abs(di), max(abs(dj), abs(dk))) != r) continue;
          int a = ci + di, b = cj + dj, c = ck + dk;
          if (a < 0 || b < 0 || c < 0 || a >= g || b >= g || c >= g) continue;
          int v = cell[a + (size_t)g * (b + (size_t)g * c)];
          best = v < best ? v : best;
        }
    if (best != INT_MAX) return best;
  }
  return 0;
}

// ---------------------------------------------------------------- device-wide exclusive scan
//
// out[0..n] = exclusive prefix sums of in[0..n) (out[n] = total), in three
// launches (per-block sums, scan of the block sums, per-block scan).  When
// `gate` is non-null the kernels run only if *gate == want, so a scan can be
// enqueued for a path the device may not take.
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

__global__ __launch_bounds__(kBlock) void k_scan_sums(const int *in, long long n, int *bsum, const int *gate,
                                                      int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; j++) s += (i0 + j < n) ? in[i0 + j] : 0;
  int tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

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

__global__ __launch_bounds__(kBlock) void k_scan_write(const int *in, long long n, const int *bsum, int *out,
                                                       const int *gate, int want) {
  if (gate_off(gate, want)) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  int v[kScanItems], s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; j++) {
    v[j] = (i0 + j < n) ? in[i0 + j] : 0;
    s += v[j];
  }
  int tot;
  int pre = bsum[blockIdx.x] + block_excl_scan(s, &tot);
#pragma unroll
  for (int j = 0; j < kScanItems; j++) {
    if (i0 + j < n) out[i0 + j] = pre;
    pre += v[j];
  }
  if (i0 <= n && n < i0 + kScanItems) out[n] = pre; // the thread holding the end writes the total
}

// ---------------------------------------------------------------- seed grid axis maps

// the per-axis histogram of every `stride`-th background vertex:
// H[block][d][bin] (kHistBlocks blocks, no atomics outside LDS)
__global__ __launch_bounds__(kBlock) void k_axis_hist(const double *xyz, int np, const Frame *fr, int stride, int *H) {
  __shared__ int h[3][kMapBins];
  for (int j = threadIdx.x; j < 3 * kMapBins; j += kBlock) (&h[0][0])[j] = 0;
  __syncthreads();
  const long long ns = ((long long)np + stride - 1) / stride;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < ns; j += (long long)gridDim.x * blockDim.x) {
    const long long i = j * stride;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const double e = fr->ext[d];
      double b = e > 0.0 ? (xyz[3 * i + d] - fr->lo[d]) * ((double)kMapBins / e) : 0.0;
      const int bi = b > 0.0 ? (b < (double)kMapBins ? (int)b : kMapBins - 1) : 0;
      atomicAdd(&h[d][bi], 1);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * kMapBins; j += kBlock) H[(size_t)blockIdx.x * 3 * kMapBins + j] = (&h[0][0])[j];
}

// one block per axis: counts -> quantile map, adaptive bit
__global__ __launch_bounds__(kBlock) void k_axis_map(const int *H, Frame *fr) {
  constexpr int R = kMapBins / kBlock; // bins per thread
  const int d = blockIdx.x;
  int cnt[R], s = 0, mx = 0, occ = 0;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int b = R * threadIdx.x + q;
    int v = 0;
    for (int k = 0; k < kHistBlocks; k++) v += H[(size_t)k * 3 * kMapBins + d * kMapBins + b];
    cnt[q] = v;
    s += v;
    mx = v > mx ? v : mx;
    occ += v > 0 ? 1 : 0;
  }
  int tot;
  const int pre = block_excl_scan(s, &tot);
  __shared__ int smx[kBlock], socc[kBlock];
  smx[threadIdx.x] = mx;
  socc[threadIdx.x] = occ;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      smx[threadIdx.x] = smx[threadIdx.x + o] > smx[threadIdx.x] ? smx[threadIdx.x + o] : smx[threadIdx.x];
      socc[threadIdx.x] += socc[threadIdx.x + o];
    }
    __syncthreads();
  }
  // adaptive: the densest bin holds more than kMapRatio x the mean occupied bin
  const bool adapt = tot > 0 && (long long)smx[0] * socc[0] > (long long)kMapRatio * tot;
  int run = pre;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int b = R * threadIdx.x + q;
    fr->map[d][b] = adapt ? (float)((double)run / (double)tot) : (float)b / (float)kMapBins;
    run += cnt[q];
  }
  if (threadIdx.x == kBlock - 1) fr->map[d][kMapBins] = 1.0f;
  if (threadIdx.x == 0 && adapt) atomicOr(&fr->adaptive, 1 << d);
}

// ---------------------------------------------------------------- query order

// Is the input numbering spatially coherent?  Distances between consecutive
// points at 4096 pseudo-random positions against the mean spacing h of np
// points in the bbox of the sample: coherent when at least half of them are
// below 4h (a median test: the jumps at the ends of lattice rows or of Mmg's
// local numbering runs do not count; a shuffled numbering has almost every
// distance at the scale of the bbox).  force: 1 always Morton-bin, 0 never,
// -1 test.  Writes st->sorted.
__global__ __launch_bounds__(kBlock) void k_coherence(const double *xyz, int np, DevStats *st, int force) {
  if (force >= 0) {
    if (threadIdx.x == 0) st->sorted = force;
    return;
  }
  constexpr int nsamp = 4096, per = nsamp / kBlock;
  __shared__ double slo[3][kBlock], shi[3][kBlock];
  __shared__ double s_h;
  __shared__ int s_near[kBlock];
  double dist[per], lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
#pragma unroll
  for (int q = 0; q < per; q++) {
    const int smp = threadIdx.x + q * kBlock;
    dist[q] = 0.0;
    if (np < 2) continue;
    // pseudo-random positions (splitmix64 of the sample index): an evenly
    // strided sample can alias with the row length of a lattice numbering
    unsigned long long z = (unsigned long long)smp * 0x9E3779B97F4A7C15ULL + 0x5EED2025ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    const long long i = (long long)(z % (unsigned long long)(np - 1));
    double d2 = 0.0;
    for (int d = 0; d < 3; d++) {
      double a = xyz[3 * (size_t)i + d], b = xyz[3 * (size_t)(i + 1) + d];
      double t = b - a;
      d2 += t * t;
      lo[d] = fmin(lo[d], a);
      hi[d] = fmax(hi[d], a);
    }
    dist[q] = sqrt(d2);
  }
  for (int d = 0; d < 3; d++) {
    slo[d][threadIdx.x] = lo[d];
    shi[d][threadIdx.x] = hi[d];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L[3] = {1e300, 1e300, 1e300}, H[3] = {-1e300, -1e300, -1e300};
    for (int j = 0; j < kBlock; j++)
      for (int d = 0; d < 3; d++) {
        L[d] = fmin(L[d], slo[d][j]);
        H[d] = fmax(H[d], shi[d][j]);
      }
    double vol = fmax(H[0] - L[0], 1e-300) * fmax(H[1] - L[1], 1e-300) * fmax(H[2] - L[2], 1e-300);
    s_h = cbrt(vol / (double)(np > 1 ? np : 1));
  }
  __syncthreads();
  int near = 0;
#pragma unroll
  for (int q = 0; q < per; q++) near += dist[q] < 4.0 * s_h ? 1 : 0;
  s_near[threadIdx.x] = near;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int j = 0; j < kBlock; j++) tot += s_near[j];
    st->sorted = (np > 1 && 2 * tot >= nsamp) ? 0 : 1;
  }
}

// ---------------------------------------------------------------- Morton binning (st->sorted == 1 only)
//
// Queries of a numbering without spatial coherence are processed in Morton
// order of a 64^3 grid over the frame, in two counting passes without global
// atomics (r03; the r02 binning took one returning device-scope atomicAdd per
// query on 2M bins: 1.9 ms at cfg4 on a shuffled numbering):
//   pass 1 (k_bin_hist, scan, k_bin_place) — digit = (class, coarse cell: the
//     top 3 bits per axis, 512 cells): per-block LDS histograms in a
//     digit-major matrix, one device-wide scan gives every (digit, block) its
//     range, the block places its queries there through LDS counters; a
//     placed query carries {id, fine key} and its coordinates;
//   pass 2 (k_bin_chunks, k_bin_fine_hist, scan, k_bin_fine_place) — the
//     same counting sort inside every digit by the fine key (the low 4 bits
//     per axis, 512 cells), on chunks of at most 4096 queries of one digit;
//     the result is the order list plus a copy of the coordinates in that
//     order (the walk then loads its queries coalesced).
// Order inside a fine cell is not deterministic (LDS counters); every query's
// result is a pure function of the query, so no output depends on it.
constexpr int kBinBitsAxis = 6;                  // 64^3 grid (Frame::inv_bin)
constexpr int kBinCoarse = 512;                  // 8^3 coarse cells per class
constexpr int kBinDigits = 2 * kBinCoarse;       // volume digits first, then surface
constexpr int kBinFine = 512;                    // 8^3 fine cells per coarse cell
constexpr int kBinChunk = kBlock * 16;           // queries per pass-2 chunk

// digit (-1: neither a volume nor a surface query) and fine key of query i
__device__ __forceinline__ int bin_key(const double *xyz, const uint8_t *pclass, long long i, const Frame *fr,
                                       int *fine, double *x) {
  const int c = pclass[i];
  if (c != PMMG_PT_VOL && c != PMMG_PT_BDY) return -1;
  uint32_t q[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    x[d] = xyz[3 * i + d];
    q[d] = (uint32_t)cell_coord(x[d], fr->lo[d], fr->inv_bin[d], 1 << kBinBitsAxis);
  }
  const uint32_t lo = 7u;
  *fine = (int)((expand10(q[0] & lo) << 2) | (expand10(q[1] & lo) << 1) | expand10(q[2] & lo));
  const int coarse = (int)((expand10(q[0] >> 3) << 2) | (expand10(q[1] >> 3) << 1) | expand10(q[2] >> 3));
  return coarse + (c == PMMG_PT_BDY ? kBinCoarse : 0);
}

// block b's contiguous tile of the queries
__device__ __forceinline__ void bin_tile(int np, int nblk, long long *lo, long long *hi) {
  const long long per = ((long long)np + nblk - 1) / nblk;
  *lo = (long long)blockIdx.x * per;
  *hi = *lo + per < np ? *lo + per : np;
}

// pass 1: H[digit * nblk + block] = the block's count (gridDim.x == nblk)
__global__ __launch_bounds__(kBlock) void k_bin_hist(const double *xyz, const uint8_t *pclass, int np, const Frame *fr,
                                                     int *H, const DevStats *st) {
  if (!st->sorted) return;
  __shared__ int h[kBinDigits];
  for (int j = threadIdx.x; j < kBinDigits; j += kBlock) h[j] = 0;
  __syncthreads();
  long long lo, hi;
  bin_tile(np, gridDim.x, &lo, &hi);
  for (long long i = lo + threadIdx.x; i < hi; i += kBlock) {
    int f;
    double x[3];
    const int d = bin_key(xyz, pclass, i, fr, &f, x);
    if (d >= 0) atomicAdd(&h[d], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < kBinDigits; j += kBlock) H[(size_t)j * gridDim.x + blockIdx.x] = h[j];
}

// pass 1: O = exclusive scan of H; the block's queries of digit d go to
// [O[d * nblk + b], ...): {id, fine} and the coordinates
__global__ __launch_bounds__(kBlock) void k_bin_place(const double *xyz, const uint8_t *pclass, int np,
                                                      const Frame *fr, const int *O, int2 *key1, double *xs1,
                                                      const DevStats *st) {
  if (!st->sorted) return;
  __shared__ int cur[kBinDigits];
  for (int j = threadIdx.x; j < kBinDigits; j += kBlock) cur[j] = O[(size_t)j * gridDim.x + blockIdx.x];
  __syncthreads();
  long long lo, hi;
  bin_tile(np, gridDim.x, &lo, &hi);
  for (long long i = lo + threadIdx.x; i < hi; i += kBlock) {
    int f;
    double x[3];
    const int d = bin_key(xyz, pclass, i, fr, &f, x);
    if (d < 0) continue;
    const int p = atomicAdd(&cur[d], 1);
    key1[p] = make_int2((int)(i + 1), f);
    xs1[3 * (size_t)p] = x[0];
    xs1[3 * (size_t)p + 1] = x[1];
    xs1[3 * (size_t)p + 2] = x[2];
  }
}

// pass 2 works on chunks of at most kBinChunk queries that never straddle a
// digit: digit d's n_d queries form ceil(n_d / kBinChunk) chunks, chunk ids
// in digit order (cbase[d] = chunks before digit d, cbase[kBinDigits] = all)
__global__ __launch_bounds__(kBlock) void k_bin_chunks(const int *O, int nblk, int *cbase, const DevStats *st) {
  if (!st->sorted) return;
  constexpr int R = kBinDigits / kBlock;
  int n[R], s = 0;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int d = R * threadIdx.x + q;
    const int cnt = O[(size_t)(d + 1) * nblk] - O[(size_t)d * nblk];
    n[q] = (cnt + kBinChunk - 1) / kBinChunk;
    s += n[q];
  }
  int tot;
  int pre = block_excl_scan(s, &tot);
#pragma unroll
  for (int q = 0; q < R; q++) {
    cbase[R * threadIdx.x + q] = pre;
    pre += n[q];
  }
  if (threadIdx.x == 0) cbase[kBinDigits] = tot;
}

// chunk b of pass 2 (b < cbase[kBinDigits]): its digit d (binary search),
// its index j inside the digit, the digit's chunk count and the queries
// [q0, q1) of key1 / xs1
struct BinChunk {
  int d, j, nch, q0, q1;
};
__device__ __forceinline__ bool bin_chunk(const int *O, int nblk, const int *cbase, int b, BinChunk *c) {
  if (b >= cbase[kBinDigits]) return false;
  int lo = 0, hi = kBinDigits; // cbase[lo] <= b < cbase[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cbase[mid] <= b) lo = mid;
    else hi = mid;
  }
  c->d = lo;
  c->j = b - cbase[lo];
  c->nch = cbase[lo + 1] - cbase[lo];
  const int b0 = O[(size_t)lo * nblk], b1 = O[(size_t)(lo + 1) * nblk];
  c->q0 = b0 + c->j * kBinChunk;
  c->q1 = c->q0 + kBinChunk < b1 ? c->q0 + kBinChunk : b1;
  return true;
}
// entry (d, fine f, chunk j) of the pass-2 count matrix, ordered digit,
// fine key, chunk: its exclusive scan is the final position of the first
// query of chunk j with key (d, f)
__device__ __forceinline__ size_t bin_m_index(const int *cbase, const BinChunk &c, int f) {
  return (size_t)cbase[c.d] * kBinFine + (size_t)f * c.nch + c.j;
}

// pass 2: per chunk, the LDS histogram of its fine keys into the matrix
// (grid: an upper bound of the chunk count; chunks past the real count exit)
__global__ __launch_bounds__(kBlock) void k_bin_fine_hist(const int *O, int nblk, const int *cbase, const int2 *key1,
                                                          int *M, const DevStats *st) {
  if (!st->sorted) return;
  BinChunk c;
  if (!bin_chunk(O, nblk, cbase, blockIdx.x, &c)) return;
  __shared__ int h[kBinFine];
  for (int f = threadIdx.x; f < kBinFine; f += kBlock) h[f] = 0;
  __syncthreads();
  for (int q = c.q0 + threadIdx.x; q < c.q1; q += kBlock) atomicAdd(&h[key1[q].y], 1);
  __syncthreads();
  for (int f = threadIdx.x; f < kBinFine; f += kBlock) M[bin_m_index(cbase, c, f)] = h[f];
}

// pass 2: after the scan of M, every chunk places its queries at their final
// positions: the order lists and, for volume queries, the coordinates in
// processing order (the walk then loads its queries coalesced)
__global__ __launch_bounds__(kBlock) void k_bin_fine_place(const int *O, int nblk, const int *cbase, const int2 *key1,
                                                           const double *xs1, const int *Ms, int *order_v, double *qs,
                                                           int *order_b, DevStats *st) {
  if (!st->sorted) return;
  const int nvol = O[(size_t)kBinCoarse * nblk];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->nvol = nvol;
    st->nbdy = O[(size_t)kBinDigits * nblk] - nvol;
  }
  BinChunk c;
  if (!bin_chunk(O, nblk, cbase, blockIdx.x, &c)) return;
  __shared__ int cur[kBinFine];
  for (int f = threadIdx.x; f < kBinFine; f += kBlock) cur[f] = Ms[bin_m_index(cbase, c, f)];
  __syncthreads();
  for (int q = c.q0 + threadIdx.x; q < c.q1; q += kBlock) {
    const int2 kv = key1[q];
    const int pos = atomicAdd(&cur[kv.y], 1);
    if (c.d < kBinCoarse) {
      order_v[pos] = kv.x;
      qs[3 * (size_t)pos] = xs1[3 * (size_t)q];
      qs[3 * (size_t)pos + 1] = xs1[3 * (size_t)q + 1];
      qs[3 * (size_t)pos + 2] = xs1[3 * (size_t)q + 2];
    } else {
      order_b[pos - nvol] = kv.x;
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
                                                      const DevStats *st) {
  if (st->sorted) return;
  const long long i0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kScanItems;
  int tot;
  block_excl_scan(__popc(cls_bits(pclass, np, i0, cls)), &tot);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_cls_scatter(const uint8_t *pclass, long long np, int cls,
                                                        const int *boff, int *out, const DevStats *st) {
  if (st->sorted) return;
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

} // namespace pmmg
