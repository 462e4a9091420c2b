// pmmg_hip.hip — MI355X (gfx950) old->new mesh transfer: locate every new
// vertex in the background mesh and interpolate metric + fields (fp64).
//
// Replaces, behind the C-ABI of include/parmmg_hip.h, the per-group body of
// PMMG_interpMetricsAndFields (reference src/interpmesh_pmmg.c:477-741):
//   PMMG_locatePointVol      src/locate_pmmg.c:786-883   -> step_vol / k_vol_walk, k_vol_fused
//   PMMG_interp4bar_*        src/interpmesh_pmmg.c:206-270 -> k_vol_interp<slot layout>
//   PMMG_locatePointBdy      src/locate_pmmg.c:587-723   -> k_bdy (locate + interpolate)
//   exhaustive / closest     src/locate_pmmg.c:477-515, 737-770 -> k_*_exhaust*, k_*_finish
// Device arithmetic lives in pmmg_device.hpp.
//
// Pipeline of one pmmg_hip_locate_interp (all on the context stream):
//   1. bbox of the background (ordered-integer atomics)           k_bbox
//   2. volume seed grid: per cell, the sampled tetra whose first
//      vertex is closest to the cell centre (64-bit atomicMin:
//      deterministic); surface seed grid: tria centroids           k_seed_vol, k_seed_srf
//   3. query order: Morton binning of the queries per class
//      (count / exclusive scan / scatter), or, when the input order
//      is already spatially coherent, a stable class compaction     k_bin_*, k_cls_*
//   4. volume: lean walk kernel writing the located tetra per query,
//      then an interpolation kernel specialised on the slot layout
//      so that every row gather is issued before any math           k_vol_walk, k_vol_interp
//   5. surface: tria walk + wedge/cone + interpolation              k_bdy
//   6. queries whose walk got stuck / ran too long: brute-force
//      scans with the reference's exhaustive semantics              k_*_exhaust*, k_*_finish
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "pmmg_device.hpp"
#include "pmmg_snapshot.hpp"
#include "pmmg_quality.hpp"

using namespace pmmg;

namespace {

// ---------------------------------------------------------------- prepare

// one launch initialises the per-call state: frame accumulators, stats,
// seed grids, bin counters
__global__ __launch_bounds__(kBlock) void k_reset(Frame *fr, DevStats *st, unsigned long long *grid, long long ng,
                                                  int *sgrid, long long nsg, int *cnt, long long ncnt, int keep_coherent) {
  const long long tid = blockIdx.x * (long long)blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  if (tid == 0) {
    for (int d = 0; d < 3; d++) {
      fr->key_lo[d] = ~0ULL;
      fr->key_hi[d] = 0ULL;
    }
    int coh = st->coherent;
    unsigned int *w = reinterpret_cast<unsigned int *>(st);
    for (size_t j = 0; j < sizeof(DevStats) / 4; j++) w[j] = 0u;
    if (keep_coherent) st->coherent = coh;
  }
  {
    unsigned long long *pw = reinterpret_cast<unsigned long long *>(st + 1);
    for (long long j = tid; j < (long long)(kStatParts * sizeof(StatPart) / 8); j += nth) pw[j] = 0ULL;
  }
  for (long long j = tid; j < ng; j += nth) grid[j] = ~0ULL;
  for (long long j = tid; j < nsg; j += nth) sgrid[j] = INT_MAX;
  for (long long j = tid; j < ncnt; j += nth) cnt[j] = 0;
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
    for (int d = 0; d < 3; d++) { slo[d][w] = lo[d]; shi[d][w] = hi[d]; }
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

__global__ void k_frame_final(Frame *fr, int g, int gs, int gb, int seed8) {
  fr->seed8 = seed8;
  for (int d = 0; d < 3; d++) {
    double lo = dunkey(fr->key_lo[d]), hi = dunkey(fr->key_hi[d]);
    double ext = hi - lo;
    fr->lo[d] = lo;
    fr->ext[d] = ext;
    fr->inv_vol[d] = ext > 0.0 ? (double)g / ext : 0.0;
    fr->inv_srf[d] = ext > 0.0 ? (double)gs / ext : 0.0;
    fr->inv_bin[d] = ext > 0.0 ? (double)gb / ext : 0.0;
  }
}

// volume seeds: per cell, the sampled tetra whose centroid is closest to
// the cell centre; key = (float(dist^2) bits << 32) | id -> deterministic min
// Samples are taken in runs of R consecutive tetra (R = 4: one 128-byte line
// of packed tetra records), nsamp / R runs evenly spaced over the tetra: the
// sampling cost is the lines it reads, and 4 samples per line quadruple the
// samples for the same traffic.  Lanes of a run that land in the same cell
// combine their keys first (one atomic per cell and run).
__global__ __launch_bounds__(kBlock) void k_seed_vol(Bg bg, const Frame *fr, unsigned long long *cell, int g,
                                                     long long nsamp, int mode, int R, int atom) {
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
    // run start aligned to a 4-tetra boundary (a cache line of tet8 records)
    const long long base = 4 * ((run * quads) / (nruns > 0 ? nruns : 1));
    const int k = (int)(1 + base + r);
    bool ok = s < hi && k <= bg.ne;
    int4 tv = make_int4(0, 0, 0, 0);
    if (ok) {
      // sampled records stream through once: non-temporal
      const nti4 r = __builtin_nontemporal_load(reinterpret_cast<const nti4 *>(bg.tetv + (size_t)(k - 1) * bg.tstride));
      tv = make_int4(r.x, r.y, r.z, r.w);
      ok = tv.x > 0;
    }
    unsigned long long key = ~0ULL;
    long long ci = -1;
    if (ok) {
      // representative point of the tetra: centroid (mode 0), midpoint of
      // the edge v0-v3 (1), first vertex (2); a cell's seed is the sampled
      // tetra whose point is closest to the cell centre
      double p[3];
      load_pt(bg.xyz, tv.x, p);
      if (mode == 0) {
        double a[3], b[3], e[3];
        load_pt(bg.xyz, tv.y, a);
        load_pt(bg.xyz, tv.z, b);
        load_pt(bg.xyz, tv.w, e);
        for (int d = 0; d < 3; d++) p[d] = 0.25 * (p[d] + a[d] + b[d] + e[d]);
      } else if (mode == 1) {
        double e[3];
        load_pt(bg.xyz, tv.w, e);
        for (int d = 0; d < 3; d++) p[d] = 0.5 * (p[d] + e[d]);
      }
      int c[3];
      if (fr->seed8) {
        // seed8 key: {8-bit distance^2 to the cell centre (cell units),
        // 9-bit centroid offset per axis, 29-bit id}: the cell's minimum is
        // also what the queries decode (no pass after the sampling)
        unsigned long long off = 0;
        float d2 = 0.f;
        for (int d = 0; d < 3; d++) {
          c[d] = cell_coord(p[d], fr->lo[d], fr->inv_vol[d], g);
          float f = (float)((p[d] - fr->lo[d]) * fr->inv_vol[d] - c[d]);
          f = f < 0.f ? 0.f : (f > 0.999f ? 0.999f : f);
          off |= (unsigned long long)(unsigned)(f * 512.f) << (9 * d);
          d2 += (f - 0.5f) * (f - 0.5f);
        }
        const unsigned q8 = d2 * 340.f < 255.f ? (unsigned)(d2 * 340.f) : 255u;
        key = ((unsigned long long)q8 << 56) | (off << 29) | (unsigned)k;
      } else {
        float d2 = 0.f;
        for (int d = 0; d < 3; d++) {
          c[d] = cell_coord(p[d], fr->lo[d], fr->inv_vol[d], g);
          double ctr = fr->lo[d] + (c[d] + 0.5) / (fr->inv_vol[d] > 0.0 ? fr->inv_vol[d] : 1.0);
          float dd = (float)(p[d] - ctr);
          d2 += dd * dd;
        }
        key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)k;
      }
      ci = c[0] + (long long)g * (c[1] + (long long)g * c[2]);
    }
    // combine within the run (R lanes, R divides 64): the first lane of each
    // distinct cell issues the atomic with the run's minimum for that cell
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
    if (leader) {
      if (atom) atomicMin(&cell[ci], best);
      else cell[ci] = best; // timing experiment only (racy)
    }
  }
}

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

// rare path of seed_vol (empty cell): lowest seed id in the shells of
// radius 1 then 2 around the cell; kept out of line so the walk kernels do
// not carry its registers
constexpr unsigned long long kSeedIdMask = (1ULL << 29) - 1; // seed8 keys: ids below 2^29 (the adja encoding's limit)

__device__ __forceinline__ int seed_vol_ring(const unsigned long long *cell, int g, int ci, int cj, int ck,
                                             unsigned long long idmask) {
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
          unsigned long long id = v & idmask;
          if (v != ~0ULL && id < best) best = id;
        }
    if (best != ~0ULL) return (int)best;
  }
  return 1;
}

__device__ __forceinline__ int seed_vol(const unsigned long long *cell, int g, const Frame *fr, const double *x) {
  if (!fr->seed8) {
    int ci = cell_coord(x[0], fr->lo[0], fr->inv_vol[0], g);
    int cj = cell_coord(x[1], fr->lo[1], fr->inv_vol[1], g);
    int ck = cell_coord(x[2], fr->lo[2], fr->inv_vol[2], g);
    unsigned long long s = cell[ci + (size_t)g * (cj + (size_t)g * ck)];
    if (s != ~0ULL) return (int)(unsigned)(s & 0xFFFFFFFFULL);
    return seed_vol_ring(cell, g, ci, cj, ck, 0xFFFFFFFFULL);
  }
  // the query's position in cell units; candidate cells: its own and the 7
  // neighbours of the octant it lies in; the seed whose (quantised) centroid
  // is nearest wins (ties: lower id)
  double t[3];
  int c[3], o[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    t[d] = (x[d] - fr->lo[d]) * fr->inv_vol[d];
    c[d] = cell_coord(x[d], fr->lo[d], fr->inv_vol[d], g);
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
    if (d2 < best || (d2 == best && id < bid)) { best = d2; bid = id; }
  }
  if (bid != 0xFFFFFFFFu) return (int)bid;
  return seed_vol_ring(cell, g, c[0], c[1], c[2], kSeedIdMask);
}

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
  return 1;
}

// ---------------------------------------------------------------- query order

// Is the input numbering spatially coherent?  Distances between consecutive
// points at 4096 pseudo-random positions against the mean spacing h of np points
// in the bbox of the sample: coherent when at least half of them are below
// 4h (a median test: the jumps at the ends of lattice rows or of Mmg's local
// numbering runs, which an evenly strided sample can hit in a fixed fraction
// of its positions, do not count; a shuffled numbering has almost every
// distance at the scale of the bbox).  Self-contained so it can run first and
// be read back early.
__global__ __launch_bounds__(kBlock) void k_coherence(const double *xyz, int np, DevStats *st) {
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
  for (int d = 0; d < 3; d++) { slo[d][threadIdx.x] = lo[d]; shi[d][threadIdx.x] = hi[d]; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L[3] = {1e300, 1e300, 1e300}, H[3] = {-1e300, -1e300, -1e300};
    for (int j = 0; j < kBlock; j++)
      for (int d = 0; d < 3; d++) { L[d] = fmin(L[d], slo[d][j]); H[d] = fmax(H[d], shi[d][j]); }
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
    st->coherent = (np > 1 && 2 * tot >= nsamp) ? 1 : 0;
  }
}

// Morton binning: bin = (class, Morton code of the gb^3 cell); rank inside the
// bin from the counter (order inside a bin is irrelevant: each query's result
// is a pure function of the query)
__global__ __launch_bounds__(kBlock) void k_bin_count(const double *xyz, const uint8_t *pclass, int np, const Frame *fr,
                                                      int gb, int nbins, int *cnt, int2 *binrank) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  int c = pclass[i];
  if (c != PMMG_PT_VOL && c != PMMG_PT_BDY) {
    binrank[i] = make_int2(-1, 0);
    return;
  }
  uint32_t q[3];
  for (int d = 0; d < 3; d++) q[d] = (uint32_t)cell_coord(xyz[3 * (size_t)i + d], fr->lo[d], fr->inv_bin[d], gb);
  int bin = (int)((expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2])) + (c == PMMG_PT_BDY ? nbins : 0);
  int r = atomicAdd(&cnt[bin], 1);
  binrank[i] = make_int2(bin, r);
}

__global__ __launch_bounds__(kBlock) void k_bin_scatter(int np, const int2 *binrank, const int *off, int nbins,
                                                        int *order_v, int *order_b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  int2 br = binrank[i];
  if (br.x < 0) return;
  if (br.x < nbins) order_v[off[br.x] + br.y] = i + 1;
  else order_b[off[br.x] - off[nbins] + br.y] = i + 1;
}

__global__ void k_bin_total(const int *off, const int *cnt, int nbins, DevStats *st) {
  st->nvol = off[nbins];
  st->nbdy = off[2 * nbins - 1] + cnt[2 * nbins - 1] - off[nbins];
}


// Stable class compaction (the surface list): out = the ids ip (1-based) with
// pclass[ip-1] == cls, in input order; *count = their number.  Three passes
// over the 1-byte classes (count per block, scan of the block counts,
// scatter): ~3 reads of np bytes, no global atomics.  Each block owns
// kClsChunk consecutive points, kClsItems per thread.
constexpr int kClsItems = 16, kClsChunk = kBlock * kClsItems;

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// exclusive scan of one int per thread over the block; returns the prefix
// and the block total in *tot
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

// bit j = (pclass[i0 + j] == cls); the 16 classes of a thread come in one
// 16-byte load when the array is 16-byte aligned and the run is complete
// (byte loads cost 16 instructions per wave and ran at ~130 GB/s)
__device__ __forceinline__ unsigned cls_bits(const uint8_t *pclass, long long np, long long i0, int cls) {
  unsigned m = 0;
  if (i0 + kClsItems <= np && ((uintptr_t)pclass & 15) == 0) {
    const uint4 w = *reinterpret_cast<const uint4 *>(pclass + i0);
    const unsigned words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < kClsItems; j++) m |= (((words[j >> 2] >> (8 * (j & 3))) & 0xFFu) == (unsigned)cls) ? (1u << j) : 0u;
    return m;
  }
#pragma unroll
  for (int j = 0; j < kClsItems; j++) {
    const long long i = i0 + j;
    m |= (i < np && pclass[i] == cls) ? (1u << j) : 0u;
  }
  return m;
}

__global__ __launch_bounds__(kBlock) void k_cls_count(const uint8_t *pclass, long long np, int cls, int *bcnt) {
  const long long i0 = (long long)blockIdx.x * kClsChunk + (long long)threadIdx.x * kClsItems;
  int tot;
  block_excl_scan(__popc(cls_bits(pclass, np, i0, cls)), &tot);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

// one block: bcnt[0..nb) -> exclusive offsets in place, total -> *count
__global__ __launch_bounds__(kBlock) void k_cls_scan(int *bcnt, int nb, int *count) {
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += kBlock) {
    const int b = b0 + threadIdx.x;
    const int v = b < nb ? bcnt[b] : 0;
    int tot;
    const int pre = block_excl_scan(v, &tot);
    if (b < nb) bcnt[b] = carry + pre;
    carry += tot;
  }
  if (threadIdx.x == 0) *count = carry;
}

__global__ __launch_bounds__(kBlock) void k_cls_scatter(const uint8_t *pclass, long long np, int cls,
                                                        const int *boff, int *out) {
  const long long i0 = (long long)blockIdx.x * kClsChunk + (long long)threadIdx.x * kClsItems;
  unsigned m = cls_bits(pclass, np, i0, cls);
  int tot;
  int pos = boff[blockIdx.x] + block_excl_scan(__popc(m), &tot);
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    out[pos++] = (int)(i0 + j + 1);
  }
}

// ---------------------------------------------------------------- stats

struct BlockStats {
  unsigned int cnt[16];
  unsigned long long steps;
  unsigned int stepmax;
};

__device__ __forceinline__ void bstats_init(BlockStats *b) {
  if (threadIdx.x < 16) b->cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) { b->steps = 0; b->stepmax = 0; }
}

__device__ __forceinline__ void bstats_flush(BlockStats *b, DevStats *st) {
  StatPart *pt = stat_part(st);
  if (threadIdx.x < 16 && b->cnt[threadIdx.x]) atomicAdd(&pt->cnt[threadIdx.x], (unsigned long long)b->cnt[threadIdx.x]);
  if (threadIdx.x == 0) {
    if (b->steps) atomicAdd(&pt->steps, b->steps);
    if (b->stepmax) atomicMax(&pt->stepmax, (unsigned long long)b->stepmax);
  }
}

// per-wave aggregation of the walk statistics (one LDS atomic per wave and counter)
__device__ __forceinline__ void wave_stats(BlockStats *bs, bool active, int hit, int steps) {
  unsigned int s = active ? (unsigned)steps : 0u, mx = s;
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_down(s, off);
    unsigned o = __shfl_down(mx, off);
    mx = o > mx ? o : mx;
  }
  if (__lane_id() == 0) {
    if (s) atomicAdd(&bs->steps, (unsigned long long)s);
    atomicMax(&bs->stepmax, mx);
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

// per-wave sum of a counter into a BlockStats slot
__device__ __forceinline__ void wave_count(BlockStats *bs, int slot, int v) {
  unsigned int s = (unsigned)v;
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
  if (__lane_id() == 0 && s) atomicAdd(&bs->cnt[slot], s);
}

// ---------------------------------------------------------------- volume

// PMMG_locatePointVol (locate_pmmg.c:786-883) from a grid seed instead of the
// previous point's tetra; visited set = the last kHist tetra.  vloc[i] = the
// accepting tetra, or 0 when the walk got stuck / exceeded maxstep (the query
// then goes to the exhaustive kernels).
//
// One exact division per step.  The reference accepts tetra k iff
// min_f bary[f] > -MMG5_EPS with bary[f] = -s[f]/vol (s = tet_dots).  IEEE
// division is sign-symmetric and monotone, so for vol > 0
//   min_f fl(-s[f]/vol) = -fl(max_f s[f] / vol)
// (for vol < 0 with min_f s[f]): the acceptance decision is bit-identical to
// the reference's while only one of its four divisions is evaluated.  The
// face to step through is the reference's first sorted coordinate whose
// neighbour exists and is unvisited, i.e. the eligible face of smallest
// bary = largest sign(vol)*s (ties: lowest face index); quotients that round
// to equal values may order differently than the reference's qsort, which
// changes only the path of the walk, never which tetra accept (parity
// classes of tests/parity.py).  Degenerate tetra (vol == 0) take the
// reference's four divisions and ranking.
//
// Vertices are reloaded at every step (3 of the 4 rows are L1 hits: the
// shared face) instead of carried over and permuted in registers: fewer live
// registers, so more waves per SIMD hide the dependent gathers.
__device__ __forceinline__ void pick_pt(int id, const int4 &tv, const double (*p)[3], double *out) {
  const int j = id == tv.x ? 0 : (id == tv.y ? 1 : (id == tv.z ? 2 : 3));
#pragma unroll
  for (int d = 0; d < 3; d++) out[d] = j == 0 ? p[0][d] : (j == 1 ? p[1][d] : (j == 2 ? p[2][d] : p[3][d]));
}

__device__ __forceinline__ void load_tet_pts(const Bg &bg, const int4 &tv, double (*p)[3]) {
  load_pt(bg.xyz, tv.x, p[0]);
  load_pt(bg.xyz, tv.y, p[1]);
  load_pt(bg.xyz, tv.z, p[2]);
  load_pt(bg.xyz, tv.w, p[3]);
}

// One step of the walk at tetra k: the reference's acceptance test (exact,
// one division, see above) and, when it fails, the face to leave through.
// Returns 1 inside, 0 moved (k = neighbour, hist updated), 2 stuck.
// On acceptance, loc (when given) receives the tetra's vertex ids and the
// reference's barycentric coordinates -s[f]/vol (PMMG_barycoord3d_compute,
// PMMG_barycoord_get: unsorted), bit-identical to tet_bary.
struct VolLoc {
  int4 v;
  double phi[4];
};

// vrec: the walk's result per query, read back once by the interpolation.
// Stored as three arrays (vertex ids int4, phi0..1, phi2..3) so that a
// wave-instruction writes / reads 1 KiB contiguously (whole cache lines);
// non-temporal: streamed once each way.
struct VRec {
  nti4 *v;
  ntd2 *a, *b;
};
__host__ __device__ inline VRec vrec_arrays(void *base, size_t nq) {
  VRec r;
  r.v = reinterpret_cast<nti4 *>(base);
  r.a = reinterpret_cast<ntd2 *>(r.v + nq);
  r.b = r.a + nq;
  return r;
}
__device__ __forceinline__ void vrec_store(const VRec &r, size_t i, const VolLoc &l) {
  const nti4 v = {l.v.x, l.v.y, l.v.z, l.v.w};
  const ntd2 a = {l.phi[0], l.phi[1]}, b = {l.phi[2], l.phi[3]};
  __builtin_nontemporal_store(v, r.v + i);
  __builtin_nontemporal_store(a, r.a + i);
  __builtin_nontemporal_store(b, r.b + i);
}
__device__ __forceinline__ VolLoc vrec_load(const VRec &r, size_t i) {
  VolLoc l;
  const nti4 v = __builtin_nontemporal_load(r.v + i);
  const ntd2 a = __builtin_nontemporal_load(r.a + i), b = __builtin_nontemporal_load(r.b + i);
  l.v = make_int4(v.x, v.y, v.z, v.w);
  l.phi[0] = a.x; l.phi[1] = a.y; l.phi[2] = b.x; l.phi[3] = b.y;
  return l;
}

__device__ __forceinline__ int step_vol(const Bg &bg, const double *x, int &k, int *hist, VolLoc *loc = nullptr) {
  const int4 tv = tetv_row(bg, k);
  const int4 ad = adja_row(bg, k);
  double p[4][3];
  load_tet_pts(bg, tv, p);
  double s[4];
  const double vol = tet_dots(x, p[0], p[1], p[2], p[3], s);
  double key[4]; // larger = more negative barycentric coordinate
  bool inside;
  if (vol > 0.0 || vol < 0.0) {
    double sm;
    if (vol > 0.0) {
      sm = s[0];
      sm = s[1] > sm ? s[1] : sm;
      sm = s[2] > sm ? s[2] : sm;
      sm = s[3] > sm ? s[3] : sm;
    } else {
      sm = s[0];
      sm = s[1] < sm ? s[1] : sm;
      sm = s[2] < sm ? s[2] : sm;
      sm = s[3] < sm ? s[3] : sm;
    }
    inside = -(sm / vol) > -kEps;
#pragma unroll
    for (int f = 0; f < 4; f++) key[f] = vol > 0.0 ? s[f] : -s[f];
  } else {
    double b[4];
#pragma unroll
    for (int f = 0; f < 4; f++) b[f] = -s[f] / vol;
    inside = min4(b) > -kEps;
    int r[4];
    ranks4(b, r);
#pragma unroll
    for (int f = 0; f < 4; f++) key[f] = (double)(3 - r[f]);
  }
  if (inside) {
    if (loc) {
      loc->v = tv;
#pragma unroll
      for (int f = 0; f < 4; f++) loc->phi[f] = -s[f] / vol;
    }
    return 1;
  }
  int f = -1;
  double best = 0.0;
#pragma unroll
  for (int ff = 0; ff < 4; ff++) {
    const int iel = sel4(ad, ff) >> 2;
    bool vis = false;
#pragma unroll
    for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
    if (iel != 0 && !vis && (f < 0 || key[ff] > best)) { f = ff; best = key[ff]; }
  }
  if (f < 0) return 2;
#pragma unroll
  for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
  hist[0] = k;
  k = sel4(ad, f) >> 2;
  return 0;
}

// the walk of one query; returns 1 found (k, tv = its vertices), 2 stuck,
// 3 over-long
__device__ __forceinline__ int walk_vol(const Bg &bg, const unsigned long long *grid, int g, const Frame *fr,
                                        const double *x, int maxstep, int &k, int4 &tv, int &steps) {
  k = seed_vol(grid, g, fr, x);
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  for (;;) {
    ++steps;
    const int r = step_vol(bg, x, k, hist);
    if (r == 1) {
      tv = tetv_row(bg, k);
      return 1;
    }
    if (r == 2) return 2;
    if (steps >= maxstep) return 3;
  }
}

// Volume walks (default pipeline: k_vol_walk [+ k_vol_walk_cont], then
// k_vol_interp).
//
// One query per lane, the 64 lanes of a wave on 64 consecutive queries of
// the processing order: neighbouring walks run in lockstep through the same
// tetra, so their tetra records and vertex rows share cache lines inside
// each wave-instruction (flattened per-lane chains that desynchronise the
// lanes, and walks carrying the shared face's vertices in registers, both
// measured slower).  vloc[i] = accepting tetra, 0 = stuck / over-long (the
// query then goes to the exhaustive kernels).
//
// A wave runs as long as its longest walk, so the first pass caps walks at
// `cap` steps (mean ~4 with the seed grid): walks still going are compacted
// into a continuation list {position, current tetra} and finished by
// k_vol_walk_cont with full waves.  This removes most of the idle-lane
// iterations (without the cap ~75% of the lane-iterations of a wave were
// idle, waiting for its slowest walk).

// walk from tetra k for at most `limit` more steps: 1 found (k), 2 stuck,
// 3 limit reached (k = current tetra)
__device__ __forceinline__ int walk_core(const Bg &bg, const double *x, int &k, int &steps, int limit,
                                         VolLoc *loc = nullptr) {
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  for (int n = 0;; n++) {
    if (n >= limit) return 3;
    ++steps;
    const int r = step_vol(bg, x, k, hist, loc);
    if (r == 1) return 1;
    if (r == 2) return 2;
  }
}

// Walk that carries the 3 vertices of the crossed face in registers: a step
// gathers the next tetra's record and only its opposite vertex (4 cache-line
// lookups per step instead of 10: the texture path, ~2 cycles per distinct
// line per wave-instruction, bounds the walk).  The carried vertices are
// permuted into the new tetra's local order (the reference's arithmetic
// order) with mask blends: a select chain over a register array is lowered
// to scratch-memory indexing.

__device__ __forceinline__ int walk_core_carry(const Bg &bg, const double *x, int &k, int &steps, int limit,
                                               VolLoc *loc) {
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  int4 tv = tetv_row(bg, k), ad = adja_row(bg, k);
  double p[4][3];
  load_tet_pts(bg, tv, p);
  for (int n = 0;; n++) {
    if (n >= limit) return 3;
    ++steps;
    double s[4];
    const double vol = tet_dots(x, p[0], p[1], p[2], p[3], s);
    double key[4];
    bool inside;
    if (vol > 0.0 || vol < 0.0) {
      double sm;
      if (vol > 0.0) {
        sm = s[0];
        sm = s[1] > sm ? s[1] : sm;
        sm = s[2] > sm ? s[2] : sm;
        sm = s[3] > sm ? s[3] : sm;
      } else {
        sm = s[0];
        sm = s[1] < sm ? s[1] : sm;
        sm = s[2] < sm ? s[2] : sm;
        sm = s[3] < sm ? s[3] : sm;
      }
      inside = -(sm / vol) > -kEps;
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = vol > 0.0 ? s[f] : -s[f];
    } else {
      double b[4];
#pragma unroll
      for (int f = 0; f < 4; f++) b[f] = -s[f] / vol;
      inside = min4(b) > -kEps;
      int r[4];
      ranks4(b, r);
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = (double)(3 - r[f]);
    }
    if (inside) {
      loc->v = tv;
#pragma unroll
      for (int f = 0; f < 4; f++) loc->phi[f] = -s[f] / vol;
      return 1;
    }
    int f = -1;
    double best = 0.0;
#pragma unroll
    for (int ff = 0; ff < 4; ff++) {
      const int iel = sel4(ad, ff) >> 2;
      bool vis = false;
#pragma unroll
      for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
      if (iel != 0 && !vis && (f < 0 || key[ff] > best)) { f = ff; best = key[ff]; }
    }
    if (f < 0) return 2;
#pragma unroll
    for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
    hist[0] = k;
    const int code = sel4(ad, f);
    k = code >> 2;
    const int iopp = code & 3;
    const int4 tn = tetv_row(bg, k);
    ad = adja_row(bg, k);
    double pn[3];
    load_pt(bg.xyz, sel4(tn, iopp), pn);
    double q[4][3];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      const int id = sel4(tn, l);
      const bool e1 = id == tv.y, e2 = id == tv.z, e3 = id == tv.w, en = l == iopp;
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const double c = e1 ? p[1][d] : (e2 ? p[2][d] : (e3 ? p[3][d] : p[0][d]));
        q[l][d] = en ? pn[d] : c;
      }
    }
#pragma unroll
    for (int l = 0; l < 4; l++)
#pragma unroll
      for (int d = 0; d < 3; d++) p[l][d] = q[l][d];
    tv = tn;
  }
}

// Walk with the tetra's vertex coordinates kept in LDS "slots" (per lane 4
// slots x 3 doubles, lane-interleaved: conflict-free).  A step writes only
// the new vertex into the slot of the vertex left behind and reads the four
// slots back in the new tetra's local order (m = local -> slot), so the
// reference's arithmetic order costs 12 LDS reads instead of ~100 register
// selects, and no register copy of the previous tetra's points stays live.
__device__ __forceinline__ int idx_in(int id, const int4 &t) {
  return (id == t.y ? 1 : 0) + (id == t.z ? 2 : 0) + (id == t.w ? 3 : 0);
}

struct LaneSlots { // this lane's view of the wave's slot image [slot][dim][64]
  double *base;
  __device__ __forceinline__ void put(int slot, const double *p) const {
#pragma unroll
    for (int d = 0; d < 3; d++) base[(slot * 3 + d) * 64] = p[d];
  }
  __device__ __forceinline__ void get(int slot, double *p) const {
#pragma unroll
    for (int d = 0; d < 3; d++) p[d] = base[(slot * 3 + d) * 64];
  }
};

__device__ __forceinline__ int walk_core_lds(const Bg &bg, const double *x, int &k, int &steps, int limit,
                                             VolLoc *loc, const LaneSlots &L) {
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  int4 tv = tetv_row(bg, k), ad = adja_row(bg, k);
  {
    double p[4][3];
    load_tet_pts(bg, tv, p);
#pragma unroll
    for (int l = 0; l < 4; l++) L.put(l, p[l]);
  }
  int4 m = make_int4(0, 1, 2, 3); // slot of local vertex l
  for (int n = 0;; n++) {
    if (n >= limit) return 3;
    ++steps;
    double p[4][3];
    L.get(m.x, p[0]);
    L.get(m.y, p[1]);
    L.get(m.z, p[2]);
    L.get(m.w, p[3]);
    double s[4];
    const double vol = tet_dots(x, p[0], p[1], p[2], p[3], s);
    double key[4];
    bool inside;
    if (vol > 0.0 || vol < 0.0) {
      double sm;
      if (vol > 0.0) {
        sm = s[0];
        sm = s[1] > sm ? s[1] : sm;
        sm = s[2] > sm ? s[2] : sm;
        sm = s[3] > sm ? s[3] : sm;
      } else {
        sm = s[0];
        sm = s[1] < sm ? s[1] : sm;
        sm = s[2] < sm ? s[2] : sm;
        sm = s[3] < sm ? s[3] : sm;
      }
      inside = -(sm / vol) > -kEps;
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = vol > 0.0 ? s[f] : -s[f];
    } else { // degenerate: the reference's four divisions; any face order
      double b[4];
#pragma unroll
      for (int f = 0; f < 4; f++) b[f] = -s[f] / vol;
      inside = min4(b) > -kEps;
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = s[f];
    }
    if (inside) {
      loc->v = tv;
#pragma unroll
      for (int f = 0; f < 4; f++) loc->phi[f] = -s[f] / vol;
      return 1;
    }
    int f = -1;
    double best = 0.0;
#pragma unroll
    for (int ff = 0; ff < 4; ff++) {
      const int iel = sel4(ad, ff) >> 2;
      bool vis = false;
#pragma unroll
      for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
      if (iel != 0 && !vis && (f < 0 || key[ff] > best)) { f = ff; best = key[ff]; }
    }
    if (f < 0) return 2;
#pragma unroll
    for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
    hist[0] = k;
    const int code = sel4(ad, f);
    k = code >> 2;
    const int iopp = code & 3;
    const int4 tn = tetv_row(bg, k);
    ad = adja_row(bg, k);
    double pn[3];
    load_pt(bg.xyz, sel4(tn, iopp), pn);
    const int sf = sel4(m, f); // slot of the vertex left behind
    int4 mn; // branch-free (a ternary with a costly arm becomes a divergent branch)
    mn.x = (int)bsel((unsigned)sel4(m, idx_in(tn.x, tv)), (unsigned)sf, iopp == 0);
    mn.y = (int)bsel((unsigned)sel4(m, idx_in(tn.y, tv)), (unsigned)sf, iopp == 1);
    mn.z = (int)bsel((unsigned)sel4(m, idx_in(tn.z, tv)), (unsigned)sf, iopp == 2);
    mn.w = (int)bsel((unsigned)sel4(m, idx_in(tn.w, tv)), (unsigned)sf, iopp == 3);
    L.put(sf, pn);
    m = mn;
    tv = tn;
  }
}

struct ContEntry {
  int ip; // query
  int k;  // tetra the capped walk stopped at
};

// order == nullptr: the queries are taken in input order (i = ip - 1) and
// the volume points selected here (no compaction pass; the idle lanes of
// surface / skipped points cost little next to the walks).  Otherwise the
// queries are order[0 .. st->nvol).  vloc is indexed by ip - 1.
// CARRY selects walk_core_carry; MINW > 1 asks the compiler for that many
// waves per SIMD (register budget 512 / MINW).
template <int CARRY, int MINW, int B = kBlock>
__global__ __launch_bounds__(B, MINW) void k_vol_walk(Bg bg, const Frame *fr, const unsigned long long *grid,
                                                           int g, const double *qxyz, const uint8_t *pclass,
                                                           const int *order, int np, int *vloc, VRec vrec, int *fb,
                                                           ContEntry *cont, DevStats *st, int cap, int maxstep,
                                                           int i0) {
  __shared__ BlockStats bs;
  __shared__ double slot_img[CARRY == 2 ? B / 64 : 1][CARRY == 2 ? 12 * 64 : 1];
  const LaneSlots L{&slot_img[CARRY == 2 ? threadIdx.x >> 6 : 0][CARRY == 2 ? __lane_id() : 0]};
  bstats_init(&bs);
  __syncthreads();
  const int i = i0 + xcd_block() * blockDim.x + threadIdx.x;
  bool active;
  int ip = 0;
  if (order) {
    active = i < st->nvol;
    if (active) ip = order[i];
  } else {
    active = i < np && pclass[i] == PMMG_PT_VOL;
    ip = i + 1;
  }
  int status = 0, steps = 0, k = 0;
  if (active) {
    double x[3];
    load_pt_nt(qxyz, ip, x); // streamed once: non-temporal
    k = seed_vol(grid, g, fr, x);
    VolLoc loc;
    const int lim = cap < maxstep ? cap : maxstep;
    status = CARRY == 2   ? walk_core_lds(bg, x, k, steps, lim, &loc, L)
             : CARRY == 1 ? walk_core_carry(bg, x, k, steps, lim, &loc)
                          : walk_core(bg, x, k, steps, lim, &loc);
    if (status == 3 && steps < maxstep) status = 4; // -> continuation list
    __builtin_nontemporal_store(status == 1 ? k : 0, vloc + ip - 1);
    if (status == 1) vrec_store(vrec, ip - 1, loc);
  }
  const bool fail = active && (status == 2 || status == 3);
  const int slot = wave_append(&st->nfb_vol, fail);
  if (fail) fb[slot] = ip;
  const int cslot = wave_append(&st->ncont, active && status == 4);
  if (active && status == 4) cont[cslot] = ContEntry{ip, k};
  wave_stats(&bs, active, status == 1 ? PMMG_HIT_VOL_WALK : 0, steps);
  __syncthreads();
  bstats_flush(&bs, st);
}

// the capped walks, continued from where they stopped (fresh visited
// history; the step count continues)
__global__ __launch_bounds__(kBlock) void k_vol_walk_cont(Bg bg, const double *qxyz, int *vloc, VRec vrec, int *fb,
                                                          const ContEntry *cont, DevStats *st, int cap, int maxstep) {
  __shared__ BlockStats bs;
  bstats_init(&bs);
  __syncthreads();
  const XcdChunk ch = xcd_chunk(st->ncont);
  for (int it = 0; it < ch.iters; it++) {
    const long long j = ch.start + it * ch.stride;
    const bool active = j < ch.hi;
    int status = 0, steps = cap, ip = 0;
    if (active) {
      const ContEntry e = cont[j];
      ip = e.ip;
      double x[3];
      load_pt(qxyz, ip, x);
      int k = e.k;
      VolLoc loc;
      status = walk_core(bg, x, k, steps, maxstep - cap, &loc);
      vloc[ip - 1] = status == 1 ? k : 0;
      if (status == 1) vrec_store(vrec, ip - 1, loc);
    }
    const bool fail = active && status != 1;
    const int slot = wave_append(&st->nfb_vol, fail);
    if (fail) fb[slot] = ip;
    wave_stats(&bs, active, status == 1 ? PMMG_HIT_VOL_WALK : 0, active ? steps - cap : 0);
  }
  __syncthreads();
  bstats_flush(&bs, st);
}

// interpolation of located volume queries; the slot layout is a template
// (codes 1 / 3 / 6, 0 = none) so every row gather is unconditional and can be
// issued before any arithmetic; C0 < 0 selects the runtime-layout variant
template <int C0, int C1, int C2, int C3, int C4, int C5>
__device__ __forceinline__ void interp_vol_layout(const Slots &S, int ip, const int *v, const double *phi) {
  if constexpr (C0 < 0) {
    for (int s = 0; s < S.n; s++) interp_dyn<4>(S.s[s], ip, v, phi);
  } else {
    if constexpr (C0 > 0) interp_code<4, C0>(S.s[0], ip, v, phi);
    if constexpr (C1 > 0) interp_code<4, C1>(S.s[1], ip, v, phi);
    if constexpr (C2 > 0) interp_code<4, C2>(S.s[2], ip, v, phi);
    if constexpr (C3 > 0) interp_code<4, C3>(S.s[3], ip, v, phi);
    if constexpr (C4 > 0) interp_code<4, C4>(S.s[4], ip, v, phi);
    if constexpr (C5 > 0) interp_code<4, C5>(S.s[5], ip, v, phi);
  }
}

__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Output rows of one slot for the wave's 64 consecutive queries, written as
// whole cache lines: each lane puts its row into a wave-private LDS image,
// then lane l of store instruction t writes piece t*64+l of the image (16-byte
// pieces for 6-double rows, 8-byte pieces for 3-double rows: every piece
// inside one row), skipping the rows of `mask` bit 0 (other classes, failed
// walks, failed inversions: the reference leaves those rows untouched, and
// the surface kernel writes its own rows concurrently).  A lane storing its
// own 48-byte row with three 16-byte stores instead writes partial lines in
// every instruction; that cost ~1 ms of the 2 ms interpolation at cfg4.
template <int C>
__device__ __forceinline__ void wave_store_rows(double *out, const double *row, unsigned long long mask,
                                                double *img) {
  const int lane = __lane_id();
  if constexpr (C == 1) {
    if ((mask >> lane) & 1ULL) nt_store(out + lane, row[0]);
  } else {
#pragma unroll
    for (int j = 0; j < C; j++) img[C * lane + j] = row[j];
    wait_lgkm();
    if constexpr (C == 6) {
      const ntd2 *src = reinterpret_cast<const ntd2 *>(img);
#pragma unroll
      for (int t = 0; t < 3; t++) {
        const int p = 64 * t + lane; // 16-byte piece
        if ((mask >> (p / 3)) & 1ULL) __builtin_nontemporal_store(src[p], reinterpret_cast<ntd2 *>(out) + p);
      }
    } else {
#pragma unroll
      for (int t = 0; t < C; t++) {
        const int p = 64 * t + lane; // 8-byte piece
        if ((mask >> (p / C)) & 1ULL) nt_store(out + p, img[p]);
      }
    }
    wait_lgkm(); // the image is reused by the next slot
  }
}

// one slot's row (C = 0: no slot)
template <int C>
struct SlotRow {
  double r[C > 0 ? C : 1];
  bool ok;
  __device__ __forceinline__ void eval(const Slot &sl, bool act, const int *v, const double *phi) {
    if constexpr (C > 0) ok = interp_row<4, C>(sl, v, phi, r) && act;
  }
  __device__ __forceinline__ void store(const Slot &sl, size_t i0, double *img) const {
    if constexpr (C > 0) wave_store_rows<C>(sl.out + (size_t)C * i0, r, __ballot(ok), img);
  }
};

// interpolation of the located volume queries, in input order; one lane per
// query, one pass (the grid covers np).  vrec holds the walk's vertex ids and
// exact barycentric coordinates (coalesced reads); the rows of every slot are
// gathered before any math (slot layout = template: codes 1 / 3 / 6, 0 =
// none; C0 < 0 = runtime layout, per-lane stores).
template <int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(kBlock) void k_vol_interp(const uint8_t *pclass, int np, const int *vloc, VRec vrec,
                                                       Slots S, int *elem_out, int8_t *hit_out, int i0) {
  __shared__ double img_all[kBlock / 64][64 * 6];
  double *img = img_all[threadIdx.x >> 6];
  const int i = i0 + xcd_block() * blockDim.x + threadIdx.x;
  bool act = i < np && __builtin_nontemporal_load(pclass + i) == PMMG_PT_VOL;
  const int k = act ? __builtin_nontemporal_load(vloc + i) : 0;
  act = act && k != 0;
  if (!__any(act)) return;
  VolLoc loc;
  if (act) loc = vrec_load(vrec, i);
  else { // idle lanes gather a valid row, never stored
    loc.v = make_int4(1, 1, 1, 1);
#pragma unroll
    for (int f = 0; f < 4; f++) loc.phi[f] = 0.0;
  }
  const int v[4] = {loc.v.x, loc.v.y, loc.v.z, loc.v.w};
  const int ip = i + 1;
  if constexpr (C0 < 0) {
    if (act)
      for (int s = 0; s < S.n; s++) interp_dyn<4>(S.s[s], ip, v, loc.phi);
  } else {
    // every slot's rows are gathered and evaluated before the first store
    // (the stores' LDS waits are compiler barriers)
    SlotRow<C0> r0;
    SlotRow<C1> r1;
    SlotRow<C2> r2;
    SlotRow<C3> r3;
    SlotRow<C4> r4;
    SlotRow<C5> r5;
    r0.eval(S.s[0], act, v, loc.phi);
    r1.eval(S.s[1], act, v, loc.phi);
    r2.eval(S.s[2], act, v, loc.phi);
    r3.eval(S.s[3], act, v, loc.phi);
    r4.eval(S.s[4], act, v, loc.phi);
    r5.eval(S.s[5], act, v, loc.phi);
    const size_t i0 = (size_t)(i - __lane_id());
    r0.store(S.s[0], i0, img);
    r1.store(S.s[1], i0, img);
    r2.store(S.s[2], i0, img);
    r3.store(S.s[3], i0, img);
    r4.store(S.s[4], i0, img);
    r5.store(S.s[5], i0, img);
  }
  if (!act) return;
  if (elem_out) __builtin_nontemporal_store(k, elem_out + ip - 1);
  if (hit_out) __builtin_nontemporal_store((int8_t)PMMG_HIT_VOL_WALK, hit_out + ip - 1);
}

// Cooperative row gathers (default interpolation).  The texture addresser
// is the interpolation's bound (PMC: TA busy ~92% of the kernel): its cost
// follows the distinct cache lines each wave-instruction touches, and a lane
// gathering its own 48-byte rows in three 16-byte instructions touches every
// row's lines three times, ~41 lines per instruction.  Here the 64 lanes of a
// wave gather the 256 rows (64 queries x 4 vertices) of one 3- or 6-double
// slot together: piece p = 64 t + lane of the slot's row image (16-byte pieces
// for 6-double rows, 8-byte pieces for 3-double rows, 3 pieces per row) is
// loaded by one lane, so a row's pieces share an instruction and every
// instruction covers ~21 whole rows.  The image goes through LDS, each lane
// reads its 4 rows back and evaluates the reference interpolator (same
// arithmetic, same order) from them.  Scalar slots keep per-lane gathers.
template <int C>
__device__ __forceinline__ void coop_gather(const Slot &sl, const int *vid, double *img) {
  const int lane = __lane_id();
  if constexpr (C == 6) {
    double2 b[12];
#pragma unroll
    for (int t = 0; t < 12; t++) {
      const int p = 64 * t + lane, r = p / 3, k = p - 3 * r;
      b[t] = *reinterpret_cast<const double2 *>(sl.in + (size_t)sl.stride * (vid[r] - 1) + 2 * k);
    }
#pragma unroll
    for (int t = 0; t < 12; t++) reinterpret_cast<double2 *>(img)[64 * t + lane] = b[t];
  } else {
    double b[12];
#pragma unroll
    for (int t = 0; t < 12; t++) {
      const int p = 64 * t + lane, r = p / 3, k = p - 3 * r;
      b[t] = sl.in[(size_t)sl.stride * (vid[r] - 1) + k];
    }
#pragma unroll
    for (int t = 0; t < 12; t++) img[64 * t + lane] = b[t];
  }
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
}

// the row of one slot from the wave's row image (rows 4*lane .. 4*lane+3)
template <int C>
__device__ __forceinline__ bool coop_row(const double *img, const double *phi, double *r) {
  const double *base = img + 4 * C * __lane_id();
  if constexpr (C == 6) {
    double m[4][6];
#pragma unroll
    for (int i = 0; i < 4; i++) load6(base + 6 * i, m[i]);
    double mint[6], mi[6];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      ok = invmat(m[i], mi) && ok;
#pragma unroll
      for (int q = 0; q < 6; q++) mint[q] = (i == 0) ? phi[0] * mi[q] : mint[q] + phi[i] * mi[q];
    }
    return invmat(mint, r) && ok;
  } else {
    double row[4][C];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < C; j++) row[i][j] = base[C * i + j];
#pragma unroll
    for (int j = 0; j < C; j++) r[j] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < C; j++) r[j] += phi[i] * row[i][j];
    return true;
  }
}

template <int C>
__device__ __forceinline__ void coop_slot(const Slot &sl, bool act, const int *v, const double *phi, const int *vid,
                                          double *img, size_t i0) {
  if constexpr (C > 0) {
    double r[C];
    bool ok;
    if constexpr (C == 1) {
      ok = interp_row<4, 1>(sl, v, phi, r) && act;
    } else {
      coop_gather<C>(sl, vid, img);
      ok = coop_row<C>(img, phi, r) && act;
      wait_lgkm();
      __builtin_amdgcn_wave_barrier(); // every lane has read its rows: the image becomes the store image
    }
    wave_store_rows<C>(sl.out + (size_t)C * i0, r, __ballot(ok), img);
  }
}

// Half-image variant (PMMG_HIP_COOP=2): a 6-double slot's 256 rows are
// gathered in two passes of 128 rows (vertices 0-1, then 2-3 of the wave's 64
// queries), so a wave's image is 768 doubles for every slot kind (6 KiB
// instead of 12 KiB): LDS then admits 5 blocks per CU instead of 3.
template <int PASS>
__device__ __forceinline__ void coop_gather6_pair(const Slot &sl, const int *vid, double *img, double (*m)[6]) {
  const int lane = __lane_id();
  double2 b[6];
#pragma unroll
  for (int t = 0; t < 6; t++) {
    const int p = 64 * t + lane, r = p / 3, k = p - 3 * r; // r in [0, 128): query r/2, vertex 2*PASS + r%2
    const int v = vid[4 * (r >> 1) + 2 * PASS + (r & 1)];
    b[t] = *reinterpret_cast<const double2 *>(sl.in + (size_t)sl.stride * (v - 1) + 2 * k);
  }
#pragma unroll
  for (int t = 0; t < 6; t++) reinterpret_cast<double2 *>(img)[64 * t + lane] = b[t];
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
  load6(img + 12 * lane, m[2 * PASS]);
  load6(img + 12 * lane + 6, m[2 * PASS + 1]);
  wait_lgkm();
  __builtin_amdgcn_wave_barrier(); // every lane has read its rows: the image is free again
}

template <int C>
__device__ __forceinline__ void coop_slot_half(const Slot &sl, bool act, const int *v, const double *phi,
                                               const int *vid, double *img, size_t i0) {
  if constexpr (C == 6) {
    double m[4][6];
    coop_gather6_pair<0>(sl, vid, img, m);
    coop_gather6_pair<1>(sl, vid, img, m);
    double mint[6], mi[6], r[6];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; i++) { // PMMG_interp4bar_ani, same order as coop_row<6>
      ok = invmat(m[i], mi) && ok;
#pragma unroll
      for (int q = 0; q < 6; q++) mint[q] = (i == 0) ? phi[0] * mi[q] : mint[q] + phi[i] * mi[q];
    }
    ok = invmat(mint, r) && ok && act;
    wave_store_rows<6>(sl.out + (size_t)6 * i0, r, __ballot(ok), img);
  } else {
    coop_slot<C>(sl, act, v, phi, vid, img, i0);
  }
}

template <int C0, int C1, int C2, int C3, int C4, int C5, int B = kBlock>
__global__ __launch_bounds__(B) void k_vol_interp_coop_half(const uint8_t *pclass, int np, const int *vloc, VRec vrec,
                                                            Slots S, int *elem_out, int8_t *hit_out, int i0q) {
  __shared__ double img_all[B / 64][256 * 3];
  __shared__ int vid_all[B / 64][256];
  double *img = img_all[threadIdx.x >> 6];
  int *vid = vid_all[threadIdx.x >> 6];
  const int i = i0q + xcd_block() * blockDim.x + threadIdx.x;
  bool act = i < np && __builtin_nontemporal_load(pclass + i) == PMMG_PT_VOL;
  const int k = act ? __builtin_nontemporal_load(vloc + i) : 0;
  act = act && k != 0;
  if (!__any(act)) return;
  VolLoc loc;
  if (act) loc = vrec_load(vrec, i);
  else { // idle lanes gather a valid row, never stored
    loc.v = make_int4(1, 1, 1, 1);
#pragma unroll
    for (int f = 0; f < 4; f++) loc.phi[f] = 0.0;
  }
  const int v[4] = {loc.v.x, loc.v.y, loc.v.z, loc.v.w};
  reinterpret_cast<int4 *>(vid)[__lane_id()] = loc.v;
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
  const size_t w0 = (size_t)(i - __lane_id());
  coop_slot_half<C0>(S.s[0], act, v, loc.phi, vid, img, w0);
  coop_slot_half<C1>(S.s[1], act, v, loc.phi, vid, img, w0);
  coop_slot_half<C2>(S.s[2], act, v, loc.phi, vid, img, w0);
  coop_slot_half<C3>(S.s[3], act, v, loc.phi, vid, img, w0);
  coop_slot_half<C4>(S.s[4], act, v, loc.phi, vid, img, w0);
  coop_slot_half<C5>(S.s[5], act, v, loc.phi, vid, img, w0);
  if (!act) return;
  if (elem_out) __builtin_nontemporal_store(k, elem_out + i);
  if (hit_out) __builtin_nontemporal_store((int8_t)PMMG_HIT_VOL_WALK, hit_out + i);
}

template <int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(kBlock) void k_vol_interp_coop(const uint8_t *pclass, int np, const int *vloc, VRec vrec,
                                                            Slots S, int *elem_out, int8_t *hit_out, int i0q) {
  __shared__ double img_all[kBlock / 64][256 * 6];
  __shared__ int vid_all[kBlock / 64][256];
  double *img = img_all[threadIdx.x >> 6];
  int *vid = vid_all[threadIdx.x >> 6];
  const int i = i0q + xcd_block() * blockDim.x + threadIdx.x;
  bool act = i < np && __builtin_nontemporal_load(pclass + i) == PMMG_PT_VOL;
  const int k = act ? __builtin_nontemporal_load(vloc + i) : 0;
  act = act && k != 0;
  if (!__any(act)) return;
  VolLoc loc;
  if (act) loc = vrec_load(vrec, i);
  else { // idle lanes gather a valid row, never stored
    loc.v = make_int4(1, 1, 1, 1);
#pragma unroll
    for (int f = 0; f < 4; f++) loc.phi[f] = 0.0;
  }
  const int v[4] = {loc.v.x, loc.v.y, loc.v.z, loc.v.w};
  reinterpret_cast<int4 *>(vid)[__lane_id()] = loc.v;
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
  const size_t w0 = (size_t)(i - __lane_id());
  coop_slot<C0>(S.s[0], act, v, loc.phi, vid, img, w0);
  coop_slot<C1>(S.s[1], act, v, loc.phi, vid, img, w0);
  coop_slot<C2>(S.s[2], act, v, loc.phi, vid, img, w0);
  coop_slot<C3>(S.s[3], act, v, loc.phi, vid, img, w0);
  coop_slot<C4>(S.s[4], act, v, loc.phi, vid, img, w0);
  coop_slot<C5>(S.s[5], act, v, loc.phi, vid, img, w0);
  if (!act) return;
  if (elem_out) __builtin_nontemporal_store(k, elem_out + i);
  if (hit_out) __builtin_nontemporal_store((int8_t)PMMG_HIT_VOL_WALK, hit_out + i);
}

// walk + interpolation in one pass (default): the located tetra's vertex ids
// and barycentric coordinates are still in registers for the row gathers
template <int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(kBlock) void k_vol_fused(Bg bg, const Frame *fr, const unsigned long long *grid, int g,
                                                      const double *qxyz, const int *order, Slots S, int *elem_out,
                                                      int8_t *hit_out, int *fb, DevStats *st, int maxstep) {
  __shared__ BlockStats bs;
  bstats_init(&bs);
  __syncthreads();
  const int nvol = st->nvol;
  const int stride = gridDim.x * blockDim.x;
  const int iters = (nvol + stride - 1) / stride;
  for (int it = 0; it < iters; it++) {
    const int i = it * stride + xcd_block() * blockDim.x + threadIdx.x;
    const bool active = i < nvol;
    int status = 0, steps = 0, k = 0, ip = 0;
    if (active) {
      ip = order[i];
      int4 tv;
      double x[3], b[4], p[4][3];
      load_pt(qxyz, ip, x);
      status = walk_vol(bg, grid, g, fr, x, maxstep, k, tv, steps);
      if (status == 1) {
        load_tet_pts(bg, tv, p);
        tet_bary(x, p[0], p[1], p[2], p[3], b); // the reference's coordinates, exactly
        const int v[4] = {tv.x, tv.y, tv.z, tv.w};
        interp_vol_layout<C0, C1, C2, C3, C4, C5>(S, ip, v, b);
        if (elem_out) elem_out[ip - 1] = k;
        if (hit_out) hit_out[ip - 1] = PMMG_HIT_VOL_WALK;
      }
    }
    int slot = wave_append(&st->nfb_vol, active && status != 1);
    if (active && status != 1) fb[slot] = ip;
    wave_stats(&bs, active, status == 1 ? PMMG_HIT_VOL_WALK : 0, steps);
  }
  __syncthreads();
  bstats_flush(&bs, st);
}

// ---------------------------------------------------------------- volume, tetra-centric scan

// Volume queries counting-sorted into a uniform row-major grid of cells (the
// sorted coordinates are stored contiguously per cell).
__global__ __launch_bounds__(kBlock) void k_qcount(const double *xyz, const uint8_t *pclass, int np, const Frame *fr,
                                                   int gq, int *cnt, int2 *binrank) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  if (pclass[i] != PMMG_PT_VOL) {
    binrank[i] = make_int2(-1, 0);
    return;
  }
  int c[3];
  for (int d = 0; d < 3; d++) c[d] = cell_coord(xyz[3 * (size_t)i + d], fr->lo[d], fr->inv_bin[d], gq);
  int cell = c[0] + gq * (c[1] + gq * c[2]);
  int r = atomicAdd(&cnt[cell], 1);
  binrank[i] = make_int2(cell, r);
}

__global__ __launch_bounds__(kBlock) void k_qscatter(int np, const double *xyz, const int2 *binrank, const int *off,
                                                     int *order, double *qs, int *res) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  int2 br = binrank[i];
  if (br.x < 0) return;
  int pos = off[br.x] + br.y;
  order[pos] = i + 1;
  qs[3 * (size_t)pos] = xyz[3 * (size_t)i];
  qs[3 * (size_t)pos + 1] = xyz[3 * (size_t)i + 1];
  qs[3 * (size_t)pos + 2] = xyz[3 * (size_t)i + 2];
  res[pos] = INT_MAX;
}

__global__ void k_qtotal(const int *off, int ncells, DevStats *st) { st->nvol = off[ncells]; }

// One thread per background tetra (contiguous tetra ranges per XCD): the
// tetra's bbox, inflated by the acceptance tolerance (an accepted point has
// every barycentric coordinate > -EPS, hence lies within 3 EPS of the tetra's
// extent of it), selects the query cells to test; an accepting tetra lowers
// res[q] with atomicMin, so res ends as the lowest-index accepting tetra —
// the reference's exhaustive-search result — for every query at once.
__global__ __launch_bounds__(kBlock) void k_vol_scan(Bg bg, const Frame *fr, int gq, const int *off, const double *qs,
                                                     int *res, DevStats *st) {
  const int x8 = blockIdx.x & 7, bpx = gridDim.x >> 3, bi = blockIdx.x >> 3;
  const long long lo_k = (long long)bg.ne * x8 / 8, hi_k = (long long)bg.ne * (x8 + 1) / 8;
  unsigned long long tests = 0;
  for (long long kk = lo_k + (long long)bi * blockDim.x + threadIdx.x; kk < hi_k; kk += (long long)bpx * blockDim.x) {
    const int k = (int)kk + 1;
    const int4 tv = tetv_row(bg, k);
    if (tv.x <= 0) continue;
    double p0[3], p1[3], p2[3], p3[3];
    load_pt(bg.xyz, tv.x, p0);
    load_pt(bg.xyz, tv.y, p1);
    load_pt(bg.xyz, tv.z, p2);
    load_pt(bg.xyz, tv.w, p3);
    double lo[3], hi[3];
    int c0[3], c1[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      lo[d] = fmin(fmin(p0[d], p1[d]), fmin(p2[d], p3[d]));
      hi[d] = fmax(fmax(p0[d], p1[d]), fmax(p2[d], p3[d]));
      double pad = 8.0 * kEps * (hi[d] - lo[d]) + 1e-300;
      lo[d] -= pad;
      hi[d] += pad;
      c0[d] = cell_coord(lo[d], fr->lo[d], fr->inv_bin[d], gq);
      c1[d] = cell_coord(hi[d], fr->lo[d], fr->inv_bin[d], gq);
    }
    for (int ck = c0[2]; ck <= c1[2]; ck++)
      for (int cj = c0[1]; cj <= c1[1]; cj++) {
        const int row = gq * (cj + gq * ck);
        const int q0 = off[row + c0[0]], q1 = off[row + c1[0] + 1];
        for (int q = q0; q < q1; q++) {
          double x[3];
          load_pt(qs, q + 1, x);
          if (x[0] < lo[0] || x[0] > hi[0] || x[1] < lo[1] || x[1] > hi[1] || x[2] < lo[2] || x[2] > hi[2]) continue;
          double b[4];
          tet_bary(x, p0, p1, p2, p3, b);
          tests++;
          if (min4(b) > -kEps) atomicMin(&res[q], k);
        }
      }
  }
  for (int o = 32; o > 0; o >>= 1) tests += __shfl_down(tests, o);
  if (__lane_id() == 0 && tests) atomicAdd(&stat_part(st)->steps, tests);
}

// interpolation of the scanned queries (sorted positions, coordinates read
// back contiguously); queries with no accepting tetra go to the closest-tetra
// fallback
template <int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(kBlock) void k_vol_interp_scan(Bg bg, const double *qs, const int *order, const int *res,
                                                            Slots S, int *elem_out, int8_t *hit_out, int *fb,
                                                            DevStats *st) {
  __shared__ unsigned int nloc;
  if (threadIdx.x == 0) nloc = 0;
  __syncthreads();
  const int nvol = st->nvol;
  const int stride = gridDim.x * blockDim.x;
  const int iters = (nvol + stride - 1) / stride;
  for (int it = 0; it < iters; it++) {
    const int i = it * stride + xcd_block() * blockDim.x + threadIdx.x;
    const bool active = i < nvol;
    int k = INT_MAX, ip = 0;
    if (active) {
      k = res[i];
      ip = order[i];
      if (k != INT_MAX) {
        double x[3], p0[3], p1[3], p2[3], p3[3], phi[4];
        load_pt(qs, i + 1, x);
        const int4 tv = tetv_row(bg, k);
        load_pt(bg.xyz, tv.x, p0);
        load_pt(bg.xyz, tv.y, p1);
        load_pt(bg.xyz, tv.z, p2);
        load_pt(bg.xyz, tv.w, p3);
        tet_bary(x, p0, p1, p2, p3, phi);
        const int v[4] = {tv.x, tv.y, tv.z, tv.w};
        interp_vol_layout<C0, C1, C2, C3, C4, C5>(S, ip, v, phi);
        if (elem_out) elem_out[ip - 1] = k;
        if (hit_out) hit_out[ip - 1] = PMMG_HIT_VOL_SCAN;
      }
    }
    const bool miss = active && k == INT_MAX;
    int slot = wave_append(&st->nfb_vol, miss);
    if (miss) fb[slot] = ip;
    unsigned long long okm = __ballot(active && k != INT_MAX);
    if (__lane_id() == 0 && okm) atomicAdd(&nloc, (unsigned)__popcll(okm));
  }
  __syncthreads();
  if (threadIdx.x == 0 && nloc) atomicAdd(&stat_part(st)->cnt[PMMG_HIT_VOL_SCAN], (unsigned long long)nloc);
}

// ---------------------------------------------------------------- surface

// one surface query (PMMG_locatePointBdy, locate_pmmg.c:587-723, and the
// surface interpolation, interpmesh_pmmg.c:550-599); returns the hit code
// (0 = not located: exhaustive list)
__device__ __forceinline__ int bdy_query(const Bg &bg, const Frame *fr, const int *sgrid, int gs, const double *qxyz,
                                         int ip, const Slots &S, int *elem_out, int8_t *hit_out, int maxstep,
                                         int &steps) {
  int hit = 0;
  double x[3];
  load_pt(qxyz, ip, x);
  int k = seed_srf(sgrid, gs, fr, x);
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  int edge = -1, vertex = -1;
  TriGeom t;
  double phi[3];
  for (;;) {
    ++steps;
    tri_load(bg, k, t);
    double b[3];
    double dist = tri_bary(x, t.p, t.q, t.n, b);
    int r[3];
    ranks3(b, r);
    double bmin = b[0];
    bmin = b[1] < bmin ? b[1] : bmin;
    bmin = b[2] < bmin ? b[2] : bmin;
    phi[0] = b[0];
    phi[1] = b[1];
    phi[2] = b[2];
    // PMMG_locatePointInTria: inside and |dist| <= hausd
    if (bmin > -kEps && !(fabs(dist) > bg.hausd)) {
      // PMMG_barycoord_isBorder on the sorted coordinates
      int f0 = r[0] == 0 ? 0 : (r[1] == 0 ? 1 : 2);
      int f1 = r[0] == 1 ? 0 : (r[1] == 1 ? 1 : 2);
      int f2 = r[0] == 2 ? 0 : (r[1] == 2 ? 1 : 2);
      double b1 = sel3d(b[0], b[1], b[2], f1);
      hit = PMMG_HIT_BDY_FACE;
      if (bmin < kEps) {
        if (b1 < kEps) { vertex = f2; hit = PMMG_HIT_BDY_VERTEX; }
        else { edge = f0; hit = PMMG_HIT_BDY_EDGE; }
      }
      break;
    }
    const int *ad = bg.adjt + 3 * (size_t)(k - 1);
    const int a0 = ad[0], a1 = ad[1], a2 = ad[2];
    int next = 0;
    bool done = false;
    for (int j = 0; j < 3 && !done && next == 0; j++) {
      int f = r[0] == j ? 0 : (r[1] == j ? 1 : 2);
      int k1 = sel3i(a0, a1, a2, f) / 3;
      if (!k1) continue;
      bool vis = false;
#pragma unroll
      for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == k1);
      if (vis) {
        double w[3];
        int il = tri_wedge(bg.hausd, t, f, x, w);
        if (il < 0) continue;
        if (il == 4) {
          phi[0] = w[0]; phi[1] = w[1]; phi[2] = w[2];
          edge = f;
          hit = PMMG_HIT_BDY_WEDGE;
          done = true;
        } else if (tri_cone(bg, k, il, t, x)) {
          vertex = il;
          hit = PMMG_HIT_BDY_CONE;
          done = true;
        }
        continue;
      }
      next = k1;
    }
    if (done) break;
    if (next == 0 || steps >= maxstep) { hit = 0; break; } // -> exhaustive
#pragma unroll
    for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
    hist[0] = k;
    k = next;
  }
  if (hit) {
    interp_bdy(S, ip, t.v, phi, edge, vertex);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)(hit | ((vertex >= 0 ? vertex : (edge >= 0 ? edge : 0)) << 4));
  }
  return hit;
}

__global__ __launch_bounds__(kBlock) void k_bdy(Bg bg, const Frame *fr, const int *sgrid, int gs, const double *qxyz,
                                                const int *order, Slots S, int *elem_out, int8_t *hit_out, int *fb,
                                                DevStats *st, int maxstep) {
  __shared__ BlockStats bs;
  bstats_init(&bs);
  __syncthreads();
  const XcdChunk ch = xcd_chunk(st->nbdy);
  for (int it = 0; it < ch.iters; it++) {
    const int i = (int)(ch.start + it * ch.stride);
    const bool active = i < ch.hi;
    int steps = 0, hit = 0, ip = 0;
    if (active) {
      ip = order[i];
      hit = bdy_query(bg, fr, sgrid, gs, qxyz, ip, S, elem_out, hit_out, maxstep, steps);
    }
    int slot = wave_append(&st->nfb_bdy, active && hit == 0);
    if (active && hit == 0) fb[slot] = ip;
    wave_stats(&bs, active, hit, steps);
  }
  __syncthreads();
  bstats_flush(&bs, st);
}

// ---------------------------------------------------------------- exhaustive fallbacks (exact reference semantics)

constexpr int kQB = 128; // fallback queries staged in LDS per pass

// lowest-index tetra accepting each fallback query (locate_pmmg.c:743-762)
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_accept(Bg bg, const double *qxyz, const int *fb,
                                                               const DevStats *st, int *best) {
  __shared__ double sx[kQB][3];
  const int nfb = st->nfb_vol;
  for (int q0 = 0; q0 < nfb; q0 += kQB) {
    int nq = min(kQB, nfb - q0);
    __syncthreads();
    for (int j = threadIdx.x; j < nq; j += blockDim.x) load_pt(qxyz, fb[q0 + j], sx[j]);
    __syncthreads();
    for (int k = 1 + blockIdx.x * blockDim.x + threadIdx.x; k <= bg.ne; k += gridDim.x * blockDim.x) {
      int4 tv = tetv_row(bg, k);
      if (tv.x <= 0) continue;
      double p0[3], p1[3], p2[3], p3[3];
      load_pt(bg.xyz, tv.x, p0);
      load_pt(bg.xyz, tv.y, p1);
      load_pt(bg.xyz, tv.z, p2);
      load_pt(bg.xyz, tv.w, p3);
      double lo[3], hi[3];
      for (int d = 0; d < 3; d++) {
        lo[d] = fmin(fmin(p0[d], p1[d]), fmin(p2[d], p3[d]));
        hi[d] = fmax(fmax(p0[d], p1[d]), fmax(p2[d], p3[d]));
        // an accepted point has every barycentric coordinate > -EPS, so it
        // lies inside the tetra's bbox inflated by 3 EPS of its extent
        double pad = 8.0 * kEps * (hi[d] - lo[d]) + 1e-300;
        lo[d] -= pad;
        hi[d] += pad;
      }
      for (int j = 0; j < nq; j++) {
        const double *x = sx[j];
        if (x[0] < lo[0] || x[0] > hi[0] || x[1] < lo[1] || x[1] > hi[1] || x[2] < lo[2] || x[2] > hi[2]) continue;
        if (best[q0 + j] <= k) continue;
        double b[4];
        tet_bary(x, p0, p1, p2, p3, b);
        if (min4(b) > -kEps) atomicMin(&best[q0 + j], k);
      }
    }
  }
}

// closest tetra of queries nobody accepts: argmin |bary_min| * vol
// (locate_pmmg.c:453-458); pass 0 finds the minimum value, pass 1 the lowest
// index reaching it
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_closest(Bg bg, const double *qxyz, const int *fb,
                                                                const DevStats *st, const int *best,
                                                                unsigned long long *ckey, int pass, int *cidx) {
  __shared__ double sx[kQB][3];
  __shared__ int sneed[kQB];
  const int nfb = st->nfb_vol;
  for (int q0 = 0; q0 < nfb; q0 += kQB) {
    int nq = min(kQB, nfb - q0);
    __syncthreads();
    for (int j = threadIdx.x; j < nq; j += blockDim.x) {
      load_pt(qxyz, fb[q0 + j], sx[j]);
      sneed[j] = best[q0 + j] == INT_MAX;
    }
    __syncthreads();
    bool any = false;
    for (int j = 0; j < nq; j++) any = any || sneed[j];
    if (!any) continue;
    for (int k = 1 + blockIdx.x * blockDim.x + threadIdx.x; k <= bg.ne; k += gridDim.x * blockDim.x) {
      int4 tv = tetv_row(bg, k);
      if (tv.x <= 0) continue;
      double p0[3], p1[3], p2[3], p3[3];
      load_pt(bg.xyz, tv.x, p0);
      load_pt(bg.xyz, tv.y, p1);
      load_pt(bg.xyz, tv.z, p2);
      load_pt(bg.xyz, tv.w, p3);
      for (int j = 0; j < nq; j++) {
        if (!sneed[j]) continue;
        double b[4];
        double vol = tet_bary(sx[j], p0, p1, p2, p3, b);
        unsigned long long key = dkey(fabs(min4(b)) * vol);
        if (pass == 0) atomicMin(&ckey[q0 + j], key);
        else if (key == ckey[q0 + j]) atomicMin(&cidx[q0 + j], k);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_vol_finish(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                       const int *best, const int *cidx, Slots S, int *elem_out,
                                                       int8_t *hit_out) {
  const int nfb = st->nfb_vol;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nfb; j += gridDim.x * blockDim.x) {
    int ip = fb[j];
    double x[3];
    load_pt(qxyz, ip, x);
    int hit, k;
    if (best[j] != INT_MAX) { k = best[j]; hit = PMMG_HIT_VOL_EXHAUST; }
    else { k = cidx[j]; hit = PMMG_HIT_VOL_CLOSEST; }
    if (k == INT_MAX || k <= 0) continue;
    int4 tv = tetv_row(bg, k);
    double p[4][3], phi[4];
    load_pt(bg.xyz, tv.x, p[0]);
    load_pt(bg.xyz, tv.y, p[1]);
    load_pt(bg.xyz, tv.z, p[2]);
    load_pt(bg.xyz, tv.w, p[3]);
    if (hit == PMMG_HIT_VOL_EXHAUST) tet_bary(x, p[0], p[1], p[2], p[3], phi);
    else closest_vertex<4>(x, p, phi);
    const int v[4] = {tv.x, tv.y, tv.z, tv.w};
    for (int s = 0; s < S.n; s++) interp_dyn<4>(S.s[s], ip, v, phi);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)hit;
    atomicAdd(&stat_part(st)->cnt[hit], 1ULL);
  }
}

// surface: pass 0 lowest-index accepting tria (locate_pmmg.c:483-503), pass 1
// minimum centroid distance, pass 2 lowest index reaching it (:400-416)
__global__ __launch_bounds__(kBlock) void k_bdy_exhaust(Bg bg, const double *qxyz, const int *fb, const DevStats *st,
                                                        int *best, unsigned long long *ckey, int pass, int *cidx) {
  __shared__ double sx[kQB][3];
  const int nfb = st->nfb_bdy;
  for (int q0 = 0; q0 < nfb; q0 += kQB) {
    int nq = min(kQB, nfb - q0);
    __syncthreads();
    for (int j = threadIdx.x; j < nq; j += blockDim.x) load_pt(qxyz, fb[q0 + j], sx[j]);
    __syncthreads();
    for (int k = 1 + blockIdx.x * blockDim.x + threadIdx.x; k <= bg.nt; k += gridDim.x * blockDim.x) {
      if (bg.triv[3 * (size_t)(k - 1)] <= 0) continue;
      TriGeom t;
      tri_load(bg, k, t);
      for (int j = 0; j < nq; j++) {
        const double *x = sx[j];
        if (pass == 0) {
          if (best[q0 + j] <= k) continue;
          double b[3];
          double dist = tri_bary(x, t.p, t.q, t.n, b);
          double bmin = fmin(b[0], fmin(b[1], b[2]));
          if (bmin > -kEps && !(fabs(dist) > bg.hausd)) atomicMin(&best[q0 + j], k);
        } else {
          if (best[q0 + j] != INT_MAX) continue;
          double d[3] = {x[0], x[1], x[2]};
          for (int v = 0; v < 3; v++)
            for (int c = 0; c < 3; c++) d[c] -= t.p[v][c] / 3.0;
          double nrm = 0;
          for (int c = 0; c < 3; c++) nrm += d[c] * d[c];
          nrm = sqrt(nrm);
          unsigned long long key = dkey(nrm);
          if (pass == 1) atomicMin(&ckey[q0 + j], key);
          else if (key == ckey[q0 + j]) atomicMin(&cidx[q0 + j], k);
        }
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_bdy_finish(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                       const int *best, const int *cidx, Slots S, int *elem_out,
                                                       int8_t *hit_out) {
  const int nfb = st->nfb_bdy;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nfb; j += gridDim.x * blockDim.x) {
    int ip = fb[j];
    double x[3];
    load_pt(qxyz, ip, x);
    int hit, k;
    double phi[3];
    TriGeom t;
    if (best[j] != INT_MAX) {
      k = best[j];
      hit = PMMG_HIT_BDY_EXHAUST;
      tri_load(bg, k, t);
      tri_bary(x, t.p, t.q, t.n, phi);
    } else {
      k = cidx[j];
      if (k == INT_MAX || k <= 0) continue;
      tri_load(bg, k, t);
      // stale re-evaluation (locate_pmmg.c:505-509): vertices and area of the
      // last tria scanned (nt), normal of the closest one
      TriGeom ts;
      tri_load(bg, bg.nt, ts);
      double b[3];
      double dist = tri_bary(x, ts.p, ts.q, t.n, b);
      double bmin = fmin(b[0], fmin(b[1], b[2]));
      if (bmin > -kEps && !(fabs(dist) > bg.hausd)) {
        hit = PMMG_HIT_BDY_STALE;
        phi[0] = b[0]; phi[1] = b[1]; phi[2] = b[2];
      } else {
        hit = PMMG_HIT_BDY_CLOSEST;
        closest_vertex<3>(x, t.p, phi);
      }
    }
    interp_bdy(S, ip, t.v, phi, -1, -1);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)hit;
    atomicAdd(&stat_part(st)->cnt[hit], 1ULL);
  }
}

__global__ void k_fallback_init(int *a, int *b, unsigned long long *c, const int *count) {
  const int n = *count;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    a[i] = INT_MAX;
    b[i] = INT_MAX;
    c[i] = ~0ULL;
  }
}

// ---------------------------------------------------------------- layout dispatch

typedef void (*VolInterpFn)(const uint8_t *, int, const int *, VRec, Slots, int *, int8_t *, int);
typedef void (*ScanInterpFn)(Bg, const double *, const int *, const int *, Slots, int *, int8_t *, int *, DevStats *);
typedef void (*FusedFn)(Bg, const Frame *, const unsigned long long *, int, const double *, const int *, Slots, int *,
                        int8_t *, int *, DevStats *, int);

struct LayoutEntry {
  int c[6];
  VolInterpFn fn;
  VolInterpFn cfn; // cooperative-gather variant (nullptr: runtime layout)
  VolInterpFn hfn; // cooperative gathers through a half-size image
  VolInterpFn hfn64; // the same in one-wave blocks
  ScanInterpFn sfn;
  FusedFn ffn;
};

#define PMMG_LAYOUT(a, b, c, d, e, f)                                                                             \
  {{a, b, c, d, e, f}, k_vol_interp<a, b, c, d, e, f>, k_vol_interp_coop<a, b, c, d, e, f>,                     \
   k_vol_interp_coop_half<a, b, c, d, e, f>, k_vol_interp_coop_half<a, b, c, d, e, f, 64>,                      \
   k_vol_interp_scan<a, b, c, d, e, f>,                                                                         \
   k_vol_fused<a, b, c, d, e, f>}
// common slot layouts (metric first): aniso metric + scalar/vector/tensor
// (BASELINE cfg3/cfg4, libexamples cube-solphys.sol), iso metric + scalars
// (cfg2, cfg5), metric only
const LayoutEntry kLayouts[] = {
    PMMG_LAYOUT(6, 1, 3, 6, 0, 0), PMMG_LAYOUT(6, 1, 3, 6, 1, 0), PMMG_LAYOUT(1, 1, 0, 0, 0, 0),
    PMMG_LAYOUT(1, 1, 1, 1, 1, 1), PMMG_LAYOUT(1, 1, 1, 0, 0, 0), PMMG_LAYOUT(6, 0, 0, 0, 0, 0),
    PMMG_LAYOUT(1, 0, 0, 0, 0, 0), PMMG_LAYOUT(6, 1, 0, 0, 0, 0), PMMG_LAYOUT(1, 1, 3, 6, 0, 0),
};
#undef PMMG_LAYOUT

const LayoutEntry kGeneric = {{-1, 0, 0, 0, 0, 0}, k_vol_interp<-1, 0, 0, 0, 0, 0>, nullptr, nullptr, nullptr,
                               k_vol_interp_scan<-1, 0, 0, 0, 0, 0>, k_vol_fused<-1, 0, 0, 0, 0, 0>};

const LayoutEntry &pick_layout(const Slots &S) {
  for (const LayoutEntry &e : kLayouts) {
    int n = 0;
    while (n < 6 && e.c[n] > 0) n++;
    if (n != S.n) continue;
    bool ok = true;
    for (int j = 0; j < n; j++) ok = ok && (S.s[j].code == e.c[j]);
    if (ok) return e;
  }
  return kGeneric;
}

} // namespace

// ================================================================ host side

constexpr int kMaxChunks = 16;

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

struct pmmg_hip_ctx {
  int device = 0;
  int options = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr; // surface branch, concurrent with the volume walk
  hipStream_t stream3 = nullptr; // volume interpolation of chunk c, concurrent with the walk of chunk c+1
  int coop = 2;         // row gathers: 0 per lane, 1 cooperative, 2 cooperative half image (PMMG_HIP_COOP)
  int seed8 = 1;        // queries pick the nearest of 8 cell seeds (PMMG_HIP_SEED8)
  int bbox_stride = 16; // frame from every 16th background vertex (PMMG_HIP_BBOXSTRIDE)
  int chunks = 1;                // volume pipeline chunks (PMMG_HIP_CHUNKS)
  int walkb = 64;                // walk block size, 64 or 256 (PMMG_HIP_WALKB)
  int bdy_early = 0;             // surface kernel enqueued before the walk (PMMG_HIP_BDYEARLY)
  int interpb = 256;             // half-image interpolation block size, 256 or 64 (PMMG_HIP_INTERPB)
  hipEvent_t evc[kMaxChunks] = {};
  bool bdy_on_s2 = false;
  int two_streams = 1; // PMMG_HIP_STREAMS=1: everything on one stream
  int carry = 2;       // 0 reload, 1 registers, 2 LDS slots (PMMG_HIP_CARRY)
  int walkw = 0;       // >= 5: walk compiled for 5 waves per SIMD (PMMG_HIP_WALKW)
  char err[512] = {0};
  Bg bg{};
  int met_size = 0;
  int nfield = 0;
  std::vector<int> fsize;
  std::vector<int> fstride; // input row strides (= sizes, or the packed record size)
  int met_stride = 0;
  std::vector<const double *> fin;
  const double *met = nullptr;
  // owned copies for PMMG_HIP_HOST inputs
  DevBuf o_xyz, o_tetv, o_adja, o_triv, o_adjt, o_met;
  std::vector<DevBuf> o_f;
  // work buffers
  DevBuf frame, stats, grid, sgrid, cnt, off, binrank, order_v, order_b, vloc, scan_tmp, qs, cls_cnt, cls_cnt2;
  DevBuf cont, vrec;
  DevBuf qmin; // tetra quality minimum (pmmg_hip_tetra_qual)
  DevBuf fb_vol, fb_bdy, best, ckey, cidx, bbest, bckey, bcidx;
  // host-mode staging
  DevBuf h_xyz, h_cls, h_met, h_elem, h_hit;
  std::vector<DevBuf> h_f;
  hipEvent_t ev[11] = {};
  bool pending = false;
  int tpc = 8;      // background tetra per volume seed cell
  int spc = 1;      // sampled tetra per seed cell
  int seed_mode = 0; // seed point of a sampled tetra: 0 centroid, 1 edge v0-v3 midpoint, 2 first vertex
  int seed_run = 4;  // consecutive tetra per sample run (1, 2, 4, 8)
  int seed_grid = 8192; // blocks of k_seed_vol (PMMG_HIP_SEEDGRID)
  int seed_atom = 1;    // 0: racy plain stores (timing experiment, PMMG_HIP_SEEDATOM)
  int qpb = 8;      // queries per Morton bin (walk path)
  int qpc = 1;      // queries per scan cell (scan path)
  int ncu = 256;     // compute units of the device
  int cap = 1 << 30; // first-pass walk cap (k_vol_walk); capped walks continue in k_vol_walk_cont.
                     // Off by default: the continuation walks lose the lockstep
                     // line sharing of neighbouring queries and measured slower
  int maxstep = 4096; // longer walks go to the exhaustive kernels (the reference caps at ne)
  int last_sorted = 0;
  int count_nvol = 0; // nvol not counted on the device (derived from the walk statistics)
  int *h_small = nullptr; // pinned host words for the two small read-backs
};

static void set_err(pmmg_hip_ctx *c, const char *fmt, ...) {
  if (!c) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(c->err, sizeof(c->err), fmt, ap);
  va_end(ap);
  fprintf(stderr, "[parmmg_hip] %s\n", c->err);
}

#define HIPCK(ctx, expr)                                                                             \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) {                                                                          \
      set_err((ctx), "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);   \
      return 0;                                                                                      \
    }                                                                                                \
  } while (0)

static int ensure(pmmg_hip_ctx *c, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 1;
  if (b.p) {
    HIPCK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  HIPCK(c, hipMalloc(&b.p, bytes));
  b.cap = bytes;
  return 1;
}

static void release(DevBuf &b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

static int upload(pmmg_hip_ctx *c, DevBuf &b, const void *src, size_t bytes) {
  if (!ensure(c, b, bytes)) return 0;
  if (bytes) HIPCK(c, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
  return 1;
}

static int env_int(const char *name, int def) { // positive values only
  const char *e = getenv(name);
  if (e && atoi(e) > 0) return atoi(e);
  return def;
}
static int env_flag(const char *name, int def) { // any integer, 0 included
  const char *e = getenv(name);
  return (e && *e) ? atoi(e) : def;
}

extern "C" {

int pmmg_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// The surface branch's stream: PMMG_HIP_S2PRIO=1 creates it with
// the device's greatest priority, so its few blocks are dispatched ahead of
// the walk's instead of after them.
static bool create_stream2(pmmg_hip_ctx *c) {
  int least = 0, greatest = 0;
  if (env_flag("PMMG_HIP_S2PRIO", 0) && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
    return hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, greatest) == hipSuccess;
  return hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) == hipSuccess;
}

pmmg_hip_ctx *pmmg_hip_create(int device, int options) {
  int n = pmmg_hip_device_count();
  if (n <= 0 || device < 0 || device >= n) {
    fprintf(stderr, "[parmmg_hip] no HIP device %d (visible: %d)\n", device, n);
    return nullptr;
  }
  pmmg_hip_ctx *c = new pmmg_hip_ctx();
  c->device = device;
  c->options = options;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      !create_stream2(c) ||
      hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess) {
    fprintf(stderr, "[parmmg_hip] cannot initialise device %d\n", device);
    delete c;
    return nullptr;
  }
  for (int i = 0; i < 11; i++) (void)hipEventCreate(&c->ev[i]);
  for (int i = 0; i < kMaxChunks; i++) (void)hipEventCreateWithFlags(&c->evc[i], hipEventDisableTiming);
  if (hipHostMalloc((void **)&c->h_small, 64, hipHostMallocDefault) != hipSuccess) {
    fprintf(stderr, "[parmmg_hip] cannot allocate pinned host memory\n");
    delete c;
    return nullptr;
  }
  c->tpc = env_int("PMMG_HIP_TPC", c->tpc);
  c->spc = env_int("PMMG_HIP_SPC", c->spc);
  if (getenv("PMMG_HIP_SEEDMODE")) c->seed_mode = atoi(getenv("PMMG_HIP_SEEDMODE"));
  c->seed_run = env_int("PMMG_HIP_SEEDRUN", c->seed_run);
  c->seed_grid = env_int("PMMG_HIP_SEEDGRID", c->seed_grid);
  c->seed_atom = env_flag("PMMG_HIP_SEEDATOM", c->seed_atom);
  if (c->seed_grid < 8) c->seed_grid = 8;
  c->two_streams = env_int("PMMG_HIP_STREAMS", 2) >= 2;
  if (getenv("PMMG_HIP_CARRY")) c->carry = atoi(getenv("PMMG_HIP_CARRY"));
  if (getenv("PMMG_HIP_WALKW")) c->walkw = atoi(getenv("PMMG_HIP_WALKW"));
  if (c->seed_run != 1 && c->seed_run != 2 && c->seed_run != 4 && c->seed_run != 8) c->seed_run = 4;
  c->qpb = env_int("PMMG_HIP_QPB", c->qpb);
  c->qpc = env_int("PMMG_HIP_QPC", c->qpc);
  c->maxstep = env_int("PMMG_HIP_MAXSTEP", c->maxstep);
  c->cap = env_int("PMMG_HIP_CAP", c->cap);
  c->chunks = env_int("PMMG_HIP_CHUNKS", c->chunks);
  c->bbox_stride = env_int("PMMG_HIP_BBOXSTRIDE", c->bbox_stride);
  c->seed8 = env_flag("PMMG_HIP_SEED8", c->seed8);
  c->coop = env_flag("PMMG_HIP_COOP", c->coop);
  c->walkb = env_int("PMMG_HIP_WALKB", c->walkb) == 256 ? 256 : 64;
  c->bdy_early = env_flag("PMMG_HIP_BDYEARLY", c->bdy_early);
  c->interpb = env_int("PMMG_HIP_INTERPB", c->interpb) == 64 ? 64 : 256;
  if (c->chunks > kMaxChunks) c->chunks = kMaxChunks;
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->ncu = prop.multiProcessorCount;
  }
  return c;
}

void pmmg_hip_destroy(pmmg_hip_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  DevBuf *bufs[] = {&c->cont, &c->vrec, &c->o_xyz, &c->o_tetv, &c->o_adja, &c->o_triv, &c->o_adjt, &c->o_met, &c->frame, &c->stats,
                    &c->grid, &c->sgrid, &c->cnt, &c->off, &c->binrank, &c->order_v, &c->order_b, &c->vloc, &c->qs,
                    &c->scan_tmp, &c->cls_cnt, &c->cls_cnt2, &c->fb_vol, &c->fb_bdy, &c->best, &c->ckey, &c->cidx, &c->bbest, &c->bckey,
                    &c->bcidx, &c->h_xyz, &c->h_cls, &c->h_met, &c->h_elem, &c->h_hit, &c->qmin};
  for (DevBuf *b : bufs) release(*b);
  for (auto &b : c->o_f) release(b);
  for (auto &b : c->h_f) release(b);
  for (int i = 0; i < 11; i++)
    if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
  for (int i = 0; i < kMaxChunks; i++)
    if (c->evc[i]) (void)hipEventDestroy(c->evc[i]);
  if (c->stream3) (void)hipStreamDestroy(c->stream3);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->h_small) (void)hipHostFree(c->h_small);
  delete c;
}

const char *pmmg_hip_last_error(pmmg_hip_ctx *c) { return c ? c->err : "null context"; }

// shared body of the two background entry points: tet8 != NULL selects the
// packed {v[4], adja[4]} records, else the separate tetv / adja arrays
static int set_background_impl(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, const int *adja,
                               const int *tet8, int nt, const int *triv, const int *adjt, double hausd, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  const bool packed = tet8 != nullptr;
  if (np <= 0 || ne <= 0 || !xyz || (!packed && (!tetv || !adja)) || nt < 0 || (nt > 0 && (!triv || !adjt))) {
    set_err(c, "set_background: invalid arguments (np=%d ne=%d nt=%d)", np, ne, nt);
    return 0;
  }
  if (ne >= (1 << 29)) {
    set_err(c, "set_background: %d tetra exceed the 4*k+i adjacency encoding (2^29)", ne);
    return 0;
  }
  c->bg.np = np;
  c->bg.ne = ne;
  c->bg.nt = nt;
  c->bg.hausd = hausd;
  c->bg.tstride = packed ? 2 : 1;
  if (where == PMMG_HIP_DEVICE) {
    const void *t0 = packed ? (const void *)tet8 : (const void *)tetv;
    if (((uintptr_t)t0 & 15) || (!packed && ((uintptr_t)adja & 15))) {
      set_err(c, "set_background: device tetra arrays must be 16-byte aligned");
      return 0;
    }
    c->bg.xyz = xyz;
    c->bg.tetv = reinterpret_cast<const int4 *>(packed ? tet8 : tetv);
    c->bg.adja = reinterpret_cast<const int4 *>(packed ? tet8 + 4 : adja);
    c->bg.triv = triv;
    c->bg.adjt = adjt;
    return 1;
  }
  if (!upload(c, c->o_xyz, xyz, sizeof(double) * 3 * (size_t)np)) return 0;
  if (packed) {
    if (!upload(c, c->o_tetv, tet8, sizeof(int) * 8 * (size_t)ne)) return 0;
  } else {
    if (!upload(c, c->o_tetv, tetv, sizeof(int) * 4 * (size_t)ne)) return 0;
    if (!upload(c, c->o_adja, adja, sizeof(int) * 4 * (size_t)ne)) return 0;
  }
  if (!upload(c, c->o_triv, triv, sizeof(int) * 3 * (size_t)nt)) return 0;
  if (!upload(c, c->o_adjt, adjt, sizeof(int) * 3 * (size_t)nt)) return 0;
  HIPCK(c, hipStreamSynchronize(c->stream));
  c->bg.xyz = (const double *)c->o_xyz.p;
  c->bg.tetv = (const int4 *)c->o_tetv.p;
  c->bg.adja = packed ? (const int4 *)c->o_tetv.p + 1 : (const int4 *)c->o_adja.p;
  c->bg.triv = (const int *)c->o_triv.p;
  c->bg.adjt = (const int *)c->o_adjt.p;
  return 1;
}

int pmmg_hip_set_background(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, const int *adja,
                            int nt, const int *triv, const int *adjt, double hausd, int where) {
  if (c && (!tetv || !adja)) {
    set_err(c, "set_background: tetv / adja is NULL");
    return 0;
  }
  return set_background_impl(c, np, xyz, ne, tetv, adja, nullptr, nt, triv, adjt, hausd, where);
}

int pmmg_hip_set_background_tet8(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tet8, int nt,
                                 const int *triv, const int *adjt, double hausd, int where) {
  if (c && !tet8) {
    set_err(c, "set_background_tet8: tet8 is NULL");
    return 0;
  }
  return set_background_impl(c, np, xyz, ne, nullptr, nullptr, tet8, nt, triv, adjt, hausd, where);
}

int pmmg_hip_set_solutions(pmmg_hip_ctx *c, int met_size, const double *met, int nfield, const int *field_size,
                           const double *const *fields, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (met_size != 0 && met_size != 1 && met_size != 6) {
    set_err(c, "set_solutions: metric size %d (expected 0, 1 or 6)", met_size);
    return 0;
  }
  if (nfield < 0 || nfield + (met_size ? 1 : 0) > kMaxSlot) {
    set_err(c, "set_solutions: %d fields exceed the %d-slot limit", nfield, kMaxSlot);
    return 0;
  }
  if (met_size && !met) {
    set_err(c, "set_solutions: metric pointer is NULL");
    return 0;
  }
  for (int j = 0; j < nfield; j++) {
    // MMG5_Scalar / MMG5_Vector / MMG5_Tensor are the only solution types at vertices
    if (!fields || !fields[j] || !(field_size[j] == 1 || field_size[j] == 3 || field_size[j] == 6)) {
      set_err(c, "set_solutions: field %d has size %d (expected 1, 3 or 6)", j, field_size ? field_size[j] : -1);
      return 0;
    }
  }
  size_t np = (size_t)c->bg.np;
  if (np == 0) {
    set_err(c, "set_solutions: call pmmg_hip_set_background first");
    return 0;
  }
  c->met_size = met_size;
  c->met_stride = met_size;
  c->nfield = nfield;
  c->fsize.assign(field_size, field_size + nfield);
  c->fstride.assign(field_size, field_size + nfield);
  c->fin.resize(nfield);
  if (where == PMMG_HIP_DEVICE) {
    c->met = met;
    for (int j = 0; j < nfield; j++) c->fin[j] = fields[j];
    return 1;
  }
  if (met_size) {
    if (!upload(c, c->o_met, met, sizeof(double) * met_size * np)) return 0;
    c->met = (const double *)c->o_met.p;
  }
  c->o_f.resize(nfield);
  for (int j = 0; j < nfield; j++) {
    if (!upload(c, c->o_f[j], fields[j], sizeof(double) * field_size[j] * np)) return 0;
    c->fin[j] = (const double *)c->o_f[j].p;
  }
  HIPCK(c, hipStreamSynchronize(c->stream));
  return 1;
}

int pmmg_hip_set_solutions_packed(pmmg_hip_ctx *c, int met_size, int met_off, int nfield, const int *field_size,
                                  const int *field_off, const double *rec, int stride, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (met_size != 0 && met_size != 1 && met_size != 6) {
    set_err(c, "set_solutions_packed: metric size %d (expected 0, 1 or 6)", met_size);
    return 0;
  }
  if (nfield < 0 || nfield + (met_size ? 1 : 0) > kMaxSlot) {
    set_err(c, "set_solutions_packed: %d fields exceed the %d-slot limit", nfield, kMaxSlot);
    return 0;
  }
  const size_t np = (size_t)c->bg.np;
  if (np == 0) {
    set_err(c, "set_solutions_packed: call pmmg_hip_set_background first");
    return 0;
  }
  if (!rec || stride <= 0 || (stride & 1) || ((uintptr_t)rec & 15)) {
    set_err(c, "set_solutions_packed: rec must be 16-byte aligned with an even stride (got %d)", stride);
    return 0;
  }
  // every column range inside the record; tensors 16-byte aligned (double2 loads)
  auto bad = [&](int size, int off) { return off < 0 || off + size > stride || (size == 6 && (off & 1)); };
  if (met_size && bad(met_size, met_off)) {
    set_err(c, "set_solutions_packed: metric columns [%d, %d) do not fit / are misaligned", met_off,
            met_off + met_size);
    return 0;
  }
  for (int j = 0; j < nfield; j++) {
    if (!field_size || !field_off || !(field_size[j] == 1 || field_size[j] == 3 || field_size[j] == 6) ||
        bad(field_size[j], field_off[j])) {
      set_err(c, "set_solutions_packed: field %d (size %d, offset %d) invalid", j, field_size ? field_size[j] : -1,
              field_off ? field_off[j] : -1);
      return 0;
    }
  }
  const double *base = rec;
  if (where != PMMG_HIP_DEVICE) {
    if (!upload(c, c->o_met, rec, sizeof(double) * (size_t)stride * np)) return 0;
    HIPCK(c, hipStreamSynchronize(c->stream));
    base = (const double *)c->o_met.p;
  }
  c->met_size = met_size;
  c->met_stride = stride;
  c->met = met_size ? base + met_off : nullptr;
  c->nfield = nfield;
  c->fsize.assign(field_size, field_size + nfield);
  c->fstride.assign(nfield, stride);
  c->fin.resize(nfield);
  for (int j = 0; j < nfield; j++) c->fin[j] = base + field_off[j];
  return 1;
}

static int grid_dim(long long n, int per_cell, int gmax) {
  double g = cbrt((double)n / (double)per_cell);
  int gi = (int)g;
  if (gi < 1) gi = 1;
  if (gi > gmax) gi = gmax;
  return gi;
}

static int blocks_for(long long n, int cap) {
  long long b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// stable compaction of the points of class cls (k_cls_*); bcnt: a per-call
// buffer of the context (one per stream that runs a compaction)
static bool class_select(pmmg_hip_ctx *c, DevBuf &bcnt, const uint8_t *pclass, long long np, int cls, int *out,
                         int *count, hipStream_t s) {
  const long long nb = np > 0 ? (np + kClsChunk - 1) / kClsChunk : 1;
  if (!ensure(c, bcnt, 4 * (size_t)nb)) return false;
  int *bc = (int *)bcnt.p;
  hipLaunchKernelGGL(k_cls_count, dim3((unsigned)nb), dim3(kBlock), 0, s, pclass, np, cls, bc);
  hipLaunchKernelGGL(k_cls_scan, dim3(1), dim3(kBlock), 0, s, bc, (int)nb, count);
  hipLaunchKernelGGL(k_cls_scatter, dim3((unsigned)nb), dim3(kBlock), 0, s, pclass, np, cls, (const int *)bc, out);
  return true;
}

// fallbacks are rare: read the two counts back and launch only what is needed
static int launch_fallbacks(pmmg_hip_ctx *c, const Slots &S, const double *xyz_new, int *elem_out, int8_t *hit_out) {
  const Bg &bg = c->bg;
  hipStream_t s = c->stream;
  DevStats *st = (DevStats *)c->stats.p;
  HIPCK(c, hipMemcpyAsync(c->h_small, &st->nfb_vol, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCK(c, hipStreamSynchronize(s));
  const int nfb_vol = c->h_small[0], nfb_bdy = c->h_small[1];
  const int fgrid = 1024;
  if (nfb_vol > 0) {
    hipLaunchKernelGGL(k_fallback_init, dim3(64), dim3(kBlock), 0, s, (int *)c->best.p, (int *)c->cidx.p,
                       (unsigned long long *)c->ckey.p, (const int *)&st->nfb_vol);
    hipLaunchKernelGGL(k_vol_exhaust_accept, dim3(fgrid), dim3(kBlock), 0, s, bg, xyz_new, (const int *)c->fb_vol.p,
                       st, (int *)c->best.p);
    for (int pass = 0; pass < 2; pass++)
      hipLaunchKernelGGL(k_vol_exhaust_closest, dim3(fgrid), dim3(kBlock), 0, s, bg, xyz_new,
                         (const int *)c->fb_vol.p, st, (const int *)c->best.p, (unsigned long long *)c->ckey.p, pass,
                         (int *)c->cidx.p);
    hipLaunchKernelGGL(k_vol_finish, dim3(64), dim3(kBlock), 0, s, bg, xyz_new, (const int *)c->fb_vol.p, st,
                       (const int *)c->best.p, (const int *)c->cidx.p, S, elem_out, hit_out);
  }
  if (bg.nt > 0 && nfb_bdy > 0) {
    hipLaunchKernelGGL(k_fallback_init, dim3(64), dim3(kBlock), 0, s, (int *)c->bbest.p, (int *)c->bcidx.p,
                       (unsigned long long *)c->bckey.p, (const int *)&st->nfb_bdy);
    for (int pass = 0; pass < 3; pass++)
      hipLaunchKernelGGL(k_bdy_exhaust, dim3(256), dim3(kBlock), 0, s, bg, xyz_new, (const int *)c->fb_bdy.p, st,
                         (int *)c->bbest.p, (unsigned long long *)c->bckey.p, pass, (int *)c->bcidx.p);
    hipLaunchKernelGGL(k_bdy_finish, dim3(64), dim3(kBlock), 0, s, bg, xyz_new, (const int *)c->fb_bdy.p, st,
                       (const int *)c->bbest.p, (const int *)c->bcidx.p, S, elem_out, hit_out);
  }
  HIPCK(c, hipGetLastError());
  return 1;
}

// default volume path: counting-sort the volume queries into a uniform grid,
// one tetra-centric scan, interpolation in cell order
static int run_scan(pmmg_hip_ctx *c, const Slots &S, int np_new, const double *xyz_new, const uint8_t *pclass,
                    int *elem_out, int8_t *hit_out, int gs) {
  const Bg &bg = c->bg;
  hipStream_t s = c->stream;
  const size_t nq = (size_t)np_new;
  const int gq = grid_dim(np_new, c->qpc, 1024);
  const long long ncells = (long long)gq * gq * gq;
  if (!ensure(c, c->cnt, 4 * (size_t)(ncells + 1)) || !ensure(c, c->off, 4 * (size_t)(ncells + 1)) ||
      !ensure(c, c->binrank, 8 * nq) || !ensure(c, c->qs, 24 * nq))
    return 0;
  Frame *fr = (Frame *)c->frame.p;
  DevStats *st = (DevStats *)c->stats.p;
  int *sgrid = (int *)c->sgrid.p;
  int *order_v = (int *)c->order_v.p, *order_b = (int *)c->order_b.p;
  int *res = (int *)c->vloc.p;
  c->last_sorted = 1;

  HIPCK(c, hipEventRecord(c->ev[0], s));
  const long long nsg = bg.nt > 0 ? (long long)gs * gs * gs : 0;
  hipLaunchKernelGGL(k_reset, dim3(blocks_for(ncells + 1 > nsg ? ncells + 1 : nsg, 2048)), dim3(kBlock), 0, s, fr, st,
                     (unsigned long long *)nullptr, 0LL, sgrid, nsg, (int *)c->cnt.p, ncells + 1, 0);
  hipLaunchKernelGGL(k_bbox, dim3(blocks_for(bg.np / c->bbox_stride + 1, 1024)), dim3(kBlock), 0, s, bg.xyz, bg.np, fr,
                     c->bbox_stride);
  hipLaunchKernelGGL(k_frame_final, dim3(1), dim3(1), 0, s, fr, 1, gs, gq, 0);
  if (bg.nt > 0) hipLaunchKernelGGL(k_seed_srf, dim3(blocks_for(bg.nt, 4096)), dim3(kBlock), 0, s, bg, fr, sgrid, gs);
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[1], s));

  size_t tb = 0;
  HIPCK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (int *)c->cnt.p, (int *)c->off.p, (int)(ncells + 1), s));
  if (!ensure(c, c->scan_tmp, tb)) return 0;
  hipLaunchKernelGGL(k_qcount, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, xyz_new, pclass, np_new, fr, gq,
                     (int *)c->cnt.p, (int2 *)c->binrank.p);
  HIPCK(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tb, (int *)c->cnt.p, (int *)c->off.p, (int)(ncells + 1), s));
  hipLaunchKernelGGL(k_qscatter, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, np_new, xyz_new,
                     (const int2 *)c->binrank.p, (const int *)c->off.p, order_v, (double *)c->qs.p, res);
  hipLaunchKernelGGL(k_qtotal, dim3(1), dim3(1), 0, s, (const int *)c->off.p, (int)ncells, st);
  if (bg.nt > 0 && !class_select(c, c->cls_cnt2, pclass, np_new, PMMG_PT_BDY, order_b, &st->nbdy, s)) return 0;
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[2], s));

  hipLaunchKernelGGL(k_vol_scan, dim3(8 * blocks_for((bg.ne + 7) / 8, 1 << 20)), dim3(kBlock), 0, s, bg, fr, gq,
                     (const int *)c->off.p, (const double *)c->qs.p, res, st);
  HIPCK(c, hipEventRecord(c->ev[6], s));
  ScanInterpFn interp = pick_layout(S).sfn;
  hipLaunchKernelGGL(interp, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, bg, (const double *)c->qs.p,
                     (const int *)order_v, (const int *)res, S, elem_out, hit_out, (int *)c->fb_vol.p, st);
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[3], s));
  const hipStream_t sb = s; // the scan path keeps everything on one stream
  c->bdy_on_s2 = false;
  HIPCK(c, hipEventRecord(c->ev[8], sb));
  if (bg.nt > 0) {
    hipLaunchKernelGGL(k_bdy, dim3(8 * blocks_for((np_new + 7) / 8, 256)), dim3(kBlock), 0, sb, bg, fr, sgrid, gs,
                       xyz_new, order_b, S, elem_out, hit_out, (int *)c->fb_bdy.p, st, c->maxstep);
    HIPCK(c, hipGetLastError());
  }
  HIPCK(c, hipEventRecord(c->ev[9], sb));
  if (c->bdy_on_s2) HIPCK(c, hipStreamWaitEvent(s, c->ev[9], 0));
  HIPCK(c, hipEventRecord(c->ev[4], s));
  if (!launch_fallbacks(c, S, xyz_new, elem_out, hit_out)) return 0;
  HIPCK(c, hipEventRecord(c->ev[5], s));
  c->pending = true;
  return 1;
}

// core pipeline on device pointers; all launches on c->stream
static int run_device(pmmg_hip_ctx *c, int np_new, const double *xyz_new, const uint8_t *pclass, double *met_out,
                      double *const *fields_out, int *elem_out, int8_t *hit_out) {
  const Bg &bg = c->bg;
  hipStream_t s = c->stream;
  Slots S{};
  S.n = 0;
  S.has_met = c->met_size ? 1 : 0;
  if (c->met_size) {
    if (!met_out) { set_err(c, "locate_interp: met_out is NULL"); return 0; }
    S.s[S.n++] = Slot{c->met, met_out, c->met_size, c->met_stride};
  }
  for (int j = 0; j < c->nfield; j++) {
    if (!fields_out || !fields_out[j]) { set_err(c, "locate_interp: fields_out[%d] is NULL", j); return 0; }
    S.s[S.n++] = Slot{c->fin[j], fields_out[j], c->fsize[j], c->fstride[j]};
  }
  const int g = grid_dim(bg.ne, c->tpc, 1024);
  const int gs = bg.nt > 0 ? grid_dim(bg.nt, 2, 512) : 1;
  int bb = 1;
  while (bb < 10 && (1LL << (3 * bb)) * c->qpb < (long long)np_new) bb++;
  const int gb = 1 << bb, nbins = 1 << (3 * bb);
  const size_t nq = (size_t)np_new;
  if (!ensure(c, c->frame, sizeof(Frame)) || !ensure(c, c->stats, sizeof(DevStats) + kStatParts * sizeof(StatPart)) ||
      !ensure(c, c->grid, 8 * (size_t)g * g * g) || !ensure(c, c->sgrid, 4 * (size_t)gs * gs * gs) ||
      !ensure(c, c->order_v, 4 * nq) || !ensure(c, c->cont, 8 * nq) ||
      !ensure(c, c->vrec, sizeof(VolLoc) * nq) || !ensure(c, c->order_b, 4 * nq) || !ensure(c, c->vloc, 4 * nq) ||
      !ensure(c, c->fb_vol, 4 * nq) || !ensure(c, c->fb_bdy, 4 * nq) || !ensure(c, c->best, 4 * nq) ||
      !ensure(c, c->ckey, 8 * nq) || !ensure(c, c->cidx, 4 * nq) || !ensure(c, c->bbest, 4 * nq) ||
      !ensure(c, c->bckey, 8 * nq) || !ensure(c, c->bcidx, 4 * nq))
    return 0;

  Frame *fr = (Frame *)c->frame.p;
  DevStats *st = (DevStats *)c->stats.p;
  unsigned long long *grid = (unsigned long long *)c->grid.p;
  int *sgrid = (int *)c->sgrid.p;
  int *order_v = (int *)c->order_v.p, *order_b = (int *)c->order_b.p;

  if (c->options & PMMG_HIP_OPT_SCAN) return run_scan(c, S, np_new, xyz_new, pclass, elem_out, hit_out, gs);

  // Query order: a 4096-point coherence sample whose 4-byte result is read
  // back while the device already builds the frame and the volume seeds (they
  // do not depend on the order); the host waits on that copy only, so the
  // GPU is not left idle across the decision.
  int sorted = 1;
  HIPCK(c, hipEventRecord(c->ev[0], s));
  const bool auto_order = !(c->options & (PMMG_HIP_OPT_NOSORT | PMMG_HIP_OPT_SORT));
  if (c->options & PMMG_HIP_OPT_NOSORT) sorted = 0;
  if (auto_order) {
    hipLaunchKernelGGL(k_coherence, dim3(1), dim3(kBlock), 0, s, xyz_new, np_new, st);
    HIPCK(c, hipMemcpyAsync(c->h_small, &st->coherent, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCK(c, hipEventRecord(c->ev[10], s));
  }

  const long long ng = (long long)g * g * g, nsg = bg.nt > 0 ? (long long)gs * gs * gs : 0;
  hipLaunchKernelGGL(k_reset, dim3(blocks_for(ng, 2048)), dim3(kBlock), 0, s, fr, st, grid, ng, sgrid, nsg, nullptr,
                     0LL, 1);
  hipLaunchKernelGGL(k_bbox, dim3(blocks_for(bg.np / c->bbox_stride + 1, 1024)), dim3(kBlock), 0, s, bg.xyz, bg.np, fr,
                     c->bbox_stride);
  hipLaunchKernelGGL(k_frame_final, dim3(1), dim3(1), 0, s, fr, g, gs, gb, c->seed8);
  HIPCK(c, hipEventRecord(c->ev[7], s)); // frame ready: the surface branch may start
  long long nsamp = (long long)c->spc * ng;
  if (nsamp > bg.ne) nsamp = bg.ne;
  hipLaunchKernelGGL(k_seed_vol, dim3((blocks_for(nsamp, c->seed_grid) + 7) & ~7), dim3(kBlock), 0, s, bg, fr, grid, g, nsamp,
                     c->seed_mode, c->seed_run, c->seed_atom);
  HIPCK(c, hipGetLastError());
  if (auto_order) {
    HIPCK(c, hipEventSynchronize(c->ev[10]));
    sorted = c->h_small[0] ? 0 : 1;
  }
  c->last_sorted = sorted;
  if (sorted) {
    if (!ensure(c, c->cnt, 4 * (size_t)2 * nbins) || !ensure(c, c->off, 4 * (size_t)2 * nbins) ||
        !ensure(c, c->binrank, 8 * nq))
      return 0;
    HIPCK(c, hipMemsetAsync(c->cnt.p, 0, 4 * (size_t)2 * nbins, s));
  }
  // The surface branch (tria seeds, surface list, k_bdy) only needs the
  // frame: on the input-order path it runs on a second stream, concurrently
  // with the volume seeds and walks (joined before the fallbacks).
  const hipStream_t sb = (!sorted && bg.nt > 0 && c->two_streams) ? c->stream2 : s;
  c->bdy_on_s2 = sb != s;
  if (c->bdy_on_s2) HIPCK(c, hipStreamWaitEvent(sb, c->ev[7], 0));
  if (bg.nt > 0) hipLaunchKernelGGL(k_seed_srf, dim3(blocks_for(bg.nt, 4096)), dim3(kBlock), 0, sb, bg, fr, sgrid, gs);
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[1], s));

  if (sorted) {
    size_t tb = 0;
    HIPCK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (int *)c->cnt.p, (int *)c->off.p, 2 * nbins, s));
    if (!ensure(c, c->scan_tmp, tb)) return 0;
    hipLaunchKernelGGL(k_bin_count, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, xyz_new, pclass, np_new, fr,
                       gb, nbins, (int *)c->cnt.p, (int2 *)c->binrank.p);
    HIPCK(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tb, (int *)c->cnt.p, (int *)c->off.p, 2 * nbins, s));
    hipLaunchKernelGGL(k_bin_scatter, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, np_new,
                       (const int2 *)c->binrank.p, (const int *)c->off.p, nbins, order_v, order_b);
    hipLaunchKernelGGL(k_bin_total, dim3(1), dim3(1), 0, s, (const int *)c->off.p, (const int *)c->cnt.p, nbins, st);
  } else {
    // stable class compaction: the surface list always (on the surface
    // branch's stream); the volume list only for the fused kernel
    // (k_vol_walk selects volume points itself)
    if ((c->options & PMMG_HIP_OPT_FUSED) &&
        !class_select(c, c->cls_cnt, pclass, np_new, PMMG_PT_VOL, order_v, &st->nvol, s))
      return 0;
    if (!class_select(c, c->cls_cnt2, pclass, np_new, PMMG_PT_BDY, order_b, &st->nbdy, sb)) return 0;
  }
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[2], s));
  c->count_nvol = !sorted && !(c->options & PMMG_HIP_OPT_FUSED);

  // surface queries (k_bdy) on the surface branch's stream
  auto launch_bdy = [&]() -> int {
    HIPCK(c, hipEventRecord(c->ev[8], sb));
    if (bg.nt > 0) {
      hipLaunchKernelGGL(k_bdy, dim3(8 * blocks_for((np_new + 7) / 8, 256)), dim3(kBlock), 0, sb, bg, fr, sgrid, gs,
                         xyz_new, order_b, S, elem_out, hit_out, (int *)c->fb_bdy.p, st, c->maxstep);
      HIPCK(c, hipGetLastError());
    }
    HIPCK(c, hipEventRecord(c->ev[9], sb));
    return 1;
  };
  // PMMG_HIP_BDYEARLY=1: enqueue k_bdy before the walk, so its blocks are
  // dispatched ahead of the walk's instead of as the walk drains
  if (c->bdy_on_s2 && c->bdy_early && !(c->options & PMMG_HIP_OPT_FUSED) && !launch_bdy()) return 0;

  if (!(c->options & PMMG_HIP_OPT_FUSED)) {
    // PMMG_HIP_WALKB=64: one-wave blocks (LDS slots then cap occupancy at
    // 26 instead of 24 waves per CU)
    const bool wb64 = c->carry == 2 && c->walkb == 64;
    auto walk = wb64 ? k_vol_walk<2, 1, 64>
                : c->carry == 2 ? (c->walkw >= 5 ? k_vol_walk<2, 5> : k_vol_walk<2, 1>)
                : c->carry    ? (c->walkw >= 5 ? k_vol_walk<1, 5> : k_vol_walk<1, 1>)
                              : (c->walkw >= 5 ? k_vol_walk<0, 5> : k_vol_walk<0, 1>);
    const LayoutEntry &lay = pick_layout(S);
    // PMMG_HIP_INTERPB=64: the half-image interpolation in one-wave blocks
    const bool ib64 = c->coop == 2 && lay.hfn64 && c->interpb == 64;
    VolInterpFn interp = ib64 ? lay.hfn64
                         : (c->coop == 2 && lay.hfn) ? lay.hfn : (c->coop && lay.cfn) ? lay.cfn : lay.fn;
    const int ib = ib64 ? 64 : kBlock;
    const VRec vr = vrec_arrays(c->vrec.p, (size_t)np_new);
    // Pipelined volume stage: the queries are cut into `nch` contiguous
    // chunks; the interpolation of chunk j (bandwidth-bound) runs on stream3
    // while the walk of chunk j+1 (latency-bound) runs on the main stream, so
    // the interpolation's traffic fills the walk's idle memory slots.  The
    // input-order path only (the Morton-binned walk is indexed by bin order).
    const bool capped = c->cap < c->maxstep;
    const int nch = (!sorted && !capped && c->chunks > 1) ? c->chunks : 1;
    const long long per = ((long long)np_new + nch - 1) / nch;
    const int chunk = (int)((per + kBlock - 1) / kBlock * kBlock);
    for (int j = 0; j < nch; j++) {
      const int a = j * chunk, n = np_new - a < chunk ? np_new - a : chunk;
      if (n <= 0) break;
      const int np_j = nch > 1 ? a + n : np_new; // lanes at or past np_j are idle
      hipLaunchKernelGGL(walk, dim3(wb64 ? (n + 63) / 64 : blocks_for(n, 1 << 30)), dim3(wb64 ? 64 : kBlock), 0, s,
                         bg, fr, grid, g, xyz_new, pclass,
                         sorted ? (const int *)order_v : nullptr, np_j, (int *)c->vloc.p, vr, (int *)c->fb_vol.p,
                         (ContEntry *)c->cont.p, st, c->cap, c->maxstep, a);
      if (nch > 1) {
        HIPCK(c, hipEventRecord(c->evc[j], s));
        HIPCK(c, hipStreamWaitEvent(c->stream3, c->evc[j], 0));
        hipLaunchKernelGGL(interp, dim3((n + ib - 1) / ib), dim3(ib), 0, c->stream3, pclass, np_j,
                           (const int *)c->vloc.p, vr, S, elem_out, hit_out, a);
      }
    }
    if (capped) // continuation pass only when capping is enabled
      hipLaunchKernelGGL(k_vol_walk_cont, dim3(8 * blocks_for((np_new + 7) / 8, 1 << 20)), dim3(kBlock), 0, s, bg,
                         xyz_new, (int *)c->vloc.p, vr, (int *)c->fb_vol.p, (const ContEntry *)c->cont.p, st, c->cap,
                         c->maxstep);
    HIPCK(c, hipEventRecord(c->ev[6], s));
    if (nch > 1) {
      HIPCK(c, hipEventRecord(c->evc[nch - 1], c->stream3));
      HIPCK(c, hipStreamWaitEvent(s, c->evc[nch - 1], 0));
    } else {
      hipLaunchKernelGGL(interp, dim3((np_new + ib - 1) / ib), dim3(ib), 0, s, pclass, np_new,
                         (const int *)c->vloc.p, vr, S, elem_out, hit_out, 0);
    }
  } else {
    FusedFn fused = pick_layout(S).ffn;
    hipLaunchKernelGGL(fused, dim3(blocks_for(np_new, 1 << 30)), dim3(kBlock), 0, s, bg, fr, grid, g, xyz_new,
                       order_v, S, elem_out, hit_out, (int *)c->fb_vol.p, st, c->maxstep);
    HIPCK(c, hipEventRecord(c->ev[6], s));
  }
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipEventRecord(c->ev[3], s));
  const bool bdy_early = c->bdy_on_s2 && c->bdy_early && !(c->options & PMMG_HIP_OPT_FUSED);
  if (!bdy_early && !launch_bdy()) return 0;
  if (c->bdy_on_s2) HIPCK(c, hipStreamWaitEvent(s, c->ev[9], 0));
  HIPCK(c, hipEventRecord(c->ev[4], s));

  if (!launch_fallbacks(c, S, xyz_new, elem_out, hit_out)) return 0;
  HIPCK(c, hipEventRecord(c->ev[5], s));
  c->pending = true;
  return 1;
}

static int collect_stats(pmmg_hip_ctx *c, pmmg_hip_stats *out) {
  DevStats h;
  std::vector<StatPart> parts(kStatParts);
  HIPCK(c, hipMemcpy(&h, c->stats.p, sizeof(DevStats), hipMemcpyDeviceToHost));
  HIPCK(c, hipMemcpy(parts.data(), (const DevStats *)c->stats.p + 1, kStatParts * sizeof(StatPart),
                     hipMemcpyDeviceToHost));
  for (const StatPart &pt : parts) {
    for (int j = 0; j < 16; j++) h.cnt[j] += pt.cnt[j];
    h.steps += pt.steps;
    if (pt.stepmax > h.stepmax) h.stepmax = (unsigned)pt.stepmax;
  }
  memset(out, 0, sizeof(*out));
  out->nvol = c->count_nvol ? (int64_t)h.cnt[PMMG_HIT_VOL_WALK] + h.nfb_vol : h.nvol;
  out->nbdy = h.nbdy;
  out->nvol_walk = (int64_t)h.cnt[PMMG_HIT_VOL_WALK];
  out->nvol_exhaust = (int64_t)h.cnt[PMMG_HIT_VOL_EXHAUST];
  out->nvol_closest = (int64_t)h.cnt[PMMG_HIT_VOL_CLOSEST];
  out->nvol_scan = (int64_t)h.cnt[PMMG_HIT_VOL_SCAN];
  out->nbdy_face = (int64_t)h.cnt[PMMG_HIT_BDY_FACE];
  out->nbdy_edge = (int64_t)h.cnt[PMMG_HIT_BDY_EDGE];
  out->nbdy_vertex = (int64_t)h.cnt[PMMG_HIT_BDY_VERTEX];
  out->nbdy_wedge = (int64_t)h.cnt[PMMG_HIT_BDY_WEDGE];
  out->nbdy_cone = (int64_t)h.cnt[PMMG_HIT_BDY_CONE];
  out->nbdy_exhaust = (int64_t)h.cnt[PMMG_HIT_BDY_EXHAUST];
  out->nbdy_stale = (int64_t)h.cnt[PMMG_HIT_BDY_STALE];
  out->nbdy_closest = (int64_t)h.cnt[PMMG_HIT_BDY_CLOSEST];
  out->steps_total = (int64_t)h.steps;
  out->stepmax = (int64_t)h.stepmax;
  out->sorted = c->last_sorted;
  float ms = 0.f;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
  out->ms_prepare = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
  out->ms_sort = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
  out->ms_vol = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[2], c->ev[6]));
  out->ms_vol_locate = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[8], c->ev[9]));
  out->ms_bdy = ms; // on the surface stream when it ran concurrently
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[4], c->ev[5]));
  out->ms_fallback = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[5]));
  out->ms_total = ms;
  return 1;
}

int pmmg_hip_sync(pmmg_hip_ctx *c, pmmg_hip_stats *stats) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  HIPCK(c, hipStreamSynchronize(c->stream));
  if (stats && c->pending) return collect_stats(c, stats);
  return 1;
}

int pmmg_hip_locate_interp(pmmg_hip_ctx *c, int np_new, const double *xyz_new, const uint8_t *pclass,
                           double *met_out, double *const *fields_out, int *elem_out, int8_t *hit_out,
                           pmmg_hip_stats *stats, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (c->bg.ne <= 0) { set_err(c, "locate_interp: no background set"); return 0; }
  if (np_new <= 0) {
    if (stats) memset(stats, 0, sizeof(*stats));
    return 1;
  }
  if (!xyz_new || !pclass) { set_err(c, "locate_interp: xyz_new / pclass is NULL"); return 0; }
  if (where == PMMG_HIP_DEVICE) {
    if (!run_device(c, np_new, xyz_new, pclass, met_out, fields_out, elem_out, hit_out)) return 0;
    if (stats) return pmmg_hip_sync(c, stats);
    return 1;
  }
  // host mode: stage inputs and the current output arrays (rows that are not
  // interpolated stay untouched), run, copy back
  size_t n = (size_t)np_new;
  if (!upload(c, c->h_xyz, xyz_new, sizeof(double) * 3 * n)) return 0;
  if (!upload(c, c->h_cls, pclass, n)) return 0;
  double *dmet = nullptr;
  if (c->met_size) {
    if (!met_out) { set_err(c, "locate_interp: met_out is NULL"); return 0; }
    if (!upload(c, c->h_met, met_out, sizeof(double) * c->met_size * n)) return 0;
    dmet = (double *)c->h_met.p;
  }
  c->h_f.resize(c->nfield);
  std::vector<double *> dfields(c->nfield > 0 ? c->nfield : 1, nullptr);
  for (int j = 0; j < c->nfield; j++) {
    if (!fields_out || !fields_out[j]) { set_err(c, "locate_interp: fields_out[%d] is NULL", j); return 0; }
    if (!upload(c, c->h_f[j], fields_out[j], sizeof(double) * c->fsize[j] * n)) return 0;
    dfields[j] = (double *)c->h_f[j].p;
  }
  int *delem = nullptr;
  int8_t *dhit = nullptr;
  if (elem_out) {
    if (!upload(c, c->h_elem, elem_out, sizeof(int) * n)) return 0;
    delem = (int *)c->h_elem.p;
  }
  if (hit_out) {
    if (!upload(c, c->h_hit, hit_out, n)) return 0;
    dhit = (int8_t *)c->h_hit.p;
  }
  if (!run_device(c, np_new, (const double *)c->h_xyz.p, (const uint8_t *)c->h_cls.p, dmet, dfields.data(), delem, dhit))
    return 0;
  if (dmet) HIPCK(c, hipMemcpyAsync(met_out, dmet, sizeof(double) * c->met_size * n, hipMemcpyDeviceToHost, c->stream));
  for (int j = 0; j < c->nfield; j++)
    HIPCK(c, hipMemcpyAsync(fields_out[j], dfields[j], sizeof(double) * c->fsize[j] * n, hipMemcpyDeviceToHost,
                            c->stream));
  if (delem) HIPCK(c, hipMemcpyAsync(elem_out, delem, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  if (dhit) HIPCK(c, hipMemcpyAsync(hit_out, dhit, n, hipMemcpyDeviceToHost, c->stream));
  HIPCK(c, hipStreamSynchronize(c->stream));
  if (stats) return collect_stats(c, stats);
  return 1;
}

// ---- background snapshot (pmmg_snapshot.hip)

static bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int pmmg_hip_build_adjacency(pmmg_hip_ctx *c, int np, int ne, const int *tetv, int *adja, int *tet8) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (np <= 0 || ne <= 0 || !tetv || (!adja && !tet8)) {
    set_err(c, "build_adjacency: invalid arguments (np=%d ne=%d)", np, ne);
    return 0;
  }
  if (ne >= (1 << 29)) {
    set_err(c, "build_adjacency: %d tetra exceed the 4*k+i adjacency encoding (2^29)", ne);
    return 0;
  }
  if (!aligned16(tetv) || (adja && !aligned16(adja)) || (tet8 && !aligned16(tet8))) {
    set_err(c, "build_adjacency: device arrays must be 16-byte aligned");
    return 0;
  }
  return pmmg_snap_adjacency(c->stream, np, ne, tetv, adja, tet8, c->err, sizeof(c->err));
}

int pmmg_hip_tetra_qual(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, int met_size,
                        const double *met, double *qual, double *minqual) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (np < 0 || ne < 0 || (ne > 0 && (!xyz || !tetv || !qual)) || !minqual ||
      (met_size == 6 && ne > 0 && !met) || (met_size != 0 && met_size != 1 && met_size != 6)) {
    set_err(c, "tetra_qual: invalid arguments (np=%d ne=%d met_size=%d)", np, ne, met_size);
    return 0;
  }
  if (ne > 0 && !aligned16(tetv)) {
    set_err(c, "tetra_qual: tetv must be 16-byte aligned");
    return 0;
  }
  if (!ensure(c, c->qmin, sizeof(unsigned long long))) return 0;
  unsigned long long bits = 0;
  if (!pmmg_qual_tetra(c->stream, np, xyz, ne, tetv, met_size, met, qual, (unsigned long long *)c->qmin.p, &bits)) {
    set_err(c, "tetra_qual: kernel launch or copy failed");
    return 0;
  }
  // MMG3D_tetraQual: minqual starts at 2/ALPHAD, returns ALPHAD * minqual
  const double alphad = 20.7846096908265; // MMG3D_ALPHAD = 12 sqrt(3): a regular tetra has quality 1
  double mn = 2.0 / alphad;
  if (bits != ~0ULL) {
    double q;
    memcpy(&q, &bits, sizeof q);
    if (q < mn) mn = q;
  }
  *minqual = alphad * mn;
  return 1;
}

int pmmg_hip_build_boundary(pmmg_hip_ctx *c, int np, int ne, const int *tet8, const int *tetv, const int *adja,
                            int cap, int *nt, int *triv, int *adjt) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  const bool packed = tet8 != nullptr;
  if (np <= 0 || ne <= 0 || !nt || (!packed && (!tetv || !adja)) || cap < 0 || (cap > 0 && !triv)) {
    set_err(c, "build_boundary: invalid arguments (np=%d ne=%d cap=%d)", np, ne, cap);
    return 0;
  }
  const int *t0 = packed ? tet8 : tetv, *a0 = packed ? tet8 + 4 : adja;
  if (!aligned16(t0) || !aligned16(a0)) {
    set_err(c, "build_boundary: device tetra arrays must be 16-byte aligned");
    return 0;
  }
  return pmmg_snap_boundary(c->stream, np, ne, t0, packed ? 2 : 1, a0, packed ? 2 : 1, cap, nt, triv, adjt, c->err,
                            sizeof(c->err));
}

void *pmmg_hip_malloc(pmmg_hip_ctx *c, int64_t bytes) {
  if (!c || bytes < 0) return nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return nullptr;
  void *p = nullptr;
  if (hipMalloc(&p, bytes > 0 ? (size_t)bytes : 16) != hipSuccess) {
    set_err(c, "hipMalloc(%lld) failed", (long long)bytes);
    return nullptr;
  }
  return p;
}

int pmmg_hip_free(pmmg_hip_ctx *c, void *p) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  HIPCK(c, hipFree(p));
  return 1;
}

int pmmg_hip_memcpy_h2d(pmmg_hip_ctx *c, void *dst, const void *src, int64_t bytes) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  HIPCK(c, hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
  HIPCK(c, hipStreamSynchronize(c->stream));
  return 1;
}

int pmmg_hip_memcpy_d2h(pmmg_hip_ctx *c, void *dst, const void *src, int64_t bytes) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  HIPCK(c, hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCK(c, hipStreamSynchronize(c->stream));
  return 1;
}

} // extern "C"
