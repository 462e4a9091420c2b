// pmmg_fallback.hpp — exhaustive searches with the reference's semantics
// (included by pmmg_hip.hip only):
//   volume:  PMMG_locatePoint_exhaustTetra (locate_pmmg.c:737-770): the
//            lowest-index accepting tetra, else the closest tetra (argmin
//            |bary_min| * vol, :453-458) and its nearest vertex
//            (PMMG_barycoord3d_getClosest, barycoord_pmmg.c:371-404)
//   surface: PMMG_locatePoint_exhaustTria (locate_pmmg.c:477-515): the
//            lowest-index accepting tria, else the closest tria by centroid
//            distance with the stale re-evaluation of :505-509
// The query lists and their counts are produced on the device by the walks;
// every kernel here reads the count itself and returns at once when its list
// is empty, so the host launches them unconditionally (no read-back).
//
// Two launches per class (r05; r04's merged scan issued one contended global
// atomicMin per (element, query) pair and took a carried ParMmg iteration
// from 0.24 to 6.7 s):
//   accept   element-major: each thread holds one element and its bounding
//            box inflated past what the acceptance test can pass, and tests
//            the queries of the list in the grid cells the box covers (a
//            grid over the list built when the list is complete); only the
//            few pairs inside the box run the reference's test (one atomicMin
//            per accepting pair).  The last block interpolates the accepted
//            queries and lists the others.
//   closest  query-major, only for the queries nothing accepted (points
//            outside the domain): elements staged in LDS tiles, every lane
//            keeps its query's running (key, index) minimum over a range of
//            elements in index order (several lanes per query when the list
//            is short), the ranges' minima merged in the last block, which
//            interpolates.  No global atomics per pair.
#pragma once

#include "pmmg_prep.hpp"

namespace pmmg {

constexpr int kFbGridVol = 1024; // blocks of the volume exhaustive kernels (fixed: the counts are on the device)
constexpr int kFbGridBdy = 256;  // blocks of the surface ones (trias: ~1-2 % of the tetra)

// one range's closest element of one query (closest scans with several ranges)
struct FbPart {
  double key;
  int idx;
  int pad;
};
constexpr long long kFbPartCap = 256LL * kFbGridVol; // FbPart entries per class (see ClosestSplit)

// distance from x to the tria's centroid, in the arithmetic of the closest
// tria search (locate_pmmg.c:400-416): x - sum_v p_v / 3, component by component
__device__ __forceinline__ double centroid_dist3(const double *x, const double (*p)[3]) {
  double d[3] = {x[0], x[1], x[2]};
  for (int v = 0; v < 3; v++)
    for (int c = 0; c < 3; c++) d[c] -= p[v][c] / 3.0;
  double nrm = 0;
  for (int c = 0; c < 3; c++) nrm += d[c] * d[c];
  return sqrt(nrm);
}

// per-block hit counters of a finishing last block, flushed once
__device__ __forceinline__ void count_hits_flush(unsigned *cnt, DevStats *st, int h0, int h1) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (cnt[0]) atomicAdd(&stat_part(st)->cnt[h0], (unsigned long long)cnt[0]);
    if (cnt[1]) atomicAdd(&stat_part(st)->cnt[h1], (unsigned long long)cnt[1]);
  }
}

// lowest-index tetra accepting each fallback query (locate_pmmg.c:743-762),
// each tetra tested against the queries of the grid cells its inflated box
// covers; the last block interpolates the accepted ones and lists the others
// (nac)
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_accept(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                               int *best, int *nac, const int *gcells,
                                                               const int *gitems, Slots S, int *elem_out,
                                                               int8_t *hit_out) {
  const int nfb = st->nfb_vol;
  if (nfb == 0) return;
  const XcdChunk ch = xcd_chunk(bg.ne); // each XCD a contiguous eighth of the tetra (shared vertex rows in its L2)
  for (int it = 0; it < ch.iters; it++) {
    const long long j0 = ch.start + it * ch.stride;
    if (j0 >= ch.hi) break;
    const int k = (int)(j0 + 1);
    const int4 tv = tetv_row(bg, k);
    if (tv.x <= 0) continue;
    double p[4][3];
    load_pt(bg.xyz, tv.x, p[0]);
    load_pt(bg.xyz, tv.y, p[1]);
    load_pt(bg.xyz, tv.z, p[2]);
    load_pt(bg.xyz, tv.w, p[3]);
    const double vol = orvol4(p[0], p[1], p[2], p[3]);
    const Box box = elem_box<4>(p, 0.0, !(fabs(vol) > 0.0) || !isfinite(vol));
    fb_grid_visit(st, 0, gcells, gitems, box, [&](int j) {
      double x[3];
      load_pt(qxyz, fb[j], x);
      if (!in_box(box, x) || best[j] <= k) return; // (a stale read only costs a test)
      double b4[4];
      tet_bary(x, p[0], p[1], p[2], p[3], b4);
      if (min4(b4) > -kEps) atomicMin(&best[j], k);
    });
  }
  if (!last_block(&st->fb_done[0], true)) return; // (only when there are fallbacks)
  __shared__ int s_nac;
  __shared__ unsigned s_cnt[2];
  if (threadIdx.x == 0) {
    s_nac = 0;
    s_cnt[0] = s_cnt[1] = 0u;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nfb; j += blockDim.x) {
    const int k = load_agent(&best[j]);
    if (k == INT_MAX) {
      nac[atomicAdd(&s_nac, 1)] = j;
      continue;
    }
    const int ip = fb[j];
    double x[3], p[4][3], phi[4];
    load_pt(qxyz, ip, x);
    const int4 tv = tetv_row(bg, k);
    load_pt(bg.xyz, tv.x, p[0]);
    load_pt(bg.xyz, tv.y, p[1]);
    load_pt(bg.xyz, tv.z, p[2]);
    load_pt(bg.xyz, tv.w, p[3]);
    tet_bary(x, p[0], p[1], p[2], p[3], phi);
    const int v[4] = {tv.x, tv.y, tv.z, tv.w};
    for (int s = 0; s < S.n; s++) interp_dyn<4>(S.s[s], ip, v, phi);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)PMMG_HIT_VOL_EXHAUST;
    atomicAdd(&s_cnt[0], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) st->nac_vol = s_nac;
  count_hits_flush(s_cnt, st, PMMG_HIT_VOL_EXHAUST, PMMG_HIT_VOL_EXHAUST);
}

// surface: the lowest-index accepting tria (locate_pmmg.c:483-503), each tria
// against the queries of the grid cells its inflated box covers; the last
// block interpolates the accepted queries and lists the others
__global__ __launch_bounds__(kBlock) void k_bdy_exhaust_accept(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                               int *best, int *nac, const int *gcells,
                                                               const int *gitems, Slots S, int *elem_out,
                                                               int8_t *hit_out) {
  const int nfb = st->nfb_bdy;
  if (nfb == 0) return;
  const XcdChunk ch = xcd_chunk(bg.nt);
  for (int it = 0; it < ch.iters; it++) {
    const long long j0 = ch.start + it * ch.stride;
    if (j0 >= ch.hi) break;
    const int k = (int)(j0 + 1);
    if (bg.triv[3 * (size_t)(k - 1)] <= 0) continue;
    TriGeom t;
    tri_load(bg, k, t);
    const Box box = elem_box<3>(t.p, bg.hausd, !(t.q > 0.0) || !isfinite(t.q));
    fb_grid_visit(st, 1, gcells, gitems, box, [&](int j) {
      double x[3];
      load_pt(qxyz, fb[j], x);
      if (!in_box(box, x) || best[j] <= k) return;
      double b3[3];
      const double dist = tri_bary(x, t.p, t.q, t.n, b3);
      const double bmin = fmin(b3[0], fmin(b3[1], b3[2]));
      if (bmin > -kEps && !(fabs(dist) > bg.hausd)) atomicMin(&best[j], k);
    });
  }
  if (!last_block(&st->fb_done[2], true)) return; // (only when there are fallbacks)
  __shared__ int s_nac;
  __shared__ unsigned s_cnt[2];
  if (threadIdx.x == 0) {
    s_nac = 0;
    s_cnt[0] = s_cnt[1] = 0u;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nfb; j += blockDim.x) {
    const int k = load_agent(&best[j]);
    if (k == INT_MAX) {
      nac[atomicAdd(&s_nac, 1)] = j;
      continue;
    }
    const int ip = fb[j];
    double x[3], phi[3];
    load_pt(qxyz, ip, x);
    TriGeom t;
    tri_load(bg, k, t);
    tri_bary(x, t.p, t.q, t.n, phi);
    interp_bdy(S, ip, t.v, phi, -1, -1);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)PMMG_HIT_BDY_EXHAUST;
    atomicAdd(&s_cnt[0], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) st->nac_bdy = s_nac;
  count_hits_flush(s_cnt, st, PMMG_HIT_BDY_EXHAUST, PMMG_HIT_BDY_EXHAUST);
}

// ---------------------------------------------------------------- closest scans

// How a closest scan deals n queries to a grid of G blocks of 256 lanes:
// groups of Qp queries (Qp = 256, or the next power of two >= n for a short
// list, whose queries then get lpq = 256 / Qp lanes each, every lane taking
// every lpq-th element of a tile), and per group nr ranges of consecutive
// elements (one block each).  n * nr <= G * 256 (= kFbPartCap for the
// volume grid), the partial minima's buffer.
struct ClosestSplit {
  int Qp, lpq, nqg, nr;
};
__device__ __forceinline__ ClosestSplit closest_split(int n, int G) {
  ClosestSplit s;
  if (n >= kBlock) {
    s.Qp = kBlock;
    s.lpq = 1;
    s.nqg = (n + kBlock - 1) / kBlock;
  } else {
    s.Qp = 1;
    while (s.Qp < n) s.Qp <<= 1;
    s.lpq = kBlock / s.Qp;
    s.nqg = 1;
  }
  s.nr = s.nqg >= G ? 1 : G / s.nqg;
  return s;
}

// (key, index) order of the closest searches: the lowest index at the minimum
// key, starting from (1e10, index 0); a NaN key never wins.  This is the
// reference's exhaustive scan on its own (it keeps the first element strictly
// closer while scanning in index order, src/locate_pmmg.c:753-765) but not its
// whole rule: the reference seeds closestDist / closestTet with what its walk
// met (:800-815, :864) and skips the walk's visited tetra (:753), so on an
// exact key tie between a walked element and a lower-index one it returns the
// walked one.  Listed as a known divergence (ties of the closest
// metric are broken by lowest index); only exact ties of |min bary| * vol
// for points outside every element can differ.
__device__ __forceinline__ bool key_before(double ka, int ia, double kb, int ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// The closest element (NV = 4: tetra, key |bary_min| * vol; NV = 3: tria,
// key centroid distance) of each query of the list nac[0, n), by ranges.
// Returns (in the block's lanes with sub == 0) the range's minimum of query
// qi; the caller stores it.
template <int NV>
__device__ __forceinline__ void closest_range(const Bg &bg, const double *x, bool active, int lpq, int sub, int k0,
                                              int k1, double &bkey, int &bidx, double (*tp)[3 * NV], int *tk) {
  constexpr int kTile = kBlock;
  for (int t0 = k0; t0 < k1; t0 += kTile) {
    __syncthreads();
    {
      const int k = t0 + (int)threadIdx.x;
      int kk = 0;
      if (k < k1) {
        if constexpr (NV == 4) {
          const int4 tv = tetv_row(bg, k);
          if (tv.x > 0) {
            kk = k;
            load_pt(bg.xyz, tv.x, &tp[threadIdx.x][0]);
            load_pt(bg.xyz, tv.y, &tp[threadIdx.x][3]);
            load_pt(bg.xyz, tv.z, &tp[threadIdx.x][6]);
            load_pt(bg.xyz, tv.w, &tp[threadIdx.x][9]);
          }
        } else {
          const int *tv = bg.triv + 3 * (size_t)(k - 1);
          if (tv[0] > 0) {
            kk = k;
            load_pt(bg.xyz, tv[0], &tp[threadIdx.x][0]);
            load_pt(bg.xyz, tv[1], &tp[threadIdx.x][3]);
            load_pt(bg.xyz, tv[2], &tp[threadIdx.x][6]);
          }
        }
      }
      tk[threadIdx.x] = kk;
    }
    __syncthreads();
    if (!active) continue;
    const int nt = min(kTile, k1 - t0);
    for (int t = sub; t < nt; t += lpq) {
      const int k = tk[t];
      if (k == 0) continue;
      double p[NV][3];
#pragma unroll
      for (int v = 0; v < NV; v++)
#pragma unroll
        for (int c = 0; c < 3; c++) p[v][c] = tp[t][3 * v + c];
      double key;
      if constexpr (NV == 4) {
        double b[4];
        const double vol = tet_bary(x, p[0], p[1], p[2], p[3], b);
        key = fabs(min4(b)) * vol;
      } else {
        key = centroid_dist3(x, p);
      }
      if (key < bkey) { // index order within a lane: strict, as the reference
        bkey = key;
        bidx = k;
      }
    }
  }
}

// the closest scan's body shared by the two classes: every block's groups
// and ranges, the lanes of a query merged in LDS, the range minima stored
// (part) or, with one range, the result itself (res)
template <int NV>
__device__ __forceinline__ void closest_scan(const Bg &bg, const double *qxyz, const int *fb, const int *nac, int n,
                                             int nelem, FbPart *part, int *res) {
  __shared__ double tp[kBlock][3 * NV];
  __shared__ int tk[kBlock];
  __shared__ double mk[kBlock];
  __shared__ int mi[kBlock];
  const ClosestSplit sp = closest_split(n, (int)gridDim.x);
  const int qsub = (int)threadIdx.x % sp.Qp, sub = (int)threadIdx.x / sp.Qp;
  const int nwork = sp.nqg * sp.nr;
  for (int w = blockIdx.x; w < nwork; w += gridDim.x) {
    const int g = w % sp.nqg, r = w / sp.nqg;
    const int qi = g * sp.Qp + qsub;
    const bool active = qi < n;
    double x[3] = {0.0, 0.0, 0.0};
    if (active) load_pt(qxyz, fb[nac[qi]], x);
    const int k0 = 1 + (int)((long long)nelem * r / sp.nr), k1 = 1 + (int)((long long)nelem * (r + 1) / sp.nr);
    double bkey = 1.0e10;
    int bidx = 0;
    closest_range<NV>(bg, x, active, sp.lpq, sub, k0, k1, bkey, bidx, tp, tk);
    if (sp.lpq > 1) {
      __syncthreads();
      mk[threadIdx.x] = bkey;
      mi[threadIdx.x] = bidx;
      __syncthreads();
      if (sub == 0)
        for (int s = 1; s < sp.lpq; s++) {
          const int o = qsub + s * sp.Qp;
          if (key_before(mk[o], mi[o], bkey, bidx)) {
            bkey = mk[o];
            bidx = mi[o];
          }
        }
    }
    if (active && sub == 0) {
      if (sp.nr == 1) res[qi] = bidx;
      else part[(long long)r * (sp.nqg * sp.Qp) + qi] = FbPart{bkey, bidx, 0};
    }
  }
}

// the last block: query qi's closest element over the ranges
__device__ __forceinline__ int closest_result(int qi, int n, const FbPart *part, const int *res) {
  const ClosestSplit sp = closest_split(n, (int)gridDim.x);
  if (sp.nr == 1) return load_agent(&res[qi]);
  double bkey = 1.0e10;
  int bidx = 0;
  for (int r = 0; r < sp.nr; r++) { // ranges in index order
    const FbPart e = part[(long long)r * (sp.nqg * sp.Qp) + qi];
    if (key_before(e.key, e.idx, bkey, bidx)) {
      bkey = e.key;
      bidx = e.idx;
    }
  }
  return bidx;
}

// closest tetra of the queries nothing accepted, then (last block) their
// nearest vertex (PMMG_barycoord3d_getClosest) and interpolation
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_closest(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                                const int *nac, FbPart *part, int *res, Slots S,
                                                                int *elem_out, int8_t *hit_out) {
  const int n = st->nac_vol;
  if (n == 0) return;
  closest_scan<4>(bg, qxyz, fb, nac, n, bg.ne, part, res);
  if (!last_block(&st->fb_done[1], true)) return; // (only when there are fallbacks)
  __shared__ unsigned s_cnt[2];
  if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0u;
  __syncthreads();
  for (int qi = threadIdx.x; qi < n; qi += blockDim.x) {
    const int k = closest_result(qi, n, part, res);
    if (k <= 0) continue; // no element closer than the reference's 1e10 start
    const int ip = fb[nac[qi]];
    double x[3], p[4][3], phi[4];
    load_pt(qxyz, ip, x);
    const int4 tv = tetv_row(bg, k);
    load_pt(bg.xyz, tv.x, p[0]);
    load_pt(bg.xyz, tv.y, p[1]);
    load_pt(bg.xyz, tv.z, p[2]);
    load_pt(bg.xyz, tv.w, p[3]);
    closest_vertex<4>(x, p, phi);
    const int v[4] = {tv.x, tv.y, tv.z, tv.w};
    for (int s = 0; s < S.n; s++) interp_dyn<4>(S.s[s], ip, v, phi);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)PMMG_HIT_VOL_CLOSEST;
    atomicAdd(&s_cnt[0], 1u);
  }
  count_hits_flush(s_cnt, st, PMMG_HIT_VOL_CLOSEST, PMMG_HIT_VOL_CLOSEST);
}

// closest tria (centroid distance) of the surface queries nothing accepted,
// then (last block) the reference's stale re-evaluation (locate_pmmg.c:505-509:
// vertices and area of the last tria scanned, nt, with the closest tria's
// normal) or its nearest vertex, and the interpolation
__global__ __launch_bounds__(kBlock) void k_bdy_exhaust_closest(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                                const int *nac, FbPart *part, int *res, Slots S,
                                                                int *elem_out, int8_t *hit_out) {
  const int n = st->nac_bdy;
  if (n == 0) return;
  closest_scan<3>(bg, qxyz, fb, nac, n, bg.nt, part, res);
  if (!last_block(&st->fb_done[3], true)) return; // (only when there are fallbacks)
  __shared__ unsigned s_cnt[2];
  if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0u;
  __syncthreads();
  for (int qi = threadIdx.x; qi < n; qi += blockDim.x) {
    const int k = closest_result(qi, n, part, res);
    if (k <= 0) continue;
    const int ip = fb[nac[qi]];
    double x[3], phi[3];
    load_pt(qxyz, ip, x);
    TriGeom t, ts;
    tri_load(bg, k, t);
    tri_load(bg, bg.nt, ts);
    double b[3];
    const double dist = tri_bary(x, ts.p, ts.q, t.n, b);
    const double bmin = fmin(b[0], fmin(b[1], b[2]));
    int hit;
    if (bmin > -kEps && !(fabs(dist) > bg.hausd)) {
      hit = PMMG_HIT_BDY_STALE;
      phi[0] = b[0];
      phi[1] = b[1];
      phi[2] = b[2];
    } else {
      hit = PMMG_HIT_BDY_CLOSEST;
      closest_vertex<3>(x, t.p, phi);
    }
    interp_bdy(S, ip, t.v, phi, -1, -1);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)hit;
    atomicAdd(&s_cnt[hit == PMMG_HIT_BDY_STALE ? 1 : 0], 1u);
  }
  count_hits_flush(s_cnt, st, PMMG_HIT_BDY_CLOSEST, PMMG_HIT_BDY_STALE);
}

} // namespace pmmg
