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
#pragma once

#include "pmmg_prep.hpp"

namespace pmmg {

constexpr int kQB = 128; // fallback queries staged in LDS per pass

// distance from x to the tria's centroid, in the arithmetic of the closest
// tria search (locate_pmmg.c:400-416): x - sum_v p_v / 3, component by component
__device__ __forceinline__ double centroid_dist(const double *x, const TriGeom &t) {
  double d[3] = {x[0], x[1], x[2]};
  for (int v = 0; v < 3; v++)
    for (int c = 0; c < 3; c++) d[c] -= t.p[v][c] / 3.0;
  double nrm = 0;
  for (int c = 0; c < 3; c++) nrm += d[c] * d[c];
  return sqrt(nrm);
}

// Exhaustive searches of the queries the walks did not settle, in two
// launches per class: a scan over every element gives each query its
// lowest-index accepting element (best) and its closest key (ckey); a second
// scan finds the lowest index at that key (cidx) for the queries nothing
// accepted, and the last block to finish it interpolates every query of the
// list (r04: the scan passes and the finish were four launches; a small
// group's step is a chain of ~20 launches of a few microseconds each).

// the last block of a grid to pass this point (after its device-scope
// atomics) gets true: the other blocks' results are then visible to it.  The
// barrier before the ticket: every wave of the block has issued its atomics
// (r04l: without it a block's later waves could still be scanning when the
// last block read the results — 4 surface points left unprocessed, once)
__device__ __forceinline__ bool last_block(unsigned *done) {
  __threadfence();
  __syncthreads();
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last) __threadfence();
  return last;
}

// lowest-index tetra accepting each fallback query (locate_pmmg.c:743-762)
// and the closest tetra's key, argmin |bary_min| * vol (:453-458)
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_scan(Bg bg, const double *qxyz, const int *fb,
                                                             const DevStats *st, int *best, unsigned long long *ckey) {
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
      for (int j = 0; j < nq; j++) {
        double b[4];
        const double vol = tet_bary(sx[j], p0, p1, p2, p3, b);
        const double bmin = min4(b);
        if (bmin > -kEps && best[q0 + j] > k) atomicMin(&best[q0 + j], k);
        atomicMin(&ckey[q0 + j], dkey(fabs(bmin) * vol));
      }
    }
  }
}

// the lowest index at the closest key (queries nothing accepted), then, in
// the last block, every query of the list located and interpolated
__global__ __launch_bounds__(kBlock) void k_vol_exhaust_pick(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                             const int *best, const unsigned long long *ckey,
                                                             int *cidx, Slots S, int *elem_out, int8_t *hit_out) {
  __shared__ double sx[kQB][3];
  __shared__ int sneed[kQB];
  const int nfb = st->nfb_vol;
  if (nfb == 0) return;
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
        const double vol = tet_bary(sx[j], p0, p1, p2, p3, b);
        if (dkey(fabs(min4(b)) * vol) == ckey[q0 + j]) atomicMin(&cidx[q0 + j], k);
      }
    }
  }
  if (!last_block(&st->fb_done[0])) return;
  for (int j = threadIdx.x; j < nfb; j += blockDim.x) {
    int ip = fb[j];
    double x[3];
    load_pt(qxyz, ip, x);
    int hit, k;
    if (best[j] != INT_MAX) {
      k = best[j];
      hit = PMMG_HIT_VOL_EXHAUST;
    } else {
      k = atomicOr(&cidx[j], 0); // the other blocks' atomicMin results
      hit = PMMG_HIT_VOL_CLOSEST;
    }
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

// surface: the lowest-index accepting tria (locate_pmmg.c:483-503) and the
// minimum centroid distance (:400-416) in one scan
__global__ __launch_bounds__(kBlock) void k_bdy_exhaust_scan(Bg bg, const double *qxyz, const int *fb,
                                                             const DevStats *st, int *best, unsigned long long *ckey) {
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
        if (best[q0 + j] > k) {
          double b[3];
          double dist = tri_bary(x, t.p, t.q, t.n, b);
          double bmin = fmin(b[0], fmin(b[1], b[2]));
          if (bmin > -kEps && !(fabs(dist) > bg.hausd)) atomicMin(&best[q0 + j], k);
        }
        atomicMin(&ckey[q0 + j], dkey(centroid_dist(x, t)));
      }
    }
  }
}

// the lowest index at the minimum distance (queries nothing accepted), then,
// in the last block, every query of the list interpolated
__global__ __launch_bounds__(kBlock) void k_bdy_exhaust_pick(Bg bg, const double *qxyz, const int *fb, DevStats *st,
                                                             const int *best, const unsigned long long *ckey,
                                                             int *cidx, Slots S, int *elem_out, int8_t *hit_out) {
  __shared__ double sx[kQB][3];
  const int nfb = st->nfb_bdy;
  if (nfb == 0) return;
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
        if (best[q0 + j] != INT_MAX) continue;
        if (dkey(centroid_dist(sx[j], t)) == ckey[q0 + j]) atomicMin(&cidx[q0 + j], k);
      }
    }
  }
  if (!last_block(&st->fb_done[1])) return;
  for (int j = threadIdx.x; j < nfb; j += blockDim.x) {
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
      k = atomicOr(&cidx[j], 0); // the other blocks' atomicMin results
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
        phi[0] = b[0];
        phi[1] = b[1];
        phi[2] = b[2];
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

} // namespace pmmg
