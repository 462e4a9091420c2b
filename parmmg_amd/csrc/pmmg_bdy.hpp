// pmmg_bdy.hpp — surface (MG_BDY) points of the transfer step (included by
// pmmg_hip.hip only): PMMG_locatePointBdy (locate_pmmg.c:587-723) with the
// wedge / cone tests and the surface interpolation (interpmesh_pmmg.c:550-599).
#pragma once

#include "pmmg_prep.hpp"

namespace pmmg {

// one surface query; returns the hit code (0 = not located: exhaustive list)
__device__ __forceinline__ int bdy_query(const Bg &bg, const Frame *fr, const unsigned long long *sgrid, int gs,
                                         const double *qxyz,
                                         int ip, const Slots &S, int *elem_out, int8_t *hit_out, int maxstep,
                                         int &steps, int &scans, bool interp = true) {
  int hit = 0;
  double x[3];
  load_pt(qxyz, ip, x);
  int k = seed_srf(sgrid, gs, fr, x);
  if (k == 0) return 0;
  int hist[kHist];
#pragma unroll
  for (int h = 0; h < kHist; h++) hist[h] = 0;
  int edge = -1, vertex = -1;
  TriGeom t;
  double phi[3];
  for (;;) {
    ++steps;
    // (r05: 128-byte walk records per tria — coordinates, normal, ids,
    // adjacency, one line per step — built by k_seed_srf made the surface
    // branch 0.44 -> 0.50 ms at cfg4 and the volume stage +3 %: not kept,
    // profiles/r05u)
    tri_load(bg, k, t);
    int ad[3];
    for (int j = 0; j < 3; j++) ad[j] = bg.adjt[3 * (size_t)(k - 1) + j];
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
        if (b1 < kEps) {
          vertex = f2;
          hit = PMMG_HIT_BDY_VERTEX;
        } else {
          edge = f0;
          hit = PMMG_HIT_BDY_EDGE;
        }
      }
      break;
    }
    // step through the first edge (sorted order) whose neighbour exists; a
    // visited neighbour triggers the wedge test of that edge and, outside
    // it, the cone test of the wedge's end vertex (locate_pmmg.c:629-668)
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
          phi[0] = w[0];
          phi[1] = w[1];
          phi[2] = w[2];
          edge = f;
          hit = PMMG_HIT_BDY_WEDGE;
          done = true;
        } else if (tri_cone(bg, k, il, t, x, scans)) {
          vertex = il;
          hit = PMMG_HIT_BDY_CONE;
          done = true;
        }
        continue;
      }
      next = k1;
    }
    if (done) break;
    if (next == 0 || steps >= maxstep) { // -> exhaustive
      hit = 0;
      break;
    }
#pragma unroll
    for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
    hist[0] = k;
    k = next;
  }
  if (hit) {
    if (interp) interp_bdy(S, ip, t.v, phi, edge, vertex);
    if (elem_out) elem_out[ip - 1] = k;
    if (hit_out) hit_out[ip - 1] = (int8_t)(hit | ((vertex >= 0 ? vertex : (edge >= 0 ? edge : 0)) << 4));
  }
  return hit;
}

// One lane per surface query, the static XCD-chunked split of the grid
// (default), or (dyn, PMMG_HIP_BDYDYN=1) every wave claiming the next 64
// queries of its XCD's eighth from a counter: measured, the claiming waves
// slowed the volume kernel beside them (profiles/r03y).
// (r05: a register budget for 5 or 6 waves per SIMD instead of the compiler's
// 4: the step +-0 / +2 %, the 8-way rank's surface branch +-0, profiles/r05ak)
__global__ __launch_bounds__(kBlock) void k_bdy(Bg bg, const Frame *fr, const unsigned long long *sgrid, int gs,
                                                const double *qxyz,
                                                const int *order, Slots S, int *elem_out, int8_t *hit_out, int *fb,
                                                DevStats *st, int maxstep, int dyn, FbInit fi, FbGridBufs gb,
                                                const int *gate, int want, unsigned long long *wt) {
  if (want >= 0 && gate[0] != want) return; // (one of the two orders' launches, as k_vol)
#ifdef PMMG_HIP_MEASURE
  // measurement build, PMMG_HIP_WAVETIME=1: per wave {start, end, longest walk, active lanes} (wall clock)
  const unsigned long long wt0 = wt ? wall_clock64() : 0ULL;
  unsigned wt_steps = 0, wt_act = 0;
#endif
  __shared__ BlockStats bs;
  bstats_init(&bs);
  __syncthreads();
  const long long n = st->nbdy;
  const int x = blockIdx.x & 7;
  const long long lo = n * x / 8, hi = n * (x + 1) / 8;
  const XcdChunk ch = xcd_chunk(n); // static split (dyn == 0)
  for (int it = 0;; it++) {
    long long i;
    if (dyn & 1) {
      int base = 0;
      if (__lane_id() == 0) base = atomicAdd(&st->bdy_next[x], 64);
      base = __shfl(base, 0);
      if (lo + base >= hi) break;
      i = lo + base + __lane_id();
    } else {
      if (it >= ch.iters) break;
      i = ch.start + it * ch.stride;
    }
    const bool active = i < ((dyn & 1) ? hi : ch.hi);
    int steps = 0, hit = 0, ip = 0, scans = 0;
    if (active) {
      ip = order[i];
      // (measurement build, dyn bit 1 = PMMG_HIP_BDYNOINTERP=1: the walks without the interpolation; r06w:
      // the interpolation is ~half of a surface wave's lifetime.  r06x: a cooperative version — the three
      // vertices' rows gathered by the wave through LDS, 8-byte pieces — made the waves longer, 32 vs 30 us,
      // and the step +27 us: not kept)
#ifdef PMMG_HIP_MEASURE
      hit = bdy_query(bg, fr, sgrid, gs, qxyz, ip, S, elem_out, hit_out, maxstep, steps, scans, !(dyn & 2));
#else
      hit = bdy_query(bg, fr, sgrid, gs, qxyz, ip, S, elem_out, hit_out, maxstep, steps, scans);
#endif
    }
    wave_count(&bs, kCntFanScan, active && scans > 0);
    int slot = wave_append(&st->nfb_bdy, active && hit == 0);
    if (active && hit == 0) {
      fb[slot] = ip;
      fi.at(slot);
    }
    wave_stats(&bs, active, hit, steps);
#ifdef PMMG_HIP_MEASURE
    if (wt) {
      unsigned m = active ? (unsigned)steps : 0u;
      for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
      wt_steps = max(wt_steps, m);
      wt_act += (unsigned)__popcll(__ballot(active));
    }
#endif
  }
#ifdef PMMG_HIP_MEASURE
  if (wt && __lane_id() == 0) {
    unsigned long long *w = wt + 4 * (size_t)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    w[0] = wt0;
    w[1] = wall_clock64();
    w[2] = wt_steps;
    w[3] = wt_act;
  }
#endif
  __syncthreads();
  bstats_flush(&bs, st);
  // (the surface fallback list's query grid: k_fb_grid, launched next)
}

} // namespace pmmg
