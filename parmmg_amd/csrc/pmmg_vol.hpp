// pmmg_vol.hpp — volume points of the transfer step (included by
// pmmg_hip.hip only): PMMG_locatePointVol (locate_pmmg.c:786-883) and the
// interpolation PMMG_interp4bar_{iso,ani} (interpmesh_pmmg.c:206-270).
//
//   k_vol             per query: fp32 filter walk from a grid seed to a
//                     candidate tetra, the reference's exact fp64 acceptance
//                     test there (and its exact coordinates), interpolation
//                     of the metric and fields
//   k_vol_walk_exact  the few queries the filter could not settle, walked and
//                     interpolated in the reference's fp64 arithmetic (then
//                     the exhaustive kernels, pmmg_fallback.hpp)
#pragma once

#include "pmmg_prep.hpp"

namespace pmmg {

__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// a located query: the tetra's vertex ids and the reference's (exact,
// unsorted) barycentric coordinates
struct VolLoc {
  int4 v;
  double phi[4];
};

struct ContEntry {
  int ip; // query
  int k;  // tetra the exact walk starts from (0: no seed)
};

// Located records of the split volume stage (r06): the walk kernel writes, per
// processing index i, the accepted tetra's vertex ids (v.x = 0: nothing to
// interpolate — another class, a handed-over or failed walk) and its four
// exact coordinates; k_vol_interp reads them back in the same order.  Three
// arrays of 16-byte rows, so that each wave-instruction writes or reads 1 KiB
// of consecutive bytes.  Null v: the fused kernel interpolates itself.
typedef int nti4 __attribute__((ext_vector_type(4)));
struct LocBuf {
  nti4 *v;
  ntd2 *p01, *p23;
};

__device__ __forceinline__ void load_tet_pts(const Bg &bg, const int4 &tv, double (*p)[3]) {
  load_pt(bg.xyz, tv.x, p[0]);
  load_pt(bg.xyz, tv.y, p[1]);
  load_pt(bg.xyz, tv.z, p[2]);
  load_pt(bg.xyz, tv.w, p[3]);
}

// The reference's acceptance test of tetra (tv) for x, exactly
// (PMMG_locatePointInTetra, locate_pmmg.c:441-461 + barycoord3d_evaluate):
// accept iff min_f bary[f] > -MMG5_EPS, bary[f] = -s[f]/vol.  IEEE division
// is sign-symmetric and monotone, so for vol > 0
//   min_f fl(-s[f]/vol) = -fl(max_f s[f] / vol)
// (for vol < 0 with min_f s[f]): one division decides, bit-identically to the
// reference's four.  Degenerate tetra (vol == 0) take the four divisions.
// On acceptance loc receives the vertex ids and -s[f]/vol (the reference's
// coordinates, PMMG_barycoord_get: unsorted).  key[f] (when non-null): larger
// = more negative coordinate (the reference's walk order of faces).
__device__ __forceinline__ bool exact_accept(const double *x, const double (*p)[3], const int4 &tv, VolLoc *loc,
                                             double *key) {
  double s[4];
  const double vol = tet_dots(x, p[0], p[1], p[2], p[3], s);
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
    if (key)
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = vol > 0.0 ? s[f] : -s[f];
  } else {
    double b[4];
#pragma unroll
    for (int f = 0; f < 4; f++) b[f] = -s[f] / vol;
    inside = min4(b) > -kEps;
    if (key)
#pragma unroll
      for (int f = 0; f < 4; f++) key[f] = s[f];
  }
  if (inside) {
    loc->v = tv;
#pragma unroll
    for (int f = 0; f < 4; f++) loc->phi[f] = -s[f] / vol;
  }
  return inside;
}

// index of id in t (0 when it is t.x or absent)
__device__ __forceinline__ int idx_in(int id, const int4 &t) {
  return (id == t.y ? 1 : 0) + (id == t.z ? 2 : 0) + (id == t.w ? 3 : 0);
}

// the eligible face with the largest key (the reference steps through the
// first face, in its sorted order, whose neighbour exists and is unvisited,
// locate_pmmg.c:819-833; ties: lowest face); -1 when none
template <typename T>
__device__ __forceinline__ int pick_face(const int4 &ad, const int *hist, const T *key) {
  int f = -1;
  T best = 0;
#pragma unroll
  for (int ff = 0; ff < 4; ff++) {
    const int iel = sel4(ad, ff) >> 2;
    bool vis = false;
#pragma unroll
    for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
    if (iel != 0 && !vis && (f < 0 || key[ff] > best)) {
      f = ff;
      best = key[ff];
    }
  }
  return f;
}

// Past kDetSteps steps a walk takes the stochastic rule instead (Devillers,
// Pion & Teillaud, "Walking in a triangulation": the remembering stochastic
// walk terminates with probability 1 on any triangulation): the first
// eligible face, in a cyclic order starting at a pseudo-random face, beyond
// which the point lies (key > 0); the usual rule when there is none.  The
// most-negative rule can cycle on sheared, strongly graded meshes (cfgG:
// cycles longer than the 4-entry history sent ~0.1 % of the queries through
// 4096 exact steps into the exhaustive search).  The path only decides which
// of the accepting tetra a class (ii) point ends in; rsel is a hash of
// (query, step), so the result stays a pure function of the query.
constexpr int kDetSteps = 24;
__device__ __forceinline__ unsigned walk_rsel(int ip, int steps) {
  if (steps <= kDetSteps) return 0u;
  unsigned h = (unsigned)ip * 0x9E3779B1u ^ (unsigned)steps * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h | 0x80000000u; // nonzero
}
template <typename T>
__device__ __forceinline__ int pick_face_walk(const int4 &ad, const int *hist, const T *key, unsigned rsel) {
  if (rsel) {
    const int f0 = (int)(rsel & 3u);
    int f = -1;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int ff = (f0 + j) & 3;
      const int iel = sel4(ad, ff) >> 2;
      bool vis = false;
#pragma unroll
      for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
      if (f < 0 && iel != 0 && !vis && key[ff] > (T)0) f = ff;
    }
    if (f >= 0) return f;
  }
  return pick_face<T>(ad, hist, key);
}

// the vertices of the tetra reached through face f: the new tetra tn's local
// vertex l sits in the slot of the same vertex of the previous tetra tv (slot
// map m), except its vertex opposite the crossed face (iopp), which takes the
// slot of the vertex left behind (f)
__device__ __forceinline__ int4 next_slots(const int4 &m, const int4 &tv, const int4 &tn, int f, int iopp) {
  const int sf = sel4(m, f);
  int4 mn; // branch-free (a ternary with a costly arm becomes a divergent branch)
  mn.x = (int)bsel((unsigned)sel4(m, idx_in(tn.x, tv)), (unsigned)sf, iopp == 0);
  mn.y = (int)bsel((unsigned)sel4(m, idx_in(tn.y, tv)), (unsigned)sf, iopp == 1);
  mn.z = (int)bsel((unsigned)sel4(m, idx_in(tn.z, tv)), (unsigned)sf, iopp == 2);
  mn.w = (int)bsel((unsigned)sel4(m, idx_in(tn.w, tv)), (unsigned)sf, iopp == 3);
  return mn;
}

// The same on a packed slot map (2 bits per local vertex: slot of local l =
// bits 2l..2l+1), the fp32 filter walk's form: a lookup is one bit-field
// extract instead of a select chain
__device__ __forceinline__ unsigned pslot(unsigned m, int l) { return (m >> (2 * l)) & 3u; }
__device__ __forceinline__ unsigned next_slots_packed(unsigned m, const int4 &tv, const int4 &tn, int f, int iopp) {
  const unsigned sf = pslot(m, f);
  const int ids[4] = {tn.x, tn.y, tn.z, tn.w};
  unsigned mn = 0u;
#pragma unroll
  for (int l = 0; l < 4; l++) {
    const unsigned s = l == iopp ? sf : pslot(m, idx_in(ids[l], tv));
    mn |= s << (2 * l);
  }
  return mn;
}

// ---------------------------------------------------------------- fp32 filter walk
//
// The walk itself only has to reach the accepting tetra; the reference's
// exact arithmetic is needed for the acceptance decision and the coordinates
// of that one tetra.  So each step runs in fp32 on the vertices relative to
// the query (q = p - x, rounded once), where the four face numerators are
// triple products: with x at the origin
//   s_f = (x - a_f) . ((b_f - a_f) x (c_f - a_f)) = -det(a_f, b_f, c_f)
// (faces idir = {1,2,3}, {0,3,2}, {0,1,3}, {0,2,1}), three cross products
// shared by the four faces, and vol = orvol = -(s0 + s1 + s2 + s3).
// A step stops the walk when min_f bary[f] > -(EPS + kFilterMargin) in fp32:
// every tetra the reference's test could accept passes (the fp32 error of a
// coordinate, ~1e-6 at most for the meshes at hand, is far below the
// margin).  The exact test then runs once per query, at the candidate; a
// query it rejects (within the margin of a face, ~1e-3 of the queries)
// continues in exact arithmetic (k_vol_walk_exact).  Every located
// tetra is therefore accepted by the reference's own test, with its exact
// coordinates.
//
// The fp32 step is ~30 single-precision operations instead of ~100
// double-precision ones plus a division, and it keeps the vertices as 12-byte
// LDS slots instead of 24-byte ones: fewer registers, more waves in flight
// for a walk whose steps are two dependent gathers each.
constexpr float kFilterMargin = 1.220703125e-4f; // 2^-13

// (an address-space-3 pointer: the slot offsets are 32-bit LDS arithmetic;
// through a generic pointer they were 64-bit multiply-adds)
typedef __attribute__((address_space(3))) float lds_float;
struct LaneSlotsF { // this lane's view of the wave's slot image [slot*3 + dim][64]
  lds_float *base;
  __device__ __forceinline__ void put(int slot, const float *q) const {
#pragma unroll
    for (int d = 0; d < 3; d++) base[(unsigned)(slot * 3 + d) * 64u] = q[d];
  }
  __device__ __forceinline__ void get(int slot, float *q) const {
#pragma unroll
    for (int d = 0; d < 3; d++) q[d] = base[(unsigned)(slot * 3 + d) * 64u];
  }
};

// vertex v relative to the query, from the fixed-point copy (exact integer
// difference, one rounding to fp32)
__device__ __forceinline__ void rel_pt(const int *xq, int v, const int *xqq, float *q) {
  if constexpr (kXqStride == 4) {
    const int4 p = reinterpret_cast<const int4 *>(xq)[v - 1];
    q[0] = (float)(p.x - xqq[0]);
    q[1] = (float)(p.y - xqq[1]);
    q[2] = (float)(p.z - xqq[2]);
  } else {
    const int *p = xq + kXqStride * (size_t)(v - 1);
    q[0] = (float)(p[0] - xqq[0]);
    q[1] = (float)(p[1] - xqq[1]);
    q[2] = (float)(p[2] - xqq[2]);
  }
}

// The filter's arithmetic needs no particular rounding (its margin is ~100x
// its error, and every accepted tetra passes the reference's exact test), so
// it takes fused multiply-adds: fewer VALU instructions per step (the module is
// built with -ffp-contract=off for the fp64 paths; fmaf is explicit)
__device__ __forceinline__ void cross3(const float *a, const float *b, float *c) {
  c[0] = __builtin_fmaf(a[1], b[2], -(a[2] * b[1]));
  c[1] = __builtin_fmaf(a[2], b[0], -(a[0] * b[2]));
  c[2] = __builtin_fmaf(a[0], b[1], -(a[1] * b[0]));
}
__device__ __forceinline__ float dot3(const float *a, const float *b) {
  return __builtin_fmaf(a[0], b[0], __builtin_fmaf(a[1], b[1], a[2] * b[2]));
}

// the face the walk leaves through: the largest key among the faces with a
// neighbour (ties: lowest face); only when that neighbour is in the visited
// history does the full rule (pick_face) run — the same face either way
template <typename T>
__device__ __forceinline__ int pick_face_fast(const int4 &ad, const int *hist, const T *key, unsigned rsel) {
  if (rsel) return pick_face_walk<T>(ad, hist, key, rsel);
  int f = -1;
  T best = 0;
#pragma unroll
  for (int ff = 0; ff < 4; ff++) {
    const int iel = sel4(ad, ff) >> 2;
    if (iel != 0 && (f < 0 || key[ff] > best)) {
      f = ff;
      best = key[ff];
    }
  }
  if (f >= 0) {
    const int iel = sel4(ad, f) >> 2;
    bool vis = false;
#pragma unroll
    for (int h = 0; h < kHist; h++) vis = vis || (hist[h] == iel);
    if (vis) f = pick_face<T>(ad, hist, key);
  }
  return f;
}

// returns 1 candidate (filter passed), 0 moved (k, tv, ad, m, hist updated),
// 2 stuck (no eligible neighbour).  (r04f: the neighbour records loaded by
// lane pairs, one sector access per record, wave-uniform loop: +4 %;
// profiles/r04f/pair_records.patch.txt.)
__device__ __forceinline__ int step_f32(const Bg &bg, const int *x, int &k, int4 &tv, int4 &ad, unsigned &m, int *hist,
                                        const LaneSlotsF &L, unsigned rsel) {
  float q[4][3];
  L.get(pslot(m, 0), q[0]);
  L.get(pslot(m, 1), q[1]);
  L.get(pslot(m, 2), q[2]);
  L.get(pslot(m, 3), q[3]);
  float c23[3], c13[3], c12[3], s[4];
  cross3(q[2], q[3], c23);
  cross3(q[1], q[3], c13);
  cross3(q[1], q[2], c12);
  s[0] = -dot3(q[1], c23);
  s[1] = dot3(q[0], c23);
  s[2] = -dot3(q[0], c13);
  s[3] = dot3(q[0], c12);
  const float vol = -((s[0] + s[1]) + (s[2] + s[3]));
  float key[4];
#pragma unroll
  for (int ff = 0; ff < 4; ff++) key[ff] = vol < 0.f ? -s[ff] : s[ff];
  const float kmax = fmaxf(fmaxf(key[0], key[1]), fmaxf(key[2], key[3]));
  if (vol != 0.f && kmax < (float)(kEps + kFilterMargin) * fabsf(vol)) return 1;
  const int f = pick_face_fast<float>(ad, hist, key, rsel);
  if (f < 0) return 2;
#pragma unroll
  for (int h = kHist - 1; h > 0; h--) hist[h] = hist[h - 1];
  hist[0] = k;
  const int code = sel4(ad, f);
  k = code >> 2;
  const int iopp = code & 3;
  const int4 tn = tetv_row(bg, k);
  ad = adja_row(bg, k);
  float qn[3];
  rel_pt(bg.xq, sel4(tn, iopp), x, qn);
  const int sf = (int)pslot(m, f);
  m = next_slots_packed(m, tv, tn, f, iopp);
  L.put(sf, qn);
  tv = tn;
  return 0;
}

// ---------------------------------------------------------------- exact continuation

// fp64 walk with the tetra's vertices kept in LDS slots (per lane 4 slots x 3
// doubles, lane-interleaved: conflict-free): the reference's arithmetic at
// every step.  Returns 1 found (loc), 2 stuck, 3 limit reached.
struct LaneSlotsD {
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

// An accepted tetra whose smallest coordinate is within MMG5_EPS of a face
// (min phi <= EPS) may have a face neighbour that holds the point strictly
// (min phi > EPS): on a graded mesh, where the heights of two neighbours
// across a face differ by orders of magnitude, a point inside the thin one
// by more than EPS of its height is within EPS of the tall one's height
// outside it, and both pass the reference's test.  The reference ends in
// whichever its walk meets first; here the strict one is preferred, so that
// a point with min barycentric > EPS (class (i) of tests/parity.py, the
// north_star's bit-exact class) lands in its tetra whatever the path
// (cfgG: 1 point in 3.9M otherwise).  The neighbour across the face of the
// smallest coordinate is checked with the reference's own arithmetic.
// (inlined: as an out-of-line call its pointer arguments kept the caller's
// locals in scratch memory, 208 B per lane of k_vol_walk_exact in r03)
__device__ __forceinline__ void prefer_strict(const Bg &bg, const double *x, const int4 &ad, int &k, VolLoc *loc) {
  if (min4(loc->phi) > kEps) return;
  int f = 0; // the first smallest coordinate (compile-time indices only: phi stays in registers)
  double mn = loc->phi[0];
#pragma unroll
  for (int j = 1; j < 4; j++)
    if (loc->phi[j] < mn) {
      mn = loc->phi[j];
      f = j;
    }
  const int nb = sel4(ad, f) >> 2;
  if (nb == 0) return;
  const int4 tn = tetv_row(bg, nb);
  double q[4][3];
  load_tet_pts(bg, tn, q);
  VolLoc l2;
  if (exact_accept(x, q, tn, &l2, nullptr) && min4(l2.phi) > kEps) {
    *loc = l2;
    k = nb;
  }
}

__device__ __forceinline__ int walk_exact(const Bg &bg, const double *x, int ip, int &k, int &steps, int limit,
                                          VolLoc *loc, const LaneSlotsD &L) {
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
  int4 m = make_int4(0, 1, 2, 3);
  for (int n = 0;; n++) {
    if (n >= limit) return 3;
    ++steps;
    double p[4][3];
    L.get(m.x, p[0]);
    L.get(m.y, p[1]);
    L.get(m.z, p[2]);
    L.get(m.w, p[3]);
    double key[4];
    if (exact_accept(x, p, tv, loc, key)) {
      prefer_strict(bg, x, ad, k, loc);
      return 1;
    }
    const int f = pick_face_walk<double>(ad, hist, key, walk_rsel(ip, n + 1));
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
    const int sf = sel4(m, f);
    m = next_slots(m, tv, tn, f, iopp);
    L.put(sf, pn);
    tv = tn;
  }
}

// the queries the filter walk handed over, walked in exact arithmetic from
// where it stopped (fresh visited history) and interpolated here (per-lane
// gathers: these are few); failures -> the exhaustive list.  Fixed grid: the
// count is read on the device.
__global__ __launch_bounds__(64) void k_vol_walk_exact(Bg bg, const double *qxyz, int *fb, const ContEntry *cont,
                                                       DevStats *st, Slots S, int *elem_out, int8_t *hit_out,
                                                       int maxstep, FbInit fi, FbGridBufs gb) {
  __shared__ BlockStats bs;
  __shared__ double slot_img[12 * 64];
  const LaneSlotsD L{&slot_img[__lane_id()]};
  bstats_init(&bs);
  __syncthreads();
  const XcdChunk ch = xcd_chunk(st->ncont);
  for (int it = 0; it < ch.iters; it++) {
    const long long j = ch.start + it * ch.stride;
    const bool active = j < ch.hi;
    int status = 0, steps = 0, ip = 0;
    if (active) {
      const ContEntry e = cont[j];
      ip = e.ip;
      int k = e.k;
      if (k > 0) {
        double x[3];
        load_pt(qxyz, ip, x);
        VolLoc loc;
        status = walk_exact(bg, x, ip, k, steps, maxstep, &loc, L);
        if (status == 1) {
          const int v[4] = {loc.v.x, loc.v.y, loc.v.z, loc.v.w};
          for (int sl = 0; sl < S.n; sl++) interp_dyn<4>(S.s[sl], ip, v, loc.phi);
          if (elem_out) elem_out[ip - 1] = k;
          if (hit_out) hit_out[ip - 1] = (int8_t)PMMG_HIT_VOL_WALK;
        }
      }
    }
    const bool fail = active && status != 1;
    const int slot = wave_append(&st->nfb_vol, fail);
    if (fail) {
      fb[slot] = ip;
      fi.at(slot);
    }
    wave_count(&bs, kCntStuck, fail && status == 2);
    wave_count(&bs, kCntLimit, fail && status == 3);
    wave_stats(&bs, active, status == 1 ? PMMG_HIT_VOL_WALK : 0, steps);
  }
  __syncthreads();
  bstats_flush(&bs, st);
  // (the volume fallback list's query grid: k_fb_grid, launched next)
}

// ---------------------------------------------------------------- interpolation


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

// The same for the Morton-binned order, where row r goes to its own query ip
// of lane r (scattered): the rows still go through the LDS image, so that
// one store instruction writes the pieces of ~21 rows (one to two lines
// each) instead of one piece of 64 rows.  Plain (cached) stores: L2 merges
// the partial lines that queries of other waves complete.
template <int C>
__device__ __forceinline__ void wave_store_rows_scat(double *out, const double *row, unsigned long long mask,
                                                     double *img, int ip) {
  const int lane = __lane_id();
  if constexpr (C == 1) {
    if ((mask >> lane) & 1ULL) out[ip - 1] = row[0];
  } else {
#pragma unroll
    for (int j = 0; j < C; j++) img[C * lane + j] = row[j];
    wait_lgkm();
    constexpr int PR = C == 6 ? 3 : C; // pieces per row: 16-byte (6-double rows) or 8-byte
#pragma unroll
    for (int t = 0; t < PR; t++) {
      const int p = 64 * t + lane, r = p / PR, k = p - PR * r;
      const int dst = __shfl(ip, r);
      if ((mask >> r) & 1ULL) {
        if constexpr (C == 6)
          reinterpret_cast<double2 *>(out + (size_t)6 * (dst - 1))[k] = reinterpret_cast<const double2 *>(img)[p];
        else
          out[(size_t)C * (dst - 1) + k] = img[p];
      }
    }
    wait_lgkm(); // the image is reused by the next slot
  }
}

// Where the rows of a wave go: input order — the wave's 64 consecutive
// queries' rows as whole lines at w0 (wave_store_rows); Morton order — every
// row to its own query ip (wave_store_rows_scat).  (r03 measured a third,
// staged, form for numberings without coherence — records in processing
// order copied back by an un-permute kernel — and dropped it: the same
// volume-stage time, profiles/r03m/staged_path.patch.txt.)
struct Sink {
  bool coalesced;
  size_t w0; // the wave's first processing index
  int ip;    // this lane's query (1-based)
};

template <int C>
__device__ __forceinline__ void sink_rows(const Slot &sl, const double *r, bool ok, double *img, const Sink &k) {
  if (k.coalesced) wave_store_rows<C>(sl.out + (size_t)C * k.w0, r, __ballot(ok), img);
  else wave_store_rows_scat<C>(sl.out, r, __ballot(ok), img, k.ip);
}

// ---------------------------------------------------------------- fused volume kernel
//
// One query per lane, the 64 lanes of a one-wave block on 64 consecutive
// queries of the processing order, in three phases per wave:
//   1. the fp32 filter walk from the grid seed to a candidate tetra
//      (neighbouring walks run in lockstep through the same tetra and share
//      cache lines inside each wave-instruction);
//   2. the reference's exact test at the candidate (its 4 vertex rows are
//      still in L1/L2 from the walk's last step), which gives the exact
//      coordinates; rejected candidates, stuck and over-long walks go to the
//      continuation list (k_vol_walk_exact);
//   3. the interpolation of every slot (layout = template: codes 1 / 3 / 6,
//      0 = none; C0 < 0 = runtime layout, per-lane).  A 3- or 6-double slot
//      is gathered one vertex at a time: in pass i the 64 lanes load the 64
//      rows of vertex i of the wave's queries cooperatively (3 pieces of a
//      row in one wave-instruction, lane l of instruction t loading piece
//      64t+l of the rows' image) into LDS, each lane reads back its own row
//      and accumulates it in the reference's order (PMMG_interp4bar_ani:
//      mint = sum_i phi_i invmat(M_i), then invmat(mint)), so only one row is
//      live per lane; vertex i+1's loads are issued before vertex i's rows
//      go through LDS (coop_issue* / coop_land*).  In input order the rows are stored as whole cache lines
//      through the same LDS image; Morton-binned queries store per lane.
// The walk's vertex slots and the gather image share one 4 KiB LDS buffer
// (the phases are sequential within the wave).  (r04e: the tensor slots'
// gathers by LDS DMA, with the next vertex in flight in a second image
// instead of registers, measured equal; 5 waves per SIMD with 8 VGPRs
// spilled, +3 %.  r04b measured a third use —
// an image of the wave's distinct vertices, sorted, for the exact test and the
// interpolation: 20 % fewer L1 accesses, +23 % VALU for the sort, +10 % time;
// profiles/r04b/unique_vertex_rows.patch.txt.)
// (the image of the array layout holds 8 doubles per lane: 4.3 KB per block
// where the packed records' 16 take 8.4 KB, which would hold a 6-wave layout
// (80 VGPRs) to 19 blocks per CU)
template <int PK>
struct VolShared {
  BlockStats bs;
  unsigned short okm[PK > 0 ? 64 : 1]; // output records: the doubles of each lane's record that are written (bit j)
  union {
    float slots[12 * 64]; // walk: the vertex slots [slot*3 + dim][lane]
    double dslots[12 * 64]; // the exact continuation's fp64 vertex slots (LaneSlotsD)
    double img[(PK > 0 ? 16 : 8) * 64]; // interpolation: 64 rows of up to 6 doubles, or 64 records of up to 16
  } u;
};

// The exact continuation inside k_vol (r06): a lane whose filter walk did not
// end in an accepted tetra walks on in fp64 from where it stopped, as
// k_vol_walk_exact does (same start, fresh history, same arithmetic: the
// same tetra), and joins the wave's interpolation; only its failures go to
// the exhaustive list.  Before, the continuations (~0.07 % of the queries)
// were a list and a kernel of their own after the volume kernel, 40-80 us on
// the volume stage's tail beside the surface kernel's blocks.
struct ContArgs {
  int *fb;     // the volume fallback list (ids)
  FbInit fi;   // its best-index initialisation
  int maxstep; // the exact walk's step cap
  int fuse;    // 1: continue in k_vol (0: the list + k_vol_walk_exact)
};

// Rows of one vertex of the wave's 64 queries, gathered cooperatively: piece
// p = 64t + lane of the rows' image (row r = query r, 3 pieces per row: 16
// bytes of a 6-double row, 8 of a 3-double row) is loaded by lane p % 64 of
// instruction t.  In two halves, so that the next vertex's gathers are in
// flight while this vertex's rows go through LDS: coop_issue* loads this
// lane's three pieces into registers, coop_land* puts them into the image
// and returns this lane's row.  (The pieces live in named registers: an
// array of them indexed per vertex went to scratch memory and cost 40 %.)
__device__ __forceinline__ void coop_issue6(const double *in, int stride, int myv, double2 &p0, double2 &p1,
                                            double2 &p2) {
  const int lane = __lane_id();
  const int q0 = lane, q1 = 64 + lane, q2 = 128 + lane;
  const int v0 = __shfl(myv, q0 / 3), v1 = __shfl(myv, q1 / 3), v2 = __shfl(myv, q2 / 3);
  p0 = *reinterpret_cast<const double2 *>(in + (size_t)stride * (v0 - 1) + 2 * (q0 % 3));
  p1 = *reinterpret_cast<const double2 *>(in + (size_t)stride * (v1 - 1) + 2 * (q1 % 3));
  p2 = *reinterpret_cast<const double2 *>(in + (size_t)stride * (v2 - 1) + 2 * (q2 % 3));
}
__device__ __forceinline__ void coop_land6(const double2 &p0, const double2 &p1, const double2 &p2, double *img,
                                           double *row) {
  const int lane = __lane_id();
  reinterpret_cast<double2 *>(img)[lane] = p0;
  reinterpret_cast<double2 *>(img)[64 + lane] = p1;
  reinterpret_cast<double2 *>(img)[128 + lane] = p2;
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 6; j++) row[j] = img[6 * lane + j];
  wait_lgkm();
  __builtin_amdgcn_wave_barrier(); // every lane has read its row: the image is free again
}
__device__ __forceinline__ void coop_issue3(const double *in, int stride, int myv, double &p0, double &p1,
                                            double &p2) {
  const int lane = __lane_id();
  const int q0 = lane, q1 = 64 + lane, q2 = 128 + lane;
  const int v0 = __shfl(myv, q0 / 3), v1 = __shfl(myv, q1 / 3), v2 = __shfl(myv, q2 / 3);
  p0 = in[(size_t)stride * (v0 - 1) + q0 % 3];
  p1 = in[(size_t)stride * (v1 - 1) + q1 % 3];
  p2 = in[(size_t)stride * (v2 - 1) + q2 % 3];
}
__device__ __forceinline__ void coop_land3(double p0, double p1, double p2, double *img, double *row) {
  const int lane = __lane_id();
  img[lane] = p0;
  img[64 + lane] = p1;
  img[128 + lane] = p2;
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 3; j++) row[j] = img[3 * lane + j];
  wait_lgkm();
  __builtin_amdgcn_wave_barrier();
}

// one slot of the wave's queries: rows gathered, interpolated, stored
template <int C>
__device__ __forceinline__ void vol_slot(const Slot &sl, bool act, const int4 &v, const double *phi, double *img,
                                         const Sink &k) {
  if constexpr (C > 0) {
    double r[C];
    bool ok = act;
    if constexpr (C == 6) { // vertex i + 1's gathers in flight while vertex i goes through LDS
      double mint[6], m[6], mi[6];
      double2 a0, a1, a2, b0, b1, b2;
#define PMMG_ACC6(i)                                                                               \
  do {                                                                                             \
    ok = invmat(m, mi) && ok;                                                                      \
    _Pragma("unroll") for (int q = 0; q < 6; q++) mint[q] = (i == 0) ? phi[0] * mi[q] : mint[q] + phi[i] * mi[q]; \
  } while (0)
      coop_issue6(sl.in, sl.istride, v.x, a0, a1, a2);
      coop_issue6(sl.in, sl.istride, v.y, b0, b1, b2);
      coop_land6(a0, a1, a2, img, m);
      PMMG_ACC6(0);
      coop_issue6(sl.in, sl.istride, v.z, a0, a1, a2);
      coop_land6(b0, b1, b2, img, m);
      PMMG_ACC6(1);
      coop_issue6(sl.in, sl.istride, v.w, b0, b1, b2);
      coop_land6(a0, a1, a2, img, m);
      PMMG_ACC6(2);
      coop_land6(b0, b1, b2, img, m);
      PMMG_ACC6(3);
      ok = invmat(mint, r) && ok;
#undef PMMG_ACC6
    } else if constexpr (C == 3) {
      double m[3], a0, a1, a2, b0, b1, b2;
#define PMMG_ACC3(i)                                                                               \
  do {                                                                                             \
    _Pragma("unroll") for (int q = 0; q < 3; q++) r[q] = (i == 0) ? 0.0 + phi[0] * m[q] : r[q] + phi[i] * m[q]; \
  } while (0)
      coop_issue3(sl.in, sl.istride, v.x, a0, a1, a2);
      coop_issue3(sl.in, sl.istride, v.y, b0, b1, b2);
      coop_land3(a0, a1, a2, img, m);
      PMMG_ACC3(0);
      coop_issue3(sl.in, sl.istride, v.z, a0, a1, a2);
      coop_land3(b0, b1, b2, img, m);
      PMMG_ACC3(1);
      coop_issue3(sl.in, sl.istride, v.w, b0, b1, b2);
      coop_land3(a0, a1, a2, img, m);
      PMMG_ACC3(2);
      coop_land3(b0, b1, b2, img, m);
      PMMG_ACC3(3);
#undef PMMG_ACC3
    } else {
      const int vv[4] = {v.x, v.y, v.z, v.w};
      interp_iso_row<4, 1>(sl.in, sl.istride, vv, phi, r);
    }
    sink_rows<C>(sl, r, ok, img, k);
  }
}

// ---------------------------------------------------------------- packed records
//
// With packed per-vertex records (pmmg_hip_set_solutions_packed: the slots'
// rows back to back, [slot 0 | slot 1 | ...], RS doubles per vertex) a
// vertex's whole solution is one record — one 128-byte line for K <= 16
// doubles (cfg3 / cfg4: 16) — so the interpolation gathers, per vertex of the
// wave's 64 queries, the 64 records in RS / 2 load instructions of 16 bytes
// per lane, each instruction covering whole records (one line access per
// record and vertex, against ~4.6 for the four separate arrays' rows), into
// an LDS image; each lane reads its own record's doubles back from it and
// accumulates every slot in the reference's order.
//
// NP passes over the record (NP = 1: the whole record per gather, every
// slot's accumulator live over the four vertices; NP = 2: the record's two
// halves in turn, a slot's accumulator live only over the passes holding its
// components, a tensor never across the halves).  r04h ran NP = 2 with 8-byte
// image reads at a 64-byte lane stride (16-way bank conflicts); r05 swizzles
// the image so that the cooperative writes and each lane's reads of its own
// record are conflict-free: piece k of record r sits at
// PP r + (k ^ ((r >> SH) & (PP - 1))) (PP pieces of 16 bytes per record and
// pass, a power of two; SH chosen so that 16 consecutive lanes reading piece
// k of their records hit 16 distinct 16-byte bank groups).
template <int C0, int C1, int C2, int C3, int C4, int C5>
struct PackedLayout {
  static constexpr int c[6] = {C0 > 0 ? C0 : 0, C1, C2, C3, C4, C5};
  static constexpr int K = c[0] + c[1] + c[2] + c[3] + c[4] + c[5];
  static constexpr int RS = (K + 1) & ~1; // record stride (doubles)
  static constexpr int off(int s) { return s == 0 ? 0 : off(s - 1) + c[s - 1]; }
  static constexpr bool valid() { return C0 >= 0 && K > 0 && RS <= 16; }
  // NP passes possible: RS / 2 pieces split evenly, no tensor across a pass boundary
  static constexpr bool passes_ok(int np) {
    if ((RS / 2) % np) return false;
    const int pw = RS / np; // doubles per pass
    for (int s = 0; s < 6; s++)
      if (c[s] == 6 && off(s) / pw != (off(s) + 5) / pw) return false;
    return true;
  }
};

template <int C>
struct SlotAcc {
  double v[C > 0 ? C : 1];
  bool ok = true;
  // component q of vertex i's row = x (iso) — PMMG_interp4bar_iso order
  __device__ __forceinline__ void iso(int i, double ph, int q, double x) {
    v[q] = (i == 0) ? 0.0 + ph * x : v[q] + ph * x;
  }
  // vertex i's tensor row m — PMMG_interp4bar_ani: mint = sum_i phi_i invmat(M_i)
  __device__ __forceinline__ void ani(int i, double ph, const double *m) {
    double mi[6];
    ok = invmat(m, mi) && ok;
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = (i == 0) ? ph * mi[q] : v[q] + ph * mi[q];
  }
};

template <int PP>
__device__ __forceinline__ constexpr int packed_swizzle_shift() {
  return PP >= 8 ? 1 : (PP == 4 ? 2 : (PP == 2 ? 3 : 0));
}
template <int PP>
__device__ __forceinline__ int packed_pos(int r, int k) {
  if constexpr ((PP & (PP - 1)) == 0 && PP > 1) return PP * r + (k ^ ((r >> packed_swizzle_shift<PP>()) & (PP - 1)));
  else return PP * r + k;
}
// double j (of this pass's PW = 2 PP doubles) of this lane's record in the image
template <int PP>
__device__ __forceinline__ double packed_dbl(const double *img, int lane, int j) {
  return img[2 * packed_pos<PP>(lane, j >> 1) + (j & 1)];
}

// slot S's components of vertex i that live in pass `pass`, read from the
// image as they are needed (only one slot's pieces in registers at a time)
template <class L, int NP, int S, int C>
__device__ __forceinline__ void packed_take(SlotAcc<C> &a, int pass, int i, double ph, const double *img, int lane) {
  if constexpr (C > 0) {
    constexpr int o = L::off(S), PW = L::RS / NP, PP = PW / 2;
    if constexpr (C == 6) {
      if (o / PW == pass) {
        double m[6];
#pragma unroll
        for (int q = 0; q < 6; q++) m[q] = packed_dbl<PP>(img, lane, o + q - PW * pass);
        a.ani(i, ph, m);
      }
    } else {
#pragma unroll
      for (int q = 0; q < C; q++)
        if ((o + q) / PW == pass) a.iso(i, ph, q, packed_dbl<PP>(img, lane, o + q - PW * pass));
    }
  }
}

template <int C>
__device__ __forceinline__ void packed_store(const Slot &sl, SlotAcc<C> &a, double *img, const Sink &k) {
  if constexpr (C > 0) {
    double r[C];
    bool ok = a.ok;
    if constexpr (C == 6) ok = invmat(a.v, r) && ok;
    else
#pragma unroll
      for (int q = 0; q < C; q++) r[q] = a.v[q];
    sink_rows<C>(sl, r, ok, img, k);
  }
}

// Output records (pmmg_hip_locate_interp_rec): each finished slot's row goes
// into an LDS image of the wave's 64 output records, in two halves of 8
// doubles (half 0 = record doubles 0-7 at img + 512 doubles, half 1 = 8-15 at
// img), each 4 swizzled 16-byte pieces per record; half 1 is written only
// after the last gather pass, so that with two passes the first pass's slots
// are staged while the second pass gathers into img[0, 512).  Then the wave
// stores whole records (kOutRecPieces pieces of 16 bytes each), one line per
// 16-double record and instruction-covered records whole, in input order or
// to each query's own record (Morton order).  okm: the doubles each lane
// writes (a failed MMG5_invmat leaves its slot's doubles untouched).
__device__ __forceinline__ double *rec_half(double *img, int h) { return h == 0 ? img + 512 : img; }
__device__ __forceinline__ void rec_put(double *img, int lane, int j, double x) {
  double *reg = rec_half(img, j >> 3);
  const int jj = j & 7;
  reg[2 * packed_pos<4>(lane, jj >> 1) + (jj & 1)] = x;
}

template <class L, int S, int C>
__device__ __forceinline__ void packed_stage(SlotAcc<C> &a, bool act, double *img, unsigned short *okm) {
  if constexpr (C > 0) {
    constexpr int o = L::off(S);
    const int lane = __lane_id();
    double r[C];
    bool ok = a.ok && act;
    if constexpr (C == 6) ok = invmat(a.v, r) && ok;
    else
#pragma unroll
      for (int q = 0; q < C; q++) r[q] = a.v[q];
#pragma unroll
    for (int q = 0; q < C; q++) rec_put(img, lane, o + q, r[q]);
    if (ok) okm[lane] |= (unsigned short)(((1u << C) - 1u) << o);
  }
}

// slot S is finished (stored) after the pass holding its last component
template <class L, int NP, int S, int C>
__device__ __forceinline__ void packed_finish(const Slots &Sl, SlotAcc<C> &a, int pass, double *img, const Sink &k,
                                              bool act, unsigned short *okm) {
  if constexpr (C > 0) {
    constexpr int PW = L::RS / NP;
    if (pass != (L::off(S) + C - 1) / PW) return;
    if (Sl.rec_out) packed_stage<L, S, C>(a, act, img, okm);
    else packed_store<C>(Sl.s[S], a, img, k);
  }
}

// the wave's staged output records to memory (see rec_half)
template <int RS>
__device__ __forceinline__ void rec_flush(double *out, const double *img, const unsigned short *okm, const Sink &k) {
  constexpr int PR = RS / 2; // 16-byte pieces per record
  const int lane = __lane_id();
#pragma unroll
  for (int t = 0; t < PR; t++) {
    const int p = 64 * t + lane, r = p / PR, kk = p - PR * r;
    const int dst = __shfl(k.ip, r);
    const unsigned m = (okm[r] >> (2 * kk)) & 3u;
    const double *reg = rec_half(const_cast<double *>(img), kk >> 2);
    const double2 v = reinterpret_cast<const double2 *>(reg)[packed_pos<4>(r, kk & 3)];
    double *q = out + (size_t)RS * (k.coalesced ? k.w0 + (size_t)r : (size_t)(dst - 1)) + 2 * kk;
    if (m == 3u) {
      if (k.coalesced) nt_store2(q, v.x, v.y);
      else *reinterpret_cast<double2 *>(q) = v;
    } else {
      if (m & 1u) q[0] = v.x;
      if (m & 2u) q[1] = v.y;
    }
  }
}

template <int NP, int C0, int C1, int C2, int C3, int C4, int C5>
__device__ __forceinline__ void vol_interp_packed(const Slots &S, bool acc, const VolLoc &loc, double *img,
                                                  const Sink &k, unsigned short *okm) {
  using L = PackedLayout<C0, C1, C2, C3, C4, C5>;
  constexpr int PW = L::RS / NP, PP = PW / 2; // doubles / 16-byte pieces per record and pass
  const int lane = __lane_id();
  SlotAcc<C0> a0;
  SlotAcc<C1> a1;
  SlotAcc<C2> a2;
  SlotAcc<C3> a3;
  SlotAcc<C4> a4;
  SlotAcc<C5> a5;
  if (!acc) { // idle lanes accumulate a valid row, never stored
    a0.ok = a1.ok = a2.ok = a3.ok = a4.ok = a5.ok = false;
  }
  const double2 *rec = reinterpret_cast<const double2 *>(S.rec);
  double2 *img2 = reinterpret_cast<double2 *>(img);
  if (S.rec_out) okm[lane] = 0;
#pragma unroll
  for (int pass = 0; pass < NP; pass++) {
    // the vertex loop is not unrolled: unrolled, the four vertices' copies of
    // a tensor slot's MMG5_invmat temporaries pushed the kernel past 128 VGPRs
#pragma unroll 1
    for (int i = 0; i < 4; i++) {
      const int myv = sel4(loc.v, i);
      const double ph = i == 0 ? loc.phi[0] : (i == 1 ? loc.phi[1] : (i == 2 ? loc.phi[2] : loc.phi[3]));
      // piece p = 64t + lane of the wave's records: record p / PP, piece p % PP
      // (every load instruction covers whole records: one line access per
      // record).  In batches of at most 4 instructions, each landed in LDS
      // before the next is issued: 16 VGPRs of loads in flight instead of 32
      constexpr int TB = PP < 4 ? PP : 4;
#pragma unroll
      for (int t0 = 0; t0 < PP; t0 += TB) {
        double2 b[TB];
#pragma unroll
        for (int t = 0; t < TB; t++) {
          const int p = 64 * (t0 + t) + lane, r = p / PP, kk = p - PP * r;
          const int v = __shfl(myv, r);
          b[t] = rec[(size_t)(L::RS / 2) * (v - 1) + PP * pass + kk];
        }
#pragma unroll
        for (int t = 0; t < TB; t++) {
          const int p = 64 * (t0 + t) + lane, r = p / PP, kk = p - PP * r;
          img2[packed_pos<PP>(r, kk)] = b[t];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      wait_lgkm();
      __builtin_amdgcn_wave_barrier();
      packed_take<L, NP, 0>(a0, pass, i, ph, img, lane);
      packed_take<L, NP, 1>(a1, pass, i, ph, img, lane);
      packed_take<L, NP, 2>(a2, pass, i, ph, img, lane);
      packed_take<L, NP, 3>(a3, pass, i, ph, img, lane);
      packed_take<L, NP, 4>(a4, pass, i, ph, img, lane);
      packed_take<L, NP, 5>(a5, pass, i, ph, img, lane);
      wait_lgkm();
      __builtin_amdgcn_wave_barrier(); // every lane has read its record: the image is free again
      // one vertex's pieces in registers at a time (left alone, the scheduler
      // hoists the four vertices' gathers together)
      __builtin_amdgcn_sched_barrier(0);
    }
    packed_finish<L, NP, 0>(S, a0, pass, img, k, acc, okm);
    packed_finish<L, NP, 1>(S, a1, pass, img, k, acc, okm);
    packed_finish<L, NP, 2>(S, a2, pass, img, k, acc, okm);
    packed_finish<L, NP, 3>(S, a3, pass, img, k, acc, okm);
    packed_finish<L, NP, 4>(S, a4, pass, img, k, acc, okm);
    packed_finish<L, NP, 5>(S, a5, pass, img, k, acc, okm);
  }
  if (S.rec_out) {
    wait_lgkm();
    __builtin_amdgcn_wave_barrier(); // every lane's record staged
    rec_flush<L::RS>(S.rec_out, img, okm, k);
    wait_lgkm();
    __builtin_amdgcn_wave_barrier();
  }
}

// The interpolation of the wave's 64 queries (lanes with acc); the walk's LDS
// slots must be dead (img aliases them in k_vol)
template <int PK, int C0, int C1, int C2, int C3, int C4, int C5>
__device__ __forceinline__ void vol_interp_wave(const Slots &S, bool acc, VolLoc &loc, int ip, double *img,
                                                const Sink &snk, unsigned short *okm) {
  if (!acc) { // idle lanes gather a valid row, never stored
    loc.v = make_int4(1, 1, 1, 1);
#pragma unroll
    for (int f = 0; f < 4; f++) loc.phi[f] = 0.0;
  }
  __builtin_amdgcn_wave_barrier(); // the walk's slots are dead: the buffer becomes the gather image
  if constexpr (PK > 0) {
    vol_interp_packed<PK, C0, C1, C2, C3, C4, C5>(S, acc, loc, img, snk, okm);
  } else if constexpr (C0 < 0) {
    if (acc) {
      const int vv[4] = {loc.v.x, loc.v.y, loc.v.z, loc.v.w};
      for (int s2 = 0; s2 < S.n; s2++) interp_dyn<4>(S.s[s2], ip, vv, loc.phi);
    }
  } else {
    vol_slot<C0>(S.s[0], acc, loc.v, loc.phi, img, snk);
    vol_slot<C1>(S.s[1], acc, loc.v, loc.phi, img, snk);
    vol_slot<C2>(S.s[2], acc, loc.v, loc.phi, img, snk);
    vol_slot<C3>(S.s[3], acc, loc.v, loc.phi, img, snk);
    vol_slot<C4>(S.s[4], acc, loc.v, loc.phi, img, snk);
    vol_slot<C5>(S.s[5], acc, loc.v, loc.phi, img, snk);
  }
}

// PK: 0 = one array per solution, 1 / 2 = packed records in 1 / 2 passes.
// lb.v non-null (split volume stage, r06; launched as the locate-only layout):
// the located records go to lb and k_vol_interp interpolates them.
template <int PK, int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(64) void k_vol(Bg bg, const Frame *fr, const unsigned long long *grid, int g,
                                            const double *qxyz, const uint8_t *pclass, const int *order,
                                            const double *qs, int np, ContEntry *cont, DevStats *st, Slots S,
                                            int *elem_out, int8_t *hit_out, int filter_steps,
                                            const int *order_flag, int xcd_run, int pad, int want, LocBuf lb,
                                            int blk0, ContArgs ca) {
  // want >= 0: the launch for one of the two orders (auto mode launches both, each after its own lists;
  // the other returns at once)
  if (want >= 0 && order_flag[0] != want) return;
  __shared__ VolShared<PK> sh;
  bstats_init(&sh.bs);
  __syncthreads();
  const LaneSlotsF L{(lds_float *)&sh.u.slots[__lane_id()]};
  const int i = (blk0 + xcd_block_runs(xcd_run)) * 64 + threadIdx.x;
  const bool sorted = order_flag[0] == 1; // the call's query order, decided on the device (the coherence test in k_bbox)
  bool active;
  int ip = 0;
  if (sorted) {
    active = i < st->nvol;
    if (active) ip = order[i];
  } else {
    active = i < np && __builtin_nontemporal_load(pclass + i) == PMMG_PT_VOL;
    ip = i + 1;
  }
  // 1. filter walk
  int status = 0, steps = 0, k = 0;
  double x[3];
  int4 tv = make_int4(1, 1, 1, 1);
  bool noseed = false;
  // the queries' coordinates, streamed once (non-temporal).  In input order
  // (and in the binning's processing-order copy) the wave's 64 rows are one
  // contiguous 1.5 KiB block: two instructions of 16-byte pieces through LDS
  // touch its 24 sectors once, where three per-lane double loads touched
  // them three times
  {
    const double *qrow = sorted ? qs : qxyz;
    const long long w0 = (long long)(i - __lane_id());
    if (qrow && w0 + 64 <= (sorted ? (long long)st->nvol : (long long)np) && ((uintptr_t)qrow & 15) == 0) {
      const ntd2 *src = reinterpret_cast<const ntd2 *>(qrow + 3 * w0);
      ntd2 *dst = reinterpret_cast<ntd2 *>(sh.u.slots);
      const int lane = __lane_id();
      const ntd2 a = __builtin_nontemporal_load(src + lane);
      ntd2 b = {0.0, 0.0};
      if (lane < 32) b = __builtin_nontemporal_load(src + 64 + lane);
      dst[lane] = a;
      if (lane < 32) dst[64 + lane] = b;
      wait_lgkm();
      __builtin_amdgcn_wave_barrier();
      const double *row = reinterpret_cast<const double *>(sh.u.slots) + 3 * lane;
      x[0] = row[0];
      x[1] = row[1];
      x[2] = row[2];
      wait_lgkm();
      __builtin_amdgcn_wave_barrier(); // the buffer holds the walk's vertex slots next
    } else if (active) {
      load_pt_nt(sorted && qs ? qs : qxyz, sorted && qs ? i + 1 : ip, x);
    }
  }
  if (active) {
    k = seed_vol(grid, g, fr, x, noseed);
    if (k == 0) {
      status = 2;
    } else {
      const int xq[3] = {quant(x[0], fr, 0), quant(x[1], fr, 1), quant(x[2], fr, 2)};
      tv = tetv_row(bg, k);
      int4 ad = adja_row(bg, k);
      unsigned m = 0xE4u; // local l in slot l
      {
        float q[3];
        rel_pt(bg.xq, tv.x, xq, q);
        L.put(0, q);
        rel_pt(bg.xq, tv.y, xq, q);
        L.put(1, q);
        rel_pt(bg.xq, tv.z, xq, q);
        L.put(2, q);
        rel_pt(bg.xq, tv.w, xq, q);
        L.put(3, q);
      }
      int hist[kHist];
#pragma unroll
      for (int h = 0; h < kHist; h++) hist[h] = 0;
      for (;;) {
        if (steps >= filter_steps) {
          status = 3;
          break;
        }
        ++steps;
#ifdef PMMG_HIP_MEASURE
        // measurement build, PMMG_HIP_PAD = v + 65536 t: v extra VALU
        // instructions and t extra L1 accesses (re-loads of the current
        // record) per walk step, to price each resource in the step
        if (pad & 0x1FFFFFFF) {
          float acc = (float)steps;
          for (int j = 0; j < (pad & 0xFFFF); j++) asm volatile("v_add_f32 %0, %0, %0" : "+v"(acc));
          int dummy = 0;
          for (int j = 0; j < ((pad >> 16) & 0x1FFF); j++)
            dummy += reinterpret_cast<const volatile int *>(bg.tetv + (size_t)(k - 1) * bg.tstride)[j & 3];
          if (acc == -1.0f && dummy == 0x7FFFFFFF) steps += 0; // keep both chains alive
          asm volatile("" ::"v"(acc), "v"(dummy));
        }
#endif
        const int r = step_f32(bg, xq, k, tv, ad, m, hist, L, walk_rsel(ip, steps));
        if (r != 0) {
          status = r;
          break;
        }
      }
    }
  }
  // 2. the reference's exact test at the candidate.  (r06: the candidates'
  // fp64 rows gathered by the wave cooperatively — ~1.1 line accesses per row
  // instead of two, 16 + 8 bytes per lane — took the volume stage +50 us at
  // cfg4, +25 at cfg3: the LDS round trip and the wave-wide wait cost more
  // than the accesses saved, profiles/r06q)
  VolLoc loc;
  bool acc = false;
  if (status == 1) {
    double p[4][3];
    load_tet_pts(bg, tv, p);
    // within EPS of a face: the exact continuation decides between this
    // tetra and its neighbour (prefer_strict)
    acc = exact_accept(x, p, tv, &loc, nullptr) && min4(loc.phi) > kEps;
  }
  const bool more = active && !acc;
  if (ca.fuse && !lb.v) {
    if (__any(more)) {
      const LaneSlotsD LD{&sh.u.dslots[__lane_id()]};
      __builtin_amdgcn_wave_barrier(); // the filter walk's slots are dead
      int st2 = 0, steps2 = 0;
      if (more && k > 0) {
        st2 = walk_exact(bg, x, ip, k, steps2, ca.maxstep, &loc, LD);
        acc = st2 == 1;
      }
      const bool fail = more && !acc;
      const int fslot = wave_append(&st->nfb_vol, fail);
      if (fail) {
        ca.fb[fslot] = ip;
        ca.fi.at(fslot);
      }
      wave_count(&sh.bs, kCntStuck, fail && st2 == 2);
      wave_count(&sh.bs, kCntLimit, fail && st2 == 3);
      steps += steps2;
      __builtin_amdgcn_wave_barrier(); // (the interpolation's image aliases the fp64 slots)
    }
  } else {
    const int slot = wave_append(&st->ncont, more);
    if (more) cont[slot] = ContEntry{ip, k};
  }
  wave_stats(&sh.bs, active, acc ? PMMG_HIT_VOL_WALK : 0, steps);
  wave_count(&sh.bs, kCntVolQueries, active);
  wave_count(&sh.bs, kCntExact, more);
  wave_count(&sh.bs, kCntNoSeed, active && noseed);
  if (lb.v && (sorted ? i < st->nvol : i < np)) { // split stage: the located record of processing index i
    __builtin_nontemporal_store(acc ? nti4{loc.v.x, loc.v.y, loc.v.z, loc.v.w} : nti4{0, 0, 0, 0}, lb.v + i);
    if (acc) {
      __builtin_nontemporal_store(ntd2{loc.phi[0], loc.phi[1]}, lb.p01 + i);
      __builtin_nontemporal_store(ntd2{loc.phi[2], loc.phi[3]}, lb.p23 + i);
    }
  }
  // 3. interpolation
#ifdef PMMG_HIP_MEASURE
  // measurement build: PMMG_HIP_PAD bit 30 — Morton order stores whole lines
  // at the processing position (wrong rows, the scattered stores' price);
  // bit 29 — no row stores in Morton order
  const Sink snk{!sorted || ((pad >> 30) & 1), (size_t)(i - __lane_id()), ip};
  if (sorted && ((pad >> 29) & 1)) acc = false;
#else
  const Sink snk{!sorted, (size_t)(i - __lane_id()), ip};
#endif
  if (__any(acc)) {
    if constexpr (PK > 0 || C0 != 0) vol_interp_wave<PK, C0, C1, C2, C3, C4, C5>(S, acc, loc, ip, sh.u.img, snk, sh.okm);
    if (acc) {
      if (sorted) { // scattered: cached stores (see wave_store_rows_scat)
        if (elem_out) elem_out[ip - 1] = k;
        if (hit_out) hit_out[ip - 1] = (int8_t)PMMG_HIT_VOL_WALK;
      } else {
        if (elem_out) __builtin_nontemporal_store(k, elem_out + ip - 1);
        if (hit_out) __builtin_nontemporal_store((int8_t)PMMG_HIT_VOL_WALK, hit_out + ip - 1);
      }
    }
  }
  __syncthreads();
  bstats_flush(&sh.bs, st);
}

// ---------------------------------------------------------------- split interpolation (r06)
//
// The second kernel of the split volume stage: the located records of 64
// consecutive processing indices per one-wave block (the walk kernel's block
// order), read as whole lines, then the same wave-cooperative interpolation
// as the fused kernel's third phase — but under its own register budget and
// occupancy, where in the fused kernel the interpolation's gathers were issued
// under the walk's.  Launched right after the walk kernel
// on the same stream.
template <int PK>
struct InterpShared {
  unsigned short okm[PK > 0 ? 64 : 1];
  double img[(PK > 0 ? 16 : 8) * 64];
};

template <int PK, int C0, int C1, int C2, int C3, int C4, int C5>
__global__ __launch_bounds__(64) void k_vol_interp(LocBuf lb, const int *order, const DevStats *st, int np, Slots S,
                                                   const int *order_flag, int xcd_run, int want, int blk0) {
  if (want >= 0 && order_flag[0] != want) return;
  __shared__ InterpShared<PK> sh;
  const int i = (blk0 + xcd_block_runs(xcd_run)) * 64 + threadIdx.x;
  const bool sorted = order_flag[0] == 1;
  const int bound = sorted ? st->nvol : np;
  VolLoc loc;
  bool acc = false;
  int ip = 0;
  if (i < bound) {
    const nti4 v = __builtin_nontemporal_load(lb.v + i);
    acc = v.x != 0;
    loc.v = make_int4(v.x, v.y, v.z, v.w);
    if (acc) {
      const ntd2 a = __builtin_nontemporal_load(lb.p01 + i), b = __builtin_nontemporal_load(lb.p23 + i);
      loc.phi[0] = a.x;
      loc.phi[1] = a.y;
      loc.phi[2] = b.x;
      loc.phi[3] = b.y;
    }
    ip = sorted ? order[i] : i + 1;
  }
  if (!__any(acc)) return;
  const Sink snk{!sorted, (size_t)(i - __lane_id()), ip};
  vol_interp_wave<PK, C0, C1, C2, C3, C4, C5>(S, acc, loc, ip, sh.img, snk, sh.okm);
}

} // namespace pmmg
