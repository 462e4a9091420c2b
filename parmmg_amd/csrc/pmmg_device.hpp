// pmmg_device.hpp — device-side arithmetic of the transfer step (included by
// pmmg_hip.hip only).
//
// Every floating-point expression keeps the reference's operation order
// (files cited per function) and the module is built with -ffp-contract=off,
// so the same element gives bit-identical barycentric coordinates and
// interpolated values as the reference arithmetic (oracle/pmmg_oracle.c).
// All small arrays are indexed with compile-time indices only (runtime picks
// go through the sel* helpers), which keeps them in registers: a runtime
// index into a local array sends it to scratch memory on CDNA.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "parmmg_hip.h"

namespace pmmg {

constexpr double kEps = 1.e-06;     // MMG5_EPS
constexpr double kEpsD2 = 1.0e-200; // MMG5_EPSD2
constexpr int kMaxSlot = 8;         // metric + up to 7 fields
constexpr int kHist = 4;            // visited-element history of a walk
constexpr int kBlock = 256;
#ifndef PMMG_XQ_STRIDE
#define PMMG_XQ_STRIDE 3
#endif
constexpr int kXqStride = PMMG_XQ_STRIDE; // ints per row of the fixed-point vertex copy (4: one aligned 16-byte load)

// Background mesh.  Tetra rows are read through tetv_row / adja_row: either
// two separate arrays (the reference's MMG5_Tetra.v and adja layouts,
// tstride 1) or one packed 32-byte record per tetra {v[4], adja[4]}
// (tetv = rec, adja = rec + 1, tstride 2), whose two halves share a cache
// line, so a walk step costs one line request for the tetra instead of two.
struct Bg {
  const double *xyz;
  const int *xq; // fixed-point copy of xyz (kXqStride int32 per vertex, Frame::quant), built per call
  const int4 *tetv;
  const int4 *adja;
  const int *triv;
  const int *adjt;
  int np, ne, nt;
  int tstride;
  double hausd;
  int fanmax; // cone test: fans longer than this take the full tria scan (kFanMax; test-only PMMG_HIP_FANMAX)
};

__device__ __forceinline__ int4 tetv_row(const Bg &bg, int k) { return bg.tetv[(size_t)(k - 1) * bg.tstride]; }
__device__ __forceinline__ int4 adja_row(const Bg &bg, int k) { return bg.adja[(size_t)(k - 1) * bg.tstride]; }

// one solution array in the reference layout (row of vertex v at
// in + code*(v-1)): code 1 = scalar, 3 = vector (both P1 iso interpolation),
// 6 = symmetric tensor (inverse-tensor interpolation)
struct Slot {
  const double *in; // row of vertex v at in + istride*(v-1)
  double *out;      // row of point ip at out + ostride*(ip-1)
  int code;
  int istride; // doubles between input rows: code (one array per solution) or the record stride (packed)
  int ostride; // doubles between output rows: code, or the output record stride (pmmg_hip_locate_interp_rec)
};

struct Slots {
  Slot s[kMaxSlot];
  int n;
  int has_met;        // slot 0 is the metric (boundary points treat it differently)
  const double *rec;  // packed per-vertex records (pmmg_hip_set_solutions_packed), else null
  double *rec_out;    // output records of the new points (same layout as rec), else null
};

// ------------------------------------------------------------ small helpers

__device__ __forceinline__ unsigned long long dkey(double d) {
  unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double dunkey(unsigned long long k) {
  unsigned long long u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
  return __longlong_as_double((long long)u);
}

// Element i of a register tuple, branch-free: a ternary chain on i is turned
// into a switch, i.e. divergent branches (exec-mask juggling per lane
// pattern) in the walk loops.
__device__ __forceinline__ unsigned bsel(unsigned a, unsigned b, unsigned bit) { return a ^ ((a ^ b) & (0u - bit)); }
__device__ __forceinline__ int sel4(const int4 &a, int i) {
  const unsigned b0 = (unsigned)i & 1u, b1 = ((unsigned)i >> 1) & 1u;
  return (int)bsel(bsel((unsigned)a.x, (unsigned)a.y, b0), bsel((unsigned)a.z, (unsigned)a.w, b0), b1);
}
__device__ __forceinline__ int sel3i(int a, int b, int c, int i) { return sel4(make_int4(a, b, c, c), i); }
__device__ __forceinline__ double sel3d(double a, double b, double c, int i) { return i == 0 ? a : (i == 1 ? b : c); }

__device__ __forceinline__ void load_pt(const double *xyz, int v, double *p) {
  const double *q = xyz + 3 * (size_t)(v - 1);
  p[0] = q[0];
  p[1] = q[1];
  p[2] = q[2];
}

__device__ __forceinline__ void load_pt_nt(const double *xyz, int v, double *p) {
  const double *q = xyz + 3 * (size_t)(v - 1);
  p[0] = __builtin_nontemporal_load(q);
  p[1] = __builtin_nontemporal_load(q + 1);
  p[2] = __builtin_nontemporal_load(q + 2);
}

__device__ __forceinline__ int wave_append(int *counter, bool pred) {
  unsigned long long m = __ballot(pred);
  if (m == 0ULL) return -1;
  int lane = __lane_id();
  int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  int rank = __popcll(m & ((1ULL << lane) - 1ULL));
  return pred ? base + rank : -1;
}

// XCD-aware block order (cdna_hip_programming.md T1): blocks are dealt
// round-robin over the 8 XCDs, each with a private 4 MiB L2.  Giving XCD x the
// contiguous range of logical blocks [x*n/8, (x+1)*n/8) keeps spatially
// adjacent queries (which walk the same tetra) on one L2.  Bijective for any n.
__device__ __forceinline__ int xcd_block() {
  const int b = blockIdx.x, n = gridDim.x;
  const int x = b & 7, q = n >> 3, r = n & 7;
  const int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + (b >> 3);
}

// The same in runs of G logical blocks dealt round-robin over the XCDs
// (G <= 0: xcd_block's contiguous eighths): each XCD still walks spatially
// adjacent queries within a run, but a costly stretch of the input (the
// appended points of an Mmg-like numbering, the last sixth of the range) is
// shared by all eight XCDs instead of landing on one or two of them while the
// others idle (r04a: 15.0 -> 10.7 resident waves per CU).  Bijective for any n.
__device__ __forceinline__ int xcd_block_runs(int G) {
  if (G <= 0) return xcd_block();
  const int b = blockIdx.x, n = gridDim.x;
  const int x = b & 7, j = b >> 3;      // the j-th block dispatched to XCD x
  const int nruns = (n + G - 1) / G;     // runs of G logical blocks (the last one short)
  const int full = n / (8 * G);          // rounds in which every XCD takes a whole run
  if (j < full * G) return ((j / G) * 8 + x) * G + j % G;
  // the tail: the remaining n - 8 G full blocks, in contiguous eighths
  const int base = 8 * G * full, m = n - base;
  const int q = m >> 3, r = m & 7;
  const int jj = j - full * G;
  (void)nruns;
  return base + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + jj;
}

// Grid-stride iteration over [0, n) split into 8 contiguous chunks, one per
// XCD (blockIdx % 8), for kernels launched with a fixed grid (a multiple of 8).
// iters is uniform across a block, so wave-collective code may run per iteration.
struct XcdChunk {
  long long start, hi, stride;
  int iters;
};
__device__ __forceinline__ XcdChunk xcd_chunk(long long n) {
  const int x = blockIdx.x & 7, bpx = gridDim.x >> 3, bi = blockIdx.x >> 3;
  XcdChunk c;
  const long long lo = n * x / 8;
  c.hi = n * (x + 1) / 8;
  c.stride = (long long)bpx * blockDim.x;
  c.iters = (int)((c.hi - lo + c.stride - 1) / c.stride);
  c.start = lo + (long long)bi * blockDim.x + threadIdx.x;
  return c;
}

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ __forceinline__ int cell_coord(double x, double lo, double inv, int g) {
  double t = (x - lo) * inv;
  int c = (t > 0.0) ? (int)t : 0;
  return c < g ? c : g - 1;
}

// ------------------------------------------------------------ tetra geometry

// MMG5_nonUnitNorPts: (b-a)x(c-a)
__device__ __forceinline__ void nonunit_normal(const double *a, const double *b, const double *c, double *n) {
  double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  n[0] = aby * acz - abz * acy;
  n[1] = abz * acx - abx * acz;
  n[2] = abx * acy - aby * acx;
}

// MMG5_orvol
__device__ __forceinline__ double orvol4(const double *p0, const double *p1, const double *p2, const double *p3) {
  double ax = p2[0] - p0[0], ay = p2[1] - p0[1], az = p2[2] - p0[2];
  double bx = p3[0] - p0[0], by = p3[1] - p0[1], bz = p3[2] - p0[2];
  return (p1[0] - p0[0]) * (ay * bz - az * by) + (p1[1] - p0[1]) * (az * bx - ax * bz) +
         (p1[2] - p0[2]) * (ax * by - ay * bx);
}

// Numerators of PMMG_barycoord3d_compute (barycoord_pmmg.c:238-257) on face
// normals recomputed from the vertices (PMMG_precompute_faceAreas,
// locate_pmmg.c:107-119; the reference's 96 B/tetra faceAreas array is never
// stored): s[f] = (x - p_idir[f][0]) . n_f, so that bary[f] = -s[f] / vol.
// Returns vol = MMG5_orvol.
__device__ __forceinline__ double tet_dots(const double *x, const double *p0, const double *p1, const double *p2,
                                           const double *p3, double *s) {
  // sched_barrier: compute the faces one after the other.  Left alone, the
  // scheduler interleaves all four for ILP and the walk kernels need ~100
  // VGPRs (4 waves/SIMD); latency-bound walks gain more from occupancy.
  double vol = orvol4(p0, p1, p2, p3);
  __builtin_amdgcn_sched_barrier(0);
  double n[3];
  nonunit_normal(p1, p2, p3, n); // face 0: idir {1,2,3}
  s[0] = (x[0] - p1[0]) * n[0] + (x[1] - p1[1]) * n[1] + (x[2] - p1[2]) * n[2];
  __builtin_amdgcn_sched_barrier(0);
  nonunit_normal(p0, p3, p2, n); // face 1: idir {0,3,2}
  s[1] = (x[0] - p0[0]) * n[0] + (x[1] - p0[1]) * n[1] + (x[2] - p0[2]) * n[2];
  __builtin_amdgcn_sched_barrier(0);
  nonunit_normal(p0, p1, p3, n); // face 2: idir {0,1,3}
  s[2] = (x[0] - p0[0]) * n[0] + (x[1] - p0[1]) * n[1] + (x[2] - p0[2]) * n[2];
  __builtin_amdgcn_sched_barrier(0);
  nonunit_normal(p0, p2, p1, n); // face 3: idir {0,2,1}
  s[3] = (x[0] - p0[0]) * n[0] + (x[1] - p0[1]) * n[1] + (x[2] - p0[2]) * n[2];
  return vol;
}

// PMMG_barycoord3d_compute: b[f] = -s[f] / vol, unsorted
__device__ __forceinline__ double tet_bary(const double *x, const double *p0, const double *p1, const double *p2,
                                           const double *p3, double *b) {
  double s[4];
  double vol = tet_dots(x, p0, p1, p2, p3, s);
#pragma unroll
  for (int f = 0; f < 4; f++) b[f] = -s[f] / vol;
  return vol;
}

// Order of the reference's qsort (glibc merge sort: stable) = ascending
// (value, index).  The reference only consumes the sorted order for the inside
// test, the walk direction and isBorder; PMMG_barycoord_get de-permutes the
// values again, so the interpolation uses the unsorted b[] directly.
__device__ __forceinline__ bool before(double va, int a, double vb, int b) {
  return (va < vb) || (va == vb && a < b);
}

__device__ __forceinline__ void ranks4(const double *b, int *r) {
#pragma unroll
  for (int f = 0; f < 4; f++) {
    int c = 0;
#pragma unroll
    for (int g = 0; g < 4; g++)
      if (g != f && before(b[g], g, b[f], f)) c++;
    r[f] = c;
  }
}

__device__ __forceinline__ void ranks3(const double *b, int *r) {
#pragma unroll
  for (int f = 0; f < 3; f++) {
    int c = 0;
#pragma unroll
    for (int g = 0; g < 3; g++)
      if (g != f && before(b[g], g, b[f], f)) c++;
    r[f] = c;
  }
}

__device__ __forceinline__ double min4(const double *b) {
  double m = b[0];
  m = b[1] < m ? b[1] : m;
  m = b[2] < m ? b[2] : m;
  m = b[3] < m ? b[3] : m;
  return m;
}

// PMMG_barycoord3d_getClosest / 2d_getClosest (barycoord_pmmg.c:371-404): unit
// coordinate on the nearest vertex (first minimum in vertex order)
template <int NV>
__device__ __forceinline__ void closest_vertex(const double *x, const double (*p)[3], double *phi) {
  double d[3];
  for (int i = 0; i < 3; i++) d[i] = x[i] - p[0][i];
  double mn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  int it = 0;
#pragma unroll
  for (int j = 1; j < NV; j++) {
    for (int i = 0; i < 3; i++) d[i] = x[i] - p[j][i];
    double nrm = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (nrm < mn) { mn = nrm; it = j; }
  }
#pragma unroll
  for (int j = 0; j < NV; j++) phi[j] = (j == it) ? 1.0 : 0.0;
}

// ------------------------------------------------------------ MMG5_invmat

// Symmetric 3x3 inverse (m11,m12,m13,m22,m23,m33), restated from Mmg
// @889d408: diagonal shortcut below MMG5_EPS off-diagonal, failure on a zero
// matrix or |det| < MMG5_EPSD2.  Results are produced in registers and only
// stored when the inversion succeeds.
__device__ __forceinline__ bool invmat(const double *m, double *mi) {
  double vmax = fabs(m[1]), maxx = fabs(m[2]);
  if (maxx > vmax) vmax = maxx;
  maxx = fabs(m[4]);
  if (maxx > vmax) vmax = maxx;
  double r0, r1, r2, r3, r4, r5;
  bool ok;
  if (vmax < kEps) {
    r0 = 1. / m[0];
    r3 = 1. / m[3];
    r5 = 1. / m[5];
    r1 = r2 = r4 = 0.0;
    ok = true;
  } else {
    double vm = fabs(m[0]);
#pragma unroll
    for (int k = 1; k < 6; k++) {
      double mx = fabs(m[k]);
      if (mx > vm) vm = mx;
    }
    double aa = m[3] * m[5] - m[4] * m[4];
    double bb = m[4] * m[2] - m[1] * m[5];
    double cc = m[1] * m[4] - m[2] * m[3];
    double det = m[0] * aa + m[1] * bb + m[2] * cc;
    ok = !(vm == 0.0) && !(fabs(det) < kEpsD2);
    det = 1.0 / det;
    r0 = aa * det;
    r1 = bb * det;
    r2 = cc * det;
    r3 = (m[0] * m[5] - m[2] * m[2]) * det;
    r4 = (m[1] * m[2] - m[0] * m[4]) * det;
    r5 = (m[0] * m[3] - m[1] * m[1]) * det;
  }
  mi[0] = r0; mi[1] = r1; mi[2] = r2; mi[3] = r3; mi[4] = r4; mi[5] = r5;
  return ok;
}

__device__ __forceinline__ void load6(const double *p, double *m) {
  const double2 *q = reinterpret_cast<const double2 *>(p);
  double2 a = q[0], b = q[1], c = q[2];
  m[0] = a.x; m[1] = a.y; m[2] = b.x; m[3] = b.y; m[4] = c.x; m[5] = c.y;
}

// Output rows are written once and never re-read by the step: non-temporal
// stores keep them from displacing the gathered background rows in L2.
typedef double ntd2 __attribute__((ext_vector_type(2)));
typedef int nti4 __attribute__((ext_vector_type(4)));
typedef int nti2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void nt_store(double *p, double v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void nt_store2(double *p, double a, double b) {
  ntd2 v = {a, b};
  __builtin_nontemporal_store(v, reinterpret_cast<ntd2 *>(p));
}

// One lane's own row at a scattered position (the surface points, the exact
// continuation, the fallbacks): non-temporal pieces (r03ab: plain stores
// here made the surface branch alone 0.40 -> 0.67 ms)
__device__ __forceinline__ void store6(double *p, const double *m) {
  if (((uintptr_t)p & 15) == 0) {
    nt_store2(p, m[0], m[1]);
    nt_store2(p + 2, m[2], m[3]);
    nt_store2(p + 4, m[4], m[5]);
  } else { // a tensor at an odd offset of an output record
#pragma unroll
    for (int j = 0; j < 6; j++) nt_store(p + j, m[j]);
  }
}

// ------------------------------------------------------------ interpolators

// PMMG_interp{3,4}bar_iso (interpmesh_pmmg.c:125-149, 206-230):
// out[j] = 0; out[j] += phi_i * old[v_i][j], i ascending
// PMMG_interp{3,4}bar_iso (interpmesh_pmmg.c:125-165, 206-246): the row
// value acc = sum_i phi_i * row_i (accumulated from 0.0 in vertex order)
template <int NV, int SZ>
__device__ __forceinline__ void interp_iso_row(const double *in, int stride, const int *v, const double *phi,
                                               double *acc) {
  double row[NV][SZ];
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j < SZ; j++) row[i][j] = in[(size_t)stride * (v[i] - 1) + j];
#pragma unroll
  for (int j = 0; j < SZ; j++) acc[j] = 0.0;
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j < SZ; j++) acc[j] += phi[i] * row[i][j];
}

// PMMG_interp{3,4}bar_ani (interpmesh_pmmg.c:166-190, 247-270):
// M = invmat( sum_i phi_i invmat(M_i) ); false (row left untouched by the
// reference) if any inversion fails
template <int NV>
__device__ __forceinline__ bool interp_ani_row(const double *in, int stride, const int *v, const double *phi,
                                               double *r) {
  double m[NV][6];
#pragma unroll
  for (int i = 0; i < NV; i++) load6(in + (size_t)stride * (v[i] - 1), m[i]);
  double mint[6], mi[6];
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    ok = invmat(m[i], mi) && ok;
#pragma unroll
    for (int s = 0; s < 6; s++) mint[s] = (i == 0) ? phi[0] * mi[s] : mint[s] + phi[i] * mi[s];
  }
  return invmat(mint, r) && ok;
}

// the row of one slot: returns false when the reference leaves it untouched
template <int NV, int CODE>
__device__ __forceinline__ bool interp_row(const Slot &sl, const int *v, const double *phi, double *r) {
  if constexpr (CODE == 6) return interp_ani_row<NV>(sl.in, sl.istride, v, phi, r);
  else {
    interp_iso_row<NV, CODE>(sl.in, sl.istride, v, phi, r);
    return true;
  }
}

template <int NV, int CODE>
__device__ __forceinline__ void interp_code(const Slot &sl, int ip, const int *v, const double *phi) {
  double r[CODE];
  if (!interp_row<NV, CODE>(sl, v, phi, r)) return;
  double *out = sl.out + (size_t)sl.ostride * (ip - 1);
  if constexpr (CODE == 6) store6(out, r);
  else {
#pragma unroll
    for (int j = 0; j < CODE; j++) nt_store(out + j, r[j]);
  }
}

template <int NV>
__device__ __forceinline__ void interp_dyn(const Slot &sl, int ip, const int *v, const double *phi) {
  if (sl.code == 6) interp_code<NV, 6>(sl, ip, v, phi);
  else if (sl.code == 3) interp_code<NV, 3>(sl, ip, v, phi);
  else interp_code<NV, 1>(sl, ip, v, phi);
}

// PMMG_interp2bar_{iso,ani} (interpmesh_pmmg.c:50-110) on edge l of a tria
__device__ __forceinline__ void interp_edge(const Slot &sl, int ip, const int *v, int l, const double *phi) {
  const int i0 = l == 0 ? 1 : (l == 1 ? 2 : 0); // MMG5_inxt2[l]
  const int i1 = l == 0 ? 2 : (l == 1 ? 0 : 1); // MMG5_iprv2[l]
  const int v0 = sel3i(v[0], v[1], v[2], i0), v1 = sel3i(v[0], v[1], v[2], i1);
  const double f0 = sel3d(phi[0], phi[1], phi[2], i0), f1 = sel3d(phi[0], phi[1], phi[2], i1);
  if (sl.code == 6) {
    double m[6], mi0[6], mi1[6], mint[6], r[6];
    load6(sl.in + (size_t)sl.istride * (v0 - 1), m);
    bool ok = invmat(m, mi0);
    load6(sl.in + (size_t)sl.istride * (v1 - 1), m);
    ok = invmat(m, mi1) && ok;
#pragma unroll
    for (int s = 0; s < 6; s++) mint[s] = f0 * mi0[s] + f1 * mi1[s];
    if (invmat(mint, r) && ok) store6(sl.out + (size_t)sl.ostride * (ip - 1), r);
  } else {
    // sizes 1 and 3 (a vertex / edge hit of the metric is size 1 or 6; the
    // fields always go through interp3bar)
    for (int j = 0; j < sl.code; j++)
      sl.out[(size_t)sl.ostride * (ip - 1) + j] =
          f0 * sl.in[(size_t)sl.istride * (v0 - 1) + j] + f1 * sl.in[(size_t)sl.istride * (v1 - 1) + j];
  }
}

__device__ __forceinline__ void copy_row(const Slot &sl, int ip, int vsrc) {
  double *out = sl.out + (size_t)sl.ostride * (ip - 1);
  const double *in = sl.in + (size_t)sl.istride * (vsrc - 1);
  if (sl.code == 6) {
    double m[6];
    load6(in, m);
    store6(out, m);
  } else if (sl.code == 3) {
    out[0] = in[0]; out[1] = in[1]; out[2] = in[2];
  } else {
    out[0] = in[0];
  }
}

// boundary point (interpmesh_pmmg.c:563-595): metric by vertex copy / edge /
// face, every field by interp3bar
__device__ __forceinline__ void interp_bdy(const Slots &S, int ip, const int *v, const double *phi, int edge,
                                           int vertex) {
  for (int s = 0; s < S.n; s++) {
    const Slot &sl = S.s[s];
    if (s == 0 && S.has_met) {
      if (vertex >= 0) copy_row(sl, ip, sel3i(v[0], v[1], v[2], vertex));
      else if (edge >= 0) interp_edge(sl, ip, v, edge, phi);
      else interp_dyn<3>(sl, ip, v, phi);
    } else {
      interp_dyn<3>(sl, ip, v, phi);
    }
  }
}

// ------------------------------------------------------------ tria geometry

struct TriGeom {
  int v[3];
  double p[3][3];
  double n[3]; // unit normal
  double q;    // |nonunit normal| (ptr->qual)
};

// vertices + PMMG_precompute_triaNormals (locate_pmmg.c:74-87)
__device__ __forceinline__ void tri_load(const Bg &bg, int k, TriGeom &t) {
  const int *tv = bg.triv + 3 * (size_t)(k - 1);
  t.v[0] = tv[0];
  t.v[1] = tv[1];
  t.v[2] = tv[2];
  load_pt(bg.xyz, t.v[0], t.p[0]);
  load_pt(bg.xyz, t.v[1], t.p[1]);
  load_pt(bg.xyz, t.v[2], t.p[2]);
  nonunit_normal(t.p[0], t.p[1], t.p[2], t.n);
  t.q = sqrt(t.n[0] * t.n[0] + t.n[1] * t.n[1] + t.n[2] * t.n[2]);
  double dd = 1.0 / t.q;
  t.n[0] *= dd;
  t.n[1] *= dd;
  t.n[2] *= dd;
}

// PMMG_quickarea (barycoord_pmmg.c:44-61)
__device__ __forceinline__ double quickarea(const double *a, const double *b, const double *c, const double *n) {
  double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  double a0 = aby * acz - abz * acy, a1 = abz * acx - abx * acz, a2 = abx * acy - aby * acx;
  return a0 * n[0] + a1 * n[1] + a2 * n[2];
}

// PMMG_barycoord2d_compute (barycoord_pmmg.c:191-223): vertices / area of
// `pv`, unit normal n; returns the normal distance
__device__ __forceinline__ double tri_bary(const double *x, const double (*pv)[3], double q, const double *n, double *b) {
  double dist = 0.0, proj[3];
  for (int i = 0; i < 3; i++) dist += (x[i] - pv[0][i]) * n[i];
  for (int i = 0; i < 3; i++) proj[i] = x[i] - dist * n[i];
  b[0] = quickarea(proj, pv[1], pv[2], n) / q;
  b[1] = quickarea(proj, pv[2], pv[0], n) / q;
  b[2] = quickarea(proj, pv[0], pv[1], n) / q;
  return dist;
}

__device__ __forceinline__ void tri_pick(const TriGeom &t, int i, double *p) {
  p[0] = sel3d(t.p[0][0], t.p[1][0], t.p[2][0], i);
  p[1] = sel3d(t.p[0][1], t.p[1][1], t.p[2][1], i);
  p[2] = sel3d(t.p[0][2], t.p[1][2], t.p[2][2], i);
}

// PMMG_locatePointInWedge (locate_pmmg.c:286-334): -1 too far, 4 inside (phi
// written), else the local vertex whose cone must be tested
__device__ __forceinline__ int tri_wedge(double hausd, const TriGeom &t, int l, const double *x, double *phi) {
  const int i0 = l == 0 ? 1 : (l == 1 ? 2 : 0), i1 = l == 0 ? 2 : (l == 1 ? 0 : 1);
  double p0[3], p1[3];
  tri_pick(t, i0, p0);
  tri_pick(t, i1, p1);
  double p[3], a[3], norm2 = 0.0, alpha = 0.0, dist = 0.0;
  for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
  for (int d = 0; d < 3; d++) a[d] = p1[d] - p0[d];
  for (int d = 0; d < 3; d++) norm2 += a[d] * a[d];
  for (int d = 0; d < 3; d++) alpha += a[d] * p[d];
  for (int d = 0; d < 3; d++) p[d] -= (alpha / norm2) * a[d];
  for (int d = 0; d < 3; d++) dist += p[d] * p[d];
  dist = sqrt(dist);
  if (dist > hausd) return -1;
  if (alpha < 0.0) return i0;
  if (alpha > norm2) return i1;
  const double w0 = 1.0 - alpha / norm2, w1 = alpha / norm2;
  phi[0] = (l == 0) ? 0.0 : (i0 == 0 ? w0 : w1);
  phi[1] = (l == 1) ? 0.0 : (i0 == 1 ? w0 : w1);
  phi[2] = (l == 2) ? 0.0 : (i0 == 2 ? w0 : w1);
  return 4;
}

// PMMG_locatePointInCone (locate_pmmg.c:209-270) with a fresh visited state
// per query: x is in the shadow cone of vertex ip iff every surface edge
// leaving ip (every other vertex of every tria of ip, the node->tria list of
// PMMG_precompute_nodeTrias) makes a non-acute angle with x - p(ip), and
// |x - p(ip)| <= hausd (tested inside the scan, as the reference does).
// The reference skips neighbours flagged by earlier queries of the same
// vertex (a state leak, :248-249; the oracle's ORC_MODE_FAITHFUL); here every
// neighbour is tested.
//
// The trias of ip are reached by rotating through adjt around ip from tria k
// in both directions.  When the rotation comes back to k the fan is complete
// (a manifold vertex).  Otherwise (a border edge, a non-manifold edge — adjt
// is 0 on edges of more than two trias — or a fan longer than kFanMax) the
// test scans every tria for those containing ip: the exact node->tria list,
// at O(nt) for the rare query that needs it, instead of building the list for
// every vertex on every call.
constexpr int kFanMax = 64;

__device__ __forceinline__ int cone_tria(const Bg &bg, int tt, int ip, const double *p0, const double *p,
                                         double dist) {
  // 1 ok, 0 outside the cone
  const int *tv = bg.triv + 3 * (size_t)(tt - 1);
  for (int l = 0; l < 3; l++) {
    const int jp = tv[l];
    if (jp == ip) continue;
    if (dist > bg.hausd) return 0;
    double p1[3], e[3], alpha = 0.0;
    load_pt(bg.xyz, jp, p1);
    for (int d = 0; d < 3; d++) e[d] = p1[d] - p0[d];
    for (int d = 0; d < 3; d++) alpha += e[d] * p[d];
    if (alpha > 0.0) return 0;
  }
  return 1;
}

// the O(nt) scan of the rare open / non-manifold / long fan.  Out of line,
// and every argument passed by value: a pointer to the caller's local arrays
// (or a reference to its Bg) across a call boundary puts them in scratch
// memory for the whole kernel (k_bdy: 144 B per lane in r02).
__device__ __noinline__ bool tri_cone_scan(const int *triv, const double *xyz, int nt, double hausd, int ip,
                                           double p0x, double p0y, double p0z, double px, double py, double pz,
                                           double dist) {
  if (dist > hausd) { // cone_tria's test before the first edge of the first tria of ip
    for (int tt = 1; tt <= nt; tt++) {
      const int *tv = triv + 3 * (size_t)(tt - 1);
      if (tv[0] > 0 && (tv[0] == ip || tv[1] == ip || tv[2] == ip)) return false;
    }
    return true;
  }
  for (int tt = 1; tt <= nt; tt++) {
    const int *tv = triv + 3 * (size_t)(tt - 1);
    if (tv[0] <= 0 || (tv[0] != ip && tv[1] != ip && tv[2] != ip)) continue;
    for (int l = 0; l < 3; l++) { // cone_tria (the distance test passed above)
      const int jp = tv[l];
      if (jp == ip) continue;
      const double *q = xyz + 3 * (size_t)(jp - 1);
      const double e0 = q[0] - p0x, e1 = q[1] - p0y, e2 = q[2] - p0z;
      double alpha = 0.0;
      alpha += e0 * px;
      alpha += e1 * py;
      alpha += e2 * pz;
      if (alpha > 0.0) return false;
    }
  }
  return true;
}

__device__ __forceinline__ bool tri_cone(const Bg &bg, int k, int iloc, const TriGeom &t, const double *x,
                                         int &scans) {
  const int ip = sel3i(t.v[0], t.v[1], t.v[2], iloc);
  double p0[3], p[3], dist = 0.0;
  tri_pick(t, iloc, p0);
  for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
  for (int d = 0; d < 3; d++) dist += p[d] * p[d];
  dist = sqrt(dist);
  if (!cone_tria(bg, k, ip, p0, p, dist)) return false;
  for (int dir = 0; dir < 2; dir++) {
    int tcur = k;
    int e = dir == 0 ? (iloc + 1) % 3 : (iloc + 2) % 3; // an edge of tcur incident to ip
    for (int it = 0;; it++) {
      if (it == bg.fanmax) {
        ++scans;
        return tri_cone_scan(bg.triv, bg.xyz, bg.nt, bg.hausd, ip, p0[0], p0[1], p0[2], p[0], p[1], p[2], dist);
      }
      const int code = bg.adjt[3 * (size_t)(tcur - 1) + e];
      const int tn = code / 3, en = code % 3;
      if (tn == 0) { // open or non-manifold fan
        ++scans;
        return tri_cone_scan(bg.triv, bg.xyz, bg.nt, bg.hausd, ip, p0[0], p0[1], p0[2], p[0], p[1], p[2], dist);
      }
      if (tn == k) return true;                                // the fan closed: every tria tested
      if (!cone_tria(bg, tn, ip, p0, p, dist)) return false;
      const int *tvn = bg.triv + 3 * (size_t)(tn - 1);
      const int lvn = (tvn[0] == ip) ? 0 : ((tvn[1] == ip) ? 1 : 2);
      const int ea = (lvn + 1) % 3, eb = (lvn + 2) % 3;
      e = (ea == en) ? eb : ea;
      tcur = tn;
    }
  }
  return true;
}

} // namespace pmmg
