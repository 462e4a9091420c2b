/*
 * pmmg_oracle.c — sequential CPU restatement of PMMG_interpMetricsAndFields.
 *
 * TEST INFRASTRUCTURE ONLY (see pmmg_oracle.h for the parity status and the
 * rule that the product path never touches this file).
 *
 * Every function names the reference code it restates.  Floating-point
 * expressions keep the reference's operation order and are compiled with
 * -ffp-contract=off, so the HIP module (built the same way) can be compared
 * bit for bit.  The Mmg primitives (MMG5_orvol, MMG5_nonUnitNorPts,
 * MMG5_invmat, MMG5_idir/inxt2/iprv2, MMG5_EPS) are restated from Mmg
 * @889d408's published source; they are not in the container.
 */
#define _POSIX_C_SOURCE 199309L
#include "pmmg_oracle.h"
#include <pthread.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* Mmg tables (src/common/mmgcommon.h @889d408) */
static const int kIdir[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}}; /* MMG5_idir  */
static const int kInxt2[5] = {1, 2, 0, 1, 2};                                /* MMG5_inxt2 */
static const int kIprv2[3] = {2, 0, 1};                                      /* MMG5_iprv2 */

enum {
  HIT_NONE = 0, HIT_VOL_WALK, HIT_VOL_EXHAUST, HIT_VOL_CLOSEST, HIT_BDY_FACE, HIT_BDY_EDGE,
  HIT_BDY_VERTEX, HIT_BDY_WEDGE, HIT_BDY_CONE, HIT_BDY_EXHAUST, HIT_BDY_STALE, HIT_BDY_CLOSEST,
};

/* PMMG_barycoord, src/barycoord_pmmg.h:41-44 */
typedef struct { int idx; double val; } bcoord;

#define PT(bg, ip) ((bg)->xyz + 3 * (size_t)((ip) - 1))
#define TETV(bg, k, i) ((bg)->tetv[4 * (size_t)((k) - 1) + (i)])
#define ADJA(bg, k, i) ((bg)->adja[4 * (size_t)((k) - 1) + (i)])
#define TRIV(bg, k, i) ((bg)->triv[3 * (size_t)((k) - 1) + (i)])
#define ADJT(bg, k, i) ((bg)->adjt[3 * (size_t)((k) - 1) + (i)])

/* ---------------- Mmg arithmetic (restated, unpinned) ---------------- */

/* MMG5_orvol: 6x oriented volume (p1-p0).((p2-p0)x(p3-p0)) */
static double orvol4(const double *p0, const double *p1, const double *p2, const double *p3) {
  double ax = p2[0] - p0[0], ay = p2[1] - p0[1], az = p2[2] - p0[2];
  double bx = p3[0] - p0[0], by = p3[1] - p0[1], bz = p3[2] - p0[2];
  return (p1[0] - p0[0]) * (ay * bz - az * by) + (p1[1] - p0[1]) * (az * bx - ax * bz) +
         (p1[2] - p0[2]) * (ax * by - ay * bx);
}

/* MMG5_nonUnitNorPts: (b-a)x(c-a) */
static void nonunit_normal(const double *a, const double *b, const double *c, double *n) {
  double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  n[0] = aby * acz - abz * acy;
  n[1] = abz * acx - abx * acz;
  n[2] = abx * acy - aby * acx;
}

/* MMG5_invmat: inverse of a symmetric 3x3 stored m11,m12,m13,m22,m23,m33 */
int orc_invmat(const double *m, double *mi) {
  double vmax = fabs(m[1]), maxx = fabs(m[2]);
  if (maxx > vmax) vmax = maxx;
  maxx = fabs(m[4]);
  if (maxx > vmax) vmax = maxx;
  if (vmax < ORC_EPS) { /* diagonal shortcut */
    mi[0] = 1. / m[0];
    mi[3] = 1. / m[3];
    mi[5] = 1. / m[5];
    mi[1] = mi[2] = mi[4] = 0.0;
    return 1;
  }
  vmax = fabs(m[0]);
  for (int k = 1; k < 6; k++) {
    maxx = fabs(m[k]);
    if (maxx > vmax) vmax = maxx;
  }
  if (vmax == 0.0) return 0;
  double aa = m[3] * m[5] - m[4] * m[4];
  double bb = m[4] * m[2] - m[1] * m[5];
  double cc = m[1] * m[4] - m[2] * m[3];
  double det = m[0] * aa + m[1] * bb + m[2] * cc;
  if (fabs(det) < ORC_EPSD2) return 0;
  det = 1.0 / det;
  mi[0] = aa * det;
  mi[1] = bb * det;
  mi[2] = cc * det;
  mi[3] = (m[0] * m[5] - m[2] * m[2]) * det;
  mi[4] = (m[1] * m[2] - m[0] * m[4]) * det;
  mi[5] = (m[0] * m[3] - m[1] * m[1]) * det;
  return 1;
}

/* ---------------- barycentric coordinates (src/barycoord_pmmg.c) ---------------- */

/* PMMG_barycoord_compare + qsort: ascending, ties keep input order (glibc
 * 2.35 qsort is a merge sort for these sizes, i.e. stable). */
static void bc_sort(bcoord *b, int n) {
  for (int i = 1; i < n; i++) {
    bcoord t = b[i];
    int j = i - 1;
    while (j >= 0 && b[j].val > t.val) { b[j + 1] = b[j]; j--; }
    b[j + 1] = t;
  }
}

/* PMMG_barycoord_get, barycoord_pmmg.c:72-78 */
static void bc_get(double *val, const bcoord *phi, int ndim) {
  for (int i = 0; i < ndim; i++) val[phi[i].idx] = phi[i].val;
}

/* PMMG_barycoord3d_compute, barycoord_pmmg.c:238-257, with face normals and
 * volume supplied (faceAreas / pt->qual of the reference) */
static void bc3d_compute(const orc_background *bg, int k, const double *fa, double vol,
                         const double *x, bcoord *b) {
  for (int f = 0; f < 4; f++) {
    const double *n = fa + 3 * f;
    const double *c0 = PT(bg, TETV(bg, k, kIdir[f][0]));
    b[f].val = -((x[0] - c0[0]) * n[0] + (x[1] - c0[1]) * n[1] + (x[2] - c0[2]) * n[2]) / vol;
    b[f].idx = f;
  }
}

/* face normals + volume of tetra k (PMMG_precompute_faceAreas, locate_pmmg.c:101-122) */
static double tet_geom(const orc_background *bg, int k, double *fa) {
  const double *p[4];
  for (int i = 0; i < 4; i++) p[i] = PT(bg, TETV(bg, k, i));
  for (int f = 0; f < 4; f++) nonunit_normal(p[kIdir[f][0]], p[kIdir[f][1]], p[kIdir[f][2]], fa + 3 * f);
  return orvol4(p[0], p[1], p[2], p[3]);
}

/* PMMG_barycoord3d_evaluate + isInside, barycoord_pmmg.c:300-310,102-107 */
static int bc3d_evaluate(const orc_background *bg, int k, const double *fa, double vol,
                         const double *x, bcoord *b) {
  bc3d_compute(bg, k, fa, vol, x, b);
  bc_sort(b, 4);
  return b[0].val > -ORC_EPS;
}

/* unit tria normal and |n| (PMMG_precompute_triaNormals, locate_pmmg.c:68-90) */
static double tria_geom(const orc_background *bg, int k, double *n) {
  nonunit_normal(PT(bg, TRIV(bg, k, 0)), PT(bg, TRIV(bg, k, 1)), PT(bg, TRIV(bg, k, 2)), n);
  double q = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  double dd = 1.0 / q;
  n[0] *= dd;
  n[1] *= dd;
  n[2] *= dd;
  return q;
}

/* PMMG_quickarea, barycoord_pmmg.c:44-61 */
static double quickarea(const double *a, const double *b, const double *c, const double *n) {
  double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  double a0 = aby * acz - abz * acy, a1 = abz * acx - abx * acz, a2 = abx * acy - aby * acx;
  return a0 * n[0] + a1 * n[1] + a2 * n[2];
}

/* PMMG_barycoord2d_compute, barycoord_pmmg.c:191-223: vertices and area of
 * tria kv, unit normal n (normally the same tria; the stale exhaustive
 * re-evaluation mixes them, locate_pmmg.c:505-509) */
static void bc2d_compute(const orc_background *bg, int kv, double vol, const double *x,
                         const double *n, bcoord *b) {
  const double *c1 = PT(bg, TRIV(bg, kv, 0));
  double dist = 0.0, proj[3];
  for (int i = 0; i < 3; i++) dist += (x[i] - c1[i]) * n[i];
  for (int i = 0; i < 3; i++) proj[i] = x[i] - dist * n[i];
  for (int ia = 0; ia < 3; ia++) {
    const double *a = PT(bg, TRIV(bg, kv, kInxt2[ia]));
    const double *c = PT(bg, TRIV(bg, kv, kInxt2[ia + 1]));
    b[ia].val = quickarea(proj, a, c, n) / vol;
    b[ia].idx = ia;
  }
  b[3].val = dist;
  b[3].idx = 3;
}

/* PMMG_barycoord_isBorder, barycoord_pmmg.c:109-120 */
static void bc_is_border(const bcoord *phi, int *edge, int *vertex) {
  if (phi[0].val < ORC_EPS) {
    if (phi[1].val < ORC_EPS) *vertex = phi[2].idx;
    else *edge = phi[0].idx;
  }
}

/* PMMG_barycoord3d_getClosest / 2d_getClosest, barycoord_pmmg.c:371-404, 324-357 */
static void bc_closest(const orc_background *bg, const int *v, int nv, const double *x, bcoord *b) {
  const double *c = PT(bg, v[0]);
  double d[3];
  for (int i = 0; i < 3; i++) d[i] = x[i] - c[i];
  double mn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  int it = 0;
  for (int j = 1; j < nv; j++) {
    c = PT(bg, v[j]);
    for (int i = 0; i < 3; i++) d[i] = x[i] - c[i];
    double nrm = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (nrm < mn) { mn = nrm; it = j; }
  }
  for (int j = 0; j < nv; j++) { b[j].val = 0.0; b[j].idx = j; }
  b[it].val = 1.0;
}

static void tet_closest(const orc_background *bg, int k, const double *x, bcoord *b) {
  int v[4];
  for (int i = 0; i < 4; i++) v[i] = TETV(bg, k, i);
  bc_closest(bg, v, 4, x, b);
}

static void tria_closest(const orc_background *bg, int k, const double *x, bcoord *b) {
  int v[3];
  for (int i = 0; i < 3; i++) v[i] = TRIV(bg, k, i);
  bc_closest(bg, v, 3, x, b);
}

/* ---------------- interpolators (src/interpmesh_pmmg.c:50-296) ---------------- */

static void interp_iso(int size, const double *old, const int *v, int nv, const double *phi, double *out) {
  for (int j = 0; j < size; j++) out[j] = 0.0;
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < size; j++) out[j] += phi[i] * old[(size_t)size * (v[i] - 1) + j];
}

/* interp{3,4}bar_ani: M = invmat(sum_i phi_i invmat(M_i)) */
static int interp_ani(const double *old, const int *v, int nv, const double *phi, double *out) {
  double mi[4][6], mint[6];
  for (int i = 0; i < nv; i++)
    if (!orc_invmat(old + 6 * (size_t)(v[i] - 1), mi[i])) return 0;
  for (int s = 0; s < 6; s++) {
    if (nv == 4) mint[s] = phi[0] * mi[0][s] + phi[1] * mi[1][s] + phi[2] * mi[2][s] + phi[3] * mi[3][s];
    else mint[s] = phi[0] * mi[0][s] + phi[1] * mi[1][s] + phi[2] * mi[2][s];
  }
  return orc_invmat(mint, out);
}

/* interp2bar_iso / _ani, interpmesh_pmmg.c:50-110 */
static int interp_edge(int size, const double *old, const int *v, int l, const double *phi, double *out) {
  int i0 = kInxt2[l], i1 = kIprv2[l];
  if (size == 6) {
    double mi[2][6], mint[6];
    if (!orc_invmat(old + 6 * (size_t)(v[i0] - 1), mi[0])) return 0;
    if (!orc_invmat(old + 6 * (size_t)(v[i1] - 1), mi[1])) return 0;
    for (int s = 0; s < 6; s++) mint[s] = phi[i0] * mi[0][s] + phi[i1] * mi[1][s];
    return orc_invmat(mint, out);
  }
  out[0] = phi[i0] * old[v[i0] - 1] + phi[i1] * old[v[i1] - 1];
  return 1;
}

static void interp_sol(int size, const double *old, const int *v, int nv, const double *phi, double *out) {
  if (size == 6) interp_ani(old, v, nv, phi, out);
  else interp_iso(size, old, v, nv, phi, out);
}

/* volume point: metric via PMMG_interp4bar, fields via 4bar_{ani,iso} (:612-636) */
static void apply_vol(const orc_background *bg, int k, const bcoord *b, double *met_row,
                      double *const *field_rows) {
  double phi[4];
  int v[4];
  bc_get(phi, b, 4);
  for (int i = 0; i < 4; i++) v[i] = TETV(bg, k, i);
  if (bg->met_size && met_row) interp_sol(bg->met_size, bg->met, v, 4, phi, met_row);
  for (int j = 0; j < bg->nfield; j++)
    if (field_rows && field_rows[j]) interp_sol(bg->field_size[j], bg->field[j], v, 4, phi, field_rows[j]);
}

/* boundary point (:563-595): metric by vertex copy / edge / face, fields always face */
static void apply_bdy(const orc_background *bg, int k, const bcoord *b, int edge, int vertex,
                      double *met_row, double *const *field_rows) {
  double phi[3];
  int v[3];
  bc_get(phi, b, 3);
  for (int i = 0; i < 3; i++) v[i] = TRIV(bg, k, i);
  if (bg->met_size && met_row) {
    int ms = bg->met_size;
    if (vertex != ORC_UNSET) {
      for (int s = 0; s < ms; s++) met_row[s] = bg->met[(size_t)ms * (v[vertex] - 1) + s];
    } else if (edge != ORC_UNSET) {
      interp_edge(ms, bg->met, v, edge, phi, met_row);
    } else {
      interp_sol(ms, bg->met, v, 3, phi, met_row);
    }
  }
  for (int j = 0; j < bg->nfield; j++)
    if (field_rows && field_rows[j]) interp_sol(bg->field_size[j], bg->field[j], v, 3, phi, field_rows[j]);
}

/* ---------------- sequential state machine of the reference ---------------- */

typedef struct {
  const orc_background *bg;
  int mode;
  double *qual;   /* ne+1   pt->qual = orvol */
  double *farea;  /* 12*(ne+1) */
  double *tqual;  /* nt+1   ptr->qual = |n| */
  double *tnorm;  /* 3*(nt+1) */
  int *tflag, *trflag, *pflag;
  int *ntoff, *ntlist; /* node -> trias CSR, ntlist[ntoff[ip]] = count */
  int base;
} orc_state;

/* PMMG_locatePointInTetra, locate_pmmg.c:441-461 */
static int in_tetra(orc_state *S, int k, const double *x, bcoord *b, double *cdist, int *ctet) {
  S->tflag[k] = S->base;
  int found = bc3d_evaluate(S->bg, k, S->farea + 12 * (size_t)k, S->qual[k], x, b);
  double vol = S->qual[k];
  if (fabs(b[0].val) * vol < *cdist) {
    *cdist = fabs(b[0].val) * vol;
    *ctet = k;
  }
  return found;
}

/* PMMG_locatePointVol + PMMG_locatePoint_exhaustTetra, locate_pmmg.c:786-883, 737-770 */
static int locate_vol(orc_state *S, const double *x, bcoord *b, int *idx, int *steps) {
  const orc_background *bg = S->bg;
  if (!*idx) *idx = 1;
  int ctet = 0, stuck = 0, step = 0;
  double cdist = 1.0e10;
  ++S->base;
  while (step <= bg->ne && !stuck) {
    step++;
    int k = *idx;
    if (TETV(bg, k, 0) <= 0) continue; /* !MG_EOK */
    if (in_tetra(S, k, x, b, &cdist, &ctet)) break;
    int i;
    for (i = 0; i < 4; i++) {
      int iel = ADJA(bg, k, b[i].idx) / 4;
      if (!iel) continue;
      if (S->tflag[iel] == S->base) continue;
      *idx = iel;
      break;
    }
    if (i == 4) stuck = 1;
  }
  *steps = stuck ? -step : step;
  if (step > bg->ne) {
    *idx = ctet;
    tet_closest(bg, *idx, x, b);
    return HIT_VOL_CLOSEST;
  }
  if (stuck) {
    int k;
    for (k = 1; k <= bg->ne; k++) {
      (*steps)--;
      if (TETV(bg, k, 0) <= 0) continue;
      if (S->tflag[k] == S->base) continue;
      if (in_tetra(S, k, x, b, &cdist, &ctet)) break;
    }
    if (k <= bg->ne) {
      *idx = k;
      return HIT_VOL_EXHAUST;
    }
    *idx = ctet;
    tet_closest(bg, *idx, x, b);
    return HIT_VOL_CLOSEST;
  }
  return HIT_VOL_WALK;
}

/* PMMG_locateChkDistTria, locate_pmmg.c:347-366 (vertex 0 of tria kv, normal n) */
static int chk_dist_tria(const orc_background *bg, int kv, const double *x, const double *n) {
  const double *p0 = PT(bg, TRIV(bg, kv, 0));
  double d[3], nrm = 0.0;
  for (int i = 0; i < 3; i++) d[i] = x[i] - p0[i];
  for (int i = 0; i < 3; i++) nrm += d[i] * n[i];
  nrm = fabs(nrm);
  return !(nrm > bg->hausd);
}

/* PMMG_locatePointInTria, locate_pmmg.c:385-423; kv = tria whose vertices are
 * used (ptr), k = tria index used for the normal and the closest tracking */
static int in_tria(orc_state *S, int kv, int k, const double *x, bcoord *b, double *cdist, int *ctria) {
  const orc_background *bg = S->bg;
  S->trflag[kv] = S->base;
  const double *n = S->tnorm + 3 * (size_t)k;
  bc2d_compute(bg, kv, S->tqual[kv], x, n, b);
  bc_sort(b, 3);
  int found = b[0].val > -ORC_EPS;
  double d[3];
  for (int i = 0; i < 3; i++) d[i] = x[i];
  for (int j = 0; j < 3; j++) {
    const double *p = PT(bg, TRIV(bg, kv, j));
    for (int i = 0; i < 3; i++) d[i] -= p[i] / 3.0;
  }
  double nrm = 0;
  for (int i = 0; i < 3; i++) nrm += d[i] * d[i];
  nrm = sqrt(nrm);
  if (nrm < *cdist) {
    *cdist = nrm;
    *ctria = k;
  }
  if (!chk_dist_tria(bg, kv, x, n)) return 0;
  return found;
}

/* PMMG_locatePointInWedge, locate_pmmg.c:286-334 */
static int in_wedge(const orc_background *bg, orc_state *S, int k, int l, const double *x, bcoord *b) {
  int i0 = kInxt2[l], i1 = kIprv2[l];
  int v0 = TRIV(bg, k, i0), v1 = TRIV(bg, k, i1);
  const double *p0 = PT(bg, v0), *p1 = PT(bg, v1);
  double p[3], a[3], norm2 = 0.0, alpha = 0.0, dist = 0.0;
  for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
  for (int d = 0; d < 3; d++) a[d] = p1[d] - p0[d];
  for (int d = 0; d < 3; d++) norm2 += a[d] * a[d];
  for (int d = 0; d < 3; d++) alpha += a[d] * p[d];
  for (int d = 0; d < 3; d++) p[d] -= (alpha / norm2) * a[d];
  for (int d = 0; d < 3; d++) dist += p[d] * p[d];
  dist = sqrt(dist);
  if (dist > bg->hausd) return ORC_UNSET;
  if (alpha < 0.0) {
    if (S) S->pflag[v1] = S->base;
    return i0;
  } else if (alpha > norm2) {
    if (S) S->pflag[v0] = S->base;
    return i1;
  }
  if (b) {
    for (int d = 0; d < 3; d++) b[d].idx = d;
    b[l].val = 0.0;
    b[i0].val = 1.0 - alpha / norm2;
    b[i1].val = alpha / norm2;
  }
  return 4;
}

/* PMMG_locatePointInCone, locate_pmmg.c:209-270.  FAITHFUL mode keeps the
 * reference's persistent point flags; FRESH mode checks every neighbour. */
static int in_cone(orc_state *S, int k, int iloc, const double *x) {
  const orc_background *bg = S->bg;
  int ip = TRIV(bg, k, iloc);
  const double *p0 = PT(bg, ip);
  S->pflag[ip] = S->base;
  double p[3], dist = 0.0;
  for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
  for (int d = 0; d < 3; d++) dist += p[d] * p[d];
  dist = sqrt(dist);
  const int *my = S->ntlist + S->ntoff[ip];
  int cnt = my[0];
  for (int t = 0; t < cnt; t++) {
    int tr = my[t + 1];
    for (int jl = 0; jl < 3; jl++) {
      int jp = TRIV(bg, tr, jl);
      if (jp == ip) continue;
      if (S->mode == ORC_MODE_FAITHFUL) {
        if (S->pflag[jp] == ip) continue;
        S->pflag[jp] = ip;
      }
      const double *p1 = PT(bg, jp);
      double a[3], alpha = 0.0;
      for (int d = 0; d < 3; d++) a[d] = p1[d] - p0[d];
      if (dist > bg->hausd) return 0;
      for (int d = 0; d < 3; d++) alpha += a[d] * p[d];
      if (alpha > 0.0) return 0;
    }
  }
  return 1;
}

/* PMMG_locatePointBdy + PMMG_locatePoint_exhaustTria, locate_pmmg.c:587-723, 477-515.
 * (PMMG_locatePoint_foundConvex, :531-569, never updates the result: it
 * compares an unset h with itself; only its visited marks are skipped.) */
static int locate_bdy(orc_state *S, const double *x, bcoord *b, int *itria, int *edge, int *vertex, int *steps) {
  const orc_background *bg = S->bg;
  int k = *itria ? *itria : 1;
  int stuck = 0, step = 0, ctria = 0;
  double cdist = 1.0e10;
  ++S->base;
  *edge = ORC_UNSET;
  *vertex = ORC_UNSET;
  while (step <= bg->nt && !stuck) {
    step++;
    if (TRIV(bg, k, 0) <= 0) continue;
    if (in_tria(S, k, k, x, b, &cdist, &ctria)) {
      bc_is_border(b, edge, vertex);
      break;
    }
    int j;
    for (j = 0; j < 3; j++) {
      int i = b[j].idx;
      int k1 = ADJT(bg, k, i) / 3;
      if (!k1) continue;
      if (S->trflag[k1] == S->base) {
        int il = in_wedge(bg, S, k, i, x, b);
        if (il == ORC_UNSET) continue;
        if (il == 4) {
          *edge = i;
          *steps = step;
          *itria = k;
          return HIT_BDY_WEDGE;
        }
        if (in_cone(S, k, il, x)) {
          *vertex = il;
          *steps = step;
          *itria = k;
          return HIT_BDY_CONE;
        }
        continue;
      }
      k = k1;
      break;
    }
    if (j == 3) stuck = 1;
  }
  *steps = stuck ? -step : step;
  if (step > bg->nt) {
    *itria = ctria;
    tria_closest(bg, ctria, x, b);
    return HIT_BDY_CLOSEST;
  }
  *itria = k;
  if (stuck) {
    int t, last = 0;
    for (t = 1; t <= bg->nt; t++) {
      (*steps)--;
      last = t;
      if (TRIV(bg, t, 0) <= 0) continue;
      if (S->trflag[t] == S->base) continue;
      if (in_tria(S, t, t, x, b, &cdist, &ctria)) break;
    }
    if (t <= bg->nt) {
      *itria = t;
      return HIT_BDY_EXHAUST;
    }
    *itria = ctria;
    /* stale re-evaluation: vertices of the last scanned tria, normal of the closest */
    if (in_tria(S, last, ctria, x, b, &cdist, &ctria)) return HIT_BDY_STALE;
    tria_closest(bg, *itria, x, b);
    return HIT_BDY_CLOSEST;
  }
  if (*vertex != ORC_UNSET) return HIT_BDY_VERTEX;
  if (*edge != ORC_UNSET) return HIT_BDY_EDGE;
  return HIT_BDY_FACE;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void state_free(orc_state *S) {
  free(S->qual); free(S->farea); free(S->tqual); free(S->tnorm);
  free(S->tflag); free(S->trflag); free(S->pflag); free(S->ntoff); free(S->ntlist);
}

/* precompute of PMMG_interpMetricsAndFields(_mesh): faceAreas, triaNormals, nodeTrias */
static int state_init(orc_state *S, const orc_background *bg, int mode) {
  memset(S, 0, sizeof(*S));
  S->bg = bg;
  S->mode = mode;
  size_t ne = (size_t)bg->ne, nt = (size_t)bg->nt, np = (size_t)bg->np;
  S->qual = (double *)malloc(sizeof(double) * (ne + 1));
  S->farea = (double *)malloc(sizeof(double) * 12 * (ne + 1));
  S->tqual = (double *)malloc(sizeof(double) * (nt + 1));
  S->tnorm = (double *)malloc(sizeof(double) * 3 * (nt + 1));
  S->tflag = (int *)calloc(ne + 1, sizeof(int));
  S->trflag = (int *)calloc(nt + 1, sizeof(int));
  S->pflag = (int *)calloc(np + 1, sizeof(int));
  S->ntoff = (int *)calloc(np + 2, sizeof(int));
  S->ntlist = (int *)malloc(sizeof(int) * (np + 3 * nt + 1));
  if (!S->qual || !S->farea || !S->tqual || !S->tnorm || !S->tflag || !S->trflag || !S->pflag ||
      !S->ntoff || !S->ntlist)
    return 0;
  for (size_t k = 1; k <= ne; k++) S->qual[k] = tet_geom(bg, (int)k, S->farea + 12 * k);
  for (size_t k = 1; k <= nt; k++) S->tqual[k] = tria_geom(bg, (int)k, S->tnorm + 3 * k);
  /* PMMG_precompute_nodeTrias, locate_pmmg.c:134-195 (point.flag left = count) */
  for (size_t k = 1; k <= nt; k++)
    for (int l = 0; l < 3; l++) S->pflag[TRIV(bg, k, l)]++;
  int off = 0;
  for (size_t ip = 1; ip <= np; ip++) {
    S->ntoff[ip] = off;
    if (S->pflag[ip]) {
      S->ntlist[off] = 0;
      off += S->pflag[ip] + 1;
    }
  }
  for (size_t k = 1; k <= nt; k++)
    for (int l = 0; l < 3; l++) {
      int ip = TRIV(bg, k, l);
      int *c = &S->ntlist[S->ntoff[ip]];
      c[1 + c[0]] = (int)k;
      c[0]++;
    }
  /* tetra flags reset to base 0 (interpmesh_pmmg.c:521-526) */
  S->base = 0;
  return 1;
}

int orc_interp_mesh(const orc_background *bg, const orc_queries *q, orc_outputs *out, int mode,
                    double *timing) {
  return orc_interp_mesh_budget(bg, q, out, mode, 0.0, timing) >= 0;
}

/* The visit loop of PMMG_interpMetricsAndFields_mesh (interpmesh_pmmg.c:535-643)
 * over visit[v0, v1), warm start carried from point to point; stops early once
 * `deadline` (now_s() clock, <= 0: none) has passed.  Returns the visit
 * entries processed. */
static int visit_range(orc_state *S, const orc_queries *q, orc_outputs *out, int v0, int v1, double deadline) {
  const orc_background *bg = S->bg;
  int itet = 1, itria = 1; /* interpmesh_pmmg.c:529 */
  int nf = bg->nfield;
  double **frow = (double **)malloc(sizeof(double *) * (nf > 0 ? nf : 1));
  int v = v0;
  for (; v < v1; v++) {
    if (deadline > 0.0 && ((v - v0) & 255) == 0 && v > v0 && now_s() > deadline) break;
    int ip = q->visit[v];
    if (ip < 1 || ip > q->np) continue;
    int cls = q->pclass[ip - 1];
    if (cls != 1 && cls != 2) continue;
    const double *x = q->xyz + 3 * (size_t)(ip - 1);
    double *mrow = (bg->met_size && out->met) ? out->met + (size_t)bg->met_size * (ip - 1) : NULL;
    for (int j = 0; j < nf; j++)
      frow[j] = (out->field && out->field[j]) ? out->field[j] + (size_t)bg->field_size[j] * (ip - 1) : NULL;
    bcoord b[4];
    int hit, elem, steps = 0, loc = -1;
    double mb = 0.0;
    if (cls == 2) {
      int edge, vertex;
      hit = locate_bdy(S, x, b, &itria, &edge, &vertex, &steps);
      elem = itria;
      loc = (vertex != ORC_UNSET) ? vertex : edge;
      mb = b[0].val;
      apply_bdy(bg, elem, b, edge, vertex, mrow, frow);
    } else {
      hit = locate_vol(S, x, b, &itet, &steps);
      elem = itet;
      mb = b[0].val;
      apply_vol(bg, elem, b, mrow, frow);
    }
    if (out->elem) out->elem[ip - 1] = elem;
    if (out->hit) out->hit[ip - 1] = (int8_t)hit;
    if (out->loc) out->loc[ip - 1] = (int8_t)loc;
    if (out->minbary) out->minbary[ip - 1] = mb;
    if (out->steps) out->steps[ip - 1] = steps;
  }
  free(frow);
  return v - v0;
}

int orc_interp_mesh_budget(const orc_background *bg, const orc_queries *q, orc_outputs *out, int mode,
                           double budget_s, double *timing) {
  orc_state S;
  double t0 = now_s();
  if (!state_init(&S, bg, mode)) { state_free(&S); return -1; }
  double t1 = now_s();
  int n = visit_range(&S, q, out, 0, q->nvisit, budget_s > 0.0 ? t1 + budget_s : 0.0);
  double t2 = now_s();
  state_free(&S);
  if (timing) { timing[0] = t1 - t0; timing[1] = t2 - t1; }
  return n;
}

/* ---------------- threaded driver (CPU baseline) ---------------- */

typedef struct {
  orc_state S;            /* shared precompute, private visited flags */
  const orc_queries *q;
  orc_outputs *out;
  int v0, v1, done;
  int k0, k1;             /* precompute range (tetra) */
  double deadline;
} orc_job;

static void *job_precompute(void *arg) {
  orc_job *J = (orc_job *)arg;
  for (int k = J->k0; k < J->k1; k++) J->S.qual[k] = tet_geom(J->S.bg, k, J->S.farea + 12 * (size_t)k);
  return NULL;
}

static void *job_visit(void *arg) {
  orc_job *J = (orc_job *)arg;
  J->done = visit_range(&J->S, J->q, J->out, J->v0, J->v1, J->deadline);
  return NULL;
}

int orc_interp_mesh_mt(const orc_background *bg, const orc_queries *q, orc_outputs *out, int mode, int nthreads,
                       double budget_s, double *timing) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  orc_state S0;
  double t0 = now_s();
  /* the precompute of state_init with the per-tetra part (faceAreas, the
   * dominant O(ne) stream) split over the threads */
  memset(&S0, 0, sizeof(S0));
  S0.bg = bg;
  S0.mode = mode;
  size_t ne = (size_t)bg->ne, nt = (size_t)bg->nt, np = (size_t)bg->np;
  S0.qual = (double *)malloc(sizeof(double) * (ne + 1));
  S0.farea = (double *)malloc(sizeof(double) * 12 * (ne + 1));
  S0.tqual = (double *)malloc(sizeof(double) * (nt + 1));
  S0.tnorm = (double *)malloc(sizeof(double) * 3 * (nt + 1));
  S0.tflag = (int *)calloc(ne + 1, sizeof(int));
  S0.trflag = (int *)calloc(nt + 1, sizeof(int));
  S0.pflag = (int *)calloc(np + 1, sizeof(int));
  S0.ntoff = (int *)calloc(np + 2, sizeof(int));
  S0.ntlist = (int *)malloc(sizeof(int) * (np + 3 * nt + 1));
  orc_job *J = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  int ok = S0.qual && S0.farea && S0.tqual && S0.tnorm && S0.tflag && S0.trflag && S0.pflag && S0.ntoff &&
           S0.ntlist && J && th;
  if (ok) {
    for (int t = 0; t < nthreads; t++) {
      J[t].S = S0;
      J[t].k0 = 1 + (int)((ne * (size_t)t) / (size_t)nthreads);
      J[t].k1 = 1 + (int)((ne * (size_t)(t + 1)) / (size_t)nthreads);
      pthread_create(&th[t], NULL, job_precompute, &J[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    for (size_t k = 1; k <= nt; k++) S0.tqual[k] = tria_geom(bg, (int)k, S0.tnorm + 3 * k);
    for (size_t k = 1; k <= nt; k++)
      for (int l = 0; l < 3; l++) S0.pflag[TRIV(bg, k, l)]++;
    int off = 0;
    for (size_t ip = 1; ip <= np; ip++) {
      S0.ntoff[ip] = off;
      if (S0.pflag[ip]) {
        S0.ntlist[off] = 0;
        off += S0.pflag[ip] + 1;
      }
    }
    for (size_t k = 1; k <= nt; k++)
      for (int l = 0; l < 3; l++) {
        int ip = TRIV(bg, k, l);
        int *cc = &S0.ntlist[S0.ntoff[ip]];
        cc[1 + cc[0]] = (int)k;
        cc[0]++;
      }
  }
  double t1 = now_s();
  int total = 0;
  if (ok) {
    /* one contiguous visit range per thread (as one MPI rank per group),
     * each with private visited flags */
    for (int t = 0; t < nthreads && ok; t++) {
      J[t].S = S0;
      J[t].S.base = 0;
      if (t > 0) {
        J[t].S.tflag = (int *)calloc(ne + 1, sizeof(int));
        J[t].S.trflag = (int *)calloc(nt + 1, sizeof(int));
        J[t].S.pflag = (int *)malloc(sizeof(int) * (np + 1));
        ok = J[t].S.tflag && J[t].S.trflag && J[t].S.pflag;
        if (J[t].S.pflag) memcpy(J[t].S.pflag, S0.pflag, sizeof(int) * (np + 1));
      }
      J[t].q = q;
      J[t].out = out;
      J[t].v0 = (int)(((size_t)q->nvisit * (size_t)t) / (size_t)nthreads);
      J[t].v1 = (int)(((size_t)q->nvisit * (size_t)(t + 1)) / (size_t)nthreads);
    }
    t1 = now_s();
    for (int t = 0; t < nthreads && ok; t++) {
      J[t].deadline = budget_s > 0.0 ? t1 + budget_s : 0.0;
      pthread_create(&th[t], NULL, job_visit, &J[t]);
    }
    for (int t = 0; t < nthreads && ok; t++) {
      pthread_join(th[t], NULL);
      total += J[t].done;
    }
  }
  double t2 = now_s();
  for (int t = 1; J && t < nthreads; t++) {
    free(J[t].S.tflag);
    free(J[t].S.trflag);
    free(J[t].S.pflag);
  }
  state_free(&S0);
  free(J);
  free(th);
  if (timing) { timing[0] = t1 - t0; timing[1] = t2 - t1; }
  return ok ? total : -1;
}

/* ---------------- element-wise checkers ---------------- */

int orc_eval_in_element(const orc_background *bg, const double *x, int is_bdy, int elem, int hit,
                        int loc, double *met_row, double *const *field_rows) {
  bcoord b[4];
  if (!is_bdy) {
    if (elem < 1 || elem > bg->ne) return 0;
    if (hit == HIT_VOL_WALK || hit == HIT_VOL_EXHAUST) {
      double fa[12];
      double vol = tet_geom(bg, elem, fa);
      bc3d_evaluate(bg, elem, fa, vol, x, b);
    } else if (hit == HIT_VOL_CLOSEST) {
      tet_closest(bg, elem, x, b);
    } else {
      return 0;
    }
    apply_vol(bg, elem, b, met_row, field_rows);
    return 1;
  }
  if (elem < 1 || elem > bg->nt) return 0;
  double n[3];
  int edge = ORC_UNSET, vertex = ORC_UNSET;
  switch (hit) {
    case HIT_BDY_FACE: case HIT_BDY_EDGE: case HIT_BDY_VERTEX: case HIT_BDY_CONE: case HIT_BDY_EXHAUST: {
      double q = tria_geom(bg, elem, n);
      bc2d_compute(bg, elem, q, x, n, b);
      bc_sort(b, 3);
      if (hit == HIT_BDY_EDGE) edge = loc;
      if (hit == HIT_BDY_VERTEX || hit == HIT_BDY_CONE) vertex = loc;
    } break;
    case HIT_BDY_WEDGE: {
      /* wedge coordinates of edge loc, locate_pmmg.c:297-331 */
      int i0 = kInxt2[loc], i1 = kIprv2[loc];
      const double *p0 = PT(bg, TRIV(bg, elem, i0)), *p1 = PT(bg, TRIV(bg, elem, i1));
      double p[3], a[3], norm2 = 0.0, alpha = 0.0;
      for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
      for (int d = 0; d < 3; d++) a[d] = p1[d] - p0[d];
      for (int d = 0; d < 3; d++) norm2 += a[d] * a[d];
      for (int d = 0; d < 3; d++) alpha += a[d] * p[d];
      for (int d = 0; d < 3; d++) b[d].idx = d;
      b[loc].val = 0.0;
      b[i0].val = 1.0 - alpha / norm2;
      b[i1].val = alpha / norm2;
    }
      edge = loc;
      break;
    case HIT_BDY_STALE: {
      /* vertices + area of the last tria (nt), normal of the closest (elem) */
      double ns[3];
      tria_geom(bg, elem, n);
      double qs = tria_geom(bg, bg->nt, ns);
      bc2d_compute(bg, bg->nt, qs, x, n, b);
      bc_sort(b, 3);
    } break;
    case HIT_BDY_CLOSEST:
      tria_closest(bg, elem, x, b);
      break;
    default:
      return 0;
  }
  apply_bdy(bg, elem, b, edge, vertex, met_row, field_rows);
  return 1;
}

double orc_tetra_minbary(const orc_background *bg, int k, const double *x) {
  double fa[12];
  bcoord b[4];
  double vol = tet_geom(bg, k, fa);
  bc3d_evaluate(bg, k, fa, vol, x, b);
  return b[0].val;
}

int orc_tria_accepts(const orc_background *bg, int k, const double *x, double *mb) {
  double n[3];
  bcoord b[4];
  double q = tria_geom(bg, k, n);
  bc2d_compute(bg, k, q, x, n, b);
  bc_sort(b, 3);
  if (mb) *mb = b[0].val;
  return (b[0].val > -ORC_EPS) && chk_dist_tria(bg, k, x, n);
}

int orc_first_accepting_tetra(const orc_background *bg, const double *x) {
  for (int k = 1; k <= bg->ne; k++) {
    if (TETV(bg, k, 0) <= 0) continue;
    if (orc_tetra_minbary(bg, k, x) > -ORC_EPS) return k;
  }
  return 0;
}

double orc_closest_value(const orc_background *bg, int k, const double *x) {
  double fa[12];
  bcoord b[4];
  double vol = tet_geom(bg, k, fa);
  bc3d_evaluate(bg, k, fa, vol, x, b);
  return fabs(b[0].val) * vol;
}

int orc_closest_tetra(const orc_background *bg, const double *x) {
  double best = 1.0e10;
  int kb = 0;
  for (int k = 1; k <= bg->ne; k++) {
    if (TETV(bg, k, 0) <= 0) continue;
    double fa[12];
    bcoord b[4];
    double vol = tet_geom(bg, k, fa);
    bc3d_evaluate(bg, k, fa, vol, x, b);
    if (fabs(b[0].val) * vol < best) { best = fabs(b[0].val) * vol; kb = k; }
  }
  return kb;
}

int orc_first_accepting_tria(const orc_background *bg, const double *x) {
  for (int k = 1; k <= bg->nt; k++) {
    if (TRIV(bg, k, 0) <= 0) continue;
    if (orc_tria_accepts(bg, k, x, NULL)) return k;
  }
  return 0;
}

int orc_closest_tria(const orc_background *bg, const double *x) {
  double best = 1.0e10;
  int kb = 0;
  for (int k = 1; k <= bg->nt; k++) {
    if (TRIV(bg, k, 0) <= 0) continue;
    double d[3];
    for (int i = 0; i < 3; i++) d[i] = x[i];
    for (int j = 0; j < 3; j++) {
      const double *p = PT(bg, TRIV(bg, k, j));
      for (int i = 0; i < 3; i++) d[i] -= p[i] / 3.0;
    }
    double nrm = 0;
    for (int i = 0; i < 3; i++) nrm += d[i] * d[i];
    nrm = sqrt(nrm);
    if (nrm < best) { best = nrm; kb = k; }
  }
  return kb;
}

int orc_wedge_test(const orc_background *bg, int k, int l, const double *x) {
  return in_wedge(bg, NULL, k, l, x, NULL);
}

int orc_cone_test(const orc_background *bg, int k, int iloc, const double *x) {
  int ip = TRIV(bg, k, iloc);
  const double *p0 = PT(bg, ip);
  double p[3], dist = 0.0;
  for (int d = 0; d < 3; d++) p[d] = x[d] - p0[d];
  for (int d = 0; d < 3; d++) dist += p[d] * p[d];
  dist = sqrt(dist);
  int any = 0;
  for (int t = 1; t <= bg->nt; t++) {
    int has = 0;
    for (int l = 0; l < 3; l++) has |= (TRIV(bg, t, l) == ip);
    if (!has) continue;
    for (int l = 0; l < 3; l++) {
      int jp = TRIV(bg, t, l);
      if (jp == ip) continue;
      any = 1;
      const double *p1 = PT(bg, jp);
      double a[3], alpha = 0.0;
      for (int d = 0; d < 3; d++) a[d] = p1[d] - p0[d];
      if (dist > bg->hausd) return 0;
      for (int d = 0; d < 3; d++) alpha += a[d] * p[d];
      if (alpha > 0.0) return 0;
    }
  }
  (void)any;
  return 1;
}

/* ---------------------------------------------------------------- batch parity check
 * The contract of tests/parity.py::check (BASELINE.json north_star, SURVEY.md
 * §8(a) row A1) for many points at once, over threads:
 *  (ii)  the element each point was located in is accepted by the reference's
 *        own test for its hit kind (walk / exhaustive / closest / tria /
 *        wedge / cone / stale);
 *  (iii) its values equal the reference interpolator evaluated in that
 *        element (bitwise count + maximum relative error);
 *  (i)   with a reference run given: points whose reference tetra has min
 *        barycentric > EPS are located in the identical tetra. */
static int same_bits(double a, double b) {
  return (a == b) || (isnan(a) && isnan(b));
}
static double rel_err(double a, double b) {
  if (isnan(a) && isnan(b)) return 0.0;
  if (isnan(a) || isnan(b)) return INFINITY;
  double d = fabs(a - b), s = fmax(fabs(a), fabs(b));
  return s > 0.0 ? d / s : d;
}

typedef struct {
  const orc_background *bg;
  const double *xyz;
  const uint8_t *pclass;
  const int *idx;
  int64_t i0, i1;
  const int *elem;
  const int8_t *hit;
  const double *met_out;
  const double *const *field_out;
  const int *ref_elem;
  const int8_t *ref_hit;
  const double *ref_minbary;
  double rel_tol;
  orc_check_report rep;
} chk_job;

static void *job_check(void *arg) {
  chk_job *J = (chk_job *)arg;
  const orc_background *bg = J->bg;
  orc_check_report *R = &J->rep;
  int ms = bg->met_size, nf = bg->nfield;
  double met_row[6], frow[64][6];
  double *fptr[64];
  for (int j = 0; j < nf && j < 64; j++) fptr[j] = frow[j];
  for (int64_t t = J->i0; t < J->i1; t++) {
    int64_t i = J->idx ? J->idx[t] : t;
    int pc = J->pclass[i];
    int h = J->hit[i] & 15, l = (J->hit[i] >> 4) & 3, k = J->elem[i];
    if (pc == 0) {
      if (h != 0) R->skipped_written++;
      continue;
    }
    if (h == 0) {
      R->unprocessed++;
      if (R->first_fail < 0) R->first_fail = i;
      continue;
    }
    R->hits[h]++;
    const double *x = J->xyz + 3 * i;
    int is_bdy = pc == 2, ok = 0;
    switch (h) {
      case HIT_VOL_WALK:
        ok = !is_bdy && k >= 1 && k <= bg->ne && orc_tetra_minbary(bg, k, x) > -ORC_EPS;
        break;
      case HIT_VOL_EXHAUST:
        ok = !is_bdy && k == orc_first_accepting_tetra(bg, x);
        break;
      case HIT_VOL_CLOSEST: {
        int kb = orc_closest_tetra(bg, x);
        ok = !is_bdy && orc_first_accepting_tetra(bg, x) == 0 && k >= 1 && k <= bg->ne &&
             (k == kb || orc_closest_value(bg, k, x) == orc_closest_value(bg, kb, x));
      } break;
      case HIT_BDY_FACE: case HIT_BDY_EDGE: case HIT_BDY_VERTEX:
        ok = is_bdy && k >= 1 && k <= bg->nt && orc_tria_accepts(bg, k, x, NULL);
        break;
      case HIT_BDY_WEDGE:
        ok = is_bdy && k >= 1 && k <= bg->nt && in_wedge(bg, NULL, k, l, x, NULL) == 4;
        break;
      case HIT_BDY_CONE:
        ok = is_bdy && k >= 1 && k <= bg->nt && orc_cone_test(bg, k, l, x) == 1;
        break;
      case HIT_BDY_EXHAUST:
        ok = is_bdy && k == orc_first_accepting_tria(bg, x);
        break;
      case HIT_BDY_STALE: case HIT_BDY_CLOSEST:
        ok = is_bdy && orc_first_accepting_tria(bg, x) == 0 && k == orc_closest_tria(bg, x);
        break;
      default:
        ok = 0;
    }
    if (!ok) {
      R->accept_fail++;
      if (R->first_fail < 0) R->first_fail = i;
      continue;
    }
    for (int c = 0; c < 6; c++) met_row[c] = NAN;
    for (int j = 0; j < nf && j < 64; j++)
      for (int c = 0; c < 6; c++) frow[j][c] = NAN;
    if (!orc_eval_in_element(bg, x, is_bdy, k, h, l, ms ? met_row : NULL, fptr)) {
      R->value_fail++;
      if (R->first_fail < 0) R->first_fail = i;
      continue;
    }
    int same = 1;
    double rel = 0.0;
    for (int c = 0; c < ms; c++) {
      double g = J->met_out[(size_t)ms * i + c];
      same = same && same_bits(g, met_row[c]);
      rel = fmax(rel, rel_err(g, met_row[c]));
    }
    for (int j = 0; j < nf && j < 64; j++) {
      int fs = bg->field_size[j];
      for (int c = 0; c < fs; c++) {
        double g = J->field_out[j][(size_t)fs * i + c];
        same = same && same_bits(g, frow[j][c]);
        rel = fmax(rel, rel_err(g, frow[j][c]));
      }
    }
    R->n++;
    R->exact += same;
    if (rel > R->maxrel) R->maxrel = rel;
    if (rel > J->rel_tol) {
      R->value_fail++;
      if (R->first_fail < 0) R->first_fail = i;
    }
    if (J->ref_elem && J->ref_hit) {
      int rh = J->ref_hit[i] & 15;
      double mb = J->ref_minbary ? J->ref_minbary[i] : 1.0;
      if ((rh == HIT_VOL_WALK || rh == HIT_VOL_EXHAUST) && mb > ORC_EPS) {
        R->class_i++;
        if (J->ref_elem[i] == k) R->class_i_same++;
        else if (R->first_fail < 0) R->first_fail = i;
      }
    }
  }
  return NULL;
}

int orc_check_batch(const orc_background *bg, const double *xyz, const uint8_t *pclass, const int *idx, int64_t n,
                    const int *elem, const int8_t *hit, const double *met_out, const double *const *field_out,
                    const int *ref_elem, const int8_t *ref_hit, const double *ref_minbary, int nthreads,
                    double rel_tol, orc_check_report *rep) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if (bg->nfield > 64) return 0;
  chk_job *J = (chk_job *)calloc((size_t)nthreads, sizeof(chk_job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!J || !th) {
    free(J);
    free(th);
    return 0;
  }
  for (int t = 0; t < nthreads; t++) {
    chk_job *j = &J[t];
    j->bg = bg; j->xyz = xyz; j->pclass = pclass; j->idx = idx;
    j->i0 = (n * t) / nthreads; j->i1 = (n * (t + 1)) / nthreads;
    j->elem = elem; j->hit = hit; j->met_out = met_out; j->field_out = field_out;
    j->ref_elem = ref_elem; j->ref_hit = ref_hit; j->ref_minbary = ref_minbary; j->rel_tol = rel_tol;
    j->rep.first_fail = -1;
    pthread_create(&th[t], NULL, job_check, j);
  }
  memset(rep, 0, sizeof(*rep));
  rep->first_fail = -1;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    const orc_check_report *r = &J[t].rep;
    rep->n += r->n; rep->exact += r->exact; rep->class_i += r->class_i; rep->class_i_same += r->class_i_same;
    rep->accept_fail += r->accept_fail; rep->value_fail += r->value_fail; rep->unprocessed += r->unprocessed;
    rep->skipped_written += r->skipped_written;
    if (r->maxrel > rep->maxrel) rep->maxrel = r->maxrel;
    for (int h = 0; h < 16; h++) rep->hits[h] += r->hits[h];
    if (rep->first_fail < 0 && r->first_fail >= 0) rep->first_fail = r->first_fail;
  }
  free(J);
  free(th);
  return 1;
}

/* ---------------------------------------------------------------- tetra quality
 * MMG3D_tetraQual / MMG5_caltet_iso / MMG5_caltet_ani (Mmg @889d408,
 * src/mmg3d/quality_3d.c, restated; reached from PMMG_tetraQual,
 * src/quality_pmmg.c:720-733).  Edges in the order ab, ac, ad, bc, bd, cd. */
#define ORC_EPSOK  1.e-20  /* MMG5_EPSOK */
#define ORC_ALPHAD 20.7846096908265 /* MMG3D_ALPHAD = 12 sqrt(3): a regular tetra has quality 1 */

static void orc_edges(const double *p[4], double e[6][3]) {
  static const int ea[6] = {0, 0, 0, 1, 1, 2}, eb[6] = {1, 2, 3, 2, 3, 3};
  for (int i = 0; i < 6; i++)
    for (int d = 0; d < 3; d++) e[i][d] = p[eb[i]][d] - p[ea[i]][d];
}

static double orc_vol6(double e[6][3]) {
  /* (b-a) . ((c-a) x (d-a)) */
  double v1 = e[1][1] * e[2][2] - e[1][2] * e[2][1];
  double v2 = e[1][2] * e[2][0] - e[1][0] * e[2][2];
  double v3 = e[1][0] * e[2][1] - e[1][1] * e[2][0];
  return e[0][0] * v1 + e[0][1] * v2 + e[0][2] * v3;
}

static double orc_caltet_iso(const double *p[4]) {
  double e[6][3];
  orc_edges(p, e);
  double vol = orc_vol6(e);
  if (vol < ORC_EPSD2) return 0.0;
  double rap = e[0][0] * e[0][0] + e[0][1] * e[0][1] + e[0][2] * e[0][2];
  for (int i = 1; i < 6; i++) rap += e[i][0] * e[i][0] + e[i][1] * e[i][1] + e[i][2] * e[i][2];
  if (rap < ORC_EPSD2) return 0.0;
  rap = rap * sqrt(rap);
  return vol / rap;
}

static double orc_caltet_ani(const double *p[4], const double *mm) {
  double e[6][3], h[6];
  orc_edges(p, e);
  double vol = orc_vol6(e);
  if (vol <= 0.0) return 0.0;
  double det = mm[0] * (mm[3] * mm[5] - mm[4] * mm[4]) - mm[1] * (mm[1] * mm[5] - mm[2] * mm[4]) +
               mm[2] * (mm[1] * mm[4] - mm[2] * mm[3]);
  if (det < ORC_EPSOK) return 0.0;
  det = sqrt(det) * vol;
  for (int i = 0; i < 6; i++) {
    const double x = e[i][0], y = e[i][1], z = e[i][2];
    h[i] = mm[0] * x * x + mm[3] * y * y + mm[5] * z * z + 2.0 * (mm[1] * x * y + mm[2] * x * z + mm[4] * y * z);
  }
  double rap = h[0] + h[1] + h[2] + h[3] + h[4] + h[5];
  double num = sqrt(rap) * rap;
  return det / num;
}

double orc_tetra_qual(int np, const double *xyz, int ne, const int *tetv, int met_size, const double *met,
                      double *qual) {
  double minqual = 2.0 / ORC_ALPHAD;
  (void)np;
  for (int k = 0; k < ne; k++) {
    const int *v = tetv + 4 * (int64_t)k;
    if (v[0] <= 0) {
      qual[k] = 0.0;
      continue;
    }
    const double *p[4];
    for (int i = 0; i < 4; i++) p[i] = xyz + 3 * (int64_t)(v[i] - 1);
    double q;
    if (met_size == 6) {
      double mm[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 6; j++) mm[j] += met[6 * (int64_t)(v[i] - 1) + j];
      for (int j = 0; j < 6; j++) mm[j] *= 0.25;
      q = orc_caltet_ani(p, mm);
    } else {
      q = orc_caltet_iso(p);
    }
    qual[k] = q;
    if (q < minqual) minqual = q;
  }
  return ORC_ALPHAD * minqual;
}

/* ------------------------------------------------------------------ metis weights
 * PMMG_computeWgt (src/metis_pmmg.c:280-300) and PMMG_computeWgt_mesh
 * (:242-266): per tetra face, the three face edges' lengths in the metric
 * (MMG5_lenedg: MMG5_lenedgCoor_iso / MMG5_lenedgCoor_ani of Mmg @889d408,
 * restated from its published source — Mmg is not in the image, parity
 * unpinned; aniso edges use the general formula, Mmg's special ridge-point
 * storage (MG_GEO edges) is not modelled), res = sum over the edges of
 * (len - 1) for len <= 1 else (1/len - 1), weight = min(1/exp(28 res / 3),
 * PMMG_WGTVAL_HUGEINT); without a metric the weight is PMMG_WGTVAL_HUGEINT. */
static const int kIare[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}}; /* MMG5_iare */
static const int kIarf[4][3] = {{5, 4, 3}, {5, 1, 2}, {4, 2, 0}, {3, 0, 1}};     /* MMG5_iarf */
#define ORC_WGTVAL_HUGEINT 1000000
#define ORC_MMG5_EPS 1.0e-06

static double lenedg_iso(const double *ca, const double *cb, double h1, double h2) {
  double l = (cb[0] - ca[0]) * (cb[0] - ca[0]) + (cb[1] - ca[1]) * (cb[1] - ca[1]) + (cb[2] - ca[2]) * (cb[2] - ca[2]);
  l = sqrt(l);
  const double r = h2 / h1 - 1.0;
  return (fabs(r) < ORC_MMG5_EPS) ? (l / h1) : (l / (h2 - h1) * log1p(r));
}

static double lenedg_ani(const double *ca, const double *cb, const double *sa, const double *sb) {
  const double ux = cb[0] - ca[0], uy = cb[1] - ca[1], uz = cb[2] - ca[2];
  double dd1 = sa[0] * ux * ux + sa[3] * uy * uy + sa[5] * uz * uz + 2.0 * (sa[1] * ux * uy + sa[2] * ux * uz + sa[4] * uy * uz);
  if (dd1 <= 0.0) dd1 = 0.0;
  double dd2 = sb[0] * ux * ux + sb[3] * uy * uy + sb[5] * uz * uz + 2.0 * (sb[1] * ux * uy + sb[2] * ux * uz + sb[4] * uy * uz);
  if (dd2 <= 0.0) dd2 = 0.0;
  if (fabs(dd1 - dd2) < 0.05) return sqrt(0.5 * (dd1 + dd2));
  return (sqrt(dd1) + sqrt(dd2) + 4.0 * sqrt(0.5 * (dd1 + dd2))) / 6.0;
}

double orc_face_wgt(const double *xyz, const int *v, int ifac, int met_size, const double *met) {
  if (met_size != 1 && met_size != 6) return (double)ORC_WGTVAL_HUGEINT;
  double res = 0.0;
  for (int i = 0; i < 3; i++) {
    const int ia = kIarf[ifac][i];
    const int ip1 = v[kIare[ia][0]], ip2 = v[kIare[ia][1]];
    const double *ca = xyz + 3 * (int64_t)(ip1 - 1), *cb = xyz + 3 * (int64_t)(ip2 - 1);
    const double len = met_size == 1 ? lenedg_iso(ca, cb, met[ip1 - 1], met[ip2 - 1])
                                     : lenedg_ani(ca, cb, met + 6 * (int64_t)(ip1 - 1), met + 6 * (int64_t)(ip2 - 1));
    if (len <= 1.0)
      res += len - 1.0;
    else
      res += 1.0 / len - 1.0;
  }
  const double w = 1.0 / exp(28.0 * res / 3.0);
  return w < (double)ORC_WGTVAL_HUGEINT ? w : (double)ORC_WGTVAL_HUGEINT;
}

void orc_compute_wgt_mesh(int ne, const int *tetv, const int *xt, const uint16_t *ftag, const double *xyz,
                          int met_size, const double *met, int tag, double *qual) {
  for (int k = 0; k < ne; k++) {
    const int *v = tetv + 4 * (int64_t)k;
    if (v[0] <= 0 || !xt[k]) continue; /* !MG_EOK, or no xtetra: qual untouched */
    double q = 0.0;
    for (int f = 0; f < 4; f++)
      if (ftag[4 * (int64_t)k + f] & tag) q += orc_face_wgt(xyz, v, f, met_size, met);
    qual[k] = q;
  }
}
