/*
 * pmmg_shard.c — halo shards of a background group.
 *
 * ParMmg distributes the background by group and each rank transfers its own
 * new points against its own part (src/interpmesh_pmmg.c:690).  For a group
 * too large to replicate on every GPU, a rank that owns a contiguous Morton
 * range of the new points needs only the background tetra around that
 * range: the tetra whose bounding box meets the range's box grown by a halo
 * (pmmg_shard_mark), or, tighter, the union of the grid cells that hold the
 * range's points (pmmg_shard_mark_cells: a Morton range of a shell has a box
 * far larger than the range).
 * Every tetra that accepts a point of the range (min barycentric > -EPS)
 * meets that box once the halo exceeds EPS times its extent, so the shard
 * holds every candidate of the range's points.
 *
 * The shard keeps the global relative order of tetra, vertices and trias
 * (local ids ascend with global ids), so the exhaustive searches' "lowest
 * index accepting" rule (src/locate_pmmg.c:737-770) picks the same element
 * in the shard as in the whole group.  Adjacency codes are remapped to local
 * ids; a neighbour outside the shard becomes 0 (a wall: walks that reach the
 * cut turn back or fall back to the exhaustive search of the shard).  Trias
 * are the group's boundary trias with all three vertices in the shard.
 *
 * Two passes over caller-owned buffers: pmmg_shard_mark sizes the shard,
 * pmmg_shard_fill writes it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pmmg_host.h"

static void tet_box(const double *xyz, const int *v, double lo[3], double hi[3]) {
  for (int d = 0; d < 3; d++) {
    lo[d] = hi[d] = xyz[3 * (int64_t)(v[0] - 1) + d];
  }
  for (int i = 1; i < 4; i++)
    for (int d = 0; d < 3; d++) {
      double c = xyz[3 * (int64_t)(v[i] - 1) + d];
      if (c < lo[d]) lo[d] = c;
      if (c > hi[d]) hi[d] = c;
    }
}

double pmmg_max_tet_extent(int np, const double *xyz, int ne, const int *tetv) {
  double m = 0.0;
  (void)np;
#pragma omp parallel for reduction(max : m) schedule(static)
  for (int64_t k = 0; k < ne; k++) {
    double lo[3], hi[3];
    tet_box(xyz, tetv + 4 * k, lo, hi);
    for (int d = 0; d < 3; d++)
      if (hi[d] - lo[d] > m) m = hi[d] - lo[d];
  }
  return m;
}

/* map[i] != 0 -> its rank among the nonzero entries (1-based), in index
 * order; returns the count.  Chunked in parallel: per-chunk counts, their
 * prefix, then the numbering (the shard keeps the group's relative order). */
static int number_marks(int *map, int64_t n) {
  enum { kChunks = 256 };
  int64_t cnt[kChunks + 1];
  const int64_t per = (n + kChunks - 1) / kChunks;
#pragma omp parallel for schedule(static)
  for (int c = 0; c < kChunks; c++) {
    int64_t a = c * per, b = a + per < n ? a + per : n, k = 0;
    for (int64_t i = a; i < b; i++) k += map[i] != 0;
    cnt[c + 1] = k;
  }
  cnt[0] = 0;
  for (int c = 0; c < kChunks; c++) cnt[c + 1] += cnt[c];
#pragma omp parallel for schedule(static)
  for (int c = 0; c < kChunks; c++) {
    int64_t a = c * per, b = a + per < n ? a + per : n;
    int next = (int)cnt[c];
    for (int64_t i = a; i < b; i++)
      if (map[i]) map[i] = ++next;
  }
  return (int)cnt[kChunks];
}

int pmmg_shard_mark(int np, const double *xyz, int ne, const int *tetv, const double box_lo[3],
                    const double box_hi[3], double halo, int *tet_map, int *vert_map, int64_t counts[2]) {
  double lo[3], hi[3];
  if (np < 0 || ne < 0 || !counts || (ne > 0 && (!xyz || !tetv || !tet_map)) || (np > 0 && !vert_map))
    return 0;
  if (halo < 0.0) halo = -halo * pmmg_max_tet_extent(np, xyz, ne, tetv);
  for (int d = 0; d < 3; d++) {
    lo[d] = box_lo[d] - halo;
    hi[d] = box_hi[d] + halo;
  }
  memset(vert_map, 0, sizeof(int) * (size_t)np);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t k = 0; k < ne; k++) {
    const int *v = tetv + 4 * k;
    double tl[3], th[3];
    int ok = 1;
    for (int i = 0; i < 4; i++)
      if (v[i] < 1 || v[i] > np) ok = 0;
    if (!ok) {
      bad = 1;
      tet_map[k] = 0;
      continue;
    }
    tet_box(xyz, v, tl, th);
    int meets = 1;
    for (int d = 0; d < 3; d++)
      if (th[d] < lo[d] || tl[d] > hi[d]) meets = 0;
    tet_map[k] = meets;
    if (meets)
      for (int i = 0; i < 4; i++) {
        /* several threads may mark one vertex: atomic stores (all store 1) */
#pragma omp atomic write
        vert_map[v[i] - 1] = 1;
      }
  }
  if (bad) return 0;
  counts[0] = number_marks(tet_map, ne);
  counts[1] = number_marks(vert_map, np);
  return 1;
}

/* bounding box of the occupied cells of a region's grid: a cheap first test
 * (empty grid: clo > chi) */
static void occ_bounds(const int g_n[3], const uint8_t *occ, int clo[3], int chi[3]) {
  for (int d = 0; d < 3; d++) {
    clo[d] = g_n[d];
    chi[d] = -1;
  }
  for (int k = 0; k < g_n[2]; k++)
    for (int j = 0; j < g_n[1]; j++)
      for (int i = 0; i < g_n[0]; i++)
        if (occ[i + (int64_t)g_n[0] * (j + (int64_t)g_n[1] * k)]) {
          const int c[3] = {i, j, k};
          for (int d = 0; d < 3; d++) {
            if (c[d] < clo[d]) clo[d] = c[d];
            if (c[d] > chi[d]) chi[d] = c[d];
          }
        }
}

/* the region test of the shard builders: the element's box [tl, th] grown by
 * the halo meets the points' box (when given) and an occupied cell */
static int region_meets(const double *box_lo, const double *box_hi, const double g_lo[3], double cell,
                        const int g_n[3], const uint8_t *occ, double halo, const int clo[3], const int chi[3],
                        const double tl[3], const double th[3]) {
  int a[3], b[3];
  if (box_lo && box_hi)
    for (int d = 0; d < 3; d++)
      if (th[d] < box_lo[d] - halo || tl[d] > box_hi[d] + halo) return 0;
  for (int d = 0; d < 3; d++) { /* cells met by the element's box grown by the halo */
    a[d] = (int)floor((tl[d] - halo - g_lo[d]) / cell);
    b[d] = (int)floor((th[d] + halo - g_lo[d]) / cell);
    if (a[d] < clo[d]) a[d] = clo[d];
    if (b[d] > chi[d]) b[d] = chi[d];
    if (a[d] > b[d]) return 0;
  }
  for (int z = a[2]; z <= b[2]; z++)
    for (int y = a[1]; y <= b[1]; y++)
      for (int x = a[0]; x <= b[0]; x++)
        if (occ[x + (int64_t)g_n[0] * (y + (int64_t)g_n[1] * z)]) return 1;
  return 0;
}

static int region_ok(const pmmg_shard_region *R) {
  if (!R || !(R->cell > 0.0) || !R->occ || !(R->halo >= 0.0)) return 0;
  for (int d = 0; d < 3; d++)
    if (R->g_n[d] < 1) return 0;
  return 1;
}

int pmmg_shard_mark_cells(int np, const double *xyz, int ne, const int *tetv, const double box_lo[3],
                          const double box_hi[3], const double g_lo[3], double cell, const int g_n[3],
                          const uint8_t *occ, double halo, int *tet_map, int *vert_map, int64_t counts[2]) {
  if (np < 0 || ne < 0 || !counts || !(cell > 0.0) || !g_n || !occ || (ne > 0 && (!xyz || !tetv || !tet_map)) ||
      (np > 0 && !vert_map))
    return 0;
  for (int d = 0; d < 3; d++)
    if (g_n[d] < 1) return 0;
  if (halo < 0.0) halo = -halo * pmmg_max_tet_extent(np, xyz, ne, tetv);
  int clo[3], chi[3];
  occ_bounds(g_n, occ, clo, chi);
  memset(vert_map, 0, sizeof(int) * (size_t)np);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t k = 0; k < ne; k++) {
    const int *v = tetv + 4 * k;
    int ok = 1;
    for (int i = 0; i < 4; i++)
      if (v[i] < 1 || v[i] > np) ok = 0;
    if (!ok) {
      bad = 1;
      tet_map[k] = 0;
      continue;
    }
    double tl[3], th[3];
    tet_box(xyz, v, tl, th);
    const int meets = region_meets(box_lo, box_hi, g_lo, cell, g_n, occ, halo, clo, chi, tl, th);
    tet_map[k] = meets;
    if (meets)
      for (int i = 0; i < 4; i++) {
        /* several threads may mark one vertex: atomic stores (all store 1) */
#pragma omp atomic write
        vert_map[v[i] - 1] = 1;
      }
  }
  if (bad) return 0;
  counts[0] = number_marks(tet_map, ne);
  counts[1] = number_marks(vert_map, np);
  return 1;
}

static void tri_box(const double *xyz, const int *v, double lo[3], double hi[3]) {
  for (int d = 0; d < 3; d++) lo[d] = hi[d] = xyz[3 * (int64_t)(v[0] - 1) + d];
  for (int i = 1; i < 3; i++)
    for (int d = 0; d < 3; d++) {
      const double c = xyz[3 * (int64_t)(v[i] - 1) + d];
      if (c < lo[d]) lo[d] = c;
      if (c > hi[d]) hi[d] = c;
    }
}

int64_t pmmg_shard_mark_trias(int np, const double *xyz, int nt, const int *triv, const pmmg_shard_region *reg,
                              int *tria_map) {
  if (np < 0 || nt < 0 || !region_ok(reg) || (nt > 0 && (!xyz || !triv || !tria_map))) return -1;
  int clo[3], chi[3];
  occ_bounds(reg->g_n, reg->occ, clo, chi);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t t = 0; t < nt; t++) {
    const int *v = triv + 3 * t;
    if (v[0] < 1 || v[0] > np || v[1] < 1 || v[1] > np || v[2] < 1 || v[2] > np) {
      bad = 1;
      tria_map[t] = 0;
      continue;
    }
    double tl[3], th[3];
    tri_box(xyz, v, tl, th);
    tria_map[t] = region_meets(reg->box_lo, reg->box_hi, reg->g_lo, reg->cell, reg->g_n, reg->occ, reg->halo, clo,
                               chi, tl, th);
  }
  if (bad) return -1;
  return number_marks(tria_map, nt);
}

int64_t pmmg_shard_fill(int np, const double *xyz, int ne, const int *tetv, const int *adja, int nt,
                        const int *triv, const int *adjt, const int *tet_map, const int *vert_map,
                        double *s_xyz, int *s_tetv, int *s_adja, int *s_triv, int *s_adjt, int *tet_gid,
                        int *vert_gid, int *tria_gid) {
  if (np < 0 || ne < 0 || nt < 0) return -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < np; i++) {
    int l = vert_map[i];
    if (!l) continue;
    memcpy(s_xyz + 3 * (int64_t)(l - 1), xyz + 3 * i, 3 * sizeof(double));
    if (vert_gid) vert_gid[l - 1] = (int)(i + 1);
  }
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t k = 0; k < ne; k++) {
    int l = tet_map[k];
    if (!l) continue;
    int64_t o = 4 * (int64_t)(l - 1);
    for (int i = 0; i < 4; i++) {
      s_tetv[o + i] = vert_map[tetv[4 * k + i] - 1];
      int a = adja ? adja[4 * k + i] : 0, la = 0;
      if (a > 0) {
        int g = a / 4;
        if (g < 1 || g > ne) {
          bad = 1;
          continue;
        }
        la = tet_map[g - 1] ? 4 * tet_map[g - 1] + a % 4 : 0;
      }
      if (s_adja) s_adja[o + i] = la;
    }
    if (tet_gid) tet_gid[l - 1] = (int)(k + 1);
  }
  if (bad) return -1;
  /* trias: kept in global order when all three vertices are in the shard */
  int *tria_map = NULL;
  if (nt > 0) {
    tria_map = (int *)malloc(sizeof(int) * (size_t)nt);
    if (!tria_map) return -1;
  }
  int ntl = 0;
  for (int64_t t = 0; t < nt; t++) {
    const int *v = triv + 3 * t;
    int ok = 1;
    for (int i = 0; i < 3; i++)
      if (v[i] < 1 || v[i] > np || !vert_map[v[i] - 1]) ok = 0;
    tria_map[t] = ok ? ++ntl : 0;
  }
  for (int64_t t = 0; t < nt; t++) {
    int l = tria_map[t];
    if (!l) continue;
    int64_t o = 3 * (int64_t)(l - 1);
    for (int i = 0; i < 3; i++) {
      s_triv[o + i] = vert_map[triv[3 * t + i] - 1];
      int a = adjt ? adjt[3 * t + i] : 0, la = 0;
      if (a > 0) {
        int g = a / 3;
        if (g < 1 || g > nt) {
          free(tria_map);
          return -1;
        }
        la = tria_map[g - 1] ? 3 * tria_map[g - 1] + a % 3 : 0;
      }
      if (s_adjt) s_adjt[o + i] = la;
    }
    if (tria_gid) tria_gid[l - 1] = (int)(t + 1);
  }
  free(tria_map);
  return ntl;
}

int64_t pmmg_shard_fill_region(int np, const double *xyz, int ne, const int *tetv, const int *adja, int nt,
                               const int *triv, const int *adjt, const int *tet_map, const int *vert_map,
                               const int *tria_map, double *s_xyz, int *s_tetv, int *s_adja, int *s_triv,
                               int *s_adjt, int *tet_gid, int *vert_gid, int *tria_gid) {
  if (nt < 0 || (nt > 0 && (!triv || !tria_map))) return -1;
  /* vertices and tetra as pmmg_shard_fill, without its trias */
  if (pmmg_shard_fill(np, xyz, ne, tetv, adja, 0, NULL, NULL, tet_map, vert_map, s_xyz, s_tetv, s_adja, NULL, NULL,
                      tet_gid, vert_gid, NULL) < 0)
    return -1;
  int64_t ntl = 0, bad = 0;
  for (int64_t t = 0; t < nt; t++) {
    const int l = tria_map[t];
    if (!l) continue;
    ntl++;
    const int64_t o = 3 * (int64_t)(l - 1);
    for (int i = 0; i < 3; i++) {
      const int v = triv[3 * t + i];
      const int lv = (v >= 1 && v <= np) ? vert_map[v - 1] : 0;
      if (!lv) bad = 1; /* a tria of the region has its tetra (and vertices) in the shard */
      s_triv[o + i] = lv;
      int a = adjt ? adjt[3 * t + i] : 0, la = 0;
      if (a > 0) {
        const int g = a / 3;
        if (g < 1 || g > nt) return -1;
        la = tria_map[g - 1] ? 3 * tria_map[g - 1] + a % 3 : 0;
      }
      if (s_adjt) s_adjt[o + i] = la;
    }
    if (tria_gid) tria_gid[l - 1] = (int)(t + 1);
  }
  return bad ? -1 : ntl;
}

/* ---------------------------------------------------------------- parts */

/* record buffer of pmmg_shard_part_pack:
 *   int64 header[5] = {magic, K, ntet, ntri, nvert}
 *   ntet x int32[9]  {gid, v[4] (global), adja[4] (group codes)}
 *   ntri x int32[7]  {gid, v[3] (global), adjt[3] (group codes)}, padded to 8 bytes
 *   nvert x {int64 gid, double xyz[3], double sol[K]}
 * every list ascending by gid */
#define SHARD_MAGIC 0x48534d50LL /* "PMSH" */
enum { TREC = 9, RREC = 7 };

static int64_t vrec_bytes(int K) { return 8 + 24 + 8 * (int64_t)K; }
static int64_t pack_bytes(int K, int64_t ntet, int64_t ntri, int64_t nvert) {
  int64_t b = 40 + 4 * (TREC * ntet + RREC * ntri);
  b = (b + 7) & ~7LL;
  return b + nvert * vrec_bytes(K);
}

/* index of gid in the ascending ids[0..n), or -1 */
static int64_t find_gid(const int *ids, int64_t n, int gid) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) / 2;
    if (ids[m] < gid) lo = m + 1;
    else hi = m;
  }
  return (lo < n && ids[lo] == gid) ? lo : -1;
}

int64_t pmmg_shard_part_pack(const pmmg_shard_part *P, const pmmg_shard_region *reg, void *buf, int64_t cap) {
  if (!P || !region_ok(reg) || P->np < 0 || P->ne < 0 || P->nt < 0 || P->K < 0 || (P->K > 0 && P->np > 0 && !P->sol) ||
      (P->np > 0 && (!P->vert_gid || !P->xyz)) || (P->ne > 0 && (!P->tet_gid || !P->tetv || !P->adja)) ||
      (P->nt > 0 && (!P->tria_gid || !P->triv)))
    return -1;
  int clo[3], chi[3];
  occ_bounds(reg->g_n, reg->occ, clo, chi);
  int *tsel = (int *)calloc((size_t)P->ne + 1, sizeof(int));
  int *rsel = (int *)calloc((size_t)P->nt + 1, sizeof(int));
  int *vsel = (int *)calloc((size_t)P->np + 1, sizeof(int));
  if (!tsel || !rsel || !vsel) {
    free(tsel);
    free(rsel);
    free(vsel);
    return -1;
  }
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t k = 0; k < P->ne; k++) {
    int64_t lv[4];
    double tl[3], th[3];
    for (int i = 0; i < 4; i++) {
      lv[i] = find_gid(P->vert_gid, P->np, P->tetv[4 * k + i]);
      if (lv[i] < 0) bad = 1;
    }
    if (bad) continue;
    for (int d = 0; d < 3; d++) tl[d] = th[d] = P->xyz[3 * lv[0] + d];
    for (int i = 1; i < 4; i++)
      for (int d = 0; d < 3; d++) {
        const double c = P->xyz[3 * lv[i] + d];
        if (c < tl[d]) tl[d] = c;
        if (c > th[d]) th[d] = c;
      }
    if (region_meets(reg->box_lo, reg->box_hi, reg->g_lo, reg->cell, reg->g_n, reg->occ, reg->halo, clo, chi, tl,
                     th)) {
      tsel[k] = 1;
      for (int i = 0; i < 4; i++) {
#pragma omp atomic write
        vsel[lv[i]] = 1;
      }
    }
  }
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t t = 0; t < P->nt; t++) {
    int64_t lv[3];
    double tl[3], th[3];
    for (int i = 0; i < 3; i++) {
      lv[i] = find_gid(P->vert_gid, P->np, P->triv[3 * t + i]);
      if (lv[i] < 0) bad = 1;
    }
    if (bad) continue;
    for (int d = 0; d < 3; d++) tl[d] = th[d] = P->xyz[3 * lv[0] + d];
    for (int i = 1; i < 3; i++)
      for (int d = 0; d < 3; d++) {
        const double c = P->xyz[3 * lv[i] + d];
        if (c < tl[d]) tl[d] = c;
        if (c > th[d]) th[d] = c;
      }
    rsel[t] = region_meets(reg->box_lo, reg->box_hi, reg->g_lo, reg->cell, reg->g_n, reg->occ, reg->halo, clo, chi,
                           tl, th);
  }
  int64_t ntet = 0, ntri = 0, nvert = 0;
  for (int64_t k = 0; k < P->ne; k++) ntet += tsel[k];
  for (int64_t t = 0; t < P->nt; t++) ntri += rsel[t];
  for (int64_t i = 0; i < P->np; i++) nvert += vsel[i];
  const int64_t need = pack_bytes(P->K, ntet, ntri, nvert);
  if (!bad && buf && cap >= need) {
    int64_t *hdr = (int64_t *)buf;
    hdr[0] = SHARD_MAGIC;
    hdr[1] = P->K;
    hdr[2] = ntet;
    hdr[3] = ntri;
    hdr[4] = nvert;
    int *w = (int *)(hdr + 5);
    for (int64_t k = 0; k < P->ne; k++) {
      if (!tsel[k]) continue;
      w[0] = P->tet_gid[k];
      memcpy(w + 1, P->tetv + 4 * k, 4 * sizeof(int));
      memcpy(w + 5, P->adja + 4 * k, 4 * sizeof(int));
      w += TREC;
    }
    for (int64_t t = 0; t < P->nt; t++) {
      if (!rsel[t]) continue;
      w[0] = P->tria_gid[t];
      memcpy(w + 1, P->triv + 3 * t, 3 * sizeof(int));
      for (int i = 0; i < 3; i++) w[4 + i] = P->adjt ? P->adjt[3 * t + i] : 0;
      w += RREC;
    }
    char *vb = (char *)buf + ((40 + 4 * (TREC * ntet + RREC * ntri) + 7) & ~7LL);
    for (int64_t i = 0; i < P->np; i++) {
      if (!vsel[i]) continue;
      const int64_t g = P->vert_gid[i];
      memcpy(vb, &g, 8);
      memcpy(vb + 8, P->xyz + 3 * i, 24);
      if (P->K) memcpy(vb + 32, P->sol + (int64_t)P->K * i, 8 * (size_t)P->K);
      vb += vrec_bytes(P->K);
    }
  }
  free(tsel);
  free(rsel);
  free(vsel);
  return bad ? -1 : need;
}

typedef struct {
  const int64_t *hdr;
  const int *tet, *tri;
  const char *vert;
  int64_t ntet, ntri, nvert;
} part_view;

static int view_of(const void *b, int64_t len, int K, part_view *v) {
  if (!b || len < 40) return 0;
  v->hdr = (const int64_t *)b;
  if (v->hdr[0] != SHARD_MAGIC || v->hdr[1] != K) return 0;
  v->ntet = v->hdr[2];
  v->ntri = v->hdr[3];
  v->nvert = v->hdr[4];
  if (v->ntet < 0 || v->ntri < 0 || v->nvert < 0 || pack_bytes(K, v->ntet, v->ntri, v->nvert) > len) return 0;
  v->tet = (const int *)(v->hdr + 5);
  v->tri = v->tet + TREC * v->ntet;
  v->vert = (const char *)b + ((40 + 4 * (TREC * v->ntet + RREC * v->ntri) + 7) & ~7LL);
  return 1;
}

static int64_t vgid_at(const part_view *v, int64_t i, int K) {
  int64_t g;
  memcpy(&g, v->vert + i * vrec_bytes(K), 8);
  return g;
}

/* k-way merge of the parts' ascending id lists: next = the part whose head
 * gid is smallest (ties: the lower part, whose copy is taken; the others'
 * equal heads are skipped as duplicates) */
typedef int64_t (*head_fn)(const part_view *, int64_t, int);
static int64_t tet_head(const part_view *v, int64_t i, int K) {
  (void)K;
  return v->tet[TREC * i];
}
static int64_t tri_head(const part_view *v, int64_t i, int K) {
  (void)K;
  return v->tri[RREC * i];
}

/* merged order of one list: (part, index) pairs into out (room for the sum),
 * returns the merged count (duplicates dropped) or -1 if a part's list is
 * not ascending */
static int64_t merge_lists(int nb, const part_view *pv, int which, int K, int *opart, int64_t *oidx) {
  int64_t *pos = (int64_t *)calloc((size_t)nb + 1, sizeof(int64_t));
  if (!pos) return -1;
  int64_t n = 0, last = -1;
  for (;;) {
    int best = -1;
    int64_t bg = 0;
    for (int b = 0; b < nb; b++) {
      const int64_t cnt = which == 0 ? pv[b].ntet : (which == 1 ? pv[b].ntri : pv[b].nvert);
      if (pos[b] >= cnt) continue;
      const int64_t g = which == 0 ? tet_head(&pv[b], pos[b], K)
                                   : (which == 1 ? tri_head(&pv[b], pos[b], K) : vgid_at(&pv[b], pos[b], K));
      if (best < 0 || g < bg) {
        best = b;
        bg = g;
      }
    }
    if (best < 0) break;
    if (bg < last) {
      free(pos);
      return -1;
    }
    if (bg != last) {
      opart[n] = best;
      oidx[n] = pos[best];
      n++;
      last = bg;
    }
    pos[best]++;
  }
  free(pos);
  return n;
}

static int64_t find_gid64(const int *ids, int64_t n, int64_t gid) { return find_gid(ids, n, (int)gid); }

int pmmg_shard_assemble(int nbuf, const void *const *bufs, const int64_t *lens, int K, int64_t counts[3],
                        double *s_xyz, double *s_sol, int *s_tetv, int *s_adja, int *s_triv, int *s_adjt,
                        int *tet_gid, int *vert_gid, int *tria_gid) {
  if (nbuf < 0 || K < 0 || !counts || (nbuf > 0 && (!bufs || !lens))) return 0;
  part_view *pv = (part_view *)calloc((size_t)nbuf + 1, sizeof(part_view));
  if (!pv) return 0;
  int64_t st = 0, sr = 0, sv = 0;
  for (int b = 0; b < nbuf; b++) {
    if (!view_of(bufs[b], lens[b], K, &pv[b])) {
      free(pv);
      return 0;
    }
    st += pv[b].ntet;
    sr += pv[b].ntri;
    sv += pv[b].nvert;
  }
  int ok = 1;
  int *op = (int *)malloc(sizeof(int) * (size_t)(st > sr ? (st > sv ? st : sv) : (sr > sv ? sr : sv)) + 8);
  int64_t *oi = (int64_t *)malloc(sizeof(int64_t) * (size_t)(st > sr ? (st > sv ? st : sv) : (sr > sv ? sr : sv)) + 8);
  int *vg = NULL, *tg = NULL, *rg = NULL;
  if (!op || !oi) ok = 0;
  /* vertices: merged, duplicates dropped; the local id of a global vertex
   * is its rank in vg */
  int64_t nv = ok ? merge_lists(nbuf, pv, 2, K, op, oi) : -1;
  if (nv < 0) ok = 0;
  if (ok) {
    vg = (int *)malloc(sizeof(int) * (size_t)nv + 4);
    if (!vg) ok = 0;
  }
  if (ok)
    for (int64_t i = 0; i < nv; i++) {
      const char *r = pv[op[i]].vert + oi[i] * vrec_bytes(K);
      int64_t g;
      memcpy(&g, r, 8);
      vg[i] = (int)g;
      if (s_xyz) {
        memcpy(s_xyz + 3 * i, r + 8, 24);
        if (K && s_sol) memcpy(s_sol + (int64_t)K * i, r + 32, 8 * (size_t)K);
        if (vert_gid) vert_gid[i] = (int)g;
      }
    }
  /* tetra */
  int64_t ne = ok ? merge_lists(nbuf, pv, 0, K, op, oi) : -1;
  if (ne < 0) ok = 0;
  if (ok) {
    tg = (int *)malloc(sizeof(int) * (size_t)ne + 4);
    if (!tg) ok = 0;
  }
  if (ok) {
    for (int64_t k = 0; k < ne; k++) tg[k] = pv[op[k]].tet[TREC * oi[k]];
    if (s_xyz) {
      int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
      for (int64_t k = 0; k < ne; k++) {
        const int *r = pv[op[k]].tet + TREC * oi[k];
        for (int i = 0; i < 4; i++) {
          const int64_t lv = find_gid(vg, nv, r[1 + i]);
          if (lv < 0) bad = 1;
          s_tetv[4 * k + i] = (int)(lv + 1);
          const int a = r[5 + i];
          int la = 0;
          if (a > 0) {
            const int64_t lk = find_gid64(tg, ne, a / 4);
            la = lk >= 0 ? (int)(4 * (lk + 1) + a % 4) : 0;
          }
          if (s_adja) s_adja[4 * k + i] = la;
        }
        if (tet_gid) tet_gid[k] = r[0];
      }
      if (bad) ok = 0;
    }
  }
  /* trias */
  int64_t nt = ok ? merge_lists(nbuf, pv, 1, K, op, oi) : -1;
  if (nt < 0) ok = 0;
  if (ok) {
    rg = (int *)malloc(sizeof(int) * (size_t)nt + 4);
    if (!rg) ok = 0;
  }
  if (ok) {
    for (int64_t t = 0; t < nt; t++) rg[t] = pv[op[t]].tri[RREC * oi[t]];
    if (s_xyz) {
      for (int64_t t = 0; t < nt && ok; t++) {
        const int *r = pv[op[t]].tri + RREC * oi[t];
        for (int i = 0; i < 3; i++) {
          const int64_t lv = find_gid(vg, nv, r[1 + i]);
          if (lv < 0) ok = 0;
          s_triv[3 * t + i] = (int)(lv + 1);
          const int a = r[4 + i];
          int la = 0;
          if (a > 0) {
            const int64_t lt = find_gid64(rg, nt, a / 3);
            la = lt >= 0 ? (int)(3 * (lt + 1) + a % 3) : 0;
          }
          if (s_adjt) s_adjt[3 * t + i] = la;
        }
        if (tria_gid) tria_gid[t] = r[0];
      }
    }
  }
  if (ok) {
    counts[0] = nv;
    counts[1] = ne;
    counts[2] = nt;
  }
  free(op);
  free(oi);
  free(vg);
  free(tg);
  free(rg);
  free(pv);
  return ok;
}
