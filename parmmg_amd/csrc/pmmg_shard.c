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

int pmmg_shard_mark_cells(int np, const double *xyz, int ne, const int *tetv, const double box_lo[3],
                          const double box_hi[3], const double g_lo[3], double cell, const int g_n[3],
                          const uint8_t *occ, double halo, int *tet_map, int *vert_map, int64_t counts[2]) {
  if (np < 0 || ne < 0 || !counts || !(cell > 0.0) || !g_n || !occ || (ne > 0 && (!xyz || !tetv || !tet_map)) ||
      (np > 0 && !vert_map))
    return 0;
  for (int d = 0; d < 3; d++)
    if (g_n[d] < 1) return 0;
  if (halo < 0.0) halo = -halo * pmmg_max_tet_extent(np, xyz, ne, tetv);
  /* bounding box of the occupied cells: a cheap first test */
  int clo[3] = {g_n[0], g_n[1], g_n[2]}, chi[3] = {-1, -1, -1};
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
    int a[3], b[3], meets = 1;
    if (box_lo && box_hi) /* and the range's box grown by the halo (pmmg_shard_mark's test) */
      for (int d = 0; d < 3; d++)
        if (th[d] < box_lo[d] - halo || tl[d] > box_hi[d] + halo) meets = 0;
    for (int d = 0; d < 3 && meets; d++) { /* cells met by the tetra's box grown by the halo */
      a[d] = (int)floor((tl[d] - halo - g_lo[d]) / cell);
      b[d] = (int)floor((th[d] + halo - g_lo[d]) / cell);
      if (a[d] < clo[d]) a[d] = clo[d];
      if (b[d] > chi[d]) b[d] = chi[d];
      if (a[d] > b[d]) meets = 0;
    }
    if (meets) {
      meets = 0;
      for (int z = a[2]; z <= b[2] && !meets; z++)
        for (int y = a[1]; y <= b[1] && !meets; y++)
          for (int x = a[0]; x <= b[0] && !meets; x++)
            if (occ[x + (int64_t)g_n[0] * (y + (int64_t)g_n[1] * z)]) meets = 1;
    }
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
