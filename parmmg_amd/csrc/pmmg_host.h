/*
 * pmmg_host.h — C host layer of the transfer step (product code).
 *
 * Mirrors PMMG_interpMetricsAndFields (reference src/interpmesh_pmmg.c:663-741)
 * over plain "group views" instead of MMG5 structs, so that the ParMmg shim
 * in INTEGRATION.md only has to fill these views from parmesh->listgrp /
 * parmesh->old_listgrp and call pmmg_interp_metrics_and_fields().  It
 *   - applies the ismet / hsiz logic (src/interpmesh_pmmg.c:497-512),
 *   - classifies new points in the reference's visitation loop
 *     (src/interpmesh_pmmg.c:535-550: invalid / MG_REQ skipped, MG_BDY to the
 *     surface path, the rest to the volume path),
 *   - copies the solutions of frozen (MG_REQ) points
 *     (PMMG_copyMetricsAndFields_point, src/interpmesh_pmmg.c:432-446),
 *   - and runs the HIP module (include/parmmg_hip.h) group by group.
 */
#ifndef PMMG_HOST_H
#define PMMG_HOST_H
#include <stdint.h>
#include "parmmg_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Mmg point tags used by the path (Mmg @889d408 src/common/libmmgtypes.h;
 * restated — a real shim uses Mmg's own macros). */
#define PMMG_TAG_REQ (1 << 2)  /* MG_REQ */
#define PMMG_TAG_BDY (1 << 4)  /* MG_BDY */
#define PMMG_TAG_NUL (1 << 14) /* MG_NUL: MG_VOK(p) == (p->tag < MG_NUL) */

/* The background group (parmesh->old_listgrp[igrp] after PMMG_update_oldGrps,
 * src/grpsplit_pmmg.c:1224).  Arrays in the "row r = entity r+1" layout. */
typedef struct {
  int np, ne, nt;
  const double *xyz;   /* 3*np (MMG5_Point.c packed) */
  const uint16_t *tag; /* np point tags (may be NULL: no MG_REQ copy) */
  const int *tetv;     /* 4*ne (MMG5_Tetra.v packed) */
  const int *adja;     /* 4*ne (= &mesh->adja[1]); NULL: built on the device (MMG3D_hashTetra's result) */
  const int *triv;     /* 3*nt (MMG5_Tria.v packed); NULL with nt < 0: the boundary faces are built on
                          the device (MMG5_chkBdryTria's single-material result) */
  const int *adjt;     /* 3*nt (= &mesh->adjt[1]); NULL: built on the device (MMG3D_hashTria) */
  double hausd;        /* oldMesh->info.hausd */
  int met_size;        /* oldMet->size (0 if no metric) */
  const double *met;   /* met_size*np */
  int nfield;          /* mesh->nsols */
  const int *field_size;
  const double *const *field;
} pmmg_old_group;

/* The adapted group (parmesh->listgrp[igrp]). */
typedef struct {
  int np, ne;
  const double *xyz;   /* 3*np */
  const uint16_t *tag; /* np, Mmg point tags */
  const int *tetv;     /* 4*ne, new tetra (MG_EOK: v[0] > 0) */
  int met_size;        /* rows of met (0 = no metric array, 1 or 6) */
  double *met;         /* met_size*np output */
  double *const *field;/* nfield outputs */
  int *elem;           /* optional np diagnostics */
  int8_t *hit;         /* optional np diagnostics */
  double hsiz;         /* mesh->info.hsiz (> 0: constant metric, not interpolated) */
  double hmin, hmax;   /* mesh->info.hmin / hmax: bounds of the constant size (<= 0: unset) */
  int ani;             /* mesh->info.ani: the constant metric is a tensor (met_size 6) */
} pmmg_new_group;

/* Classification of the reference loop: pclass[np] receives PMMG_PT_*.
 * Returns the number of points to locate. */
int64_t pmmg_classify_points(const pmmg_new_group *g, uint8_t *pclass);

/* PMMG_copyMetricsAndFields_point (src/interpmesh_pmmg.c:432-446) ->
 * PMMG_copySol_point (:311-358): the rows of the old group's valid MG_REQ
 * points are copied into the new group, at the same index when
 * `!renum || !permNodGlob`, else at permNodGlob[ip] (1-based, the SCOTCH
 * renumbering, src/libparmmg1.c:692-715).  The metric only when
 * input_met == 1 and hsiz <= 0 (PMMG_copyMetrics_point, :373-383); the
 * fields always.  Returns 1, or 0 on invalid arguments / a target out of
 * range. */
int pmmg_copy_metrics_and_fields_point(const pmmg_old_group *old, pmmg_new_group *g, const int *permNodGlob,
                                       int renum, int input_met);

/* MMG3D_Set_constantSize's fill (hsiz > 0 branch of the ismet logic,
 * src/interpmesh_pmmg.c:501-505), restated from Mmg @889d408 (unpinned):
 * MMG5_Compute_constantSize rejects hsiz outside [hmin, hmax] (bounds <= 0
 * are unset; "Mismatched options", the metric is left untouched), else every
 * valid point gets hsiz (iso, info.ani == 0) or diag(1/hsiz^2) (aniso).
 * g->met_size must be 6 when g->ani, else 1.  Returns 1, or 0 on a size
 * mismatch or mismatched options. */
int pmmg_set_constant_metric(pmmg_new_group *g);

/* PMMG_interpMetricsAndFields over ngrp groups.
 *   input_met   parmesh->info.inputMet (1 = the user provided a metric)
 * Returns 1 if every group succeeded, 0 otherwise (src/interpmesh_pmmg.c:689-741). */
int pmmg_interp_metrics_and_fields(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old, pmmg_new_group *grp,
                                   int input_met, pmmg_hip_stats *stats);

/* The same over the iterations of a run (src/libparmmg1.c:653: the adapted
 * groups become the next old groups): every group's new points and the rows
 * the step wrote stay on the device (pmmg_hip_keep, slot = group index), and
 * with carried = 1 old group ig IS the previous call's new group ig — its
 * vertex i+1 is that group's point src[ig][i] (1-based, 0: not carried, e.g.
 * moved in by load balancing; src or src[ig] NULL: the same numbering) — so
 * only its connectivity and the rows the device does not hold go up
 * (pmmg_hip_carry_over).  A group whose previous rows are not kept (it was
 * skipped, or its point count changed without a map) goes up whole.  The
 * kept rows must not have been modified on the host in between. */
int pmmg_interp_metrics_and_fields_carry(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old,
                                         pmmg_new_group *grp, int input_met, int carried, const int *const *src,
                                         pmmg_hip_stats *stats);

/* ---- halo shards of a background group (pmmg_shard.c) ----
 * All arrays in the "row r = entity r+1" layout of parmmg_hip.h. */

/* Largest bounding-box side over the tetra (halo unit). */
double pmmg_max_tet_extent(int np, const double *xyz, int ne, const int *tetv);

/* Marks the tetra whose bounding box meets [box_lo - halo, box_hi + halo]
 * (halo < 0: |halo| x pmmg_max_tet_extent) and their vertices:
 * tet_map[ne] / vert_map[np] receive the 1-based local id in the shard or 0
 * (ascending with the global id).  counts = {shard tetra, shard vertices}.
 * Returns 1, or 0 on invalid input. */
int pmmg_shard_mark(int np, const double *xyz, int ne, const int *tetv, const double box_lo[3],
                    const double box_hi[3], double halo, int *tet_map, int *vert_map, int64_t counts[2]);

/* The same, tighter: the tetra whose bounding box grown by the halo meets
 * both the range's box (box_lo/box_hi, may be NULL) and one of the grid
 * cells occ[g_n[0]*g_n[1]*g_n[2]] != 0 (cell (i,j,k) = g_lo + cell *
 * [i,i+1) x [j,j+1) x [k,k+1), x fastest) that hold the range's points.  A
 * Morton range's cells hug it; its box can hold half a shell. */
int pmmg_shard_mark_cells(int np, const double *xyz, int ne, const int *tetv, const double box_lo[3],
                          const double box_hi[3], const double g_lo[3], double cell, const int g_n[3],
                          const uint8_t *occ, double halo, int *tet_map, int *vert_map, int64_t counts[2]);

/* Writes the shard: s_xyz[3*nv], s_tetv/s_adja[4*nk] (neighbours outside the
 * shard -> 0), the boundary trias with all vertices in the shard
 * s_triv/s_adjt (room for nt rows) and the 1-based global ids of the local
 * tetra / vertices / trias (each optional).  Returns the shard's tria count,
 * or -1 on invalid input. */
int64_t pmmg_shard_fill(int np, const double *xyz, int ne, const int *tetv, const int *adja, int nt,
                        const int *triv, const int *adjt, const int *tet_map, const int *vert_map,
                        double *s_xyz, int *s_tetv, int *s_adja, int *s_triv, int *s_adjt, int *tet_gid,
                        int *vert_gid, int *tria_gid);

/* ---- halo shards built from the ranks' parts of a group (r05) --------------
 * The builders above read the whole group; a rank of a distributed group
 * holds only its part.  Each rank packs, for every destination rank, the
 * tetra, trias and vertex rows of its part that the destination's region
 * needs (pmmg_shard_part_pack), the ranks exchange the buffers (MPI /
 * RCCL all-to-all; bench and tests: torch.distributed), and each rank
 * assembles its shard from what it received (pmmg_shard_assemble).  The
 * shard is the one pmmg_shard_mark_cells + pmmg_shard_fill_region build
 * from the whole group: local ids ascend with the global ids, cut faces and
 * edges are walls. */

/* A destination's region: the tetra / trias whose bounding box grown by
 * `halo` meets the box (when box_lo) and a grid cell with occ != 0 (the
 * cells holding the destination's points, as pmmg_shard_mark_cells). */
typedef struct {
  const double *box_lo, *box_hi; /* 3 each, or NULL */
  double g_lo[3];
  double cell;
  int g_n[3];
  const uint8_t *occ;
  double halo; /* absolute, >= 0 */
} pmmg_shard_region;

/* A rank's part of a background group, global ids (1-based) ascending:
 * every vertex a part tetra or tria uses is a part vertex; tetv / triv hold
 * GLOBAL vertex ids, adja / adjt the group's codes (4 gk + i, 3 gt + i). */
typedef struct {
  int np, ne, nt, K;
  const int *vert_gid;  /* np */
  const double *xyz;    /* 3 np */
  const double *sol;    /* K np (solution rows: metric | fields), NULL when K == 0 */
  const int *tet_gid;   /* ne */
  const int *tetv;      /* 4 ne */
  const int *adja;      /* 4 ne */
  const int *tria_gid;  /* nt */
  const int *triv;      /* 3 nt */
  const int *adjt;      /* 3 nt (may be NULL) */
} pmmg_shard_part;

/* Trias of the whole group meeting the region: tria_map[nt] = 1-based local
 * id (ascending) or 0; returns their count, -1 on invalid input. */
int64_t pmmg_shard_mark_trias(int np, const double *xyz, int nt, const int *triv, const pmmg_shard_region *reg,
                              int *tria_map);

/* pmmg_shard_fill with the trias of tria_map (pmmg_shard_mark_trias) instead
 * of "all three vertices in the shard": the rule the part builders share. */
int64_t pmmg_shard_fill_region(int np, const double *xyz, int ne, const int *tetv, const int *adja, int nt,
                               const int *triv, const int *adjt, const int *tet_map, const int *vert_map,
                               const int *tria_map, double *s_xyz, int *s_tetv, int *s_adja, int *s_triv,
                               int *s_adjt, int *tet_gid, int *vert_gid, int *tria_gid);

/* The records of `part` the region needs, into buf (bytes; NULL or too small:
 * only sized).  Returns the bytes needed, or -1 on invalid input. */
int64_t pmmg_shard_part_pack(const pmmg_shard_part *part, const pmmg_shard_region *reg, void *buf, int64_t cap);

/* A shard from the buffers received from every rank (nbuf of them, lens
 * bytes each; K solution doubles per vertex, the same in every buffer).
 * counts[3] = {vertices, tetra, trias}; with xyz == NULL only counts are
 * computed.  Outputs as pmmg_shard_fill_region, plus the vertex rows
 * s_sol[K nv].  Returns 1, or 0 on inconsistent buffers. */
int pmmg_shard_assemble(int nbuf, const void *const *bufs, const int64_t *lens, int K, int64_t counts[3],
                        double *s_xyz, double *s_sol, int *s_tetv, int *s_adja, int *s_triv, int *s_adjt,
                        int *tet_gid, int *vert_gid, int *tria_gid);

#ifdef __cplusplus
}
#endif
#endif
