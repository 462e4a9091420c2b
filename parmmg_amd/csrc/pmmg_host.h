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

typedef struct {
  int np, ne, nt;
  const double *xyz;   /* 3*np */
  const int *tetv;     /* 4*ne */
  const int *adja;     /* 4*ne (= &mesh->adja[1]) */
  const int *triv;     /* 3*nt */
  const int *adjt;     /* 3*nt (= &mesh->adjt[1]) */
  double hausd;        /* oldMesh->info.hausd */
  int met_size;        /* oldMet->size (0 if no metric) */
  const double *met;   /* met_size*np */
  int nfield;          /* mesh->nsols */
  const int *field_size;
  const double *const *field;
} pmmg_old_group;

typedef struct {
  int np, ne;
  const double *xyz;   /* 3*np */
  const uint16_t *tag; /* np, Mmg point tags */
  const int *tetv;     /* 4*ne, new tetra (MG_EOK: v[0] > 0) */
  double *met;         /* met_size*np output (may be NULL when no metric) */
  double *const *field;/* nfield outputs */
  int *elem;           /* optional np diagnostics */
  int8_t *hit;         /* optional np diagnostics */
} pmmg_new_group;

/* Classification of the reference loop: pclass[np] receives PMMG_PT_*.
 * Returns the number of points to locate. */
int64_t pmmg_classify_points(const pmmg_new_group *g, uint8_t *pclass);

/* PMMG_copyMetricsAndFields_point (src/interpmesh_pmmg.c:432-446): copy the
 * solutions of MG_REQ points from the old group (optionally through
 * permNodGlob, 1-based).  Returns 1. */
int pmmg_copy_required(const pmmg_old_group *old, const uint16_t *old_tag, pmmg_new_group *g,
                       const int *permNodGlob, int copy_met);

/* MMG3D_Set_constantSize's fill (hsiz > 0 branch): iso -> hsiz,
 * aniso -> diag(1/hsiz^2).  Returns 1. */
int pmmg_set_constant_metric(int np, int met_size, double hsiz, double *met);

/* PMMG_interpMetricsAndFields over ngrp groups.
 *   input_met   parmesh->info.inputMet (1 = the user provided a metric)
 *   hsiz        mesh->info.hsiz (> 0: constant metric recomputed, not interpolated)
 * Returns 1 if every group succeeded, 0 otherwise (src/interpmesh_pmmg.c:689-741). */
int pmmg_interp_metrics_and_fields(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old, pmmg_new_group *grp,
                                   int input_met, double hsiz, pmmg_hip_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
