/*
 * pmmg_host.c — C host layer of the transfer step (see pmmg_host.h).
 * Product code: it calls only the HIP module's C-ABI; there is no CPU
 * fallback — a missing device makes every entry point return 0.
 */
#include "pmmg_host.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t pmmg_classify_points(const pmmg_new_group *g, uint8_t *pclass) {
  memset(pclass, PMMG_PT_SKIP, (size_t)g->np);
  int64_t n = 0;
  /* visitation loop of src/interpmesh_pmmg.c:535-550 */
  for (int64_t k = 0; k < g->ne; k++) {
    const int *v = g->tetv + 4 * k;
    if (v[0] <= 0) continue; /* !MG_EOK */
    for (int l = 0; l < 4; l++) {
      int ip = v[l];
      if (ip < 1 || ip > g->np) continue;
      if (pclass[ip - 1] != PMMG_PT_SKIP) continue; /* already classified */
      uint16_t tag = g->tag ? g->tag[ip - 1] : 0;
      if (tag >= PMMG_TAG_NUL) continue;  /* !MG_VOK */
      if (tag & PMMG_TAG_REQ) continue;   /* copied by PMMG_copyMetricsAndFields_point */
      pclass[ip - 1] = (tag & PMMG_TAG_BDY) ? PMMG_PT_BDY : PMMG_PT_VOL;
      n++;
    }
  }
  return n;
}

int pmmg_copy_required(const pmmg_old_group *old, const uint16_t *old_tag, pmmg_new_group *g,
                       const int *permNodGlob, int copy_met) {
  /* PMMG_copySol_point, src/interpmesh_pmmg.c:311-358 */
  for (int ip = 1; ip <= old->np; ip++) {
    uint16_t tag = old_tag[ip - 1];
    if (tag >= PMMG_TAG_NUL || !(tag & PMMG_TAG_REQ)) continue;
    int dst = permNodGlob ? permNodGlob[ip] : ip;
    if (dst < 1 || dst > g->np) continue;
    if (copy_met && old->met_size && g->met)
      memcpy(g->met + (size_t)old->met_size * (dst - 1), old->met + (size_t)old->met_size * (ip - 1),
             sizeof(double) * old->met_size);
    for (int j = 0; j < old->nfield; j++)
      memcpy(g->field[j] + (size_t)old->field_size[j] * (dst - 1),
             old->field[j] + (size_t)old->field_size[j] * (ip - 1), sizeof(double) * old->field_size[j]);
  }
  return 1;
}

int pmmg_set_constant_metric(int np, int met_size, double hsiz, double *met) {
  if (met_size == 1) {
    for (int i = 0; i < np; i++) met[i] = hsiz;
  } else if (met_size == 6) {
    double isq = 1.0 / (hsiz * hsiz);
    for (int i = 0; i < np; i++) {
      double *m = met + 6 * (size_t)i;
      m[0] = isq; m[1] = 0.0; m[2] = 0.0; m[3] = isq; m[4] = 0.0; m[5] = isq;
    }
  } else {
    return 0;
  }
  return 1;
}

static void stats_add(pmmg_hip_stats *a, const pmmg_hip_stats *b) {
  a->nvol += b->nvol; a->nbdy += b->nbdy;
  a->nvol_walk += b->nvol_walk; a->nvol_exhaust += b->nvol_exhaust; a->nvol_closest += b->nvol_closest;
  a->nbdy_face += b->nbdy_face; a->nbdy_edge += b->nbdy_edge; a->nbdy_vertex += b->nbdy_vertex;
  a->nbdy_wedge += b->nbdy_wedge; a->nbdy_cone += b->nbdy_cone; a->nbdy_exhaust += b->nbdy_exhaust;
  a->nbdy_stale += b->nbdy_stale; a->nbdy_closest += b->nbdy_closest;
  a->steps_total += b->steps_total;
  if (b->stepmax > a->stepmax) a->stepmax = b->stepmax;
  a->ms_prepare += b->ms_prepare; a->ms_sort += b->ms_sort; a->ms_vol += b->ms_vol; a->ms_bdy += b->ms_bdy;
  a->ms_fallback += b->ms_fallback; a->ms_total += b->ms_total;
}

int pmmg_interp_metrics_and_fields(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old, pmmg_new_group *grp,
                                   int input_met, double hsiz, pmmg_hip_stats *stats) {
  if (!ctx) {
    fprintf(stderr, "[parmmg_host] no HIP context: the transfer step has no CPU fallback\n");
    return 0;
  }
  if (stats) memset(stats, 0, sizeof(*stats));
  int ier = 1;
  for (int ig = 0; ig < ngrp; ig++) {
    const pmmg_old_group *o = &old[ig];
    pmmg_new_group *g = &grp[ig];
    /* ismet logic, src/interpmesh_pmmg.c:497-512 */
    int ismet = (input_met == 1) && o->met_size > 0;
    if (ismet && hsiz > 0.0) {
      if (!pmmg_set_constant_metric(g->np, o->met_size, hsiz, g->met)) { ier = 0; continue; }
      ismet = 0;
    }
    if (!ismet && o->nfield == 0) continue; /* nothing to do */
    uint8_t *pclass = (uint8_t *)malloc((size_t)g->np + 1);
    /* the module's HBM layout of the tetra: packed {v[4], adja[4]} records */
    int *tet8 = (int *)malloc(sizeof(int) * 8 * (size_t)(o->ne > 0 ? o->ne : 1));
    if (!pclass || !tet8) { free(pclass); free(tet8); ier = 0; continue; }
    for (int64_t k = 0; k < o->ne; k++) {
      memcpy(tet8 + 8 * k, o->tetv + 4 * k, 4 * sizeof(int));
      memcpy(tet8 + 8 * k + 4, o->adja + 4 * k, 4 * sizeof(int));
    }
    pmmg_classify_points(g, pclass);
    int ok = pmmg_hip_set_background_tet8(ctx, o->np, o->xyz, o->ne, tet8, o->nt, o->triv, o->adjt, o->hausd,
                                          PMMG_HIP_HOST) &&
             pmmg_hip_set_solutions(ctx, ismet ? o->met_size : 0, ismet ? o->met : NULL, o->nfield,
                                    o->field_size, o->field, PMMG_HIP_HOST);
    pmmg_hip_stats st;
    if (ok)
      ok = pmmg_hip_locate_interp(ctx, g->np, g->xyz, pclass, ismet ? g->met : NULL, g->field, g->elem, g->hit,
                                  &st, PMMG_HIP_HOST);
    if (ok && stats) stats_add(stats, &st);
    if (!ok) ier = 0;
    free(pclass);
    free(tet8);
  }
  return ier;
}
