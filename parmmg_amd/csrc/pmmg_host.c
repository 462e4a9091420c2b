/*
 * pmmg_host.c — C host layer of the transfer step (see pmmg_host.h).
 * Product code: it calls only the HIP module's C-ABI; there is no CPU
 * fallback — a missing device makes every entry point return 0.
 */
#define _GNU_SOURCE
#include "pmmg_host.h"
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ---------------------------------------------------------------- point classification
 * The visitation loop of src/interpmesh_pmmg.c:535-550 classifies every
 * vertex of a valid new tetra once: skipped if !MG_VOK or MG_REQ (copied by
 * PMMG_copyMetricsAndFields_point), surface if MG_BDY, volume otherwise.  The
 * class of a point depends only on its tags and on whether a valid tetra
 * references it, so the loop runs as two parallel passes: mark the
 * referenced points (every writer stores the same byte), then classify. */

typedef struct {
  const pmmg_new_group *g;
  uint8_t *pclass;
  int64_t k0, k1; /* tetra range (pass 1) / point range (pass 2) */
  int64_t count;
} cls_job;

static void *cls_mark(void *arg) {
  cls_job *J = (cls_job *)arg;
  const pmmg_new_group *g = J->g;
  for (int64_t k = J->k0; k < J->k1; k++) {
    const int *v = g->tetv + 4 * k;
    if (v[0] <= 0) continue; /* !MG_EOK */
    for (int l = 0; l < 4; l++)
      if (v[l] >= 1 && v[l] <= g->np) J->pclass[v[l] - 1] = 1;
  }
  return NULL;
}

static void *cls_assign(void *arg) {
  cls_job *J = (cls_job *)arg;
  const pmmg_new_group *g = J->g;
  int64_t n = 0;
  for (int64_t i = J->k0; i < J->k1; i++) {
    if (!J->pclass[i]) continue;
    uint16_t tag = g->tag ? g->tag[i] : 0;
    if (tag >= PMMG_TAG_NUL || (tag & PMMG_TAG_REQ)) {
      J->pclass[i] = PMMG_PT_SKIP;
      continue;
    }
    J->pclass[i] = (tag & PMMG_TAG_BDY) ? PMMG_PT_BDY : PMMG_PT_VOL;
    n++;
  }
  J->count = n;
  return NULL;
}

static int host_threads(void) {
  long n = sysconf(_SC_NPROCESSORS_ONLN);
  const char *e = getenv("PMMG_HOST_THREADS");
  if (e && atoi(e) > 0) n = atoi(e);
  if (n < 1) n = 1;
  if (n > 16) n = 16;
  return (int)n;
}

int64_t pmmg_classify_points(const pmmg_new_group *g, uint8_t *pclass) {
  memset(pclass, PMMG_PT_SKIP, (size_t)g->np);
  int nt = host_threads();
  cls_job J[16];
  pthread_t th[16];
  for (int pass = 0; pass < 2; pass++) {
    const int64_t n = pass == 0 ? (int64_t)g->ne : (int64_t)g->np;
    for (int t = 0; t < nt; t++) {
      J[t].g = g;
      J[t].pclass = pclass;
      J[t].k0 = n * t / nt;
      J[t].k1 = n * (t + 1) / nt;
      J[t].count = 0;
      if (pthread_create(&th[t], NULL, pass == 0 ? cls_mark : cls_assign, &J[t]) != 0) {
        (pass == 0 ? cls_mark : cls_assign)(&J[t]);
        th[t] = 0;
      }
    }
    for (int t = 0; t < nt; t++)
      if (th[t]) pthread_join(th[t], NULL);
  }
  int64_t total = 0;
  for (int t = 0; t < nt; t++) total += J[t].count;
  return total;
}

/* ---------------------------------------------------------------- frozen points */

static int copy_sol_point(const pmmg_old_group *old, int size, const double *src, double *dst, int np_new,
                          const int *perm) {
  /* PMMG_copySol_point, src/interpmesh_pmmg.c:311-358 */
  for (int ip = 1; ip <= old->np; ip++) {
    uint16_t tag = old->tag[ip - 1];
    if (tag >= PMMG_TAG_NUL) continue; /* !MG_VOK */
    if (!(tag & PMMG_TAG_REQ)) continue;
    int to = perm ? perm[ip] : ip;
    if (to < 1 || to > np_new) return 0;
    memcpy(dst + (size_t)size * (to - 1), src + (size_t)size * (ip - 1), sizeof(double) * (size_t)size);
  }
  return 1;
}

int pmmg_copy_metrics_and_fields_point(const pmmg_old_group *old, pmmg_new_group *g, const int *permNodGlob,
                                       int renum, int input_met) {
  if (!old || !g || !old->tag) return 0;
  /* no permutation array, or no renumbering: the same index (:321-337) */
  const int *perm = (renum && permNodGlob) ? permNodGlob : NULL;
  /* PMMG_copyMetrics_point, src/interpmesh_pmmg.c:373-383 */
  if (input_met == 1 && !(g->hsiz > 0.0) && old->met_size > 0) {
    if (!g->met || g->met_size != old->met_size) return 0;
    if (!copy_sol_point(old, old->met_size, old->met, g->met, g->np, perm)) return 0;
  }
  /* PMMG_copyFields_point, :397-415 */
  for (int j = 0; j < old->nfield; j++)
    if (!copy_sol_point(old, old->field_size[j], old->field[j], g->field[j], g->np, perm)) return 0;
  return 1;
}

int pmmg_set_constant_metric(pmmg_new_group *g) {
  /* MMG3D_Set_constantSize: met->size from info.ani; MMG5_Compute_constantSize
   * (Mmg @889d408, not in the reference tree: parity unpinned) rejects a
   * uniform size outside the user bounds ("Mismatched options: hmin ... is
   * greater than hsiz" / "hmax ... is lower than hsiz"), and
   * PMMG_interpMetricsAndFields_mesh then fails (src/interpmesh_pmmg.c:504);
   * MMG5_Set_constantSize: valid points only */
  const int size = g->ani ? 6 : 1;
  if (!g->met || g->met_size != size || !(g->hsiz > 0.0)) return 0;
  const double h = g->hsiz;
  if ((g->hmin > 0.0 && g->hmin > h) || (g->hmax > 0.0 && g->hmax < h)) {
    fprintf(stderr, "[parmmg_host] mismatched options: hmin (%e), hmax (%e), hsiz (%e)\n", g->hmin, g->hmax, h);
    return 0;
  }
  const double isq = 1.0 / (h * h);
  for (int i = 0; i < g->np; i++) {
    if (g->tag && g->tag[i] >= PMMG_TAG_NUL) continue; /* !MG_VOK */
    double *m = g->met + (size_t)size * i;
    if (size == 1) {
      m[0] = h;
    } else {
      m[0] = isq; m[1] = 0.0; m[2] = 0.0; m[3] = isq; m[4] = 0.0; m[5] = isq;
    }
  }
  return 1;
}

static void stats_add(pmmg_hip_stats *a, const pmmg_hip_stats *b) {
  a->nvol += b->nvol; a->nbdy += b->nbdy;
  a->nvol_walk += b->nvol_walk; a->nvol_exhaust += b->nvol_exhaust; a->nvol_closest += b->nvol_closest;
  a->nvol_exact += b->nvol_exact;
  a->nbdy_face += b->nbdy_face; a->nbdy_edge += b->nbdy_edge; a->nbdy_vertex += b->nbdy_vertex;
  a->nbdy_wedge += b->nbdy_wedge; a->nbdy_cone += b->nbdy_cone; a->nbdy_exhaust += b->nbdy_exhaust;
  a->nbdy_stale += b->nbdy_stale; a->nbdy_closest += b->nbdy_closest;
  a->steps_total += b->steps_total;
  a->wave_iters += b->wave_iters;
  if (b->stepmax > a->stepmax) a->stepmax = b->stepmax;
  a->ms_prepare += b->ms_prepare; a->ms_sort += b->ms_sort; a->ms_vol += b->ms_vol; a->ms_bdy += b->ms_bdy;
  a->ms_fallback += b->ms_fallback; a->ms_total += b->ms_total; a->ms_vol_locate += b->ms_vol_locate;
  a->nvol_noseed += b->nvol_noseed; a->nvol_stuck += b->nvol_stuck; a->nvol_limit += b->nvol_limit;
  a->seed_map_axes |= b->seed_map_axes;
  a->nbdy_fanscan += b->nbdy_fanscan;
}

static int interp_groups(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old, pmmg_new_group *grp, int input_met,
                         int keep, int carried, const int *const *src, pmmg_hip_stats *stats) {
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
    int ismet = 1;
    if (input_met != 1) {
      ismet = 0;
    } else if (g->hsiz > 0.0) {
      if (!pmmg_set_constant_metric(g)) {
        if (keep) pmmg_hip_carry_over(ctx, ig, 0, NULL);
        ier = 0;
        continue;
      }
      ismet = 0;
    }
    /* a group left out drops what was kept for it (its next old group is
     * not this call's output) */
    if (!ismet && o->nfield == 0) { /* nothing to do */
      if (keep) pmmg_hip_carry_over(ctx, ig, 0, NULL);
      continue;
    }
    if (ismet && (o->met_size == 0 || g->met_size != o->met_size || !g->met)) {
      if (keep) pmmg_hip_carry_over(ctx, ig, 0, NULL);
      ier = 0;
      continue;
    }
    uint8_t *pclass = (uint8_t *)malloc((size_t)g->np + 1);
    if (!pclass) { ier = 0; continue; }
    pmmg_classify_points(g, pclass);
    /* the previous iteration's new group ig, kept on the device: carried
     * unless nothing was kept for it (then it goes up whole) */
    if (carried && !pmmg_hip_carry_over(ctx, ig, o->np, src ? src[ig] : NULL))
      fprintf(stderr, "[parmmg_host] group %d: no carry-over (%s), uploading it\n", ig, pmmg_hip_last_error(ctx));
    /* the background: adjacency and boundary trias are built on the device
     * when the caller does not hand them over (set_background, adja / triv
     * NULL) */
    int ok = pmmg_hip_set_background(ctx, o->np, o->xyz, o->ne, o->tetv, o->adja, o->nt, o->triv, o->adjt,
                                     o->hausd, PMMG_HIP_HOST) &&
             pmmg_hip_set_solutions(ctx, ismet ? o->met_size : 0, ismet ? o->met : NULL, o->nfield,
                                    o->field_size, o->field, PMMG_HIP_HOST);
    pmmg_hip_stats st;
    if (ok)
      ok = pmmg_hip_locate_interp(ctx, g->np, g->xyz, pclass, ismet ? g->met : NULL, g->field, g->elem, g->hit,
                                  &st, PMMG_HIP_HOST);
    if (ok && stats) stats_add(stats, &st);
    if (ok && keep) ok = pmmg_hip_keep(ctx, ig);
    if (!ok && keep) pmmg_hip_carry_over(ctx, ig, 0, NULL);
    if (!ok) ier = 0;
    free(pclass);
  }
  return ier;
}

int pmmg_interp_metrics_and_fields(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old, pmmg_new_group *grp,
                                   int input_met, pmmg_hip_stats *stats) {
  return interp_groups(ctx, ngrp, old, grp, input_met, 0, 0, NULL, stats);
}

int pmmg_interp_metrics_and_fields_carry(pmmg_hip_ctx *ctx, int ngrp, const pmmg_old_group *old,
                                         pmmg_new_group *grp, int input_met, int carried, const int *const *src,
                                         pmmg_hip_stats *stats) {
  return interp_groups(ctx, ngrp, old, grp, input_met, 1, carried, src, stats);
}
