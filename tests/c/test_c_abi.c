/*
 * test_c_abi.c — the drop-in boundary exercised from C, the way the ParMmg
 * shim of INTEGRATION.md drives it: group views filled from packed arrays,
 * pmmg_interp_metrics_and_fields() (PMMG_interpMetricsAndFields,
 * src/interpmesh_pmmg.c:663-741) and pmmg_copy_metrics_and_fields_point()
 * (PMMG_copyMetricsAndFields_point, :432-446) called through the C-ABI of
 * include/parmmg_hip.h + pmmg_host.h, linked against libpmmg_hip.so and
 * libpmmg_host.so (no ctypes).  Meshes come from the synthetic generator
 * (pmmg_synth.c).
 *
 * Without a device the host-only entry points are checked and the module
 * must refuse to run (no CPU fallback); with a device, a two-group transfer
 * is checked against known answers (affine fields are reproduced by the P1
 * interpolation, a constant tensor by the inverse-tensor interpolation) and
 * the device-built background (adjacency / boundary trias not handed over)
 * must give bit-identical outputs, as must the many-groups call
 * (pmmg_hip_locate_interp_groups) and a second iteration carried over from
 * the device (pmmg_interp_metrics_and_fields_carry).  Exit status 0 = pass.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parmmg_hip.h"
#include "pmmg_host.h"
#include "pmmg_medit.h"
#include "pmmg_synth.h"

static int failures = 0;
#define CHECK(cond, ...)                                                 \
  do {                                                                   \
    if (!(cond)) {                                                       \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);               \
      fprintf(stderr, __VA_ARGS__);                                      \
      fprintf(stderr, "\n");                                             \
      failures++;                                                        \
    }                                                                    \
  } while (0)

typedef struct {
  int np, ne, nt;
  double *xyz;
  int *tetv, *adja, *triv, *adjt;
  uint8_t *isbdy;
} mesh;

static mesh make_mesh(int kind, int n, double jitter, uint64_t seed) {
  mesh m;
  int64_t c[3];
  synth_counts(kind, n, c);
  m.np = (int)c[0];
  m.ne = (int)c[1];
  m.nt = (int)c[2];
  m.xyz = malloc(sizeof(double) * 3 * m.np);
  m.isbdy = malloc(m.np);
  m.tetv = malloc(sizeof(int) * 4 * m.ne);
  m.adja = malloc(sizeof(int) * 4 * m.ne);
  m.triv = malloc(sizeof(int) * 3 * (m.nt + 1));
  m.adjt = malloc(sizeof(int) * 3 * (m.nt + 1));
  synth_vertices(kind, n, jitter, seed, m.xyz, m.isbdy);
  synth_tetra(kind, n, m.tetv, m.adja);
  synth_trias(m.ne, m.tetv, m.adja, m.triv, m.adjt);
  return m;
}

static void free_mesh(mesh *m) {
  free(m->xyz); free(m->isbdy); free(m->tetv); free(m->adja); free(m->triv); free(m->adjt);
}

/* 1 + 2x - 3y + z/2 (synth field 5) */
static double affine(const double *x) { return 1.0 + 2.0 * x[0] - 3.0 * x[1] + 0.5 * x[2]; }

static void host_only_checks(void) {
  /* classification (src/interpmesh_pmmg.c:535-550) */
  mesh nm = make_mesh(SYNTH_CUBE, 4, 0.1, 7);
  uint16_t *tag = calloc(nm.np, sizeof(uint16_t));
  for (int i = 0; i < nm.np; i++) tag[i] = nm.isbdy[i] ? PMMG_TAG_BDY : 0;
  tag[0] |= PMMG_TAG_REQ;
  tag[1] = PMMG_TAG_NUL;
  pmmg_new_group g = {0};
  g.np = nm.np;
  g.ne = nm.ne;
  g.xyz = nm.xyz;
  g.tag = tag;
  g.tetv = nm.tetv;
  uint8_t *pc = malloc(nm.np);
  int64_t nloc = pmmg_classify_points(&g, pc);
  int nv = 0, nb = 0;
  for (int i = 0; i < nm.np; i++) {
    nv += pc[i] == PMMG_PT_VOL;
    nb += pc[i] == PMMG_PT_BDY;
  }
  CHECK(pc[0] == PMMG_PT_SKIP && pc[1] == PMMG_PT_SKIP, "REQ / invalid points must be skipped");
  CHECK(nloc == nv + nb && nloc == nm.np - 2, "classified %lld of %d", (long long)nloc, nm.np);

  /* PMMG_copySol_point with and without the SCOTCH permutation */
  double om[6 * 10], nmet[6 * 12];
  uint16_t otag[10] = {0};
  for (int i = 0; i < 60; i++) om[i] = i + 1.0;
  otag[2] = PMMG_TAG_REQ;
  otag[7] = PMMG_TAG_REQ;
  pmmg_old_group o = {0};
  o.np = 10;
  o.tag = otag;
  o.met_size = 6;
  o.met = om;
  pmmg_new_group ng = {0};
  ng.np = 12;
  ng.met_size = 6;
  ng.met = nmet;
  int perm[11];
  for (int i = 0; i <= 10; i++) perm[i] = 12 - i;
  for (int i = 0; i < 72; i++) nmet[i] = -1.0;
  CHECK(pmmg_copy_metrics_and_fields_point(&o, &ng, perm, 0, 1) == 1, "copy (renum off)");
  CHECK(nmet[6 * 2] == om[6 * 2] && nmet[6 * 7 + 5] == om[6 * 7 + 5] && nmet[0] == -1.0, "copy at the same index");
  for (int i = 0; i < 72; i++) nmet[i] = -1.0;
  CHECK(pmmg_copy_metrics_and_fields_point(&o, &ng, perm, 1, 1) == 1, "copy (renum on)");
  /* old vertex 3 (row 2) -> new vertex perm[3] = 9 (row 8) */
  CHECK(nmet[6 * 8] == om[6 * 2] && nmet[6 * 2] == -1.0, "copy through permNodGlob");
  for (int i = 0; i < 72; i++) nmet[i] = -1.0;
  ng.hsiz = 0.1; /* constant size: the metric is not copied */
  CHECK(pmmg_copy_metrics_and_fields_point(&o, &ng, NULL, 1, 1) == 1 && nmet[12] == -1.0, "no metric copy with hsiz");

  /* no device context: no CPU fallback */
  pmmg_old_group og = {0};
  CHECK(pmmg_interp_metrics_and_fields(NULL, 1, &og, &g, 1, NULL) == 0, "a NULL context must fail");
  free(pc);
  free(tag);
  free_mesh(&nm);
}

typedef struct {
  mesh bg, nw;
  double *met, *fs, *fv, *ft;        /* background solutions */
  double *omet, *ofs, *ofv, *oft;    /* outputs */
  uint16_t *tag;
  int *elem;
  int8_t *hit;
} group;

static void make_group(group *G, int n_old, int n_new, uint64_t seed) {
  G->bg = make_mesh(SYNTH_CUBE, n_old, 0.0, 1);
  G->nw = make_mesh(SYNTH_CUBE, n_new, 0.2, seed);
  int np = G->bg.np, nq = G->nw.np;
  G->met = malloc(sizeof(double) * 6 * np);
  G->fs = malloc(sizeof(double) * np);
  G->fv = malloc(sizeof(double) * 3 * np);
  G->ft = malloc(sizeof(double) * 6 * np);
  synth_field(1, np, G->bg.xyz, G->met);
  synth_field(5, np, G->bg.xyz, G->fs);
  synth_field(6, np, G->bg.xyz, G->fv);
  synth_field(7, np, G->bg.xyz, G->ft);
  G->omet = malloc(sizeof(double) * 6 * nq);
  G->ofs = malloc(sizeof(double) * nq);
  G->ofv = malloc(sizeof(double) * 3 * nq);
  G->oft = malloc(sizeof(double) * 6 * nq);
  G->tag = calloc(nq, sizeof(uint16_t));
  G->elem = calloc(nq, sizeof(int));
  G->hit = calloc(nq, 1);
  for (int i = 0; i < nq; i++) G->tag[i] = (G->nw.isbdy[i] ? PMMG_TAG_BDY : 0) | (i % 13 == 0 ? PMMG_TAG_REQ : 0);
}

static void free_group(group *G) {
  free_mesh(&G->bg); free_mesh(&G->nw);
  free(G->met); free(G->fs); free(G->fv); free(G->ft); free(G->omet); free(G->ofs); free(G->ofv); free(G->oft);
  free(G->tag); free(G->elem); free(G->hit);
}

static int run(pmmg_hip_ctx *ctx, group *G, int ngrp, int device_built) {
  pmmg_old_group old[2];
  pmmg_new_group nw[2];
  static const int fsz[3] = {1, 3, 6};
  const double *fin[2][3];
  double *fout[2][3];
  for (int ig = 0; ig < ngrp; ig++) {
    group *g = &G[ig];
    memset(&old[ig], 0, sizeof(old[ig]));
    memset(&nw[ig], 0, sizeof(nw[ig]));
    fin[ig][0] = g->fs; fin[ig][1] = g->fv; fin[ig][2] = g->ft;
    fout[ig][0] = g->ofs; fout[ig][1] = g->ofv; fout[ig][2] = g->oft;
    for (size_t i = 0; i < (size_t)g->nw.np; i++) {
      for (int c = 0; c < 6; c++) g->omet[6 * i + c] = g->oft[6 * i + c] = NAN;
      g->ofs[i] = NAN;
      for (int c = 0; c < 3; c++) g->ofv[3 * i + c] = NAN;
    }
    old[ig].np = g->bg.np;
    old[ig].ne = g->bg.ne;
    old[ig].nt = device_built ? -1 : g->bg.nt;
    old[ig].xyz = g->bg.xyz;
    old[ig].tetv = g->bg.tetv;
    old[ig].adja = device_built ? NULL : g->bg.adja;
    old[ig].triv = device_built ? NULL : g->bg.triv;
    old[ig].adjt = device_built ? NULL : g->bg.adjt;
    old[ig].hausd = 0.01;
    old[ig].met_size = 6;
    old[ig].met = g->met;
    old[ig].nfield = 3;
    old[ig].field_size = fsz;
    old[ig].field = fin[ig];
    nw[ig].np = g->nw.np;
    nw[ig].ne = g->nw.ne;
    nw[ig].xyz = g->nw.xyz;
    nw[ig].tag = g->tag;
    nw[ig].tetv = g->nw.tetv;
    nw[ig].met_size = 6;
    nw[ig].met = g->omet;
    nw[ig].field = fout[ig];
    nw[ig].elem = g->elem;
    nw[ig].hit = g->hit;
    nw[ig].ani = 1;
  }
  pmmg_hip_stats st;
  return pmmg_interp_metrics_and_fields(ctx, ngrp, old, nw, 1, &st);
}

static void device_checks(pmmg_hip_ctx *ctx) {
  group G[2];
  make_group(&G[0], 6, 7, 11);
  make_group(&G[1], 8, 5, 12);
  CHECK(run(ctx, G, 2, 0) == 1, "transfer failed: %s", pmmg_hip_last_error(ctx));
  for (int ig = 0; ig < 2; ig++) {
    group *g = &G[ig];
    int nq = g->nw.np, bad = 0, processed = 0;
    for (int i = 0; i < nq; i++) {
      const int req = (g->tag[i] & PMMG_TAG_REQ) != 0;
      if (req) {
        bad += !isnan(g->ofs[i]) || g->hit[i] != 0;
        continue;
      }
      processed++;
      bad += g->hit[i] == 0 || g->elem[i] <= 0;
      if (!g->nw.isbdy[i]) bad += fabs(g->ofs[i] - affine(g->nw.xyz + 3 * i)) > 1e-12;
      bad += fabs(g->oft[6 * i + 0] - 4.0) > 1e-12 || fabs(g->oft[6 * i + 5] - 2.0) > 1e-12;
      for (int c = 0; c < 6; c++) bad += !isfinite(g->omet[6 * i + c]);
    }
    CHECK(bad == 0 && processed > 0, "group %d: %d wrong rows of %d", ig, bad, processed);
  }
  /* the device-built background gives bit-identical outputs */
  group H[2];
  make_group(&H[0], 6, 7, 11);
  make_group(&H[1], 8, 5, 12);
  CHECK(run(ctx, H, 2, 1) == 1, "transfer (device-built background) failed: %s", pmmg_hip_last_error(ctx));
  for (int ig = 0; ig < 2; ig++) {
    size_t nq = (size_t)G[ig].nw.np;
    CHECK(memcmp(G[ig].omet, H[ig].omet, 48 * nq) == 0 && memcmp(G[ig].oft, H[ig].oft, 48 * nq) == 0 &&
              memcmp(G[ig].elem, H[ig].elem, 4 * nq) == 0 && memcmp(G[ig].hit, H[ig].hit, nq) == 0,
          "group %d: device-built background differs", ig);
    free_group(&G[ig]);
    free_group(&H[ig]);
  }
}

/* device allocations of one check, freed together */
typedef struct {
  void *p[64];
  int n;
} dev_list;

static void *dev_up(pmmg_hip_ctx *ctx, dev_list *L, const void *src, size_t bytes) {
  void *d = pmmg_hip_malloc(ctx, (int64_t)bytes);
  if (d && src && !pmmg_hip_memcpy_h2d(ctx, d, src, (int64_t)bytes)) d = NULL;
  if (d && L->n < 64) L->p[L->n++] = d;
  return d;
}

static void dev_free(pmmg_hip_ctx *ctx, dev_list *L) {
  for (int i = 0; i < L->n; i++) pmmg_hip_free(ctx, L->p[i]);
  L->n = 0;
}

static double *nan_rows(size_t n) {
  double *a = malloc(sizeof(double) * n);
  for (size_t i = 0; i < n; i++) a[i] = NAN;
  return a;
}

/* pmmg_hip_locate_interp_groups: two groups in device memory, one call —
 * bit-identical to the host layer's one call per group */
static void groups_checks(pmmg_hip_ctx *ctx) {
  group G[2];
  make_group(&G[0], 6, 7, 21);
  make_group(&G[1], 5, 8, 22);
  CHECK(run(ctx, G, 2, 0) == 1, "host-layer transfer failed: %s", pmmg_hip_last_error(ctx));
  static const int fsz[3] = {1, 3, 6};
  dev_list L = {{0}, 0};
  pmmg_hip_group dg[2];
  const double *din[2][3];
  double *dout[2][3];
  for (int ig = 0; ig < 2; ig++) {
    group *g = &G[ig];
    const size_t ne = (size_t)g->bg.ne, nq = (size_t)g->nw.np;
    int *tet8 = malloc(sizeof(int) * 8 * ne);
    for (size_t k = 0; k < ne; k++) {
      memcpy(tet8 + 8 * k, g->bg.tetv + 4 * k, 16);
      memcpy(tet8 + 8 * k + 4, g->bg.adja + 4 * k, 16);
    }
    pmmg_new_group ng = {0};
    ng.np = g->nw.np;
    ng.ne = g->nw.ne;
    ng.xyz = g->nw.xyz;
    ng.tag = g->tag;
    ng.tetv = g->nw.tetv;
    uint8_t *pc = malloc(nq);
    pmmg_classify_points(&ng, pc);
    double *n6 = nan_rows(6 * nq), *n3 = nan_rows(3 * nq), *n1 = nan_rows(nq);
    int *z4 = calloc(nq, sizeof(int));
    din[ig][0] = dev_up(ctx, &L, g->fs, sizeof(double) * g->bg.np);
    din[ig][1] = dev_up(ctx, &L, g->fv, sizeof(double) * 3 * g->bg.np);
    din[ig][2] = dev_up(ctx, &L, g->ft, sizeof(double) * 6 * g->bg.np);
    dout[ig][0] = dev_up(ctx, &L, n1, sizeof(double) * nq);
    dout[ig][1] = dev_up(ctx, &L, n3, sizeof(double) * 3 * nq);
    dout[ig][2] = dev_up(ctx, &L, n6, sizeof(double) * 6 * nq);
    memset(&dg[ig], 0, sizeof(dg[ig]));
    dg[ig].np = g->bg.np;
    dg[ig].ne = g->bg.ne;
    dg[ig].nt = g->bg.nt;
    dg[ig].xyz = dev_up(ctx, &L, g->bg.xyz, sizeof(double) * 3 * g->bg.np);
    dg[ig].tet8 = dev_up(ctx, &L, tet8, sizeof(int) * 8 * ne);
    dg[ig].triv = dev_up(ctx, &L, g->bg.triv, sizeof(int) * 3 * g->bg.nt);
    dg[ig].adjt = dev_up(ctx, &L, g->bg.adjt, sizeof(int) * 3 * g->bg.nt);
    dg[ig].hausd = 0.01;
    dg[ig].met_size = 6;
    dg[ig].met = dev_up(ctx, &L, g->met, sizeof(double) * 6 * g->bg.np);
    dg[ig].nfield = 3;
    dg[ig].field_size = fsz;
    dg[ig].fields = din[ig];
    dg[ig].np_new = g->nw.np;
    dg[ig].xyz_new = dev_up(ctx, &L, g->nw.xyz, sizeof(double) * 3 * nq);
    dg[ig].pclass = dev_up(ctx, &L, pc, nq);
    dg[ig].met_out = dev_up(ctx, &L, n6, sizeof(double) * 6 * nq);
    dg[ig].fields_out = dout[ig];
    dg[ig].elem_out = dev_up(ctx, &L, z4, sizeof(int) * nq);
    dg[ig].hit_out = dev_up(ctx, &L, z4, nq);
    free(tet8); free(pc); free(n6); free(n3); free(n1); free(z4);
  }
  pmmg_hip_stats st;
  CHECK(pmmg_hip_locate_interp_groups(ctx, 2, dg, &st) == 1, "groups call failed: %s", pmmg_hip_last_error(ctx));
  for (int ig = 0; ig < 2; ig++) {
    group *g = &G[ig];
    const size_t nq = (size_t)g->nw.np;
    double *m = malloc(48 * nq), *fs = malloc(8 * nq), *fv = malloc(24 * nq), *ft = malloc(48 * nq);
    int *el = malloc(4 * nq);
    int8_t *ht = malloc(nq);
    pmmg_hip_memcpy_d2h(ctx, m, dg[ig].met_out, 48 * (int64_t)nq);
    pmmg_hip_memcpy_d2h(ctx, fs, dout[ig][0], 8 * (int64_t)nq);
    pmmg_hip_memcpy_d2h(ctx, fv, dout[ig][1], 24 * (int64_t)nq);
    pmmg_hip_memcpy_d2h(ctx, ft, dout[ig][2], 48 * (int64_t)nq);
    pmmg_hip_memcpy_d2h(ctx, el, dg[ig].elem_out, 4 * (int64_t)nq);
    pmmg_hip_memcpy_d2h(ctx, ht, dg[ig].hit_out, (int64_t)nq);
    /* NaN rows compare bit for bit: both sides start from the same NaN */
    CHECK(memcmp(m, g->omet, 48 * nq) == 0 && memcmp(fs, g->ofs, 8 * nq) == 0 && memcmp(fv, g->ofv, 24 * nq) == 0 &&
              memcmp(ft, g->oft, 48 * nq) == 0 && memcmp(el, g->elem, 4 * nq) == 0 && memcmp(ht, g->hit, nq) == 0,
          "group %d: the groups call differs from the host layer", ig);
    free(m); free(fs); free(fv); free(ft); free(el); free(ht);
  }
  dev_free(ctx, &L);
  free_group(&G[0]);
  free_group(&G[1]);
}

/* pmmg_interp_metrics_and_fields_carry: the second iteration fed from the
 * rows kept on the device equals a cold call on a fresh context, with fewer
 * bytes up */
static void carry_checks(pmmg_hip_ctx *ctx) {
  group G;
  make_group(&G, 6, 7, 31);
  static const int fsz[3] = {1, 3, 6};
  /* iteration 1: G.bg -> G.nw, kept */
  pmmg_old_group o1 = {0};
  pmmg_new_group n1 = {0};
  const double *fin1[3] = {G.fs, G.fv, G.ft};
  double *fout1[3] = {G.ofs, G.ofv, G.oft};
  const size_t nq = (size_t)G.nw.np;
  for (size_t i = 0; i < 6 * nq; i++) G.omet[i] = G.oft[i] = NAN;
  for (size_t i = 0; i < nq; i++) G.ofs[i] = NAN;
  for (size_t i = 0; i < 3 * nq; i++) G.ofv[i] = NAN;
  o1.np = G.bg.np; o1.ne = G.bg.ne; o1.nt = G.bg.nt; o1.xyz = G.bg.xyz; o1.tetv = G.bg.tetv; o1.adja = G.bg.adja;
  o1.triv = G.bg.triv; o1.adjt = G.bg.adjt; o1.hausd = 0.01; o1.met_size = 6; o1.met = G.met; o1.nfield = 3;
  o1.field_size = fsz; o1.field = fin1;
  n1.np = G.nw.np; n1.ne = G.nw.ne; n1.xyz = G.nw.xyz; n1.tag = G.tag; n1.tetv = G.nw.tetv; n1.met_size = 6;
  n1.met = G.omet; n1.field = fout1; n1.ani = 1;
  pmmg_hip_stats st;
  CHECK(pmmg_interp_metrics_and_fields_carry(ctx, 1, &o1, &n1, 1, 0, NULL, &st) == 1, "iteration 1: %s",
        pmmg_hip_last_error(ctx));
  /* the skipped (MG_REQ) rows as PMMG_copyMetricsAndFields_point fills them */
  for (size_t i = 0; i < nq; i++)
    if (G.tag[i] & PMMG_TAG_REQ) {
      for (int c = 0; c < 6; c++) G.omet[6 * i + c] = G.oft[6 * i + c] = 0.5 + c;
      G.ofs[i] = -1.0;
      for (int c = 0; c < 3; c++) G.ofv[3 * i + c] = 2.0;
    }
  /* iteration 2: old group = G.nw with those rows, new group = another lattice */
  mesh nx = make_mesh(SYNTH_CUBE, 5, 0.2, 33);
  const size_t nq2 = (size_t)nx.np;
  uint16_t *tag2 = calloc(nq2, sizeof(uint16_t));
  for (size_t i = 0; i < nq2; i++) tag2[i] = nx.isbdy[i] ? PMMG_TAG_BDY : 0;
  pmmg_old_group o2 = {0};
  const double *fin2[3] = {G.ofs, G.ofv, G.oft};
  o2.np = G.nw.np; o2.ne = G.nw.ne; o2.nt = -1; o2.xyz = G.nw.xyz; o2.tetv = G.nw.tetv; o2.hausd = 0.01;
  o2.met_size = 6; o2.met = G.omet; o2.nfield = 3; o2.field_size = fsz; o2.field = fin2;
  double *res[2][4];
  int64_t up[2];
  for (int pass = 0; pass < 2; pass++) { /* 0: carried, 1: cold on a fresh context */
    pmmg_hip_ctx *c = pass == 0 ? ctx : pmmg_hip_create(0, 0);
    res[pass][0] = nan_rows(6 * nq2); res[pass][1] = nan_rows(nq2); res[pass][2] = nan_rows(3 * nq2);
    res[pass][3] = nan_rows(6 * nq2);
    double *fo[3] = {res[pass][1], res[pass][2], res[pass][3]};
    pmmg_new_group n2 = {0};
    n2.np = nx.np; n2.ne = nx.ne; n2.xyz = nx.xyz; n2.tag = tag2; n2.tetv = nx.tetv; n2.met_size = 6;
    n2.met = res[pass][0]; n2.field = fo; n2.ani = 1;
    pmmg_hip_bytes_up(c, 1);
    const int ok = pass == 0 ? pmmg_interp_metrics_and_fields_carry(c, 1, &o2, &n2, 1, 1, NULL, &st)
                             : pmmg_interp_metrics_and_fields(c, 1, &o2, &n2, 1, &st);
    CHECK(ok == 1, "iteration 2 (%s): %s", pass == 0 ? "carried" : "cold", pmmg_hip_last_error(c));
    up[pass] = pmmg_hip_bytes_up(c, 0);
    if (pass == 1) pmmg_hip_destroy(c);
  }
  const size_t sz[4] = {48 * nq2, 8 * nq2, 24 * nq2, 48 * nq2};
  int same = 1;
  for (int a = 0; a < 4; a++) same = same && memcmp(res[0][a], res[1][a], sz[a]) == 0;
  CHECK(same, "the carried iteration differs from the cold one");
  const int64_t rows = (int64_t)nq * (24 + 48 + 8 + 24 + 48);
  CHECK(up[0] <= up[1] - rows / 2, "carried iteration uploaded %lld bytes, cold %lld", (long long)up[0],
        (long long)up[1]);
  printf("test_c_abi: carried iteration %lld bytes up, cold %lld\n", (long long)up[0], (long long)up[1]);
  for (int p = 0; p < 2; p++)
    for (int a = 0; a < 4; a++) free(res[p][a]);
  free(tag2);
  free_mesh(&nx);
  free_group(&G);
}

/* the reference's libexamples/adaptation_example0 cube read by the C Medit
 * reader (cube.mesh, cube-met.sol, cube-solphys.sol), transferred to its
 * tetra centroids (volume points: P1 values = mean of the 4 vertex values)
 * and to its own vertices as MG_BDY points (vertex hits: the vertex rows
 * copied bit for bit) */
static void fixture_checks(pmmg_hip_ctx *ctx, const char *dir) {
  char path[1024], err[256];
  pmmg_medit_mesh m;
  pmmg_medit_sol met, phys;
  snprintf(path, sizeof path, "%s/cube.mesh", dir);
  CHECK(pmmg_medit_read_mesh(path, &m, err, sizeof err) == 1, "%s", err);
  snprintf(path, sizeof path, "%s/cube-met.sol", dir);
  CHECK(pmmg_medit_read_sol(path, &met, err, sizeof err) == 1, "%s", err);
  snprintf(path, sizeof path, "%s/cube-solphys.sol", dir);
  CHECK(pmmg_medit_read_sol(path, &phys, err, sizeof err) == 1, "%s", err);
  if (failures) return;
  CHECK(met.nsol == 1 && met.size[0] == 1 && phys.nsol == 3 && met.np == m.np, "fixture solutions");
  const int nq = m.ne + m.np;
  double *xq = malloc(sizeof(double) * 3 * nq);
  uint16_t *tag = calloc(nq, sizeof(uint16_t));
  for (int k = 0; k < m.ne; k++)
    for (int d = 0; d < 3; d++) {
      double c = 0.0;
      for (int i = 0; i < 4; i++) c += m.xyz[3 * (m.tetv[4 * k + i] - 1) + d];
      xq[3 * k + d] = 0.25 * c;
    }
  memcpy(xq + 3 * m.ne, m.xyz, sizeof(double) * 3 * m.np);
  for (int i = 0; i < m.np; i++) tag[m.ne + i] = PMMG_TAG_BDY;
  /* new tetra (the reference visits the new points through them): centroid
   * k with faces of background tetra k, so every point appears */
  int *ntet = malloc(sizeof(int) * 8 * m.ne);
  for (int k = 0; k < m.ne; k++) {
    ntet[8 * k] = ntet[8 * k + 4] = k + 1;
    for (int i = 0; i < 3; i++) {
      ntet[8 * k + 1 + i] = m.ne + m.tetv[4 * k + i];
      ntet[8 * k + 5 + i] = m.ne + m.tetv[4 * k + 1 + i];
    }
  }
  double *omet = malloc(sizeof(double) * nq), *of[3];
  for (int j = 0; j < 3; j++) of[j] = malloc(sizeof(double) * phys.size[j] * nq);
  int *elem = calloc(nq, sizeof(int));
  int8_t *hit = calloc(nq, 1);
  pmmg_old_group o = {0};
  o.np = m.np;
  o.ne = m.ne;
  o.nt = -1; /* boundary trias built on the device */
  o.xyz = m.xyz;
  o.tetv = m.tetv;
  o.hausd = 0.01;
  o.met_size = 1;
  o.met = met.val[0];
  o.nfield = 3;
  o.field_size = phys.size;
  o.field = (const double *const *)phys.val;
  pmmg_new_group g = {0};
  g.np = nq;
  g.ne = 2 * m.ne;
  g.tetv = ntet;
  g.xyz = xq;
  g.tag = tag;
  g.met_size = 1;
  g.met = omet;
  g.field = of;
  g.elem = elem;
  g.hit = hit;
  pmmg_hip_stats st;
  CHECK(pmmg_interp_metrics_and_fields(ctx, 1, &o, &g, 1, &st) == 1, "fixture transfer: %s", pmmg_hip_last_error(ctx));
  int bad = 0;
  for (int k = 0; k < m.ne; k++) { /* centroids: P1 = mean of the vertex values */
    bad += (hit[k] & 15) != 1;
    bad += fabs(omet[k] - met.val[0][m.tetv[4 * k] - 1]) > 1e-12 * fabs(omet[k]); /* constant size */
    for (int j = 0; j < 2; j++)
      for (int c = 0; c < phys.size[j]; c++) {
        double mean = 0.0;
        for (int i = 0; i < 4; i++) mean += 0.25 * phys.val[j][phys.size[j] * (m.tetv[4 * k + i] - 1) + c];
        bad += fabs(of[j][phys.size[j] * k + c] - mean) > 1e-12 * (fabs(mean) + 1.0);
      }
    for (int c = 0; c < 6; c++) bad += !isfinite(of[2][6 * k + c]);
  }
  for (int i = 0; i < m.np; i++) { /* vertices: copied rows */
    const int q = m.ne + i;
    bad += (hit[q] & 15) != 6;
    bad += omet[q] != met.val[0][i];
    for (int j = 0; j < 3; j++)
      bad += memcmp(of[j] + phys.size[j] * q, phys.val[j] + phys.size[j] * i, sizeof(double) * phys.size[j]) != 0;
  }
  CHECK(bad == 0, "reference cube fixture: %d wrong values", bad);
  printf("test_c_abi: reference cube fixture (%d tetra, %d points) transferred, %d wrong values\n", m.ne, nq, bad);
  free(xq); free(tag); free(omet); free(elem); free(hit); free(ntet);
  for (int j = 0; j < 3; j++) free(of[j]);
  pmmg_medit_free_mesh(&m);
  pmmg_medit_free_sol(&met);
  pmmg_medit_free_sol(&phys);
}

int main(int argc, char **argv) {
  const char *fixtures = argc > 1 ? argv[1] : "tests/golden";
  host_only_checks();
  const int ndev = pmmg_hip_device_count();
  pmmg_hip_ctx *ctx = pmmg_hip_create(0, 0);
  if (ndev <= 0) {
    CHECK(ctx == NULL, "pmmg_hip_create must fail without a device");
    printf("test_c_abi: host-only checks %s; device part SKIPPED (no HIP device)\n", failures ? "FAILED" : "passed");
  } else {
    CHECK(ctx != NULL, "pmmg_hip_create(0) failed");
    if (ctx) device_checks(ctx);
    if (ctx) groups_checks(ctx);
    if (ctx) carry_checks(ctx);
    if (ctx) fixture_checks(ctx, fixtures);
    pmmg_hip_destroy(ctx);
    printf("test_c_abi: host-only and device checks %s\n", failures ? "FAILED" : "passed");
  }
  return failures ? 1 : 0;
}
