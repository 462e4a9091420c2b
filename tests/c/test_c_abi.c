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
 * must give bit-identical outputs.  Exit status 0 = pass.
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
    if (ctx) fixture_checks(ctx, fixtures);
    pmmg_hip_destroy(ctx);
    printf("test_c_abi: host-only and device checks %s\n", failures ? "FAILED" : "passed");
  }
  return failures ? 1 : 0;
}
