/*
 * pmmg_oracle.h — CPU restatement of ParMmg's old->new transfer step.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (parmmg_amd/, the
 * HIP module, the C host shim) may include, link or call this code; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as
 * the checker and as the CPU baseline.
 *
 * PARITY STATUS: the reference path cannot be built in this image (it needs
 * Mmg @889d408, absent and unfetchable; building it against stand-in headers
 * is not allowed), and the reference ships no value-level golden data for
 * this path.  This restatement is therefore checked
 * against analytic known answers derived from the reference's own fixtures
 * (libexamples/adaptation_example0) and documented algorithm — value-level
 * parity with the reference binary is UNPINNED, in particular at the Mmg
 * arithmetic boundary (MMG5_invmat, MMG5_orvol, MMG5_nonUnitNorPts,
 * MMG5_EPS, MMG5_idir), which is restated from Mmg's published source.
 *
 * Layouts follow include/parmmg_hip.h ("row r = entity r+1", 1-based ids
 * inside arrays).
 */
#ifndef PMMG_ORACLE_H
#define PMMG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mmg constants restated (Mmg src/common/mmgcommon.h @889d408): */
#define ORC_EPS   1.e-06   /* MMG5_EPS   */
#define ORC_EPSD2 1.0e-200 /* MMG5_EPSD2 */
#define ORC_UNSET (-1)     /* PMMG_UNSET, src/libparmmgtypes.h:236 */

typedef struct {
  int np, ne, nt;
  const double *xyz;   /* 3*np */
  const int *tetv;     /* 4*ne */
  const int *adja;     /* 4*ne */
  const int *triv;     /* 3*nt */
  const int *adjt;     /* 3*nt */
  double hausd;
  int met_size;        /* 0, 1 or 6 */
  const double *met;   /* met_size*np */
  int nfield;
  const int *field_size;
  const double *const *field;
} orc_background;

typedef struct {
  int np;
  const double *xyz;       /* 3*np */
  const uint8_t *pclass;   /* np: 0 skip, 1 volume, 2 boundary */
  int nvisit;              /* points in reference visitation order */
  const int *visit;        /* 1-based ids (new-tetra first-appearance order) */
} orc_queries;

typedef struct {
  double *met;             /* met_size*np, may be NULL */
  double *const *field;    /* nfield arrays, may be NULL */
  int *elem;               /* np, may be NULL */
  int8_t *hit;             /* np, PMMG_HIT_* codes, may be NULL */
  int8_t *loc;             /* np, local edge/vertex index, may be NULL */
  double *minbary;         /* np, smallest barycentric coordinate (volume), may be NULL */
  int *steps;              /* np, reference ppt->s (negative = exhaustive), may be NULL */
} orc_outputs;

/* ORC_MODE_FAITHFUL reproduces the reference's persistent point-flag state in
 * the cone test (src/locate_pmmg.c:219,248-249,319-322 and the nodeTrias
 * counts left in point.flag, :157,190); ORC_MODE_FRESH gives every query a
 * fresh visited state (what the GPU module implements). */
#define ORC_MODE_FAITHFUL 0
#define ORC_MODE_FRESH    1

/* Full sequential run in reference order (PMMG_interpMetricsAndFields_mesh,
 * src/interpmesh_pmmg.c:477-649), warm start from the previous point's
 * element.  Returns 1.  If `timing` is non-NULL, timing[0] = precompute
 * seconds, timing[1] = locate+interp seconds. */
int orc_interp_mesh(const orc_background *bg, const orc_queries *q, orc_outputs *out,
                    int mode, double *timing);

/* Same run, stopped once the locate+interp phase has used `budget_s` seconds
 * (checked every 256 visited points; budget_s <= 0: no limit).  Returns the
 * number of visit entries processed (CPU-baseline sampling in bench.py), or
 * -1 on failure. */
int orc_interp_mesh_budget(const orc_background *bg, const orc_queries *q, orc_outputs *out,
                           int mode, double budget_s, double *timing);

/* Threaded CPU baseline: the precompute's per-tetra stream split over
 * nthreads, then nthreads contiguous ranges of visit[] processed in parallel
 * (each as its own sequential reference run with warm start and private
 * visited flags, like one MPI rank per group), each stopping after budget_s
 * seconds (<= 0: none).  Returns the visit entries processed in total (the
 * ranges' prefixes), or -1.  timing[0] precompute, timing[1] locate wall. */
int orc_interp_mesh_mt(const orc_background *bg, const orc_queries *q, orc_outputs *out,
                       int mode, int nthreads, double budget_s, double *timing);

/* Re-evaluate one query in a given element / hit kind (as the GPU reports
 * it) with the reference arithmetic, writing the interpolated values into
 * met_row / field_rows (rows of the point, not whole arrays).  Used to check
 * parity class (iii).  Returns 1, or 0 for an unknown hit code. */
int orc_eval_in_element(const orc_background *bg, const double *x, int is_bdy,
                        int elem, int hit, int loc, double *met_row,
                        double *const *field_rows);

/* Acceptance tests of the reference (for checking GPU classes):
 * tetra: min barycentric coordinate of x in tetra k (sorted[0], src/barycoord_pmmg.c:300-310)
 * tria : 1 if PMMG_locatePointInTria would accept x in tria k (bary > -EPS and
 *        |normal distance| <= hausd), minbary returned through *mb. */
double orc_tetra_minbary(const orc_background *bg, int k, const double *x);
int orc_tria_accepts(const orc_background *bg, int k, const double *x, double *mb);
/* Brute force over all elements: lowest-index accepting tetra / tria (0 if
 * none); closest tetra by |bary_min|*vol, closest tria by centroid distance. */
int orc_first_accepting_tetra(const orc_background *bg, const double *x);
int orc_closest_tetra(const orc_background *bg, const double *x);
/* |bary_min| * vol of x in tetra k: the reference's closest-tetra metric
 * (locate_pmmg.c:453-458); exact ties are broken by evaluation order in the
 * reference (walk first, then index order) and by lowest index here. */
double orc_closest_value(const orc_background *bg, int k, const double *x);
int orc_first_accepting_tria(const orc_background *bg, const double *x);
int orc_closest_tria(const orc_background *bg, const double *x);
/* Fresh-state shadow tests (wedge returns 4 when x lies in the shadow wedge of
 * edge l of tria k, cone returns 1 when x lies in the shadow cone of local
 * vertex iloc of tria k). */
int orc_wedge_test(const orc_background *bg, int k, int l, const double *x);
int orc_cone_test(const orc_background *bg, int k, int iloc, const double *x);

/* Batch parity check (the contract of tests/parity.py::check) of a module's
 * outputs over n points (idx[0..n) 0-based point ids, or all np points when
 * idx is NULL and n == np), over nthreads threads.  ref_elem / ref_hit /
 * ref_minbary: a reference run's per-point outputs (class (i) identity; may
 * be NULL).  Returns 1 (report filled), 0 on invalid input. */
typedef struct {
  int64_t n;               /* points whose element was accepted and values evaluated */
  int64_t exact;           /* of those, every value bit-identical */
  int64_t class_i, class_i_same;
  int64_t accept_fail;     /* element not accepted by the reference's test for its hit kind */
  int64_t value_fail;      /* relative error above rel_tol (or not evaluable) */
  int64_t unprocessed;     /* pclass != 0 but no hit code */
  int64_t skipped_written; /* pclass == 0 but a hit code */
  int64_t first_fail;      /* first failing point (0-based) or -1 */
  double maxrel;
  int64_t hits[16];
} orc_check_report;

int orc_check_batch(const orc_background *bg, const double *xyz, const uint8_t *pclass, const int *idx, int64_t n,
                    const int *elem, const int8_t *hit, const double *met_out, const double *const *field_out,
                    const int *ref_elem, const int8_t *ref_hit, const double *ref_minbary, int nthreads,
                    double rel_tol, orc_check_report *rep);

/* MMG5_invmat restated; exposed for unit tests. */
int orc_invmat(const double *m, double *mi);

/* MMG3D_tetraQual(mesh, met, 1) as PMMG_tetraQual calls it
 * (src/quality_pmmg.c:720-733): qual[ne] = MMG5_caltet_iso (no aniso metric)
 * or MMG5_caltet_ani (metric averaged over the vertices) of every tetra
 * (0 for tetv rows with v[0] <= 0); returns MMG3D_ALPHAD * min.  Restated
 * from Mmg's published source (unpinned). */
double orc_tetra_qual(int np, const double *xyz, int ne, const int *tetv, int met_size, const double *met,
                      double *qual);

/* PMMG_computeWgt (src/metis_pmmg.c:280-300) of face ifac of the tetra with
 * vertices v[4] (1-based), and PMMG_computeWgt_mesh (:242-266): for every
 * used tetra with xt[k] != 0, qual[k] = sum over faces with ftag[4k+f] & tag
 * of the face weight (other tetra untouched). */
double orc_face_wgt(const double *xyz, const int *v, int ifac, int met_size, const double *met);
void orc_compute_wgt_mesh(int ne, const int *tetv, const int *xt, const uint16_t *ftag, const double *xyz,
                          int met_size, const double *met, int tag, double *qual);

#ifdef __cplusplus
}
#endif
#endif
