/*
 * parmmg_hip.h — C-ABI of the MI355X (gfx950) old->new mesh transfer module.
 *
 * This is the drop-in boundary for ParMmg's metric/field interpolation step.
 * It replaces, per group, the body of
 *
 *   int PMMG_interpMetricsAndFields(PMMG_pParMesh parmesh, int *permNodGlob)
 *       reference: src/interpmesh_pmmg.c:663-741, prototype src/parmmg.h:472,
 *       called once per remeshing iteration from src/libparmmg1.c:829
 *
 * and, below it, the static per-group worker
 *
 *   PMMG_interpMetricsAndFields_mesh(...)      src/interpmesh_pmmg.c:477-649
 *
 * together with everything it reaches: PMMG_locatePointVol / _Bdy
 * (src/locate_pmmg.c:786-883, :587-723), the barycentric evaluation
 * (src/barycoord_pmmg.c) and the interpolators bound through the
 * PMMG_interp{2,3,4}bar function pointers (src/parmmgexterns.c:4-6,
 * bound by PMMG_setfunc src/libparmmg_tools.c:595-612).
 *
 * Conventions (all entry points):
 *  - Plain pointers and sizes only; no torch or HIP types in signatures.
 *  - Return 1 on success, 0 on failure: the internal ParMmg convention of
 *    PMMG_interpMetricsAndFields (NOT the public PMMG_SUCCESS=0 convention).
 *  - Arrays are "row r = entity r+1": ParMmg entities are 1-based, entry 0 is
 *    unused.  A host shim passes e.g. `met->m + met->size` for the metric and
 *    `mesh->adja + 1` for the tetra adjacency, so no copy is needed for those.
 *  - Entity ids stored INSIDE arrays keep the reference encoding: vertex ids
 *    in tetv/triv are 1-based, adja holds 4*k'+i' (0 = boundary face,
 *    src/locate_pmmg.c:821), adjt holds 3*k'+i' (0 = surface border,
 *    src/locate_pmmg.c:635).
 *  - `where` = PMMG_HIP_HOST: pointers are host memory, calls copy (through
 *    pinned staging buffers of the context) and are synchronous.  `where` = PMMG_HIP_DEVICE: pointers are device memory on
 *    the context's device; set_* calls only record the pointers (no copy) and
 *    pmmg_hip_locate_interp only enqueues work on the context's streams (no
 *    host synchronisation inside the call: every decision — query order,
 *    fallback launches — is taken on the device); use pmmg_hip_sync before
 *    reading results or stats.
 *  - The module is reentrant per context (the reference is not: it uses
 *    static warning flags and global function pointers).
 */
#ifndef PARMMG_HIP_H
#define PARMMG_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PMMG_HIP_HOST   0
#define PMMG_HIP_DEVICE 1

/* Per-point classification supplied by the caller (the host shim derives it
 * from Mmg tags in the reference's visitation loop, src/interpmesh_pmmg.c:535-550). */
#define PMMG_PT_SKIP 0   /* invalid, MG_REQ (copied by PMMG_copyMetricsAndFields_point) or unreferenced */
#define PMMG_PT_VOL  1   /* volume point   -> PMMG_locatePointVol path */
#define PMMG_PT_BDY  2   /* MG_BDY point   -> PMMG_locatePointBdy path */

/* Located-element kind written to hit_out (diagnostics + parity checking). */
#define PMMG_HIT_NONE         0  /* not processed (PMMG_PT_SKIP) */
#define PMMG_HIT_VOL_WALK     1  /* adjacency walk accepted the tetra          locate_pmmg.c:814-815 */
#define PMMG_HIT_VOL_EXHAUST  2  /* exhaustive scan: lowest-index accepted      locate_pmmg.c:743-762 */
#define PMMG_HIT_VOL_CLOSEST  3  /* not located: closest tetra, nearest vertex  locate_pmmg.c:764-767 */
#define PMMG_HIT_BDY_FACE     4  /* tria walk accepted, interior of the tria    locate_pmmg.c:624-627 */
#define PMMG_HIT_BDY_EDGE     5  /* tria walk accepted, on an edge (isBorder)   barycoord_pmmg.c:109-120 */
#define PMMG_HIT_BDY_VERTEX   6  /* tria walk accepted, at a vertex (isBorder)  barycoord_pmmg.c:109-120 */
#define PMMG_HIT_BDY_WEDGE    7  /* edge shadow wedge                           locate_pmmg.c:643-649 */
#define PMMG_HIT_BDY_CONE     8  /* vertex shadow cone                          locate_pmmg.c:651-657 */
#define PMMG_HIT_BDY_EXHAUST  9  /* exhaustive tria scan: lowest-index accepted locate_pmmg.c:483-503 */
#define PMMG_HIT_BDY_STALE   10  /* not located, re-evaluation accepted         locate_pmmg.c:505-509 */
#define PMMG_HIT_BDY_CLOSEST 11  /* not located: closest tria, nearest vertex   locate_pmmg.c:511,681 */

#define PMMG_HIT_CODE(h) ((h) & 15)
#define PMMG_HIT_LOC(h)  (((h) >> 4) & 3)

typedef struct pmmg_hip_ctx pmmg_hip_ctx;

/* Counters of one pmmg_hip_locate_interp call (the reference's debug-only
 * PMMG_locateStats, src/locate_pmmg.h:45-50, plus per-phase device times). */
typedef struct {
  int64_t nvol;          /* volume queries */
  int64_t nbdy;          /* surface queries */
  int64_t nvol_walk, nvol_exhaust, nvol_closest;
  int64_t nvol_exact;    /* volume queries the fp32 filter walk handed to the exact (fp64) walk */
  int64_t nbdy_face, nbdy_edge, nbdy_vertex, nbdy_wedge, nbdy_cone;
  int64_t nbdy_exhaust, nbdy_stale, nbdy_closest;
  int64_t steps_total;   /* walk steps, volume + surface */
  int64_t stepmax;
  int64_t wave_iters;    /* sum over wavefronts of their longest walk (lockstep cost; steps_total /
                            (64 * wave_iters) = lockstep efficiency) */
  int64_t sorted;        /* 1 if the queries were Morton-binned, 0 if processed in input order */
  /* device time in milliseconds, measured with HIP events on the context stream */
  float ms_prepare;      /* bbox, seed grids, input-order coherence test */
  float ms_sort;         /* query order: Morton binning, or stable class compaction */
  float ms_vol;          /* volume locate + interpolate kernels */
  float ms_bdy;          /* surface branch: locate + interpolate, its exhaustive / closest kernels */
  float ms_fallback;     /* exhaustive / closest kernels of the volume queries */
  float ms_total;        /* whole call, first to last event */
  float ms_vol_locate;   /* the volume walk kernel alone (part of ms_vol) */
  int64_t nvol_noseed;   /* volume queries with no seed within 6 seed-grid cells: walked from the lowest
                            in-use tetra the grid sampled */
  int64_t nvol_stuck;    /* exact volume walks stuck (no eligible neighbour) -> exhaustive */
  int64_t nvol_limit;    /* exact volume walks stopped at maxstep -> exhaustive */
  int64_t seed_map_axes; /* bit d: axis d of the volume seed grid followed the vertex quantiles */
  int64_t nbdy_fanscan;  /* surface queries whose cone test scanned every tria for a vertex's ball (its fan
                            open, non-manifold or longer than 64: e.g. at a halo shard's cut) */
  int64_t reserved[6];   /* zero; room for later counters without changing the struct's size */
} pmmg_hip_stats;

/* ABI of this header (r06): a shim built against it checks, once at load,
 *     pmmg_hip_abi_version() == PMMG_HIP_ABI_VERSION
 *     pmmg_hip_stats_size()  == sizeof(pmmg_hip_stats)
 * and refuses a library that differs: the library writes a whole
 * pmmg_hip_stats into the caller's struct (round 5 appended nbdy_fanscan, so a
 * shim built against the round-4 header would have been overrun by 8 bytes). */
#define PMMG_HIP_ABI_VERSION 6
int pmmg_hip_abi_version(void);
int64_t pmmg_hip_stats_size(void);

/* Options (bit flags) for pmmg_hip_create.  Default: Morton-bin the queries
 * unless a sampled test on the device finds the input numbering already
 * spatially coherent (3 in 4 consecutive points closer than 4 mean
 * spacings), and groups of fewer than 2^20 new points keep their input order. */
#define PMMG_HIP_OPT_NOSORT 1   /* always process queries in input order */
#define PMMG_HIP_OPT_SORT   2   /* always Morton-bin the queries */

/* Create a context on HIP device `device`.  Returns NULL on failure. */
pmmg_hip_ctx *pmmg_hip_create(int device, int options);
void pmmg_hip_destroy(pmmg_hip_ctx *ctx);

/* Background (pre-remesh) mesh of one group: the reference's oldMesh after
 * PMMG_update_oldGrps (src/grpsplit_pmmg.c:1224).
 *   np    vertices, xyz[3*np]        (MMG5_Point.c, packed)
 *   ne    tetrahedra, tetv[4*ne]     (MMG5_Tetra.v, packed), adja[4*ne] (= &mesh->adja[1])
 *   nt    boundary trias, triv[3*nt] (MMG5_Tria.v, packed),  adjt[3*nt] (= &mesh->adjt[1])
 *   hausd surface distance tolerance (oldMesh->info.hausd, src/locate_pmmg.c:253,315,363)
 * What PMMG_create_oldGrp derives from the connectivity (src/grpsplit_pmmg.c:
 * 350-415) may instead be built on the device:
 *   adja == NULL            the tetra adjacency (MMG3D_hashTetra's result)
 *   triv == NULL, nt < 0    the boundary trias, in (tetra, face) order oriented
 *                           by MMG5_idir, and their adjacency (MMG5_chkBdryTria
 *                           + MMG3D_hashTria for a single-material old mesh
 *                           without input trias)
 *   adjt == NULL, triv set  the tria adjacency (MMG3D_hashTria)
 * In host mode this also spares the PCIe upload of those arrays (the
 * adjacency is as large as the connectivity).  nt may be 0 (then no
 * PMMG_PT_BDY query may be submitted). */
int pmmg_hip_set_background(pmmg_hip_ctx *ctx, int np, const double *xyz,
                            int ne, const int *tetv, const int *adja,
                            int nt, const int *triv, const int *adjt,
                            double hausd, int where);

/* Same background with the tetrahedra as packed 32-byte records
 *   tet8[8*ne] = {v0, v1, v2, v3, adja0, adja1, adja2, adja3} per tetra
 * (MMG5_Tetra.v followed by the tetra's 4 adja codes 4*k+i).  This is the
 * module's preferred HBM layout: a walk step reads one record (one cache
 * line) instead of a tetv row plus an adja row.  A host shim builds it in the
 * same pass that packs MMG5_Tetra.v.  In device mode tet8
 * must be 16-byte aligned. */
int pmmg_hip_set_background_tet8(pmmg_hip_ctx *ctx, int np, const double *xyz,
                                 int ne, const int *tet8,
                                 int nt, const int *triv, const int *adjt,
                                 double hausd, int where);

/* Background solutions: the metric (met_size 0 = none, 1 = iso, 6 = aniso,
 * storage m11,m12,m13,m22,m23,m33 as MMG5 stores it) and nfield fields of
 * size field_size[j] (1, 3 or 6; size 6 fields use the inverse-tensor
 * interpolation, src/interpmesh_pmmg.c:582-593,623-634).
 * met[met_size*np], fields[j][field_size[j]*np] (= sol->m + sol->size).
 * Device-mode size-6 arrays must be 16-byte aligned. */
int pmmg_hip_set_solutions(pmmg_hip_ctx *ctx, int met_size, const double *met,
                           int nfield, const int *field_size,
                           const double *const *fields, int where);

/* Locate every new point with pclass != PMMG_PT_SKIP and interpolate the
 * metric and fields into it.
 *   np_new         new-mesh vertices; xyz_new[3*np_new], pclass[np_new]
 *   met_out        [met_size*np_new] (may be NULL iff met_size == 0)
 *   fields_out[j]  [field_size[j]*np_new]
 *   elem_out       [np_new] located tetra/tria id (1-based), may be NULL
 *   hit_out        [np_new] PMMG_HIT_* code in bits 0-3; for EDGE / WEDGE the
 *                  local edge, for VERTEX / CONE the local vertex of the tria
 *                  in bits 4-5 (PMMG_HIT_CODE / PMMG_HIT_LOC); may be NULL
 *   stats          may be NULL (with PMMG_HIP_DEVICE it is filled at pmmg_hip_sync)
 * Rows of points that are skipped, and rows whose tensor inversion fails
 * (MMG5_invmat, src/interpmesh_pmmg.c:258-267), are left untouched, as in the
 * reference. */
int pmmg_hip_locate_interp(pmmg_hip_ctx *ctx, int np_new, const double *xyz_new,
                           const uint8_t *pclass, double *met_out,
                           double *const *fields_out, int *elem_out,
                           int8_t *hit_out, pmmg_hip_stats *stats, int where);

/* Wait for all work queued on the context (groups calls included); fills the
 * stats of the last PMMG_HIP_DEVICE pmmg_hip_locate_interp call.  Returns 1/0. */
int pmmg_hip_sync(pmmg_hip_ctx *ctx, pmmg_hip_stats *stats);

/* ---- Carry-over of the new mesh into the next iteration ----------------------
 * ParMmg's next iteration takes the adapted group as its old group
 * (src/libparmmg1.c:653 -> PMMG_update_oldGrps, src/grpsplit_pmmg.c:1224-1248):
 * its vertices are the points this step located and its solutions the rows
 * this step wrote.  After a PMMG_HIP_HOST pmmg_hip_locate_interp they are
 * still in HBM:
 *   pmmg_hip_keep(ctx, slot)    keeps that call's new points and written rows
 *                               in `slot` (0..1023; no copy)
 *   pmmg_hip_carry_over(ctx, slot, np, src)
 *                               arms the next PMMG_HIP_HOST set_background +
 *                               set_solutions: vertex i+1 of the new background
 *                               is kept point src[i] (1-based; NULL: the
 *                               identity, np = the kept count).  Those calls
 *                               still take the full host arrays, but upload
 *                               only the vertices with src[i] == 0 (moved in,
 *                               e.g. by load balancing) and the solution rows
 *                               the step did not write (skipped points, whose
 *                               values the caller copies on the host, and
 *                               MMG5_invmat failures); a metric / field whose
 *                               size differs from the kept one goes up whole.
 * pmmg_hip_carry_over(ctx, slot, 0, NULL) drops the slot and frees its device
 * buffers.  A carry consumes its slot (keep again for the next iteration);
 * any failure of the armed set_background / set_solutions disarms it, and an
 * armed carry rejects pmmg_hip_set_solutions_packed and PMMG_HIP_DEVICE
 * calls.  The kept rows must not have been changed on the host in between;
 * the connectivity always comes from the host.  Both return 1/0. */
int pmmg_hip_keep(pmmg_hip_ctx *ctx, int slot);
int pmmg_hip_carry_over(pmmg_hip_ctx *ctx, int slot, int np, const int *src);

/* Host -> device bytes moved by host-mode calls since the last reset. */
int64_t pmmg_hip_bytes_up(pmmg_hip_ctx *ctx, int reset);

/* Free the context's reusable scratch: the snapshot builders' buckets (12 B x
 * 4 x ne for the adjacency: ~4.8 GB at 101M tetra), the Morton binning's
 * second key / value arrays and digit tables, and the group lanes (contexts
 * of their own, re-created by the next groups call).  The next call that
 * needs any of them allocates it again.  Waits for the context's work first.
 * The background, solutions, kept slots and seed grids stay.  Returns 1/0. */
int pmmg_hip_release_scratch(pmmg_hip_ctx *ctx);

/* ---- Many groups in one call ------------------------------------------------
 * ParMmg transfers group by group (the loop of src/interpmesh_pmmg.c:690 over
 * up to PMMG_REMESHER_NGRPS_MAX = 100 groups per rank, src/parmmg.h:212);
 * a group of a few hundred thousand points is launch-bound on one stream.  One
 * group: the arguments of pmmg_hip_set_background(_tet8) +
 * pmmg_hip_set_solutions + pmmg_hip_locate_interp, all PMMG_HIP_DEVICE
 * pointers (same alignment rules). */
typedef struct {
  /* background (old group): tet8 != NULL selects packed records, else tetv +
   * adja (adja NULL: adjacency built on the device, which synchronises); nt <
   * 0 with triv NULL: boundary trias built on the device (synchronises) */
  int np, ne, nt;
  const double *xyz;
  const int *tet8;
  const int *tetv, *adja;
  const int *triv, *adjt;
  double hausd;
  /* solutions at the background vertices */
  int met_size;
  const double *met;
  int nfield;
  const int *field_size;
  const double *const *fields;
  /* the new group's points and outputs */
  int np_new;
  const double *xyz_new;
  const uint8_t *pclass;
  double *met_out;
  double *const *fields_out;
  int *elem_out;
  int8_t *hit_out;
} pmmg_hip_group;

/* Enqueue the transfer of ngroup groups: group i runs on lane i % L of the
 * context (L = ceil(ngroup / rounds), rounds = ceil(ngroup / Lmax), Lmax =
 * PMMG_HIP_GROUP_LANES, default 5: every lane gets the same number of groups
 * give or take one, in the fewest rounds; a lane is a
 * pair of streams with its own work buffers, so the groups of different lanes
 * overlap on the device).  stats == NULL: the call only enqueues (nothing is
 * read back; use pmmg_hip_sync before reading outputs).  stats != NULL: the
 * call waits after each round of L groups and returns the counters summed
 * over all groups (ms_* summed as well, stepmax the largest, sorted the
 * number of groups whose queries were Morton-binned).  Results are identical to one
 * pmmg_hip_locate_interp per group.  The lanes are contexts of their own
 * (lane 0 enqueues on ctx's streams): ctx's background, solutions and armed
 * carry-over are left as they were.  Returns 1 if every group was enqueued
 * (and, with stats, completed), 0 at the first invalid group (the error names
 * its index; groups before it are enqueued). */
int pmmg_hip_locate_interp_groups(pmmg_hip_ctx *ctx, int ngroup, const pmmg_hip_group *groups,
                                  pmmg_hip_stats *stats);

/* ---- Background snapshot on the device -------------------------------------
 * ParMmg rebuilds the background's derived arrays on the host every
 * iteration: PMMG_create_oldGrp (src/grpsplit_pmmg.c:207-418) copies the
 * adjacency computed by MMG3D_hashTetra (src/libparmmg1.c:495,730), rebuilds
 * the boundary trias (MMG5_chkBdryTria, :404) and hashes the tria adjacency
 * (MMG3D_hashTria, :410).  These two entry points build the same arrays on
 * the device from the connectivity, so the arrays pmmg_hip_set_background*
 * consumes never take a host round trip.  All pointers are device memory on
 * the context's device, 16-byte aligned; calls are synchronous. */

/* Tetra adjacency of a conforming mesh from tetv[4*ne] (1-based vertex ids):
 *   adja[4*ne]  (may be NULL)  4*k'+i' of the tetra sharing face i, 0 on the boundary
 *   tet8[8*ne]  (may be NULL)  packed {v[4], adja[4]} records (set_background_tet8)
 * Returns 0 (message in pmmg_hip_last_error) for ids outside [1, np], repeated
 * ids in a tetra, or a face shared by more than two tetra. */
int pmmg_hip_build_adjacency(pmmg_hip_ctx *ctx, int np, int ne, const int *tetv,
                             int *adja, int *tet8);

/* Boundary trias: the faces with no neighbour — and, when tref[ne] (the
 * tetra references, MMG5_Tetra.ref) is given, the faces towards a neighbour
 * of smaller reference (MMG5_chkBdryTria's rule for a multi-material old mesh,
 * restated from Mmg @889d408: unpinned) — in (tetra, face) order, with
 * vertices v[MMG5_idir[i]] (outward for positively oriented tetra), and their
 * adjacency adjt[3*nt] (3*t'+j' across edge j, 0 on borders and on edges of
 * more than two trias).  Tetra from tet8 (packed records) when non-NULL, else
 * from tetv + adja.  *nt receives the number of trias; when it exceeds `cap`
 * nothing is written and 0 is returned.  tref and adjt may be NULL. */
int pmmg_hip_build_boundary(pmmg_hip_ctx *ctx, int np, int ne, const int *tet8,
                            const int *tetv, const int *adja, const int *tref,
                            int cap, int *nt, int *triv, int *adjt);

/* Element quality in the interpolated metric:
 * replaces MMG3D_tetraQual(mesh, met, 1) inside PMMG_tetraQual
 * (src/quality_pmmg.c:720-733, called at src/libparmmg1.c:845).  Device
 * pointers (the metric where pmmg_hip_locate_interp wrote it), synchronous:
 *   qual[ne]   pt->qual of every tetra (Mmg's unscaled caltet value; 0 for
 *              unused tetra, tetv row with v[0] <= 0)
 *   *minqual   MMG3D_ALPHAD * min over used tetra (2 when none is used)
 * met_size 0/1: geometric quality (MMG5_caltet_iso); 6: MMG5_caltet_ani with
 * the metric averaged over the 4 vertices.  As in the reference, a caller
 * treats *minqual == 0 as the "Quality computation problem" failure.
 * Returns 1, or 0 on invalid arguments. */
int pmmg_hip_tetra_qual(pmmg_hip_ctx *ctx, int np, const double *xyz, int ne,
                        const int *tetv, int met_size, const double *met,
                        double *qual, double *minqual);

/* Solutions as packed per-vertex records: rec[RS*np], vertex v's record at
 * rec + RS*(v-1) = [metric (met_size) | field 0 | field 1 | ...] with
 * RS = (met_size + sum field_size) rounded up to even.  The module's
 * preferred HBM layout (one 128-byte line per vertex for up to 16 doubles:
 * one gather per vertex instead of one per solution); a shim builds it in the
 * pass that packs MMG5_Point.c.  Supported: at most 16 doubles in the
 * compiled slot layouts (BASELINE's configs: metric, scalar, vector, tensor;
 * iso metric + scalars); otherwise 0 is returned and pmmg_hip_set_solutions
 * takes the arrays.  Device records: 16-byte aligned (RS * 8 bytes apart: a
 * 128-byte-aligned base puts a 16-double record on one cache line).
 * Returns 1/0. */
int pmmg_hip_set_solutions_packed(pmmg_hip_ctx *ctx, int met_size, int nfield,
                                  const int *field_size, const double *rec, int where);

/* pmmg_hip_locate_interp with the new points' values written as records of
 * the same layout as the packed input (rec_out[RS*np_new], point ip's record
 * at rec_out + RS*(ip-1): [metric | field 0 | ...]): after
 * pmmg_hip_set_solutions_packed, device pointers only (rec_out 16-byte
 * aligned; 128-byte aligned puts each 16-double record on one line).  What a
 * record is not written for keeps its previous content, per solution as in
 * the reference (skipped points, MMG5_invmat failures).  The records a step
 * writes are the next iteration's background records as they are (the
 * adapted group becomes the old group, src/libparmmg1.c:653): a resident
 * pipeline never repacks.  Same results, bit for bit, as
 * pmmg_hip_locate_interp.  Returns 1/0. */
int pmmg_hip_locate_interp_rec(pmmg_hip_ctx *ctx, int np_new, const double *xyz_new, const uint8_t *pclass,
                               double *rec_out, int *elem_out, int8_t *hit_out, pmmg_hip_stats *stats, int where);

/* Load-balancing weights from the interpolated metric (SURVEY.md §8(f)
 * rank 2, the second consumer after PMMG_tetraQual), device arrays, 1-based
 * vertex ids, synchronous.
 *
 * pmmg_hip_compute_wgt_mesh replaces PMMG_computeWgt_mesh
 * (src/metis_pmmg.c:242-266): for every used tetra k (tetv[4k] > 0) with an
 * xtetra (xt[k] != 0), qual[k] = sum over its faces f with (ftag[4k+f] & tag)
 * of PMMG_computeWgt(mesh, met, pt, f) (:280-300); the other entries of qual
 * are left untouched.  ftag = the xtetra face tags gathered per tetra
 * (pxt->ftag[0..3]).
 *
 * pmmg_hip_compute_wgt_faces: PMMG_computeWgt of a list of faces
 * face[2j] = tetra (1-based), face[2j+1] = local face index (the graph
 * weights of src/metis_pmmg.c:812, :959) into wgt[j].
 *
 * PMMG_computeWgt: the three edges of the face have lengths len in the
 * metric (MMG5_lenedg: met_size 1 MMG5_lenedgCoor_iso, 6
 * MMG5_lenedgCoor_ani); res = sum (len - 1) for len <= 1 else (1/len - 1);
 * weight = min(1/exp(28 res / 3), PMMG_WGTVAL_HUGEINT); met_size 0 (no
 * metric): PMMG_WGTVAL_HUGEINT.  Mmg's special metric storage at ridge
 * points (MG_GEO edges of an aniso metric) is not modelled.
 * Returns 1, or 0 on invalid arguments. */
int pmmg_hip_compute_wgt_mesh(pmmg_hip_ctx *ctx, int np, const double *xyz, int ne,
                              const int *tetv, const int *xt, const uint16_t *ftag,
                              int met_size, const double *met, int tag, double *qual);
int pmmg_hip_compute_wgt_faces(pmmg_hip_ctx *ctx, int np, const double *xyz,
                               const int *tetv, int nface, const int *face,
                               int met_size, const double *met, double *wgt);

/* ---- One group split over the GPUs of a node -------------
 * One process per GPU (ParMmg's MPI ranks; GPU = node-local rank,
 * src/parmmg.c:121).  Each rank transfers its part of the group's new points
 * (its own pmmg_hip_locate_interp, against a replicated or halo-sharded
 * background), then the located element ids, hit codes and interpolated rows
 * of every part are collected on every rank with one RCCL all-gather over
 * xGMI.  ParMmg's only process boundary is MPI (src/libparmmg1.c:831); a shim
 * creates the communicator with MPI:
 *     char id[PMMG_HIP_COMM_ID_BYTES];
 *     if (rank == 0) pmmg_hip_comm_unique_id(id);
 *     MPI_Bcast(id, PMMG_HIP_COMM_ID_BYTES, MPI_BYTE, 0, comm_node);
 *     pmmg_hip_comm_init(ctx, nranks, rank, id);       (collective)
 * or hands over an ncclComm_t it owns (pmmg_hip_comm_attach).  RCCL
 * (librccl.so.1) is loaded at the first of these calls.  Returns 1/0. */
#define PMMG_HIP_COMM_ID_BYTES 128
int pmmg_hip_comm_unique_id(void *id);
int pmmg_hip_comm_init(pmmg_hip_ctx *ctx, int nranks, int rank, const void *id);
int pmmg_hip_comm_attach(pmmg_hip_ctx *ctx, void *nccl_comm, int nranks, int rank);

/* All-gather of the parts' results (collective over the communicator; every
 * rank passes the same counts[], nslot, slot_size[] and the same choice of
 * elem / hit given or NULL — the ranks first agree on that and on their
 * arguments' validity, and all return 0 together when one differs or fails):
 * counts[nranks] points per rank (rank order), this rank's part in
 * rows[s] (slot_size[s] doubles per point: the metric / field rows
 * pmmg_hip_locate_interp wrote), elem, hit (both optional, NULL on every
 * rank or on none); outputs rows_all[s], elem_all, hit_all hold the parts
 * concatenated in rank order (sum counts points).  Device pointers;
 * returns when the outputs are written.  Returns 1/0. */
int pmmg_hip_allgather_points(pmmg_hip_ctx *ctx, const int64_t *counts, int nslot, const int *slot_size,
                              const double *const *rows, double *const *rows_all, const int *elem, int *elem_all,
                              const int8_t *hit, int8_t *hit_all);

/* Device memory helpers for callers that keep data resident (bench, shims
 * that reuse buffers across iterations). */
void *pmmg_hip_malloc(pmmg_hip_ctx *ctx, int64_t bytes);
int   pmmg_hip_free(pmmg_hip_ctx *ctx, void *dptr);
int   pmmg_hip_memcpy_h2d(pmmg_hip_ctx *ctx, void *dst, const void *src, int64_t bytes);
int   pmmg_hip_memcpy_d2h(pmmg_hip_ctx *ctx, void *dst, const void *src, int64_t bytes);

/* Last error message of the context (static storage inside ctx). */
const char *pmmg_hip_last_error(pmmg_hip_ctx *ctx);

/* Number of visible HIP devices (0 when none / no driver). */
int pmmg_hip_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* PARMMG_HIP_H */
