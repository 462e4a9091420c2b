/*
 * pmmg_synth.h — synthetic background / adapted meshes for the transfer step.
 *
 * Test and benchmark support (SURVEY.md §8(d) "Synthetic inputs"): Kuhn
 * (6-tetra) lattices of the unit cube, or of a cube shell [-1,1]^3 minus
 * (-1/2,1/2)^3 mapped radially onto the spherical shell r in [1/2,1]
 * (x = y*|y|_inf/|y|_2).  Connectivity, tetra adjacency (reference encoding
 * 4*k+i, src/locate_pmmg.c:821), boundary trias and tria adjacency (3*k+i,
 * src/locate_pmmg.c:635) are produced analytically / by edge matching, in the
 * packed "row r = entity r+1" layout of include/parmmg_hip.h.
 *
 * Vertex jitter uses a counter-based splitmix64 keyed by (seed, vertex id),
 * so a vertex's position does not depend on sharding or evaluation order.
 */
#ifndef PMMG_SYNTH_H
#define PMMG_SYNTH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYNTH_CUBE  0
#define SYNTH_SHELL 1

/* out[0]=np, out[1]=ne, out[2]=nt.  Returns 1, or 0 for an invalid (kind,n)
 * (the shell needs n % 4 == 0). */
int synth_counts(int kind, int n, int64_t *out);

/* Vertex coordinates xyz[3*np] and boundary flags isbdy[np] (may be NULL).
 * jitter: amplitude in units of the lattice step h (0 = exact lattice);
 * interior vertices move in 3D, boundary vertices only tangentially, so they
 * stay exactly on the cube faces / spheres. */
int synth_vertices(int kind, int n, double jitter, uint64_t seed,
                   double *xyz, uint8_t *isbdy);

/* The same, every vertex's displacement capped at 0.2 of its smallest height
 * over the Kuhn tetra around it (unjittered): the lattice's tetra stay
 * positive, so the jittered points with synth_tetra's connectivity form a
 * valid mesh (a remeshed group that becomes the next background).  Vertices
 * whose cap is not reached move exactly as in synth_vertices. */
int synth_vertices_valid(int kind, int n, double jitter, uint64_t seed,
                         double *xyz, uint8_t *isbdy);

/* Tetra vertices tetv[4*ne] (1-based ids, positively oriented) and adjacency
 * adja[4*ne] (may be NULL). */
int synth_tetra(int kind, int n, int *tetv, int *adja);

/* Boundary trias (faces of tetra with adja == 0, oriented as MMG5_idir, i.e.
 * outward) and their adjacency.  Returns the number of trias written, or -1. */
int64_t synth_trias(int ne, const int *tetv, const int *adja, int *triv, int *adjt);

/* Analytic solutions at xyz[3*np]:
 *  0 iso metric size h(x)                  (size 1)
 *  1 aniso metric R^T diag(h^-2,(2h)^-2,(3h)^-2) R, diagonal in a slab (size 6)
 *  2 scalar sin(pi x) cos(pi y) + z        (size 1)
 *  3 vector (x^2, y^2, z^2)                (size 3)
 *  4 SPD tensor                            (size 6)
 *  5 affine scalar 1 + 2x - 3y + z/2       (size 1)
 *  6 affine vector                         (size 3)
 *  7 constant SPD tensor                   (size 6) */
int synth_field(int which, int64_t np, const double *xyz, double *out);
int synth_field_size(int which);

/* Point visitation order of the reference (src/interpmesh_pmmg.c:535-545):
 * first appearance of each vertex in new-tetra order.  order[] receives up to
 * np entries (1-based ids); returns the count. */
int64_t synth_visit_order(int ne, const int *tetv, int np, int *order);

/* Point classes for pmmg_hip_locate_interp: PMMG_PT_BDY for boundary
 * vertices, PMMG_PT_VOL otherwise; every `req_every`-th vertex (if > 0) is
 * PMMG_PT_SKIP (stands in for MG_REQ interface points). */
int synth_classes(int64_t np, const uint8_t *isbdy, int req_every, uint8_t *pclass);

#ifdef __cplusplus
}
#endif
#endif
