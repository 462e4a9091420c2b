/*
 * pmmg_medit.h — Medit ASCII reader for the transfer path's inputs (host
 * code, part of libpmmg_host).
 *
 * What PMMG_loadMesh_centralized / PMMG_loadAllSols_centralized (reference
 * src/inout_pmmg.c:488, :748) obtain through Mmg's MMG3D_loadMesh /
 * MMG3D_loadAllSols for the arrays this path reads: vertices (+ refs),
 * tetrahedra (+ refs), boundary triangles (+ refs) of a .mesh file, and the
 * SolAtVertices block of a .sol file (types 1 scalar, 2 vector, 3 symmetric
 * tensor).  Medit stores a 3D tensor as m11 m12 m22 m13 m23 m33 and MMG5
 * keeps m11 m12 m13 m22 m23 m33 in memory: entries 2 and 3 are swapped on
 * read, as Mmg's MMG5_loadSolAtVertices does.  Arrays use the C-ABI's "row r =
 * entity r+1" layout (include/parmmg_hip.h).  Binary .meshb / .solb files
 * (GMF versions 1-3, either byte order) are read too (pmmg_medit.c).
 */
#ifndef PMMG_MEDIT_H
#define PMMG_MEDIT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int np, ne, nt;
  double *xyz; /* 3*np */
  int *vref;   /* np */
  int *tetv;   /* 4*ne */
  int *tref;   /* ne */
  int *triv;   /* 3*nt */
  int *trref;  /* nt */
} pmmg_medit_mesh;

#define PMMG_MEDIT_MAXSOL 32

typedef struct {
  int np;                          /* vertices of the SolAtVertices block */
  int nsol;                        /* solutions at each vertex */
  int type[PMMG_MEDIT_MAXSOL];     /* Medit type: 1 scalar, 2 vector, 3 tensor */
  int size[PMMG_MEDIT_MAXSOL];     /* doubles per vertex: 1, 3, 6 */
  double *val[PMMG_MEDIT_MAXSOL];  /* size[j]*np each, MMG5 component order */
} pmmg_medit_sol;

/* Returns 1 on success, 0 on error (message in err[errlen]); the struct is
 * zeroed on error. */
int pmmg_medit_read_mesh(const char *path, pmmg_medit_mesh *m, char *err, int errlen);
int pmmg_medit_read_sol(const char *path, pmmg_medit_sol *s, char *err, int errlen);
void pmmg_medit_free_mesh(pmmg_medit_mesh *m);
void pmmg_medit_free_sol(pmmg_medit_sol *s);

#ifdef __cplusplus
}
#endif
#endif
