/*
 * pmmg_medit.c — Medit ASCII .mesh / .sol reader (see pmmg_medit.h).
 *
 * The format: whitespace-separated tokens, '#' comments to the end of the
 * line, keyword blocks `Keyword count rows...`.  Read here: Vertices (x y z
 * ref), Tetrahedra (v0 v1 v2 v3 ref), Triangles (v0 v1 v2 ref),
 * SolAtVertices (count, ntypes, types..., values per vertex in type order).
 * MeshVersionFormatted / Dimension take one value; any other keyword with a
 * count is skipped by the row width Mmg gives it when it is one of the
 * common entity blocks, otherwise the reader stops with an error (a block of
 * unknown width cannot be skipped safely).
 */
#define _POSIX_C_SOURCE 200809L
#include "pmmg_medit.h"

#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  FILE *f;
  char tok[256];
} lexer;

/* next whitespace-separated token (comments skipped); 0 at end of file */
static int next_tok(lexer *L) {
  int ch, n = 0;
  for (;;) {
    ch = fgetc(L->f);
    if (ch == EOF) return 0;
    if (ch == '#') {
      while (ch != EOF && ch != '\n') ch = fgetc(L->f);
      continue;
    }
    if (!isspace(ch)) break;
  }
  while (ch != EOF && !isspace(ch) && ch != '#') {
    if (n < (int)sizeof(L->tok) - 1) L->tok[n++] = (char)ch;
    ch = fgetc(L->f);
  }
  if (ch == '#') ungetc(ch, L->f);
  L->tok[n] = 0;
  return 1;
}

static void seterr(char *err, int errlen, const char *fmt, ...) {
  if (!err || errlen <= 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, (size_t)errlen, fmt, ap);
  va_end(ap);
}

static int read_long(lexer *L, long long *v) {
  char *end;
  if (!next_tok(L)) return 0;
  *v = strtoll(L->tok, &end, 10);
  return *end == 0;
}

static int read_double(lexer *L, double *v) {
  char *end;
  if (!next_tok(L)) return 0;
  *v = strtod(L->tok, &end);
  return *end == 0;
}

static int is_binary(const char *path) {
  const size_t n = strlen(path);
  return n >= 1 && path[n - 1] == 'b';
}

/* row widths (tokens per entity) of Medit blocks that are skipped */
static int skip_width(const char *kw) {
  static const struct {
    const char *kw;
    int w;
  } tab[] = {{"Edges", 3},        {"Quadrilaterals", 5}, {"Prisms", 7},      {"Hexahedra", 9},
             {"Corners", 1},      {"RequiredVertices", 1}, {"Ridges", 1},     {"RequiredEdges", 1},
             {"RequiredTriangles", 1}, {"RequiredTetrahedra", 1}, {"Normals", 3}, {"NormalAtVertices", 2},
             {"Tangents", 3},     {"TangentAtVertices", 2}, {"ParallelTriangles", 1}, {"ParallelVertices", 1}};
  for (size_t i = 0; i < sizeof(tab) / sizeof(tab[0]); i++)
    if (!strcmp(kw, tab[i].kw)) return tab[i].w;
  return -1;
}

void pmmg_medit_free_mesh(pmmg_medit_mesh *m) {
  if (!m) return;
  free(m->xyz);
  free(m->vref);
  free(m->tetv);
  free(m->tref);
  free(m->triv);
  free(m->trref);
  memset(m, 0, sizeof(*m));
}

void pmmg_medit_free_sol(pmmg_medit_sol *s) {
  if (!s) return;
  for (int j = 0; j < PMMG_MEDIT_MAXSOL; j++) free(s->val[j]);
  memset(s, 0, sizeof(*s));
}

int pmmg_medit_read_mesh(const char *path, pmmg_medit_mesh *m, char *err, int errlen) {
  memset(m, 0, sizeof(*m));
  if (is_binary(path)) {
    seterr(err, errlen, "%s: binary Medit files are not read", path);
    return 0;
  }
  lexer L;
  L.f = fopen(path, "r");
  if (!L.f) {
    seterr(err, errlen, "%s: cannot open", path);
    return 0;
  }
  int ok = 1, dim = 3;
  while (ok && next_tok(&L)) {
    char kw[256];
    long long n, v;
    snprintf(kw, sizeof(kw), "%s", L.tok);
    if (!strcmp(kw, "End")) break;
    if (!strcmp(kw, "MeshVersionFormatted")) {
      ok = read_long(&L, &v);
      continue;
    }
    if (!strcmp(kw, "Dimension")) {
      ok = read_long(&L, &v);
      dim = (int)v;
      if (dim != 3) {
        seterr(err, errlen, "%s: dimension %d (3 expected)", path, dim);
        ok = 0;
      }
      continue;
    }
    if (!read_long(&L, &n) || n < 0 || n > (1LL << 31) - 2) {
      seterr(err, errlen, "%s: block %s without a valid count", path, kw);
      ok = 0;
      break;
    }
    /* a repeated entity block is a format error (it would replace the arrays
       and the count the range checks below use) */
    if ((!strcmp(kw, "Vertices") && m->xyz) || (!strcmp(kw, "Tetrahedra") && m->tetv) ||
        (!strcmp(kw, "Triangles") && m->triv)) {
      seterr(err, errlen, "%s: repeated block %s", path, kw);
      ok = 0;
      break;
    }
    if (!strcmp(kw, "Vertices")) {
      m->np = (int)n;
      m->xyz = (double *)malloc(sizeof(double) * 3 * (size_t)(n ? n : 1));
      m->vref = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));
      if (!m->xyz || !m->vref) ok = 0;
      for (long long i = 0; ok && i < n; i++) {
        ok = read_double(&L, &m->xyz[3 * i]) && read_double(&L, &m->xyz[3 * i + 1]) &&
             read_double(&L, &m->xyz[3 * i + 2]) && read_long(&L, &v);
        m->vref[i] = (int)v;
      }
    } else if (!strcmp(kw, "Tetrahedra") || !strcmp(kw, "Triangles")) {
      const int nv = kw[1] == 'e' ? 4 : 3;
      int *vv = (int *)malloc(sizeof(int) * nv * (size_t)(n ? n : 1));
      int *rr = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));
      if (!vv || !rr) ok = 0;
      for (long long i = 0; ok && i < n; i++) {
        for (int k = 0; ok && k < nv; k++) {
          /* ids beyond INT_MAX would wrap in the int arrays and pass the
             range check below: rejected here, before the cast */
          ok = read_long(&L, &v) && v >= 1 && v <= 2147483647LL;
          vv[nv * i + k] = ok ? (int)v : 0;
        }
        ok = ok && read_long(&L, &v);
        rr[i] = (int)v;
      }
      if (nv == 4) {
        m->ne = (int)n;
        m->tetv = vv;
        m->tref = rr;
      } else {
        m->nt = (int)n;
        m->triv = vv;
        m->trref = rr;
      }
    } else {
      const int w = skip_width(kw);
      if (w < 0) {
        seterr(err, errlen, "%s: unknown block %s", path, kw);
        ok = 0;
        break;
      }
      for (long long i = 0; ok && i < n * w; i++) ok = next_tok(&L);
    }
    if (!ok && !(err && err[0])) seterr(err, errlen, "%s: truncated or malformed block %s", path, kw);
  }
  fclose(L.f);
  if (ok && m->np <= 0) {
    seterr(err, errlen, "%s: no vertices", path);
    ok = 0;
  }
  for (int i = 0; ok && i < 4 * m->ne; i++)
    if (m->tetv[i] < 1 || m->tetv[i] > m->np) {
      seterr(err, errlen, "%s: tetrahedron vertex %d out of range", path, m->tetv[i]);
      ok = 0;
    }
  for (int i = 0; ok && i < 3 * m->nt; i++)
    if (m->triv[i] < 1 || m->triv[i] > m->np) {
      seterr(err, errlen, "%s: triangle vertex %d out of range", path, m->triv[i]);
      ok = 0;
    }
  if (!ok) pmmg_medit_free_mesh(m);
  return ok;
}

int pmmg_medit_read_sol(const char *path, pmmg_medit_sol *s, char *err, int errlen) {
  memset(s, 0, sizeof(*s));
  if (is_binary(path)) {
    seterr(err, errlen, "%s: binary Medit files are not read", path);
    return 0;
  }
  lexer L;
  L.f = fopen(path, "r");
  if (!L.f) {
    seterr(err, errlen, "%s: cannot open", path);
    return 0;
  }
  int ok = 1, found = 0;
  while (ok && !found && next_tok(&L)) {
    long long v;
    if (!strcmp(L.tok, "End")) break;
    if (!strcmp(L.tok, "MeshVersionFormatted")) {
      ok = read_long(&L, &v);
    } else if (!strcmp(L.tok, "Dimension")) {
      ok = read_long(&L, &v) && v == 3;
      if (!ok) seterr(err, errlen, "%s: dimension (3 expected)", path);
    } else if (!strcmp(L.tok, "SolAtVertices")) {
      long long n, nt;
      found = 1;
      ok = read_long(&L, &n) && n > 0 && n < (1LL << 31) - 1 && read_long(&L, &nt) && nt >= 1 &&
           nt <= PMMG_MEDIT_MAXSOL;
      if (!ok) {
        seterr(err, errlen, "%s: invalid SolAtVertices header", path);
        break;
      }
      s->np = (int)n;
      s->nsol = (int)nt;
      for (int j = 0; ok && j < s->nsol; j++) {
        ok = read_long(&L, &v) && v >= 1 && v <= 3;
        s->type[j] = (int)v;
        s->size[j] = v == 1 ? 1 : (v == 2 ? 3 : 6);
        s->val[j] = ok ? (double *)malloc(sizeof(double) * s->size[j] * (size_t)n) : NULL;
        if (ok && !s->val[j]) ok = 0;
      }
      if (!ok) {
        seterr(err, errlen, "%s: invalid solution types", path);
        break;
      }
      for (long long i = 0; ok && i < n; i++)
        for (int j = 0; ok && j < s->nsol; j++) {
          double t[6];
          for (int k = 0; ok && k < s->size[j]; k++) ok = read_double(&L, &t[k]);
          double *dst = s->val[j] + (size_t)s->size[j] * i;
          if (s->size[j] == 6) { /* Medit m11 m12 m22 m13 m23 m33 -> MMG5 m11 m12 m13 m22 m23 m33 */
            dst[0] = t[0];
            dst[1] = t[1];
            dst[2] = t[3];
            dst[3] = t[2];
            dst[4] = t[4];
            dst[5] = t[5];
          } else {
            for (int k = 0; k < s->size[j]; k++) dst[k] = t[k];
          }
        }
      if (!ok) seterr(err, errlen, "%s: truncated SolAtVertices block", path);
    }
  }
  fclose(L.f);
  if (ok && !found) {
    seterr(err, errlen, "%s: no SolAtVertices block", path);
    ok = 0;
  }
  if (!ok) pmmg_medit_free_sol(s);
  return ok;
}
