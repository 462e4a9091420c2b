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
 *
 * Binary .meshb / .solb (r04; libMeshb's GMF layout as published, restated —
 * libMeshb is absent from the image, so this is not pinned to it): an int32
 * 1 (its byte order gives the file's), an int32 version (1: 32-bit reals,
 * 2: 64-bit reals, 3: also 64-bit keyword positions; 4, 64-bit integers, is
 * not read), then keyword blocks: int32 code, the position of the next
 * keyword (int32, int64 from version 3), the block.  Codes read: 3
 * Dimension (int32), 4 Vertices, 6 Triangles, 8 Tetrahedra (int32 count,
 * then rows of reals / int32 ids and an int32 ref), 62 SolAtVertices (count,
 * number of types, types, then the values of every vertex in type order),
 * 54 End; any other block is skipped through its next-keyword position.
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

/* ---- binary (GMF) files */
enum { kGmfDimension = 3, kGmfVertices = 4, kGmfTriangles = 6, kGmfTetrahedra = 8, kGmfEnd = 54, kGmfSolAtVertices = 62 };

typedef struct {
  FILE *f;
  int swap, ver;
  long long size; /* bytes in the file */
} bfile;

/* n rows of w bytes fit in what is left of the file (a corrupted count must
   not size an allocation) */
static int b_fits(bfile *B, long long n, long long w) {
  const long long at = (long long)ftello(B->f);
  return at >= 0 && n >= 0 && n <= (B->size - at) / (w > 0 ? w : 1);
}

static int b_read(bfile *B, void *p, size_t w) {
  if (fread(p, w, 1, B->f) != 1) return 0;
  if (B->swap) {
    unsigned char *c = (unsigned char *)p;
    for (size_t i = 0; i < w / 2; i++) {
      const unsigned char t = c[i];
      c[i] = c[w - 1 - i];
      c[w - 1 - i] = t;
    }
  }
  return 1;
}

static int b_int(bfile *B, long long *v) {
  int32_t x;
  if (!b_read(B, &x, 4)) return 0;
  *v = x;
  return 1;
}

static int b_pos(bfile *B, long long *v) {
  if (B->ver < 3) return b_int(B, v);
  int64_t x;
  if (!b_read(B, &x, 8)) return 0;
  *v = x;
  return 1;
}

static int b_real(bfile *B, double *v) {
  if (B->ver == 1) {
    float x;
    if (!b_read(B, &x, 4)) return 0;
    *v = x;
    return 1;
  }
  return b_read(B, v, 8);
}

static int b_open(const char *path, bfile *B, char *err, int errlen) {
  B->f = fopen(path, "rb");
  B->swap = 0;
  if (!B->f) {
    seterr(err, errlen, "%s: cannot open", path);
    return 0;
  }
  B->size = fseeko(B->f, 0, SEEK_END) == 0 ? (long long)ftello(B->f) : -1;
  if (B->size < 0 || fseeko(B->f, 0, SEEK_SET) != 0) {
    seterr(err, errlen, "%s: cannot read", path);
    fclose(B->f);
    return 0;
  }
  long long code = 0, ver = 0;
  if (!b_int(B, &code)) code = 0;
  if (code == 16777216) { /* 1 in the other byte order */
    B->swap = 1;
    code = 1;
  }
  if (code != 1 || !b_int(B, &ver) || ver < 1 || ver > 4) {
    seterr(err, errlen, "%s: not a binary Medit file", path);
    fclose(B->f);
    return 0;
  }
  if (ver == 4) {
    seterr(err, errlen, "%s: Medit version 4 (64-bit integers) is not read", path);
    fclose(B->f);
    return 0;
  }
  B->ver = (int)ver;
  return 1;
}

/* next keyword: its code and the next one's position (0: none); 0 at the
   end of the file */
static int b_keyword(bfile *B, long long *kw, long long *next) {
  if (!b_int(B, kw)) return 0;
  *next = 0;
  return *kw == kGmfEnd || b_pos(B, next);
}

/* forward only: a corrupted position pointing back would loop forever */
static int b_skip_to(bfile *B, long long next) {
  const long long at = (long long)ftello(B->f);
  return at >= 0 && next > at && next <= B->size && fseeko(B->f, (off_t)next, SEEK_SET) == 0;
}

static int read_mesh_binary(const char *path, pmmg_medit_mesh *m, char *err, int errlen) {
  bfile B;
  if (!b_open(path, &B, err, errlen)) return 0;
  int ok = 1;
  long long kw, next, n, v = 0;
  while (ok && b_keyword(&B, &kw, &next) && kw != kGmfEnd) {
    if (kw == kGmfDimension) {
      ok = b_int(&B, &v);
      if (ok && v != 3) {
        seterr(err, errlen, "%s: dimension %lld (3 expected)", path, v);
        ok = 0;
      }
    } else if (kw == kGmfVertices || kw == kGmfTriangles || kw == kGmfTetrahedra) {
      const long long real = B.ver == 1 ? 4 : 8;
      const long long w = kw == kGmfVertices ? 3 * real + 4 : (kw == kGmfTetrahedra ? 20 : 16);
      if (!b_int(&B, &n) || n < 0 || n > (1LL << 31) - 2 || !b_fits(&B, n, w)) {
        seterr(err, errlen, "%s: block %lld without a valid count", path, kw);
        ok = 0;
        break;
      }
      if ((kw == kGmfVertices && m->xyz) || (kw == kGmfTetrahedra && m->tetv) || (kw == kGmfTriangles && m->triv)) {
        seterr(err, errlen, "%s: repeated block %lld", path, kw);
        ok = 0;
        break;
      }
      if (kw == kGmfVertices) {
        m->np = (int)n;
        m->xyz = (double *)malloc(sizeof(double) * 3 * (size_t)(n ? n : 1));
        m->vref = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));
        if (!m->xyz || !m->vref) ok = 0;
        for (long long i = 0; ok && i < n; i++) {
          ok = b_real(&B, &m->xyz[3 * i]) && b_real(&B, &m->xyz[3 * i + 1]) && b_real(&B, &m->xyz[3 * i + 2]) &&
               b_int(&B, &v);
          m->vref[i] = (int)v;
        }
      } else {
        const int nv = kw == kGmfTetrahedra ? 4 : 3;
        int *vv = (int *)malloc(sizeof(int) * nv * (size_t)(n ? n : 1));
        int *rr = (int *)malloc(sizeof(int) * (size_t)(n ? n : 1));
        if (!vv || !rr) ok = 0;
        for (long long i = 0; ok && i < n; i++) {
          for (int k = 0; ok && k < nv; k++) {
            ok = b_int(&B, &v) && v >= 1;
            vv[nv * i + k] = ok ? (int)v : 0;
          }
          ok = ok && b_int(&B, &v);
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
      }
    } else {
      ok = b_skip_to(&B, next);
    }
    if (!ok && !(err && err[0])) seterr(err, errlen, "%s: truncated or malformed block %lld", path, kw);
  }
  fclose(B.f);
  return ok;
}

static int read_sol_binary(const char *path, pmmg_medit_sol *s, char *err, int errlen, int *found) {
  bfile B;
  if (!b_open(path, &B, err, errlen)) return 0;
  int ok = 1;
  long long kw, next, v = 0;
  while (ok && !*found && b_keyword(&B, &kw, &next) && kw != kGmfEnd) {
    if (kw == kGmfDimension) {
      ok = b_int(&B, &v) && v == 3;
      if (!ok) seterr(err, errlen, "%s: dimension (3 expected)", path);
    } else if (kw == kGmfSolAtVertices) {
      long long n, nt;
      *found = 1;
      ok = b_int(&B, &n) && n > 0 && n < (1LL << 31) - 1 && b_int(&B, &nt) && nt >= 1 && nt <= PMMG_MEDIT_MAXSOL;
      if (!ok) {
        seterr(err, errlen, "%s: invalid SolAtVertices header", path);
        break;
      }
      s->np = (int)n;
      s->nsol = (int)nt;
      long long row = 0;
      for (int j = 0; ok && j < s->nsol; j++) {
        ok = b_int(&B, &v) && v >= 1 && v <= 3;
        s->type[j] = (int)v;
        s->size[j] = v == 1 ? 1 : (v == 2 ? 3 : 6);
        row += s->size[j];
      }
      ok = ok && b_fits(&B, n, row * (B.ver == 1 ? 4 : 8));
      for (int j = 0; ok && j < s->nsol; j++) {
        s->val[j] = (double *)malloc(sizeof(double) * s->size[j] * (size_t)n);
        if (!s->val[j]) ok = 0;
      }
      if (!ok) {
        seterr(err, errlen, "%s: invalid solution types or count", path);
        break;
      }
      for (long long i = 0; ok && i < n; i++)
        for (int j = 0; ok && j < s->nsol; j++) {
          double t[6];
          for (int k = 0; ok && k < s->size[j]; k++) ok = b_real(&B, &t[k]);
          if (!ok) break;
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
    } else {
      ok = b_skip_to(&B, next);
      if (!ok) seterr(err, errlen, "%s: truncated or malformed block %lld", path, kw);
    }
  }
  fclose(B.f);
  return ok;
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
  if (err && errlen > 0) err[0] = 0;
  int ok = 1, dim = 3;
  if (is_binary(path)) {
    ok = read_mesh_binary(path, m, err, errlen);
    goto check;
  }
  lexer L;
  L.f = fopen(path, "r");
  if (!L.f) {
    seterr(err, errlen, "%s: cannot open", path);
    return 0;
  }
  while (ok && next_tok(&L)) {
    char kw[256];
    long long n, v = 0;
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
check:
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
  if (err && errlen > 0) err[0] = 0;
  int ok = 1, found = 0;
  if (is_binary(path)) {
    ok = read_sol_binary(path, s, err, errlen, &found);
    goto check;
  }
  lexer L;
  L.f = fopen(path, "r");
  if (!L.f) {
    seterr(err, errlen, "%s: cannot open", path);
    return 0;
  }
  while (ok && !found && next_tok(&L)) {
    long long v = 0;
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
check:
  if (ok && !found) {
    seterr(err, errlen, "%s: no SolAtVertices block", path);
    ok = 0;
  }
  if (!ok) pmmg_medit_free_sol(s);
  return ok;
}
