/*
 * pmmg_synth.c — synthetic Kuhn-lattice meshes (see pmmg_synth.h).
 *
 * Lattice cell c = (ci,cj,ck) is split into the 6 Kuhn tetra that share the
 * diagonal c -> c+(1,1,1): for an axis permutation (a,b,d),
 *   q0 = c, q1 = c+e_a, q2 = c+e_a+e_b, q3 = c+(1,1,1).
 * Odd permutations store (q0,q1,q3,q2) so every tetra has positive MMG5_orvol.
 * Face neighbours (face opposite q_j) are analytic:
 *   j=0: cell c+e_a, perm (b,d,a), its face opposite q3
 *   j=3: cell c-e_d, perm (d,a,b), its face opposite q0
 *   j=1: cell c,     perm (b,a,d), its face opposite q1
 *   j=2: cell c,     perm (a,d,b), its face opposite q2
 */
#include "pmmg_synth.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int kPerm[6][3] = {{0,1,2},{0,2,1},{1,0,2},{1,2,0},{2,0,1},{2,1,0}};
static const int kOdd[6]     = {0,1,1,0,0,1};
/* Face f of a tetra is opposite vertex f; its vertices, oriented outward
 * (the MMG5_idir table of Mmg). */
static const int kIdir[4][3] = {{1,2,3},{0,3,2},{0,1,3},{0,2,1}};

static int perm_index(int a, int b) {
  for (int p = 0; p < 6; p++)
    if (kPerm[p][0] == a && kPerm[p][1] == b) return p;
  return -1;
}

/* local index (0..3) of Kuhn vertex q_j in a tetra of permutation p */
static inline int local_of(int p, int j) {
  if (!kOdd[p]) return j;
  return j == 2 ? 3 : (j == 3 ? 2 : j);
}

typedef struct {
  int kind, n;
  int64_t np, ncell;
  int64_t *vrow;   /* (n+1)^2 : vertices before row (j,k) */
  int64_t *crow;   /* n^2     : cells before row (cj,ck) */
} lattice;

static int vrow_has_hole(const lattice *L, int j, int k) {
  int n = L->n;
  return L->kind == SYNTH_SHELL && j > n / 4 && j < 3 * n / 4 && k > n / 4 && k < 3 * n / 4;
}
static int crow_has_hole(const lattice *L, int cj, int ck) {
  int n = L->n;
  return L->kind == SYNTH_SHELL && cj >= n / 4 && cj < 3 * n / 4 && ck >= n / 4 && ck < 3 * n / 4;
}

static int lattice_init(lattice *L, int kind, int n) {
  memset(L, 0, sizeof(*L));
  if (n < 1 || (kind != SYNTH_CUBE && kind != SYNTH_SHELL)) return 0;
  if (kind == SYNTH_SHELL && (n % 4 != 0 || n < 8)) return 0;
  L->kind = kind;
  L->n = n;
  L->vrow = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1) * (n + 1));
  L->crow = (int64_t *)malloc(sizeof(int64_t) * (size_t)n * n);
  if (!L->vrow || !L->crow) return 0;
  int64_t acc = 0;
  for (int k = 0; k <= n; k++)
    for (int j = 0; j <= n; j++) {
      L->vrow[(size_t)k * (n + 1) + j] = acc;
      acc += (n + 1) - (vrow_has_hole(L, j, k) ? (n / 2 - 1) : 0);
    }
  L->np = acc;
  acc = 0;
  for (int ck = 0; ck < n; ck++)
    for (int cj = 0; cj < n; cj++) {
      L->crow[(size_t)ck * n + cj] = acc;
      acc += n - (crow_has_hole(L, cj, ck) ? n / 2 : 0);
    }
  L->ncell = acc;
  return 1;
}

static void lattice_free(lattice *L) {
  free(L->vrow);
  free(L->crow);
}

static inline int cell_in(const lattice *L, int ci, int cj, int ck) {
  int n = L->n;
  if (ci < 0 || cj < 0 || ck < 0 || ci >= n || cj >= n || ck >= n) return 0;
  if (L->kind == SYNTH_SHELL) {
    int lo = n / 4, hi = 3 * n / 4;
    if (ci >= lo && ci < hi && cj >= lo && cj < hi && ck >= lo && ck < hi) return 0;
  }
  return 1;
}

static inline int64_t vid(const lattice *L, int i, int j, int k) {
  int n = L->n;
  int64_t base = L->vrow[(size_t)k * (n + 1) + j];
  if (vrow_has_hole(L, j, k) && i > n / 4) return 1 + base + i - (n / 2 - 1);
  return 1 + base + i;
}

static inline int64_t cid(const lattice *L, int ci, int cj, int ck) {
  int n = L->n;
  int64_t base = L->crow[(size_t)ck * n + cj];
  if (crow_has_hole(L, cj, ck) && ci >= 3 * n / 4) return base + ci - n / 2;
  return base + ci;
}

int synth_counts(int kind, int n, int64_t *out) {
  lattice L;
  if (!lattice_init(&L, kind, n)) { lattice_free(&L); return 0; }
  out[0] = L.np;
  out[1] = 6 * L.ncell;
  if (kind == SYNTH_CUBE) out[2] = 12LL * n * n;
  else out[2] = 12LL * n * n + 12LL * (n / 2) * (n / 2);
  lattice_free(&L);
  return 1;
}

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

static inline double unit_rand(uint64_t seed, int64_t id, int c) {
  uint64_t r = splitmix64(seed ^ splitmix64((uint64_t)id * 4 + (uint64_t)c));
  return (double)(r >> 11) * (1.0 / 9007199254740992.0); /* [0,1) */
}

/* lattice point idx (jittered by jit * h per unpinned coordinate) mapped to
 * the mesh: the cube as is, the shell radially onto spheres (|p| = ninf(y)) */
static void place(int kind, int n, const int *idx, const int *pinned, double jit, uint64_t seed, int64_t v,
                  double *p) {
  double h = (kind == SYNTH_CUBE) ? 1.0 / n : 2.0 / n;
  double y[3];
  for (int d = 0; d < 3; d++) {
    y[d] = (kind == SYNTH_CUBE) ? (double)idx[d] / n : -1.0 + 2.0 * idx[d] / n;
    if (jit != 0.0 && !pinned[d]) y[d] += (2.0 * unit_rand(seed, v, d) - 1.0) * jit * h;
  }
  if (kind == SYNTH_CUBE) {
    p[0] = y[0]; p[1] = y[1]; p[2] = y[2];
  } else {
    double ninf = fmax(fabs(y[0]), fmax(fabs(y[1]), fabs(y[2])));
    double n2 = sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
    double s = ninf / n2;
    p[0] = y[0] * s; p[1] = y[1] * s; p[2] = y[2] * s;
  }
}

/* smallest height of lattice vertex idx over the Kuhn tetra around it
 * (unjittered positions): the distance to the opposite face */
static double min_height(const lattice *L, const int *idx) {
  static const int e[3][3] = {{1,0,0},{0,1,0},{0,0,1}};
  static const int zero[3] = {0, 0, 0};
  const int n = L->n;
  double hmin = HUGE_VAL;
  for (int dk = -1; dk <= 0; dk++)
    for (int dj = -1; dj <= 0; dj++)
      for (int di = -1; di <= 0; di++) {
        int cc[3] = {idx[0] + di, idx[1] + dj, idx[2] + dk};
        if (!cell_in(L, cc[0], cc[1], cc[2])) continue;
        for (int p = 0; p < 6; p++) {
          int a = kPerm[p][0], b = kPerm[p][1];
          int q[4][3], me = -1;
          for (int x = 0; x < 3; x++) {
            q[0][x] = cc[x];
            q[1][x] = cc[x] + e[a][x];
            q[2][x] = cc[x] + e[a][x] + e[b][x];
            q[3][x] = cc[x] + 1;
          }
          for (int j = 0; j < 4; j++)
            if (q[j][0] == idx[0] && q[j][1] == idx[1] && q[j][2] == idx[2]) me = j;
          if (me < 0) continue;
          double P[4][3];
          for (int j = 0; j < 4; j++) place(L->kind, n, q[j], zero, 0.0, 0, 0, P[j]);
          const double *A = P[(me + 1) & 3], *B = P[(me + 2) & 3], *C = P[(me + 3) & 3];
          double u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, w[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
          double nn[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
          double len = sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
          double hh = fabs((P[me][0] - A[0]) * nn[0] + (P[me][1] - A[1]) * nn[1] + (P[me][2] - A[2]) * nn[2]) / len;
          if (hh < hmin) hmin = hh;
        }
      }
  return hmin;
}

static int vertices(int kind, int n, double jitter, uint64_t seed, int valid, double *xyz, uint8_t *isbdy) {
  lattice L;
  if (!lattice_init(&L, kind, n)) { lattice_free(&L); return 0; }
  const int lo = n / 4, hi = 3 * n / 4;
#pragma omp parallel for schedule(static)
  for (int k = 0; k <= n; k++) {
    for (int j = 0; j <= n; j++) {
      for (int i = 0; i <= n; i++) {
        int idx[3] = {i, j, k};
        int bdy = 0, pinned[3] = {0, 0, 0};
        if (kind == SYNTH_CUBE) {
          for (int d = 0; d < 3; d++)
            if (idx[d] == 0 || idx[d] == n) { pinned[d] = 1; bdy = 1; }
        } else {
          if (i > lo && i < hi && j > lo && j < hi && k > lo && k < hi) continue; /* hole */
          int m[3], mx = 0;
          for (int d = 0; d < 3; d++) { m[d] = abs(2 * idx[d] - n); if (m[d] > mx) mx = m[d]; }
          if (mx == n || mx == n / 2) {
            bdy = 1;
            for (int d = 0; d < 3; d++) pinned[d] = (m[d] == mx);
          }
        }
        int64_t v = vid(&L, i, j, k);
        double *p = xyz + 3 * (v - 1);
        place(kind, n, idx, pinned, jitter, seed, v, p);
        if (valid && jitter != 0.0) {
          /* a vertex moves by at most kValidFrac of its smallest height, so
           * that no Kuhn tetra inverts (the shell's radial map leaves slivers
           * along the planes |y_i| = |y_j| = ninf, volume down to 7e-5 of the
           * median, which a jitter of 0.05 cell already inverts) */
          const double kValidFrac = 0.2;
          static const int zero[3] = {0, 0, 0};
          double p0[3];
          place(kind, n, idx, zero, 0.0, 0, 0, p0);
          double dd = sqrt((p[0] - p0[0]) * (p[0] - p0[0]) + (p[1] - p0[1]) * (p[1] - p0[1]) +
                           (p[2] - p0[2]) * (p[2] - p0[2]));
          double cap = kValidFrac * min_height(&L, idx);
          if (dd > cap) place(kind, n, idx, pinned, jitter * cap / dd, seed, v, p);
        }
        if (isbdy) isbdy[v - 1] = (uint8_t)bdy;
      }
    }
  }
  lattice_free(&L);
  return 1;
}

int synth_vertices(int kind, int n, double jitter, uint64_t seed, double *xyz, uint8_t *isbdy) {
  return vertices(kind, n, jitter, seed, 0, xyz, isbdy);
}

int synth_vertices_valid(int kind, int n, double jitter, uint64_t seed, double *xyz, uint8_t *isbdy) {
  return vertices(kind, n, jitter, seed, 1, xyz, isbdy);
}

int synth_tetra(int kind, int n, int *tetv, int *adja) {
  lattice L;
  if (!lattice_init(&L, kind, n)) { lattice_free(&L); return 0; }
  static const int e[3][3] = {{1,0,0},{0,1,0},{0,0,1}};
#pragma omp parallel for schedule(static)
  for (int ck = 0; ck < n; ck++) {
    for (int cj = 0; cj < n; cj++) {
      for (int ci = 0; ci < n; ci++) {
        if (!cell_in(&L, ci, cj, ck)) continue;
        int64_t c = cid(&L, ci, cj, ck);
        int cc[3] = {ci, cj, ck};
        for (int p = 0; p < 6; p++) {
          int a = kPerm[p][0], b = kPerm[p][1], d = kPerm[p][2];
          int q[4][3];
          for (int x = 0; x < 3; x++) {
            q[0][x] = cc[x];
            q[1][x] = cc[x] + e[a][x];
            q[2][x] = cc[x] + e[a][x] + e[b][x];
            q[3][x] = cc[x] + 1;
          }
          int64_t k = 6 * c + p; /* 0-based row */
          for (int jj = 0; jj < 4; jj++)
            tetv[4 * k + local_of(p, jj)] = (int)vid(&L, q[jj][0], q[jj][1], q[jj][2]);
          if (!adja) continue;
          for (int jj = 0; jj < 4; jj++) {
            int nc[3] = {cc[0], cc[1], cc[2]};
            int np_, nj;
            if (jj == 0) {
              nc[a] += 1; np_ = perm_index(b, d); nj = 3;
            } else if (jj == 3) {
              nc[d] -= 1; np_ = perm_index(d, a); nj = 0;
            } else if (jj == 1) {
              np_ = perm_index(b, a); nj = 1;
            } else {
              np_ = perm_index(a, d); nj = 2;
            }
            int code = 0;
            if (cell_in(&L, nc[0], nc[1], nc[2])) {
              int64_t kn = 6 * cid(&L, nc[0], nc[1], nc[2]) + np_ + 1; /* 1-based */
              code = (int)(4 * kn + local_of(np_, nj));
            }
            adja[4 * k + local_of(p, jj)] = code;
          }
        }
      }
    }
  }
  lattice_free(&L);
  return 1;
}

typedef struct { uint64_t key; int code; } edge_rec;

static int edge_cmp(const void *x, const void *y) {
  const edge_rec *a = (const edge_rec *)x, *b = (const edge_rec *)y;
  if (a->key < b->key) return -1;
  if (a->key > b->key) return 1;
  return (a->code > b->code) - (a->code < b->code);
}

int64_t synth_trias(int ne, const int *tetv, const int *adja, int *triv, int *adjt) {
  int64_t nt = 0;
  for (int64_t k = 0; k < ne; k++)
    for (int f = 0; f < 4; f++) {
      if (adja[4 * k + f]) continue;
      for (int l = 0; l < 3; l++) triv[3 * nt + l] = tetv[4 * k + kIdir[f][l]];
      nt++;
    }
  if (!adjt) return nt;
  edge_rec *ed = (edge_rec *)malloc(sizeof(edge_rec) * (size_t)(3 * nt + 1));
  if (!ed) return -1;
  for (int64_t t = 0; t < nt; t++)
    for (int i = 0; i < 3; i++) {
      uint32_t va = (uint32_t)triv[3 * t + (i + 1) % 3];
      uint32_t vb = (uint32_t)triv[3 * t + (i + 2) % 3];
      uint32_t lo = va < vb ? va : vb, hi = va < vb ? vb : va;
      ed[3 * t + i].key = ((uint64_t)lo << 32) | hi;
      ed[3 * t + i].code = (int)(3 * (t + 1) + i);
      adjt[3 * t + i] = 0;
    }
  qsort(ed, (size_t)(3 * nt), sizeof(edge_rec), edge_cmp);
  for (int64_t s = 0; s + 1 < 3 * nt;) {
    int64_t e2 = s + 1;
    while (e2 < 3 * nt && ed[e2].key == ed[s].key) e2++;
    if (e2 - s == 2) {
      int c0 = ed[s].code, c1 = ed[s + 1].code;
      adjt[3 * (c0 / 3 - 1) + c0 % 3] = c1;
      adjt[3 * (c1 / 3 - 1) + c1 % 3] = c0;
    }
    s = e2;
  }
  free(ed);
  return nt;
}

int synth_field_size(int which) {
  static const int sz[8] = {1, 6, 1, 3, 6, 1, 3, 6};
  return (which >= 0 && which < 8) ? sz[which] : 0;
}

/* M = R^T diag(l) R for a rotation R about axis `ax` by angle th */
static void spd_from_rot(int ax, double th, const double l[3], double *m) {
  double R[3][3] = {{1,0,0},{0,1,0},{0,0,1}};
  int u = (ax + 1) % 3, v = (ax + 2) % 3;
  double c = cos(th), s = sin(th);
  R[u][u] = c; R[u][v] = -s; R[v][u] = s; R[v][v] = c;
  double M[3][3];
  for (int j = 0; j < 3; j++)
    for (int k = 0; k < 3; k++) {
      double acc = 0.0;
      for (int i = 0; i < 3; i++) acc += R[i][j] * l[i] * R[i][k];
      M[j][k] = acc;
    }
  m[0] = M[0][0]; m[1] = M[0][1]; m[2] = M[0][2];
  m[3] = M[1][1]; m[4] = M[1][2]; m[5] = M[2][2];
}

int synth_field(int which, int64_t np, const double *xyz, double *out) {
  if (synth_field_size(which) == 0) return 0;
  const double pi = 3.14159265358979323846;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < np; i++) {
    const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    double dx = x - 0.5, dy = y - 0.5, dz = z - 0.5;
    double h = 0.02 + 0.08 * sqrt(dx * dx + dy * dy + dz * dz);
    switch (which) {
      case 0: out[i] = h; break;
      case 1: {
        double l[3] = {1.0 / (h * h), 1.0 / (4.0 * h * h), 1.0 / (9.0 * h * h)};
        double th = (x < 0.1) ? 0.0 : pi * x;
        spd_from_rot(2, th, l, out + 6 * i);
        if (x < 0.1) { out[6 * i + 1] = 0.0; out[6 * i + 2] = 0.0; out[6 * i + 4] = 0.0; }
      } break;
      case 2: out[i] = sin(pi * x) * cos(pi * y) + z; break;
      case 3: out[3 * i] = x * x; out[3 * i + 1] = y * y; out[3 * i + 2] = z * z; break;
      case 4: {
        double l[3] = {1.0 + x * x, 2.0 + y * y, 3.0 + z * z};
        spd_from_rot(0, pi * y, l, out + 6 * i);
      } break;
      case 5: out[i] = 1.0 + 2.0 * x - 3.0 * y + 0.5 * z; break;
      case 6: out[3 * i] = x + y; out[3 * i + 1] = 2.0 * y - z; out[3 * i + 2] = 3.0 * z + x - 1.0; break;
      case 7: {
        double *m = out + 6 * i;
        m[0] = 4.0; m[1] = 1.0; m[2] = 0.5; m[3] = 3.0; m[4] = 0.25; m[5] = 2.0;
      } break;
    }
  }
  return 1;
}

int64_t synth_visit_order(int ne, const int *tetv, int np, int *order) {
  uint8_t *seen = (uint8_t *)calloc((size_t)np + 1, 1);
  if (!seen) return -1;
  int64_t cnt = 0;
  for (int64_t k = 0; k < ne; k++)
    for (int l = 0; l < 4; l++) {
      int v = tetv[4 * k + l];
      if (v < 1 || v > np || seen[v]) continue;
      seen[v] = 1;
      order[cnt++] = v;
    }
  free(seen);
  return cnt;
}

int synth_classes(int64_t np, const uint8_t *isbdy, int req_every, uint8_t *pclass) {
  for (int64_t i = 0; i < np; i++) {
    uint8_t c = (isbdy && isbdy[i]) ? 2 : 1;
    if (req_every > 0 && ((i + 1) % req_every) == 0) c = 0;
    pclass[i] = c;
  }
  return 1;
}
