/*
 * fuzz_medit.c — the C Medit reader (csrc/pmmg_medit.c) on corrupted copies
 * of the reference's libexamples fixtures: truncated at every length, with
 * single bytes replaced, with counts inflated.  Built with ASan + UBSan by
 * tests/test_medit.py: every call must return 0 or 1 without memory errors
 * or leaks (the reader frees what it allocated on error).
 *   fuzz_medit <mesh> <sol> <scratch-file>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pmmg_medit.h"

static char *slurp(const char *path, long *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *b = malloc((size_t)*n + 1);
  if (fread(b, 1, (size_t)*n, f) != (size_t)*n) *n = 0;
  b[*n] = 0; /* strstr below */
  fclose(f);
  return b;
}

static void dump(const char *path, const char *b, long n) {
  FILE *f = fopen(path, "wb");
  fwrite(b, 1, (size_t)n, f);
  fclose(f);
}

static int run(const char *scratch, int is_mesh) {
  char err[256];
  if (is_mesh) {
    pmmg_medit_mesh m;
    int ok = pmmg_medit_read_mesh(scratch, &m, err, sizeof err);
    if (ok) pmmg_medit_free_mesh(&m);
    return ok;
  }
  pmmg_medit_sol s;
  int ok = pmmg_medit_read_sol(scratch, &s, err, sizeof err);
  if (ok) pmmg_medit_free_sol(&s);
  return ok;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const char *scratch = argv[3];
  long calls = 0, oks = 0;
  for (int which = 0; which < 2; which++) {
    long n;
    char *b = slurp(argv[1 + which], &n);
    if (!b || n <= 0) return 2;
    char *t = malloc((size_t)n + 64);
    for (long len = 0; len <= n; len += 1) { /* every truncation */
      dump(scratch, b, len);
      oks += run(scratch, which == 0);
      calls++;
    }
    const char repl[] = {'9', '-', '#', ' ', 'x', '\n', '0', '.'};
    for (long pos = 0; pos < n; pos += 3) /* single-byte replacements */
      for (int r = 0; r < 8; r++) {
        memcpy(t, b, (size_t)n);
        t[pos] = repl[r];
        dump(scratch, t, n);
        oks += run(scratch, which == 0);
        calls++;
      }
    /* an inflated count: the reader must stop at the end of the file */
    memcpy(t, b, (size_t)n);
    char *v = strstr(t, which == 0 ? "Vertices" : "SolAtVertices");
    if (v) {
      char *num = v + strlen(which == 0 ? "Vertices" : "SolAtVertices");
      while (*num == ' ' || *num == '\n') num++;
      if (*num >= '0' && *num <= '9') *num = '9';
      dump(scratch, t, n);
      oks += run(scratch, which == 0);
      calls++;
    }
    if (which == 0) {
      /* a vertex id past INT_MAX in the Tetrahedra block (would wrap to a
         negative int): must be rejected */
      char *tb = strstr(b, "Tetrahedra");
      if (tb) {
        char *nl = strchr(tb, '\n');
        if (nl) nl = strchr(nl + 1, '\n'); /* end of the count line */
        if (nl) {
          FILE *f = fopen(scratch, "wb");
          fwrite(b, 1, (size_t)(nl + 1 - b), f);
          fputs("4294967297 1 2 3 0\n", f);
          fwrite(nl + 1, 1, (size_t)(n - (nl + 1 - b)), f);
          fclose(f);
          const int ok = run(scratch, 1);
          printf("fuzz_medit: huge vertex id accepted=%d\n", ok);
          oks += ok;
          calls++;
        }
      }
      /* the Vertices block twice: must be rejected (no leak of the first) */
      char *vb = strstr(b, "Vertices"), *end = strstr(b, "End");
      if (vb && end && end > vb) {
        FILE *f = fopen(scratch, "wb");
        fwrite(b, 1, (size_t)(end - b), f);
        fwrite(vb, 1, (size_t)(end - vb), f);
        fputs("End\n", f);
        fclose(f);
        const int ok = run(scratch, 1);
        printf("fuzz_medit: repeated block accepted=%d\n", ok);
        oks += ok;
        calls++;
      }
    }
    free(t);
    free(b);
  }
  printf("fuzz_medit: %ld calls, %ld accepted\n", calls, oks);
  return 0;
}
