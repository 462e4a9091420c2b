// pmmg_snapshot.hip — background snapshot on the device.
//
// ParMmg takes a copy of each group before remeshing it, PMMG_create_oldGrp
// (reference src/grpsplit_pmmg.c:207-418): tetra, adjacency, points and
// solutions are copied, then the boundary trias of the old mesh are rebuilt
// (MMG5_chkBdryTria, :404) and hashed for the tria adjacency adjt
// (MMG3D_hashTria, :410).  The adjacency itself comes from MMG3D_hashTetra
// (called e.g. at src/libparmmg1.c:495,730).  Those three host O(ne) steps
// feed the transfer step (PMMG_interpMetricsAndFields) its `adja`, `triv`,
// `adjt`; here they run on the GPU from the connectivity alone, so a
// connectivity uploaded (or produced) on the device never needs a host-side
// hash or a re-upload of the derived arrays.
//
// Conventions (Mmg @889d408, restated, not pinned: Mmg is absent from the
// image): face i of tetra k is the face opposite vertex i; adja[4(k-1)+i] =
// 4k'+i' for the tetra k' sharing it, 0 on the boundary; boundary trias are
// the faces with adja == 0 in (tetra, face) order, vertices v[MMG5_idir[i]]
// (outward for positively oriented tetra); adjt[3(t-1)+j] = 3t'+j' for the
// tria sharing edge j (the edge opposite local vertex j), 0 on borders and on
// edges shared by more than two trias.
//
// Algorithm (both hashes): bucket every face (edge) under its smallest vertex
// id — count with atomics, exclusive scan, scatter {other ids, code} — then
// each face (edge) scans its own bucket (~24 faces per vertex in a tetra
// mesh) for its twin.  The match is a pure function of the connectivity, so
// the result does not depend on the atomic order.  Everything is a stream of
// the connectivity plus small L2-resident bucket scans: HBM-bound.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <stdio.h>

#include "pmmg_snapshot.hpp"

namespace {

constexpr int kB = 256;

__constant__ int kIdirS[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};

__device__ __forceinline__ int sel(const int4 &t, int i) { return i == 0 ? t.x : (i == 1 ? t.y : (i == 2 ? t.z : t.w)); }

// sorted vertex ids of face i of a tetra
__device__ __forceinline__ void face_ids(const int4 &t, int i, int &a, int &b, int &c) {
  int u = sel(t, kIdirS[i][0]), v = sel(t, kIdirS[i][1]), w = sel(t, kIdirS[i][2]);
  int lo = min(u, min(v, w)), hi = max(u, max(v, w));
  a = lo;
  c = hi;
  b = u + v + w - lo - hi;
}

// error bits
constexpr int kErrIds = 1, kErrNonManifold = 2;

__global__ __launch_bounds__(kB) void k_face_count(const int4 *tetv, int ne, int np, int *cnt, int *rank,
                                                   int *err) {
  const long long f = blockIdx.x * (long long)kB + threadIdx.x;
  if (f >= 4LL * ne) return;
  const int4 t = tetv[f >> 2];
  int a, b, c;
  face_ids(t, (int)(f & 3), a, b, c);
  if (a < 1 || c > np || a == b || b == c) {
    atomicOr(err, kErrIds);
    rank[f] = -1;
    return;
  }
  rank[f] = atomicAdd(&cnt[a - 1], 1);
}

__global__ __launch_bounds__(kB) void k_face_scatter(const int4 *tetv, int ne, const int *off, const int *rank,
                                                     int4 *bucket) {
  const long long f = blockIdx.x * (long long)kB + threadIdx.x;
  if (f >= 4LL * ne) return;
  const int r = rank[f];
  if (r < 0) return;
  const int4 t = tetv[f >> 2];
  int a, b, c;
  face_ids(t, (int)(f & 3), a, b, c);
  // code of this face in the reference encoding: 4*k + i with k 1-based
  bucket[off[a - 1] + r] = make_int4(b, c, (int)(4 * ((f >> 2) + 1) + (f & 3)), 0);
}

// one thread per tetra: the 4 twins, one adjacency row (and one tet8 record)
__global__ __launch_bounds__(kB) void k_face_match(const int4 *tetv, int ne, const int *off, const int *cnt,
                                                   const int4 *bucket, int4 *adja, int4 *tet8, int *err) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 t = tetv[k];
  int code[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int a, b, c;
    face_ids(t, i, a, b, c);
    code[i] = 0;
    if (a < 1) continue; // flagged by k_face_count
    const int self = 4 * (k + 1) + i;
    const int lo = off[a - 1], n = cnt[a - 1];
    int found = 0;
    for (int j = 0; j < n; j++) {
      const int4 e = bucket[lo + j];
      if (e.x == b && e.y == c && e.z != self) {
        if (!found) code[i] = e.z;
        found++;
      }
    }
    if (found > 1) atomicOr(err, kErrNonManifold);
  }
  const int4 row = make_int4(code[0], code[1], code[2], code[3]);
  if (adja) adja[k] = row;
  if (tet8) {
    tet8[2 * (size_t)k] = t;
    tet8[2 * (size_t)k + 1] = row;
  }
}

// ---- boundary trias

__global__ __launch_bounds__(kB) void k_bdy_count(const int4 *adja, int astride, int ne, int *nb) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 a = adja[(size_t)k * astride];
  nb[k] = (a.x == 0) + (a.y == 0) + (a.z == 0) + (a.w == 0);
}

__global__ __launch_bounds__(kB) void k_bdy_write(const int4 *tetv, int tstride, const int4 *adja, int astride, int ne,
                                                  const int *toff, int *triv) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 a = adja[(size_t)k * astride];
  if (a.x && a.y && a.z && a.w) return;
  const int4 t = tetv[(size_t)k * tstride];
  int pos = toff[k];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (sel(a, i)) continue;
#pragma unroll
    for (int l = 0; l < 3; l++) triv[3 * (size_t)pos + l] = sel(t, kIdirS[i][l]);
    pos++;
  }
}

__device__ __forceinline__ void edge_ids(const int *triv, long long e, int &lo, int &hi) {
  const long long t = e / 3;
  const int i = (int)(e % 3);
  const int va = triv[3 * t + (i + 1) % 3], vb = triv[3 * t + (i + 2) % 3];
  lo = min(va, vb);
  hi = max(va, vb);
}

__global__ __launch_bounds__(kB) void k_edge_count(const int *triv, int nt, int np, int *cnt, int *rank, int *err) {
  const long long e = blockIdx.x * (long long)kB + threadIdx.x;
  if (e >= 3LL * nt) return;
  int lo, hi;
  edge_ids(triv, e, lo, hi);
  if (lo < 1 || hi > np || lo == hi) {
    atomicOr(err, kErrIds);
    rank[e] = -1;
    return;
  }
  rank[e] = atomicAdd(&cnt[lo - 1], 1);
}

__global__ __launch_bounds__(kB) void k_edge_scatter(const int *triv, int nt, const int *off, const int *rank,
                                                     int2 *bucket) {
  const long long e = blockIdx.x * (long long)kB + threadIdx.x;
  if (e >= 3LL * nt) return;
  const int r = rank[e];
  if (r < 0) return;
  int lo, hi;
  edge_ids(triv, e, lo, hi);
  bucket[off[lo - 1] + r] = make_int2(hi, (int)(3 * (e / 3 + 1) + e % 3));
}

// twin of each tria edge: paired only when exactly two trias share the edge
__global__ __launch_bounds__(kB) void k_edge_match(const int *triv, int nt, const int *off, const int *cnt,
                                                   const int2 *bucket, int *adjt) {
  const long long e = blockIdx.x * (long long)kB + threadIdx.x;
  if (e >= 3LL * nt) return;
  int lo, hi;
  edge_ids(triv, e, lo, hi);
  int code = 0;
  if (lo >= 1) {
    const int self = (int)(3 * (e / 3 + 1) + e % 3);
    const int b = off[lo - 1], n = cnt[lo - 1];
    int other = 0, same = 0;
    for (int j = 0; j < n; j++) {
      const int2 x = bucket[b + j];
      if (x.x == hi) {
        same++;
        if (x.y != self) other = x.y;
      }
    }
    code = same == 2 ? other : 0;
  }
  adjt[e] = code;
}

int blocks(long long n) { return (int)((n + kB - 1) / kB > 0 ? (n + kB - 1) / kB : 1); }

struct Scratch {
  static constexpr int kMax = 16;
  void *p[kMax] = {};
  int n = 0;
  ~Scratch() {
    for (int i = 0; i < n; i++) (void)hipFree(p[i]);
  }
  template <class T>
  T *get(size_t count) {
    if (n >= kMax) return nullptr;
    void *q = nullptr;
    if (hipMalloc(&q, count * sizeof(T) > 0 ? count * sizeof(T) : 16) != hipSuccess) return nullptr;
    p[n++] = q;
    return static_cast<T *>(q);
  }
};

#define SCK(expr)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) {                                                                         \
      snprintf(msg, msglen, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return 0;                                                                                     \
    }                                                                                               \
  } while (0)

int exclusive_scan(Scratch &S, const int *in, int *out, int n, hipStream_t s, char *msg, size_t msglen) {
  size_t tb = 0;
  SCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, s));
  void *tmp = S.get<char>(tb);
  if (!tmp) { snprintf(msg, msglen, "out of device memory (scan)"); return 0; }
  SCK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, n, s));
  return 1;
}

} // namespace

int pmmg_snap_adjacency(hipStream_t s, int np, int ne, const int *tetv, int *adja, int *tet8, char *msg,
                        size_t msglen) {
  Scratch S;
  const long long nf = 4LL * ne;
  int *cnt = S.get<int>((size_t)np), *off = S.get<int>((size_t)np), *rank = S.get<int>((size_t)nf),
      *err = S.get<int>(1);
  int4 *bucket = S.get<int4>((size_t)nf);
  if (!cnt || !off || !rank || !err || !bucket) {
    snprintf(msg, msglen, "build_adjacency: out of device memory (%lld faces)", nf);
    return 0;
  }
  SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
  SCK(hipMemsetAsync(err, 0, sizeof(int), s));
  const int4 *tv = reinterpret_cast<const int4 *>(tetv);
  hipLaunchKernelGGL(k_face_count, dim3(blocks(nf)), dim3(kB), 0, s, tv, ne, np, cnt, rank, err);
  if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
  hipLaunchKernelGGL(k_face_scatter, dim3(blocks(nf)), dim3(kB), 0, s, tv, ne, off, rank, bucket);
  hipLaunchKernelGGL(k_face_match, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, off, cnt, bucket,
                     reinterpret_cast<int4 *>(adja), reinterpret_cast<int4 *>(tet8), err);
  SCK(hipGetLastError());
  int h_err = 0;
  SCK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  if (h_err & kErrIds) { snprintf(msg, msglen, "build_adjacency: vertex ids out of [1, np] or repeated in a tetra"); return 0; }
  if (h_err & kErrNonManifold) { snprintf(msg, msglen, "build_adjacency: a face is shared by more than two tetra"); return 0; }
  return 1;
}

int pmmg_snap_boundary(hipStream_t s, int np, int ne, const int *tetv, int tstride, const int *adja, int astride,
                       int cap, int *nt_out, int *triv, int *adjt, char *msg, size_t msglen) {
  Scratch S;
  int *nb = S.get<int>((size_t)ne), *toff = S.get<int>((size_t)ne), *err = S.get<int>(1);
  if (!nb || !toff || !err) { snprintf(msg, msglen, "build_boundary: out of device memory"); return 0; }
  const int4 *tv = reinterpret_cast<const int4 *>(tetv), *ad = reinterpret_cast<const int4 *>(adja);
  hipLaunchKernelGGL(k_bdy_count, dim3(blocks(ne)), dim3(kB), 0, s, ad, astride, ne, nb);
  if (!exclusive_scan(S, nb, toff, ne, s, msg, msglen)) return 0;
  int last[2] = {0, 0};
  SCK(hipMemcpyAsync(&last[0], toff + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipMemcpyAsync(&last[1], nb + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  const int nt = last[0] + last[1];
  *nt_out = nt;
  if (nt > cap) { snprintf(msg, msglen, "build_boundary: %d boundary trias exceed the capacity %d", nt, cap); return 0; }
  if (nt == 0) return 1;
  hipLaunchKernelGGL(k_bdy_write, dim3(blocks(ne)), dim3(kB), 0, s, tv, tstride, ad, astride, ne, toff, triv);
  if (adjt) {
    const long long nedge = 3LL * nt;
    int *cnt = S.get<int>((size_t)np), *off = S.get<int>((size_t)np), *rank = S.get<int>((size_t)nedge);
    int2 *bucket = S.get<int2>((size_t)nedge);
    if (!cnt || !off || !rank || !bucket) { snprintf(msg, msglen, "build_boundary: out of device memory"); return 0; }
    SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
    SCK(hipMemsetAsync(err, 0, sizeof(int), s));
    hipLaunchKernelGGL(k_edge_count, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, np, cnt, rank, err);
    if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
    hipLaunchKernelGGL(k_edge_scatter, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, off, rank, bucket);
    hipLaunchKernelGGL(k_edge_match, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, off, cnt, bucket, adjt);
  }
  SCK(hipGetLastError());
  SCK(hipStreamSynchronize(s));
  return 1;
}
