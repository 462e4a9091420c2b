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

// The faces of a tetra whose sorted vertices are s0 < s1 < s2 < s3: the
// three faces containing s0 (opposite s1, s2, s3) share the bucket of s0, the
// face opposite s0 is in the bucket of s1.  One atomic reserves the three
// slots in s0's bucket, one the slot in s1's; one scan of s0's bucket serves
// all three faces in the match.

// local index (0..3) of the smallest and second smallest vertex of a tetra
__device__ __forceinline__ void two_smallest(const int4 &t, int &i0, int &i1) {
  int v[4] = {t.x, t.y, t.z, t.w};
  i0 = 0;
#pragma unroll
  for (int i = 1; i < 4; i++) i0 = v[i] < v[i0] ? i : i0;
  i1 = i0 == 0 ? 1 : 0;
#pragma unroll
  for (int i = 0; i < 4; i++) i1 = (i != i0 && v[i] < v[i1]) ? i : i1;
}

__device__ __forceinline__ bool tet_ids_ok(const int4 &t, int np) {
  const int v[4] = {t.x, t.y, t.z, t.w};
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    ok = ok && v[i] >= 1 && v[i] <= np;
#pragma unroll
    for (int j = i + 1; j < 4; j++) ok = ok && v[i] != v[j];
  }
  return ok;
}

// rank[k] = {slot of the s0 faces (3 consecutive), slot of the s1 face}
__global__ __launch_bounds__(kB) void k_face_count(const int4 *tetv, int ne, int np, int *cnt, int2 *rank,
                                                   int *err) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 t = tetv[k];
  if (!tet_ids_ok(t, np)) {
    atomicOr(err, kErrIds);
    rank[k] = make_int2(-1, -1);
    return;
  }
  int i0, i1;
  two_smallest(t, i0, i1);
  const int r0 = atomicAdd(&cnt[sel(t, i0) - 1], 3);
  const int r1 = atomicAdd(&cnt[sel(t, i1) - 1], 1);
  rank[k] = make_int2(r0, r1);
}

__global__ __launch_bounds__(kB) void k_face_scatter(const int4 *tetv, int ne, const int *off, const int2 *rank,
                                                     int4 *bucket) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int2 r = rank[k];
  if (r.x < 0) return;
  const int4 t = tetv[k];
  int i0, i1;
  two_smallest(t, i0, i1);
  int n = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int a, b, c;
    face_ids(t, i, a, b, c);
    // code of this face in the reference encoding: 4*k + i with k 1-based
    const int4 e = make_int4(b, c, 4 * (k + 1) + i, 0);
    if (i == i0) bucket[off[a - 1] + r.y] = e; // face opposite s0: bucket of s1
    else bucket[off[a - 1] + r.x + n++] = e;
  }
}

// one thread per tetra: the 4 twins, one adjacency row (and one tet8 record)
__global__ __launch_bounds__(kB) void k_face_match(const int4 *tetv, int ne, int np, const int *off, const int *cnt,
                                                   const int4 *bucket, int4 *adja, int4 *tet8, int *err) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 t = tetv[k];
  int code[4] = {0, 0, 0, 0};
  if (tet_ids_ok(t, np)) { // invalid tetra were flagged by k_face_count
    int i0, i1;
    two_smallest(t, i0, i1);
    int fb[4], fc[4], found[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int a;
      face_ids(t, i, a, fb[i], fc[i]);
    }
    // bucket of s0: the three faces other than i0; bucket of s1: face i0
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
      const int v = pass == 0 ? sel(t, i0) : sel(t, i1);
      const int lo = off[v - 1], n = cnt[v - 1];
      for (int j = 0; j < n; j++) {
        const int4 e = bucket[lo + j];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          if ((i == i0) != (pass == 1)) continue;
          if (e.x == fb[i] && e.y == fc[i] && e.z != 4 * (k + 1) + i) {
            if (!found[i]) code[i] = e.z;
            found[i]++;
          }
        }
      }
    }
    if (found[0] > 1 || found[1] > 1 || found[2] > 1 || found[3] > 1) atomicOr(err, kErrNonManifold);
  }
  const int4 row = make_int4(code[0], code[1], code[2], code[3]);
  if (adja) adja[k] = row;
  if (tet8) {
    tet8[2 * (size_t)k] = t;
    tet8[2 * (size_t)k + 1] = row;
  }
}

// ---- boundary trias
//
// A face is a boundary tria when it has no neighbour, or (with tetra
// references, a multi-material mesh) when the neighbour's reference is
// smaller than the tetra's: MMG5_chkBdryTria's rule for an old mesh without
// input trias (adj == 0 || pt->ref > pt1->ref), restated from Mmg @889d408
// (absent from the image: unpinned), each interface face emitted once, from
// the tetra of the larger reference, oriented by MMG5_idir.

__device__ __forceinline__ bool bdy_face(int code, int k, const int *tref) {
  if (code == 0) return true;
  return tref && tref[k] > tref[(code >> 2) - 1];
}

__global__ __launch_bounds__(kB) void k_bdy_count(const int4 *adja, int astride, const int *tref, int ne, int *nb) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 a = adja[(size_t)k * astride];
  nb[k] = bdy_face(a.x, k, tref) + bdy_face(a.y, k, tref) + bdy_face(a.z, k, tref) + bdy_face(a.w, k, tref);
}

__global__ __launch_bounds__(kB) void k_bdy_write(const int4 *tetv, int tstride, const int4 *adja, int astride,
                                                  const int *tref, int ne, const int *toff, int *triv) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne) return;
  const int4 a = adja[(size_t)k * astride];
  if (!tref && a.x && a.y && a.z && a.w) return;
  const int4 t = tetv[(size_t)k * tstride];
  int pos = toff[k];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (!bdy_face(sel(a, i), k, tref)) continue;
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
  int *cnt = S.get<int>((size_t)np), *off = S.get<int>((size_t)np), *err = S.get<int>(1);
  int2 *rank = S.get<int2>((size_t)ne);
  int4 *bucket = S.get<int4>((size_t)nf);
  if (!cnt || !off || !rank || !err || !bucket) {
    snprintf(msg, msglen, "build_adjacency: out of device memory (%lld faces)", nf);
    return 0;
  }
  SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
  SCK(hipMemsetAsync(err, 0, sizeof(int), s));
  const int4 *tv = reinterpret_cast<const int4 *>(tetv);
  hipLaunchKernelGGL(k_face_count, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, np, cnt, rank, err);
  if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
  hipLaunchKernelGGL(k_face_scatter, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, off, rank, bucket);
  hipLaunchKernelGGL(k_face_match, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, np, off, cnt, bucket,
                     reinterpret_cast<int4 *>(adja), reinterpret_cast<int4 *>(tet8), err);
  SCK(hipGetLastError());
  int h_err = 0;
  SCK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  if (h_err & kErrIds) { snprintf(msg, msglen, "build_adjacency: vertex ids out of [1, np] or repeated in a tetra"); return 0; }
  if (h_err & kErrNonManifold) { snprintf(msg, msglen, "build_adjacency: a face is shared by more than two tetra"); return 0; }
  return 1;
}

int pmmg_snap_tria_adjacency(hipStream_t s, int np, int nt, const int *triv, int *adjt, char *msg, size_t msglen) {
  if (nt == 0) return 1;
  Scratch S;
  const long long nedge = 3LL * nt;
  int *cnt = S.get<int>((size_t)np), *off = S.get<int>((size_t)np), *rank = S.get<int>((size_t)nedge);
  int2 *bucket = S.get<int2>((size_t)nedge);
  int *err = S.get<int>(1);
  if (!cnt || !off || !rank || !bucket || !err) {
    snprintf(msg, msglen, "tria adjacency: out of device memory");
    return 0;
  }
  SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
  SCK(hipMemsetAsync(err, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_edge_count, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, np, cnt, rank, err);
  if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
  hipLaunchKernelGGL(k_edge_scatter, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, off, rank, bucket);
  hipLaunchKernelGGL(k_edge_match, dim3(blocks(nedge)), dim3(kB), 0, s, triv, nt, off, cnt, bucket, adjt);
  SCK(hipGetLastError());
  int h_err = 0;
  SCK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  if (h_err) {
    snprintf(msg, msglen, "tria adjacency: tria vertex ids out of [1, np]");
    return 0;
  }
  return 1;
}

int pmmg_snap_boundary(hipStream_t s, int np, int ne, const int *tetv, int tstride, const int *adja, int astride,
                       const int *tref, int cap, int *nt_out, int *triv, int *adjt, char *msg, size_t msglen) {
  Scratch S;
  int *nb = S.get<int>((size_t)ne), *toff = S.get<int>((size_t)ne);
  if (!nb || !toff) { snprintf(msg, msglen, "build_boundary: out of device memory"); return 0; }
  const int4 *tv = reinterpret_cast<const int4 *>(tetv), *ad = reinterpret_cast<const int4 *>(adja);
  hipLaunchKernelGGL(k_bdy_count, dim3(blocks(ne)), dim3(kB), 0, s, ad, astride, tref, ne, nb);
  if (!exclusive_scan(S, nb, toff, ne, s, msg, msglen)) return 0;
  int last[2] = {0, 0};
  SCK(hipMemcpyAsync(&last[0], toff + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipMemcpyAsync(&last[1], nb + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  const int nt = last[0] + last[1];
  *nt_out = nt;
  if (nt > cap) { snprintf(msg, msglen, "build_boundary: %d boundary trias exceed the capacity %d", nt, cap); return 0; }
  if (nt == 0) return 1;
  hipLaunchKernelGGL(k_bdy_write, dim3(blocks(ne)), dim3(kB), 0, s, tv, tstride, ad, astride, tref, ne, toff, triv);
  SCK(hipGetLastError());
  if (adjt && !pmmg_snap_tria_adjacency(s, np, nt, triv, adjt, msg, msglen)) return 0;
  SCK(hipStreamSynchronize(s));
  return 1;
}
