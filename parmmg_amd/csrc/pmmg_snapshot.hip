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
// the result does not depend on the atomic order.  Tetra faces (r04): the
// counting atomics are combined per wave (consecutive tetra share their
// smallest vertex), and the twins are found bucket by bucket — a block loads
// the buckets of 64 consecutive vertices into LDS with one coalesced read and
// every face scans its bucket there, writing its adjacency entry (r03: one
// thread per tetra scanning two buckets in HBM, 9.3 of the 22 ms, latency-
// bound).  Scratch buffers are kept by the context (SnapCache).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <stdio.h>

#include "pmmg_snapshot.hpp"

namespace {

constexpr int kB = 256;

// XCD-contiguous block order: hardware deals workgroup b to XCD b % 8; the
// logical block returned gives XCD x the contiguous range [x n / 8, (x + 1)
// n / 8), so the bucket / adjacency lines a tetra range writes fill in one
// XCD's L2 instead of being written in parts from all eight (bijective)
__device__ __forceinline__ long long xcd_blk() {
  const long long b = blockIdx.x, n = gridDim.x;
  const long long x = b & 7, q = n >> 3, r = n & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}


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

// cnt[idx] += val for the active lanes, returning each lane's old value plus
// the contributions of the lower lanes with the same idx: lanes with equal
// idx share one atomic (up to kAggRounds distinct idx per wave; the rest
// issue their own)
constexpr int kAggRounds = 6;
__device__ __forceinline__ int wave_add(int *cnt, int idx, int val, bool act) {
  const int lane = __lane_id();
  unsigned long long todo = __ballot(act);
  int res = 0;
#pragma unroll 1
  for (int r = 0; r < kAggRounds && todo; r++) {
    const int leader = __ffsll((long long)todo) - 1;
    const int li = __shfl(idx, leader);
    const unsigned long long m = __ballot(act && idx == li) & todo;
    int old = 0;
    if (lane == leader) old = atomicAdd(&cnt[li], val * __popcll(m));
    old = __shfl(old, leader);
    if ((m >> lane) & 1ULL) res = old + val * __popcll(m & ((1ULL << lane) - 1ULL));
    todo &= ~m;
  }
  if ((todo >> lane) & 1ULL) res = atomicAdd(&cnt[idx], val);
  return res;
}

// rank[k] = {slot of the s0 faces (3 consecutive), slot of the s1 face};
// the vertex half of the tet8 record goes out here (the adjacency half is
// written face by face by k_face_match)
__global__ __launch_bounds__(kB) void k_face_count(const int4 *tetv, int ne, int np, int *cnt, int2 *rank,
                                                   int4 *tet8, int *err) {
  const int k = (int)(xcd_blk() * kB + threadIdx.x);
  const bool in = k < ne;
  const int4 t = in ? tetv[k] : make_int4(1, 2, 3, 4);
  const bool ok = in && tet_ids_ok(t, np);
  if (in && !ok) atomicOr(err, kErrIds);
  int i0 = 0, i1 = 1;
  two_smallest(t, i0, i1);
  const int r0 = wave_add(cnt, sel(t, i0) - 1, 3, ok);
  const int r1 = wave_add(cnt, sel(t, i1) - 1, 1, ok);
  if (in) {
    rank[k] = ok ? make_int2(r0, r1) : make_int2(-1, -1);
    if (tet8) tet8[2 * (size_t)k] = t;
  }
}

__global__ __launch_bounds__(kB) void k_face_scatter(const int4 *tetv, int ne, const int *off, const int2 *rank,
                                                     int4 *bucket) {
  const int k = (int)(xcd_blk() * kB + threadIdx.x);
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

// The buckets of kMatchVerts consecutive vertices per block (contiguous
// entries), staged in LDS when they fit in kMatchCap entries, else scanned
// in place; every face writes its entry of the adjacency: its twin's code, 0
// on the boundary.  Invalid tetra (flagged by k_face_count) have no faces in
// the buckets: their rows are zeroed by k_face_invalid.
constexpr int kMatchVerts = 64, kMatchCap = 2048;
__global__ __launch_bounds__(kB) void k_face_match(int np, const int *off, const int *cnt, const int4 *bucket,
                                                   int *adja, int *tet8, int *err) {
  __shared__ int4 ent[kMatchCap];
  __shared__ int loff[kMatchVerts + 1];
  const int v0 = (int)xcd_blk() * kMatchVerts, nv = min(kMatchVerts, np - v0);
  if (threadIdx.x <= nv) loff[threadIdx.x] = threadIdx.x < nv ? off[v0 + threadIdx.x] : off[v0 + nv - 1] + cnt[v0 + nv - 1];
  __syncthreads();
  const int e0 = loff[0], n = loff[nv] - e0;
  const bool staged = n <= kMatchCap;
  if (staged)
    for (int j = threadIdx.x; j < n; j += kB) ent[j] = bucket[e0 + j];
  __syncthreads();
  const int4 *src = staged ? ent : bucket + e0;
  int bad = 0;
  for (int j = threadIdx.x; j < n; j += kB) {
    // the bucket of entry j: the last local offset <= j
    int lo = 0, hi = nv; // loff[lo] - e0 <= j < loff[hi] - e0
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (loff[mid] - e0 <= j) lo = mid;
      else hi = mid;
    }
    const int b0 = loff[lo] - e0, b1 = loff[lo + 1] - e0;
    const int4 me = src[j];
    int twin = 0, found = 0;
    for (int q = b0; q < b1; q++) {
      const int4 o = src[q];
      if (q != j && o.x == me.x && o.y == me.y) {
        if (!found) twin = o.z;
        found++;
      }
    }
    bad |= found > 1;
    const size_t k = (size_t)(me.z >> 2) - 1, i = (size_t)(me.z & 3);
    if (adja) adja[4 * k + i] = twin;
    if (tet8) tet8[8 * k + 4 + i] = twin;
  }
  if (bad) atomicOr(err, kErrNonManifold);
}

__global__ __launch_bounds__(kB) void k_face_invalid(int ne, const int2 *rank, int4 *adja, int4 *tet8) {
  const int k = blockIdx.x * kB + threadIdx.x;
  if (k >= ne || rank[k].x >= 0) return;
  if (adja) adja[k] = make_int4(0, 0, 0, 0);
  if (tet8) tet8[2 * (size_t)k + 1] = make_int4(0, 0, 0, 0);
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

// device scratch: slot i of the context's cache (grown, never shrunk), or a
// temporary freed at the end of the call when there is no cache
struct Scratch {
  SnapCache *cache;
  void *tmp[SnapCache::kSlots] = {};
  explicit Scratch(SnapCache *c) : cache(c) {}
  ~Scratch() {
    for (void *q : tmp)
      if (q) (void)hipFree(q);
  }
  template <class T>
  T *get(int slot, size_t count) {
    const size_t bytes = count * sizeof(T) > 0 ? count * sizeof(T) : 16;
    if (cache) {
      if (cache->cap[slot] < bytes) {
        if (cache->p[slot]) (void)hipFree(cache->p[slot]);
        cache->p[slot] = nullptr;
        cache->cap[slot] = 0;
        if (hipMalloc(&cache->p[slot], bytes) != hipSuccess) return nullptr;
        cache->cap[slot] = bytes;
      }
      return static_cast<T *>(cache->p[slot]);
    }
    if (tmp[slot]) (void)hipFree(tmp[slot]);
    tmp[slot] = nullptr;
    if (hipMalloc(&tmp[slot], bytes) != hipSuccess) return nullptr;
    return static_cast<T *>(tmp[slot]);
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

constexpr int kSlotScan = SnapCache::kSlots - 1;
int exclusive_scan(Scratch &S, const int *in, int *out, int n, hipStream_t s, char *msg, size_t msglen) {
  size_t tb = 0;
  SCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, s));
  void *tmp = S.get<char>(kSlotScan, tb);
  if (!tmp) { snprintf(msg, msglen, "out of device memory (scan)"); return 0; }
  SCK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, n, s));
  return 1;
}

} // namespace

int pmmg_snap_adjacency(hipStream_t s, int np, int ne, const int *tetv, int *adja, int *tet8, SnapCache *cache,
                        char *msg, size_t msglen) {
  Scratch S(cache);
  const long long nf = 4LL * ne;
  int *cnt = S.get<int>(0, (size_t)np), *off = S.get<int>(1, (size_t)np), *err = S.get<int>(2, 1);
  int2 *rank = S.get<int2>(3, (size_t)ne);
  int4 *bucket = S.get<int4>(4, (size_t)nf);
  if (!cnt || !off || !rank || !err || !bucket) {
    snprintf(msg, msglen, "build_adjacency: out of device memory (%lld faces)", nf);
    return 0;
  }
  SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
  SCK(hipMemsetAsync(err, 0, sizeof(int), s));
  const int4 *tv = reinterpret_cast<const int4 *>(tetv);
  hipLaunchKernelGGL(k_face_count, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, np, cnt, rank,
                     reinterpret_cast<int4 *>(tet8), err);
  if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
  hipLaunchKernelGGL(k_face_scatter, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, off, rank, bucket);
  hipLaunchKernelGGL(k_face_match, dim3((np + kMatchVerts - 1) / kMatchVerts), dim3(kB), 0, s, np, off, cnt, bucket,
                     adja, tet8, err);
  hipLaunchKernelGGL(k_face_invalid, dim3(blocks(ne)), dim3(kB), 0, s, ne, rank, reinterpret_cast<int4 *>(adja),
                     reinterpret_cast<int4 *>(tet8));
  SCK(hipGetLastError());
  int h_err = 0;
  SCK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  if (h_err & kErrIds) { snprintf(msg, msglen, "build_adjacency: vertex ids out of [1, np] or repeated in a tetra"); return 0; }
  if (h_err & kErrNonManifold) { snprintf(msg, msglen, "build_adjacency: a face is shared by more than two tetra"); return 0; }
  return 1;
}

void pmmg_snap_cache_free(SnapCache *c) {
  if (!c) return;
  for (int i = 0; i < SnapCache::kSlots; i++) {
    if (c->p[i]) (void)hipFree(c->p[i]);
    c->p[i] = nullptr;
    c->cap[i] = 0;
  }
}

int pmmg_snap_tria_adjacency(hipStream_t s, int np, int nt, const int *triv, int *adjt, SnapCache *cache, char *msg,
                             size_t msglen) {
  if (nt == 0) return 1;
  Scratch S(cache);
  const long long nedge = 3LL * nt;
  int *cnt = S.get<int>(0, (size_t)np), *off = S.get<int>(1, (size_t)np), *rank = S.get<int>(3, (size_t)nedge);
  int2 *bucket = S.get<int2>(4, (size_t)nedge);
  int *err = S.get<int>(2, 1);
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
                       const int *tref, int cap, int *nt_out, int *triv, int *adjt, SnapCache *cache, char *msg,
                       size_t msglen) {
  Scratch S(cache);
  int *nb = S.get<int>(5, (size_t)ne), *toff = S.get<int>(6, (size_t)ne);
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
  if (adjt && !pmmg_snap_tria_adjacency(s, np, nt, triv, adjt, cache, msg, msglen)) return 0;
  SCK(hipStreamSynchronize(s));
  return 1;
}
