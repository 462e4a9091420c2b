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
// counting atomics are combined per wave (one atomic per distinct vertex, all
// in one instruction), the bucket entries are 12 bytes, and the twins are
// found bucket by bucket — a block loads the buckets of 24 consecutive
// vertices into LDS with one coalesced read and the faces meet in an LDS hash
// table, each writing its adjacency entry (r03: one thread per tetra scanning
// two buckets in HBM, 9.3 of the 22 ms, latency-bound).  Scratch buffers are
// kept by the context (SnapCache).
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

// cnt[idx] += val for the active lanes (idx >= 0), each lane getting the old
// value plus the contributions of the lanes before it with the same idx.  The
// wave's {idx, lane} keys are bitonic-sorted across the lanes (wave_runs), the
// first lane of every run of equal idx issues the run's atomic — all runs in
// one instruction — and the ranks go back to the lanes they belong to by
// ds_permute (run_rank).  k_face_scatter issues its two reservations'
// atomics together: one round trip per wave.  (r04: the previous form took up to 7
// dependent atomic round trips per wave, one per distinct idx; the count
// kernel was latency-bound on them at 6.8 ms for 101M tetra.)
struct WaveRun {
  unsigned long long key; // this lane's sorted {idx, lane}
  int h, n;               // first lane of its run; the run's length (at the first lane)
  bool head, valid;
};
constexpr unsigned long long kIdle = ~0ULL >> 6; // sorts after every idx, lane bits kept distinct

__device__ __forceinline__ WaveRun wave_runs(int idx, bool act) {
  const int lane = __lane_id();
  unsigned long long key = ((act ? (unsigned long long)(unsigned)idx : kIdle) << 6) | (unsigned)lane;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const unsigned long long o = __shfl_xor(key, j);
      const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
      key = keep_min ? (o < key ? o : key) : (o > key ? o : key);
    }
  }
  WaveRun w;
  w.key = key;
  const unsigned long long sid = key >> 6, prev = __shfl_up(sid, 1);
  w.valid = sid != kIdle;
  w.head = w.valid && (lane == 0 || prev != sid);
  const unsigned long long heads = __ballot(w.head), nvalid = __popcll(__ballot(w.valid));
  const unsigned long long le = lane == 63 ? ~0ULL : ((2ULL << lane) - 1ULL);
  w.h = 63 - __clzll((long long)(heads & le)); // valid lanes only
  const unsigned long long after = heads & ~le;
  w.n = (after ? __ffsll((long long)after) - 1 : (int)nvalid) - lane;
  return w;
}

// `old`: the atomic's result at the run's first lane
__device__ __forceinline__ int run_rank(const WaveRun &w, int old, int val) {
  const int lane = __lane_id();
  old = __shfl(old, w.valid ? w.h : lane);
  // back to the lane the key came from (a push: every lane receives exactly one value)
  return __builtin_amdgcn_ds_permute((int)(w.key & 63) << 2, old + val * (lane - w.h));
}

// The bucket sizes: per tetra, 3 faces in the bucket of its smallest vertex,
// 1 in that of the second smallest, counted with no-return atomics (r04: the
// slots themselves are taken in k_face_scatter, so nothing waits on these
// atomics and no per-tetra rank goes through memory).  The vertex half of
// the tet8 record goes out here (the adjacency half is written face by face
// by k_face_match).
__global__ __launch_bounds__(kB) void k_face_count(const int4 *tetv, int ne, int np, int *cnt, int4 *tet8, int *err) {
  const int k = (int)(xcd_blk() * kB + threadIdx.x);
  const bool in = k < ne;
  const int4 t = in ? tetv[k] : make_int4(1, 2, 3, 4);
  const bool ok = in && tet_ids_ok(t, np);
  if (in && !ok) atomicOr(err, kErrIds);
  int i0 = 0, i1 = 1;
  two_smallest(t, i0, i1);
  const WaveRun w0 = wave_runs(sel(t, i0) - 1, ok), w1 = wave_runs(sel(t, i1) - 1, ok);
  if (w0.head) atomicAdd(&cnt[(int)(w0.key >> 6)], 3 * w0.n);
  if (w1.head) atomicAdd(&cnt[(int)(w1.key >> 6)], w1.n);
  if (in && tet8) tet8[2 * (size_t)k] = t;
}

// The faces into their buckets: slots taken from the buckets' cursors
// (initialised to the offsets) with one atomic round trip per wave.  An
// invalid tetra (flagged by k_face_count) gets a zero adjacency row here and
// has no faces in the buckets.
__global__ __launch_bounds__(kB) void k_face_scatter(const int4 *tetv, int ne, int np, int *cursor, int3 *bucket,
                                                     int4 *adja, int4 *tet8) {
  const int k = (int)(xcd_blk() * kB + threadIdx.x);
  const bool in = k < ne;
  const int4 t = in ? tetv[k] : make_int4(1, 2, 3, 4);
  const bool ok = in && tet_ids_ok(t, np);
  int i0 = 0, i1 = 1;
  two_smallest(t, i0, i1);
  const WaveRun w0 = wave_runs(sel(t, i0) - 1, ok), w1 = wave_runs(sel(t, i1) - 1, ok);
  int c0 = 0, c1 = 0;
  if (w0.head) c0 = atomicAdd(&cursor[(int)(w0.key >> 6)], 3 * w0.n);
  if (w1.head) c1 = atomicAdd(&cursor[(int)(w1.key >> 6)], w1.n);
  const int o0 = run_rank(w0, c0, 3), o1 = run_rank(w1, c1, 1);
  if (!in) return;
  if (!ok) {
    if (adja) adja[k] = make_int4(0, 0, 0, 0);
    if (tet8) tet8[2 * (size_t)k + 1] = make_int4(0, 0, 0, 0);
    return;
  }
  int n = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int a, b, c;
    face_ids(t, i, a, b, c);
    // code of this face in the reference encoding: 4*k + i with k 1-based
    const int3 e = make_int3(b, c, 4 * (k + 1) + i);
    if (i == i0) bucket[o1] = e; // face opposite s0: bucket of s1
    else bucket[o0 + n++] = e;
  }
}

// The buckets of kMatchVerts consecutive vertices per block (contiguous
// entries), staged in LDS when they fit in kMatchCap entries, else scanned
// in place; every face writes its entry of the adjacency: its twin's code, 0
// on the boundary.  Invalid tetra (flagged by k_face_count) have no faces in
// the buckets: their rows are zeroed by k_face_scatter.
//
// r04: in LDS the twins meet in a hash table keyed by {bucket, b, c} — each
// entry probes ~1-2 slots — instead of every entry scanning its whole bucket
// (~24 entries of 16 bytes: 6.7 ms of LDS reads for 404M faces at cfg4).
// The later of two twins finds the earlier in the table and pairs them with a
// compare-and-swap on the earlier's mate; a third face with the same key
// finds the mate taken (non-manifold).  Blocks whose buckets exceed
// kMatchCap entries scan them in place.
constexpr int kMatchVerts = 24, kMatchCap = 768, kHashSlots = 1024; // 17 KB of LDS: 8 blocks per CU
__device__ __forceinline__ int bucket_of(const int *loff, int nv, int e0, int j) {
  int lo = 0, hi = nv; // loff[lo] - e0 <= j < loff[hi] - e0
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (loff[mid] - e0 <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void put_adja(int *adja, int *tet8, int code, int twin) {
  const size_t k = (size_t)(code >> 2) - 1, i = (size_t)(code & 3);
  if (adja) adja[4 * k + i] = twin;
  if (tet8) tet8[8 * k + 4 + i] = twin;
}

// One block per chunk of kMatchVerts vertices, in XCD-contiguous order.
// (r04: persistent blocks loading the next chunk's entries while matching
// the current one took 3.79 against 3.30 ms, r04u.)
__global__ __launch_bounds__(kB) void k_face_match(int np, const int *off, const int *cnt, const int3 *bucket,
                                                   int *adja, int *tet8, int *err) {
  __shared__ int3 ent[kMatchCap];         // {b, c, code}
  __shared__ unsigned char lb[kMatchCap]; // local bucket
  __shared__ int slot[kHashSlots], mate[kMatchCap];
  __shared__ int loff[kMatchVerts + 1];
  const int v0 = (int)xcd_blk() * kMatchVerts, nv = min(kMatchVerts, np - v0);
  if (threadIdx.x <= nv) loff[threadIdx.x] = threadIdx.x < nv ? off[v0 + threadIdx.x] : off[v0 + nv - 1] + cnt[v0 + nv - 1];
  __syncthreads();
  const int e0 = loff[0], n = loff[nv] - e0;
  int bad = 0;
  if (n <= kMatchCap) {
    for (int j = threadIdx.x; j < n; j += kB) {
      ent[j] = bucket[e0 + j];
      lb[j] = (unsigned char)bucket_of(loff, nv, e0, j);
      mate[j] = -1;
    }
    for (int h = threadIdx.x; h < kHashSlots; h += kB) slot[h] = -1;
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += kB) {
      const int3 me = ent[j];
      const int mb = lb[j];
      unsigned h = ((unsigned)mb * 0x9E3779B1u) ^ ((unsigned)me.x * 0x85EBCA77u) ^ ((unsigned)me.y * 0xC2B2AE3Du);
      h = (h ^ (h >> 15)) & (kHashSlots - 1);
      for (;;) {
        const int q = atomicCAS(&slot[h], -1, j);
        if (q < 0) break; // first of its key: inserted
        const int3 o = ent[q];
        if (o.x == me.x && o.y == me.y && lb[q] == mb) {
          if (atomicCAS(&mate[q], -1, j) == -1) mate[j] = q;
          else bad = 1; // a third face with this key
          break;
        }
        h = (h + 1) & (kHashSlots - 1);
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += kB) {
      const int m = mate[j];
      put_adja(adja, tet8, ent[j].z, m >= 0 ? ent[m].z : 0);
    }
  } else {
    const int3 *src = bucket + e0;
    for (int j = threadIdx.x; j < n; j += kB) {
      const int b = bucket_of(loff, nv, e0, j);
      const int b0 = loff[b] - e0, b1 = loff[b + 1] - e0;
      const int3 me = src[j];
      int twin = 0, found = 0;
      for (int q = b0; q < b1; q++) {
        const int3 o = src[q];
        if (q != j && o.x == me.x && o.y == me.y) {
          if (!found) twin = o.z;
          found++;
        }
      }
      bad |= found > 1;
      put_adja(adja, tet8, me.z, twin);
    }
  }
  if (bad) atomicOr(err, kErrNonManifold);
}

// (r04: writing the twins in bucket order and the rows by a per-tetra gather
// took 0.3 ms longer than the match's own 4-byte stores)

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

__device__ __forceinline__ int bdy_faces(const int4 &a, int k, const int *tref) {
  return bdy_face(a.x, k, tref) + bdy_face(a.y, k, tref) + bdy_face(a.z, k, tref) + bdy_face(a.w, k, tref);
}

// block-wide exclusive prefix of v (kB threads), and the block's total
__device__ __forceinline__ int block_prefix(int v, int *wsum, int &total) {
  const int lane = __lane_id(), w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int j = 0; j < kB / 64; j++) {
    before += j < w ? wsum[j] : 0;
    total += wsum[j];
  }
  __syncthreads();
  return before + x - v;
}

// Pass 1 over the tetra (r04): per block of kB tetra, its boundary faces'
// count and its tetra with any, compacted in tetra order into the block's
// own kB slots of cand (boundary tetra are few: pass 2 reads only those
// instead of every tetra's adjacency again; r03 wrote and scanned a count per
// tetra, then re-read all of them)
__global__ __launch_bounds__(kB) void k_bdy_count(const int4 *adja, int astride, const int *tref, int ne, int *cand,
                                                  int *btot, int *bcnt) {
  __shared__ int wsum[kB / 64];
  const int k = blockIdx.x * kB + threadIdx.x;
  const int nb = k < ne ? bdy_faces(adja[(size_t)k * astride], k, tref) : 0;
  // one prefix over {candidate flag, face count} (<= 256 and <= 1024 per block)
  int tot = 0;
  const int pos = block_prefix(((nb > 0) << 16) | nb, wsum, tot) >> 16;
  if (nb > 0) cand[(size_t)blockIdx.x * kB + pos] = k;
  if (threadIdx.x == 0) {
    btot[blockIdx.x] = tot & 0xFFFF;
    bcnt[blockIdx.x] = tot >> 16;
  }
}

// Pass 2: the trias of a block's candidate tetra at the block's offset
__global__ __launch_bounds__(kB) void k_bdy_write(const int4 *tetv, int tstride, const int4 *adja, int astride,
                                                  const int *tref, const int *cand, const int *bcnt, const int *boff,
                                                  int *triv) {
  __shared__ int wsum[kB / 64];
  const int n = bcnt[blockIdx.x];
  if (n == 0) return; // block-uniform
  const bool in = (int)threadIdx.x < n;
  const int k = in ? cand[(size_t)blockIdx.x * kB + threadIdx.x] : 0;
  const int4 a = in ? adja[(size_t)k * astride] : make_int4(1, 1, 1, 1);
  const int nb = in ? bdy_faces(a, k, tref) : 0;
  int tot = 0;
  int pos = boff[blockIdx.x] + block_prefix(nb, wsum, tot);
  if (!in) return;
  const int4 t = tetv[(size_t)k * tstride];
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
  int *cursor = S.get<int>(3, (size_t)np);
  int3 *bucket = S.get<int3>(4, (size_t)nf); // {b, c, code} of every face
  if (!cnt || !off || !cursor || !err || !bucket) {
    snprintf(msg, msglen, "build_adjacency: out of device memory (%lld faces)", nf);
    return 0;
  }
  SCK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)np, s));
  SCK(hipMemsetAsync(err, 0, sizeof(int), s));
  const int4 *tv = reinterpret_cast<const int4 *>(tetv);
  hipLaunchKernelGGL(k_face_count, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, np, cnt, reinterpret_cast<int4 *>(tet8),
                     err);
  if (!exclusive_scan(S, cnt, off, np, s, msg, msglen)) return 0;
  SCK(hipMemcpyAsync(cursor, off, sizeof(int) * (size_t)np, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_face_scatter, dim3(blocks(ne)), dim3(kB), 0, s, tv, ne, np, cursor, bucket,
                     reinterpret_cast<int4 *>(adja), reinterpret_cast<int4 *>(tet8));
  hipLaunchKernelGGL(k_face_match, dim3((np + kMatchVerts - 1) / kMatchVerts), dim3(kB), 0, s, np, off, cnt, bucket,
                     adja, tet8, err);
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
  const int nblk = blocks(ne);
  int *cand = S.get<int>(5, (size_t)nblk * kB), *bs = S.get<int>(6, 3 * (size_t)nblk);
  if (!cand || !bs) { snprintf(msg, msglen, "build_boundary: out of device memory"); return 0; }
  int *btot = bs, *bcnt = bs + nblk, *boff = bs + 2 * (size_t)nblk;
  const int4 *tv = reinterpret_cast<const int4 *>(tetv), *ad = reinterpret_cast<const int4 *>(adja);
  hipLaunchKernelGGL(k_bdy_count, dim3(nblk), dim3(kB), 0, s, ad, astride, tref, ne, cand, btot, bcnt);
  if (!exclusive_scan(S, btot, boff, nblk, s, msg, msglen)) return 0;
  int last[2] = {0, 0};
  SCK(hipMemcpyAsync(&last[0], boff + nblk - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipMemcpyAsync(&last[1], btot + nblk - 1, sizeof(int), hipMemcpyDeviceToHost, s));
  SCK(hipStreamSynchronize(s));
  const int nt = last[0] + last[1];
  *nt_out = nt;
  if (nt > cap) { snprintf(msg, msglen, "build_boundary: %d boundary trias exceed the capacity %d", nt, cap); return 0; }
  if (nt == 0) return 1;
  hipLaunchKernelGGL(k_bdy_write, dim3(nblk), dim3(kB), 0, s, tv, tstride, ad, astride, tref, (const int *)cand,
                     (const int *)bcnt, (const int *)boff, triv);
  SCK(hipGetLastError());
  if (adjt && !pmmg_snap_tria_adjacency(s, np, nt, triv, adjt, cache, msg, msglen)) return 0;
  SCK(hipStreamSynchronize(s));
  return 1;
}
