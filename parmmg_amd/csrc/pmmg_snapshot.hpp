// pmmg_snapshot.hpp — internal interface of pmmg_snapshot.hip (background
// snapshot on the device); the C-ABI wrappers live in pmmg_hip.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

// Device scratch of the snapshot kernels kept between calls (owned by a
// context; hipMalloc / hipFree of the GB-sized face buckets every call cost
// milliseconds and synchronise the device).  NULL: temporaries.
struct SnapCache {
  static constexpr int kSlots = 8;
  void *p[kSlots] = {};
  size_t cap[kSlots] = {};
};
void pmmg_snap_cache_free(SnapCache *c);

// adja[4*ne] (may be NULL) and/or tet8[8*ne] (may be NULL) from tetv[4*ne];
// all device pointers, 16-byte aligned.  Returns 1, or 0 with msg set.
int pmmg_snap_adjacency(hipStream_t s, int np, int ne, const int *tetv, int *adja, int *tet8, SnapCache *cache,
                        char *msg, size_t msglen);

// boundary trias (faces with adja == 0, or towards a smaller tetra reference
// when tref[ne] is given) and their adjacency.  Tetra rows are int4 rows
// `tstride` / `astride` int4s apart (1: separate arrays, 2: tet8).
int pmmg_snap_boundary(hipStream_t s, int np, int ne, const int *tetv, int tstride, const int *adja, int astride,
                       const int *tref, int cap, int *nt_out, int *triv, int *adjt, SnapCache *cache, char *msg,
                       size_t msglen);

// adjt[3*nt] of given trias (MMG3D_hashTria: 3*t'+j' across edge j, 0 on
// borders and on edges of more than two trias).  Synchronous.
int pmmg_snap_tria_adjacency(hipStream_t s, int np, int nt, const int *triv, int *adjt, SnapCache *cache, char *msg,
                             size_t msglen);
