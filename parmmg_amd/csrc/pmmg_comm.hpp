// pmmg_comm.hpp — the split of one group over the node's GPUs, C-level
// (included by pmmg_hip.hip only; SURVEY.md §8(e), BASELINE north_star: "Located element ids and
// interpolated values are collected with RCCL all-gather over xGMI").
//
// One process per GPU (ParMmg's MPI ranks, GPU = node-local rank,
// src/parmmg.c:121): every rank transfers its part of the new points, then
// one ncclAllGather collects {K doubles, element id, hit code} per point on
// every rank.  RCCL is loaded at the first communicator call (dlopen of
// librccl.so.1, the ROCm library or the copy a host process such as PyTorch
// has already loaded: the same soname), so libpmmg_hip.so itself needs no
// RCCL to load and a caller that never splits a group never touches it.
//
// All-gather of unequal parts: each rank packs its points' rows into records
// of R = 8 K + 8 bytes (K doubles, int32 element, int8 hit, padding) in a
// send buffer of max_r counts[r] records, one ncclAllGather of that many
// bytes per rank (ring over xGMI), then one kernel unpacks every rank's
// records into the rank-order concatenation of the caller's output arrays.
#pragma once

#include <dlfcn.h>
#include <rccl/rccl.h> // types only: the functions are taken from the dlopen'ed library

namespace pmmg {

struct Rccl {
  bool tried = false, ok = false;
  char why[256] = {0};
  decltype(&::ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&::ncclCommInitRank) commInitRank = nullptr;
  decltype(&::ncclCommDestroy) commDestroy = nullptr;
  decltype(&::ncclAllGather) allGather = nullptr;
  decltype(&::ncclGetErrorString) errorString = nullptr;
};

// the process's RCCL entry points (loaded once; dlopen is thread-safe, the
// races of two contexts' first calls only repeat the same lookups)
inline Rccl &rccl() {
  static Rccl R;
  if (R.tried) return R;
  void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    snprintf(R.why, sizeof(R.why), "librccl.so.1 not found: %s", dlerror());
  } else {
    R.getUniqueId = (decltype(R.getUniqueId))dlsym(h, "ncclGetUniqueId");
    R.commInitRank = (decltype(R.commInitRank))dlsym(h, "ncclCommInitRank");
    R.commDestroy = (decltype(R.commDestroy))dlsym(h, "ncclCommDestroy");
    R.allGather = (decltype(R.allGather))dlsym(h, "ncclAllGather");
    R.errorString = (decltype(R.errorString))dlsym(h, "ncclGetErrorString");
    R.ok = R.getUniqueId && R.commInitRank && R.commDestroy && R.allGather && R.errorString;
    if (!R.ok) snprintf(R.why, sizeof(R.why), "librccl.so.1 lacks the NCCL entry points");
  }
  R.tried = true;
  return R;
}

// record layout of the all-gather: the slots' rows (nslot of size[s]
// doubles), then the element id and the hit code
struct AgSlots {
  const double *in[kMaxSlot];
  double *out[kMaxSlot];
  int size[kMaxSlot];
  int n;
  int K; // doubles per record
};

__global__ __launch_bounds__(kBlock) void k_ag_pack(AgSlots S, const int *elem, const int8_t *hit, long long n,
                                                    char *send) {
  const long long R = 8LL * S.K + 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    double *row = reinterpret_cast<double *>(send + R * i);
    int o = 0;
    for (int s = 0; s < S.n; s++)
      for (int j = 0; j < S.size[s]; j++) row[o++] = S.in[s][(size_t)S.size[s] * i + j];
    int *tail = reinterpret_cast<int *>(row + S.K);
    tail[0] = elem ? elem[i] : 0;
    tail[1] = hit ? (int)hit[i] : 0;
  }
}

// rank r's records at recv + r * maxn * R -> output rows off[r] .. off[r] + cnt[r]
__global__ __launch_bounds__(kBlock) void k_ag_unpack(AgSlots S, const char *recv, long long maxn, int nranks,
                                                      const long long *off, int *elem_all, int8_t *hit_all) {
  const long long R = 8LL * S.K + 8, total = off[nranks];
  for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < total;
       g += (long long)gridDim.x * blockDim.x) {
    int r = 0;
    while (off[r + 1] <= g) r++; // ranks are few
    const long long i = g - off[r];
    const double *row = reinterpret_cast<const double *>(recv + R * ((long long)r * maxn + i));
    int o = 0;
    for (int s = 0; s < S.n; s++)
      for (int j = 0; j < S.size[s]; j++) S.out[s][(size_t)S.size[s] * g + j] = row[o++];
    const int *tail = reinterpret_cast<const int *>(row + S.K);
    if (elem_all) elem_all[g] = tail[0];
    if (hit_all) hit_all[g] = (int8_t)tail[1];
  }
}

} // namespace pmmg
