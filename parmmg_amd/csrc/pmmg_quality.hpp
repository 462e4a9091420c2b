// pmmg_quality.hpp — internal interface of pmmg_quality.hip (tetra quality in
// the interpolated metric); the C-ABI wrapper lives in pmmg_hip.hip.
#pragma once
#include <hip/hip_runtime.h>

// qual[ne] and the minimum over used tetra (bit pattern of a non-negative
// double, all ones when no tetra is used) in *h_minbits; device pointers
// except h_minbits (pinned or pageable host).  Synchronous.  Returns 1/0.
int pmmg_qual_tetra(hipStream_t s, int np, const double *xyz, int ne, const int *tetv, int met_size,
                    const double *met, double *qual, unsigned long long *d_minbits, unsigned long long *h_minbits);
