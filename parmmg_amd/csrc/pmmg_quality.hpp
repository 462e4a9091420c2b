// pmmg_quality.hpp — internal interface of pmmg_quality.hip (tetra quality in
// the interpolated metric); the C-ABI wrapper lives in pmmg_hip.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// qual[ne] and the minimum over used tetra (bit pattern of a non-negative
// double, all ones when no tetra is used) in *h_minbits; device pointers
// except h_minbits (pinned or pageable host).  Synchronous.  Returns 1/0.
int pmmg_qual_tetra(hipStream_t s, int np, const double *xyz, int ne, const int *tetv, int met_size,
                    const double *met, double *qual, unsigned long long *d_minbits, unsigned long long *h_minbits);

// PMMG_computeWgt_mesh / PMMG_computeWgt on device arrays (tetv, ftag 16-byte /
// 8-byte aligned); synchronous; 1/0
int pmmg_wgt_mesh(hipStream_t s, const double *xyz, int ne, const int *tetv, const int *xt, const uint16_t *ftag,
                  int met_size, const double *met, int tag, double *qual);
int pmmg_wgt_faces(hipStream_t s, const double *xyz, const int *tetv, int nface, const int *face, int met_size,
                   const double *met, double *wgt);
