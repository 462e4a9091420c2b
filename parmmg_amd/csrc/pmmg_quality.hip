// pmmg_quality.hip — element quality of the adapted mesh in its interpolated
// metric, on the device.
//
// PMMG_tetraQual (reference src/quality_pmmg.c:720-733, called right after
// the transfer at src/libparmmg1.c:845 with metRidTyp = 1) runs Mmg's
// MMG3D_tetraQual per group: pt->qual of every used tetra, and the group's
// minimum scaled by MMG3D_ALPHAD; a zero minimum fails the call.  With
// metRidTyp = 1 the quality is MMG5_orcal -> MMG5_caltet: the geometric
// MMG5_caltet_iso without an aniso metric, MMG5_caltet_ani (metric averaged
// over the 4 vertices) with one.  Mmg @889d408 is not in the image: the
// formulas below restate its published source (parity unpinned, like the
// rest of the Mmg boundary), with the same operation order as
// the oracle's restatement (oracle/pmmg_oracle.c orc_caltet_*), so both are
// bit-identical under -ffp-contract=off.
//
// The metric stays where the transfer wrote it (device rows, reference
// layout): quality and minimum need no D2H of the metric.  One lane per
// tetra; HBM-bound: 16 B tetv + 8 B qual per tetra plus 4 vertex rows
// (24 + 8*met_size B) that neighbouring tetra share through L2.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "pmmg_quality.hpp"

namespace {

constexpr int kQBlock = 256;
constexpr double kEPSD2 = 1.0e-200; // MMG5_EPSD2
constexpr double kEPSOK = 1.0e-20;  // MMG5_EPSOK

__device__ __forceinline__ double caltet_iso(const double *a, const double *b, const double *c, const double *d) {
  const double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  const double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  const double adx = d[0] - a[0], ady = d[1] - a[1], adz = d[2] - a[2];
  const double v1 = acy * adz - acz * ady;
  const double v2 = acz * adx - acx * adz;
  const double v3 = acx * ady - acy * adx;
  const double vol = abx * v1 + aby * v2 + abz * v3;
  if (vol < kEPSD2) return 0.0;
  const double bcx = c[0] - b[0], bcy = c[1] - b[1], bcz = c[2] - b[2];
  const double bdx = d[0] - b[0], bdy = d[1] - b[1], bdz = d[2] - b[2];
  const double cdx = d[0] - c[0], cdy = d[1] - c[1], cdz = d[2] - c[2];
  double rap = abx * abx + aby * aby + abz * abz;
  rap += acx * acx + acy * acy + acz * acz;
  rap += adx * adx + ady * ady + adz * adz;
  rap += bcx * bcx + bcy * bcy + bcz * bcz;
  rap += bdx * bdx + bdy * bdy + bdz * bdz;
  rap += cdx * cdx + cdy * cdy + cdz * cdz;
  if (rap < kEPSD2) return 0.0;
  rap = rap * sqrt(rap);
  return vol / rap;
}

__device__ __forceinline__ double metlen(const double *mm, double x, double y, double z) {
  return mm[0] * x * x + mm[3] * y * y + mm[5] * z * z + 2.0 * (mm[1] * x * y + mm[2] * x * z + mm[4] * y * z);
}

__device__ __forceinline__ double caltet_ani(const double *a, const double *b, const double *c, const double *d,
                                             const double *mm) {
  const double abx = b[0] - a[0], aby = b[1] - a[1], abz = b[2] - a[2];
  const double acx = c[0] - a[0], acy = c[1] - a[1], acz = c[2] - a[2];
  const double adx = d[0] - a[0], ady = d[1] - a[1], adz = d[2] - a[2];
  const double v1 = acy * adz - acz * ady;
  const double v2 = acz * adx - acx * adz;
  const double v3 = acx * ady - acy * adx;
  const double vol = abx * v1 + aby * v2 + abz * v3;
  if (vol <= 0.0) return 0.0;
  double det = mm[0] * (mm[3] * mm[5] - mm[4] * mm[4]) - mm[1] * (mm[1] * mm[5] - mm[2] * mm[4]) +
               mm[2] * (mm[1] * mm[4] - mm[2] * mm[3]);
  if (det < kEPSOK) return 0.0;
  det = sqrt(det) * vol;
  const double bcx = c[0] - b[0], bcy = c[1] - b[1], bcz = c[2] - b[2];
  const double bdx = d[0] - b[0], bdy = d[1] - b[1], bdz = d[2] - b[2];
  const double cdx = d[0] - c[0], cdy = d[1] - c[1], cdz = d[2] - c[2];
  const double h1 = metlen(mm, abx, aby, abz), h2 = metlen(mm, acx, acy, acz), h3 = metlen(mm, adx, ady, adz);
  const double h4 = metlen(mm, bcx, bcy, bcz), h5 = metlen(mm, bdx, bdy, bdz), h6 = metlen(mm, cdx, cdy, cdz);
  const double rap = h1 + h2 + h3 + h4 + h5 + h6;
  const double num = sqrt(rap) * rap;
  return det / num;
}

// qual[k] for every tetra (0 for unused ones: v[0] <= 0, MG_EOK false) and the
// minimum over used tetra as the bit pattern of a non-negative double
// (ordered like the value) in *minbits.
__global__ __launch_bounds__(kQBlock) void k_tetra_qual(const double *xyz, int ne, const int4 *tetv, int ani,
                                                        const double *met, double *qual, unsigned long long *minbits) {
  __shared__ unsigned long long wmin[kQBlock / 64];
  unsigned long long mine = ~0ULL;
  const int stride = gridDim.x * blockDim.x;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ne; k += stride) {
    const int4 v = tetv[k];
    double q = 0.0;
    if (v.x > 0) {
      const int id[4] = {v.x, v.y, v.z, v.w};
      double p[4][3];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) p[i][j] = xyz[3 * (size_t)(id[i] - 1) + j];
      if (ani) {
        double mm[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int j = 0; j < 6; j++) mm[j] += met[6 * (size_t)(id[i] - 1) + j];
#pragma unroll
        for (int j = 0; j < 6; j++) mm[j] *= 0.25;
        q = caltet_ani(p[0], p[1], p[2], p[3], mm);
      } else {
        q = caltet_iso(p[0], p[1], p[2], p[3]);
      }
      const unsigned long long b = (unsigned long long)__double_as_longlong(q);
      mine = b < mine ? b : mine;
    }
    __builtin_nontemporal_store(q, qual + k);
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(mine, o);
    mine = other < mine ? other : mine;
  }
  if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = wmin[0];
    for (int w = 1; w < kQBlock / 64; w++) m = wmin[w] < m ? wmin[w] : m;
    if (m != ~0ULL) atomicMin(minbits, m);
  }
}

// ---------------------------------------------------------------- metis weights
//
// PMMG_computeWgt (src/metis_pmmg.c:280-300): weight of a tetra face from the
// lengths of its three edges in the metric (MMG5_lenedg = MMG5_lenedgCoor_iso
// / MMG5_lenedgCoor_ani of Mmg @889d408, restated; aniso ridge-point storage
// not modelled), the load-balancing weight of the faces on parallel
// interfaces.  Same operation order as oracle/pmmg_oracle.c orc_face_wgt;
// exp / log1p are the device library's (within an ulp of the host's).
constexpr double kHugeWgt = 1000000.0; // PMMG_WGTVAL_HUGEINT
constexpr double kMmgEps = 1.0e-06;    // MMG5_EPS
__constant__ int kIare[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}}; // MMG5_iare
__constant__ int kIarf[4][3] = {{5, 4, 3}, {5, 1, 2}, {4, 2, 0}, {3, 0, 1}};     // MMG5_iarf

__device__ __forceinline__ double lenedg_iso(const double *ca, const double *cb, double h1, double h2) {
  double l = (cb[0] - ca[0]) * (cb[0] - ca[0]) + (cb[1] - ca[1]) * (cb[1] - ca[1]) + (cb[2] - ca[2]) * (cb[2] - ca[2]);
  l = sqrt(l);
  const double r = h2 / h1 - 1.0;
  return (fabs(r) < kMmgEps) ? (l / h1) : (l / (h2 - h1) * log1p(r));
}

__device__ __forceinline__ double lenedg_ani(const double *ca, const double *cb, const double *sa, const double *sb) {
  const double ux = cb[0] - ca[0], uy = cb[1] - ca[1], uz = cb[2] - ca[2];
  double dd1 = sa[0] * ux * ux + sa[3] * uy * uy + sa[5] * uz * uz + 2.0 * (sa[1] * ux * uy + sa[2] * ux * uz + sa[4] * uy * uz);
  if (dd1 <= 0.0) dd1 = 0.0;
  double dd2 = sb[0] * ux * ux + sb[3] * uy * uy + sb[5] * uz * uz + 2.0 * (sb[1] * ux * uy + sb[2] * ux * uz + sb[4] * uy * uz);
  if (dd2 <= 0.0) dd2 = 0.0;
  if (fabs(dd1 - dd2) < 0.05) return sqrt(0.5 * (dd1 + dd2));
  return (sqrt(dd1) + sqrt(dd2) + 4.0 * sqrt(0.5 * (dd1 + dd2))) / 6.0;
}

__device__ double face_wgt(const double *xyz, const int *v, int ifac, int met_size, const double *met) {
  if (met_size != 1 && met_size != 6) return kHugeWgt;
  double res = 0.0;
  for (int i = 0; i < 3; i++) {
    const int ia = kIarf[ifac][i];
    const int ip1 = v[kIare[ia][0]], ip2 = v[kIare[ia][1]];
    const double *ca = xyz + 3 * (size_t)(ip1 - 1), *cb = xyz + 3 * (size_t)(ip2 - 1);
    const double len = met_size == 1 ? lenedg_iso(ca, cb, met[ip1 - 1], met[ip2 - 1])
                                     : lenedg_ani(ca, cb, met + 6 * (size_t)(ip1 - 1), met + 6 * (size_t)(ip2 - 1));
    if (len <= 1.0)
      res += len - 1.0;
    else
      res += 1.0 / len - 1.0;
  }
  const double w = 1.0 / exp(28.0 * res / 3.0);
  return w < kHugeWgt ? w : kHugeWgt;
}

// PMMG_computeWgt_mesh: qual[k] = sum over the faces of k tagged `tag` of the
// face weight, for used tetra with an xtetra; the others keep qual[k]
__global__ __launch_bounds__(kQBlock) void k_wgt_mesh(const double *xyz, int ne, const int4 *tetv, const int *xt,
                                                      const uint16_t *ftag, int met_size, const double *met, int tag,
                                                      double *qual) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ne; k += gridDim.x * blockDim.x) {
    const int4 t = tetv[k];
    if (t.x <= 0 || !xt[k]) continue;
    const int v[4] = {t.x, t.y, t.z, t.w};
    const ushort4 ft = reinterpret_cast<const ushort4 *>(ftag)[k];
    const int f4[4] = {ft.x, ft.y, ft.z, ft.w};
    double q = 0.0;
    for (int f = 0; f < 4; f++)
      if (f4[f] & tag) q += face_wgt(xyz, v, f, met_size, met);
    qual[k] = q;
  }
}

// the weights of a list of (tetra, face) pairs (the graph weights of
// src/metis_pmmg.c:812, :959): face[2j] = tetra (1-based), face[2j+1] = ifac
__global__ __launch_bounds__(kQBlock) void k_wgt_faces(const double *xyz, const int4 *tetv, int nface,
                                                       const int2 *face, int met_size, const double *met,
                                                       double *wgt) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nface; j += gridDim.x * blockDim.x) {
    const int2 fj = face[j];
    const int4 t = tetv[fj.x - 1];
    const int v[4] = {t.x, t.y, t.z, t.w};
    wgt[j] = face_wgt(xyz, v, fj.y, met_size, met);
  }
}

} // namespace

int pmmg_qual_tetra(hipStream_t s, int np, const double *xyz, int ne, const int *tetv, int met_size,
                    const double *met, double *qual, unsigned long long *d_minbits, unsigned long long *h_minbits) {
  (void)np;
  if (hipMemsetAsync(d_minbits, 0xff, sizeof(unsigned long long), s) != hipSuccess) return 0;
  if (ne > 0) {
    const int need = (ne + kQBlock - 1) / kQBlock;
    const int blocks = need < 8 * 256 * 8 ? need : 8 * 256 * 8; // grid-stride beyond 16K blocks
    hipLaunchKernelGGL(k_tetra_qual, dim3(blocks), dim3(kQBlock), 0, s, xyz, ne,
                       reinterpret_cast<const int4 *>(tetv), met_size == 6 ? 1 : 0, met, qual, d_minbits);
    if (hipGetLastError() != hipSuccess) return 0;
  }
  if (hipMemcpyAsync(h_minbits, d_minbits, sizeof(unsigned long long), hipMemcpyDeviceToHost, s) != hipSuccess)
    return 0;
  return hipStreamSynchronize(s) == hipSuccess;
}

int pmmg_wgt_mesh(hipStream_t s, const double *xyz, int ne, const int *tetv, const int *xt, const uint16_t *ftag,
                  int met_size, const double *met, int tag, double *qual) {
  if (ne > 0) {
    const int need = (ne + kQBlock - 1) / kQBlock;
    hipLaunchKernelGGL(k_wgt_mesh, dim3(need < 16384 ? need : 16384), dim3(kQBlock), 0, s, xyz, ne,
                       reinterpret_cast<const int4 *>(tetv), xt, ftag, met_size, met, tag, qual);
    if (hipGetLastError() != hipSuccess) return 0;
  }
  return hipStreamSynchronize(s) == hipSuccess;
}

int pmmg_wgt_faces(hipStream_t s, const double *xyz, const int *tetv, int nface, const int *face, int met_size,
                   const double *met, double *wgt) {
  if (nface > 0) {
    const int need = (nface + kQBlock - 1) / kQBlock;
    hipLaunchKernelGGL(k_wgt_faces, dim3(need < 16384 ? need : 16384), dim3(kQBlock), 0, s, xyz,
                       reinterpret_cast<const int4 *>(tetv), nface, reinterpret_cast<const int2 *>(face), met_size,
                       met, wgt);
    if (hipGetLastError() != hipSuccess) return 0;
  }
  return hipStreamSynchronize(s) == hipSuccess;
}
