// Brick renumbering of the background — a measurement, not part of the
// transfer.
//
// A brick-resident volume stage (a workgroup stages one spatial brick's tetra
// records, vertex rows and solution rows into LDS with coalesced loads, then
// walks and interpolates its queries from there) needs each brick's data
// contiguous in HBM.  The caller's background is in the caller's numbering,
// so every call would first renumber it by bricks:
//   1. one brick key per vertex and per tetra (brick of the seed grid's cell
//      holding the vertex / the centroid, Morton order of the bricks);
//   2. both lists sorted by brick (rocPRIM's stable radix sort);
//   3. the inverse permutations;
//   4. vertex rows (fixed-point, fp64, every solution slot) gathered into
//      brick order, tetra records gathered with their vertex ids and
//      adjacencies renumbered.
// PMMG_HIP_BRICK=b (cells per brick edge, a power of two) enqueues exactly
// this on the main stream between the seed grid and the volume kernel, whose
// inputs it leaves untouched: the step's extra time is the floor a brick
// path starts from, before any of its walking.
#pragma once

namespace pmmg {

__device__ __forceinline__ unsigned brick_key(const Frame *fr, const double p[3], int g, int lb) {
  uint32_t b[3];
#pragma unroll
  for (int d = 0; d < 3; d++) b[d] = (uint32_t)seed_cell(seed_pos(fr, d, p[d], g), g) >> lb;
  return (expand10(b[0]) << 2) | (expand10(b[1]) << 1) | expand10(b[2]);
}

__device__ __forceinline__ void xq_point(const Bg &bg, const Frame *fr, int v, double p[3], double w) {
  const int *q = bg.xq + kXqStride * (size_t)(v - 1);
#pragma unroll
  for (int d = 0; d < 3; d++) p[d] += w * (fr->qc[d] + (double)q[d] / fr->qs);
}

__global__ __launch_bounds__(kBlock) void k_brick_vkeys(Bg bg, const Frame *fr, int g, int lb, unsigned *keys,
                                                        int *vals) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < bg.np; i += (long long)gridDim.x * blockDim.x) {
    double p[3] = {0.0, 0.0, 0.0};
    xq_point(bg, fr, (int)(i + 1), p, 1.0);
    keys[i] = brick_key(fr, p, g, lb);
    vals[i] = (int)i;
  }
}

__global__ __launch_bounds__(kBlock) void k_brick_tkeys(Bg bg, const Frame *fr, int g, int lb, unsigned *keys,
                                                        int *vals) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < bg.ne; i += (long long)gridDim.x * blockDim.x) {
    const int4 tv = tetv_row(bg, (int)(i + 1));
    double p[3] = {0.0, 0.0, 0.0};
    unsigned key = 0u;
    if (tv.x > 0) {
      xq_point(bg, fr, tv.x, p, 0.25);
      xq_point(bg, fr, tv.y, p, 0.25);
      xq_point(bg, fr, tv.z, p, 0.25);
      xq_point(bg, fr, tv.w, p, 0.25);
      key = brick_key(fr, p, g, lb);
    }
    keys[i] = key;
    vals[i] = (int)i;
  }
}

__global__ __launch_bounds__(kBlock) void k_brick_inv(const int *perm, long long n, int *inv) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    inv[perm[i]] = (int)i;
}

// vertex rows in brick order: fixed-point and fp64 coordinates
__global__ __launch_bounds__(kBlock) void k_brick_vrows(Bg bg, const int *vperm, int *xq_b, double *xyz_b) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < bg.np; i += (long long)gridDim.x * blockDim.x) {
    const size_t v = (size_t)vperm[i];
#pragma unroll
    for (int d = 0; d < kXqStride; d++) xq_b[kXqStride * i + d] = bg.xq[kXqStride * v + d];
#pragma unroll
    for (int d = 0; d < 3; d++) xyz_b[3 * i + d] = bg.xyz[3 * v + d];
  }
}

// one solution slot's rows in brick order, one double per thread (a row's
// pieces in neighbouring lanes)
__global__ __launch_bounds__(kBlock) void k_brick_srows(const double *in, int istride, int code, const int *vperm,
                                                        long long np, double *out) {
  const long long n = np * code;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x) {
    const long long i = j / code;
    const int r = (int)(j - i * code);
    out[j] = in[(size_t)istride * vperm[i] + r];
  }
}

// tetra records {v[4], adja[4]} in brick order, both renumbered
__global__ __launch_bounds__(kBlock) void k_brick_trec(Bg bg, const int *tperm, const int *vinv, const int *tinv,
                                                       int4 *rec_b) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < bg.ne; i += (long long)gridDim.x * blockDim.x) {
    const int k = tperm[i] + 1;
    int4 tv = tetv_row(bg, k), ad = adja_row(bg, k);
    if (tv.x > 0) {
      tv = make_int4(vinv[tv.x - 1] + 1, vinv[tv.y - 1] + 1, vinv[tv.z - 1] + 1, vinv[tv.w - 1] + 1);
      int a[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
      for (int f = 0; f < 4; f++)
        if (a[f] > 0) a[f] = 4 * (tinv[(a[f] >> 2) - 1] + 1) + (a[f] & 3);
      ad = make_int4(a[0], a[1], a[2], a[3]);
    }
    rec_b[2 * i] = tv;
    rec_b[2 * i + 1] = ad;
  }
}

} // namespace pmmg
