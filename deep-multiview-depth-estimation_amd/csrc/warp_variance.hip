// warp_variance.hip -- the unfused pieces of the reference API.
//
//   warp_kernel      homography.py:6-92 as the reference returns it: warped[N][C][D][h][w]
//                    (homography_warping); one thread per output pixel of one (sample, plane),
//                    every view and channel, direct bilinear gathers from the NCHW features.
//   variance_kernel  costvolume.py:3-16 on a materialised warped volume: two-pass population
//                    variance over the V views.
// The model uses the fused kernel (cost_volume_fwd.hip) instead of this pair.
#include "launchers.h"

namespace mvs {
namespace {

// warp only: warped[i][c][kk][p] for every image i of sample b
template <int MAXV, bool EXACT, int CU>
__global__ __launch_bounds__(kBlock) void warp_kernel(const float* __restrict__ feat,
                                                      const float* __restrict__ sampling,
                                                      float* __restrict__ warped, int nv_rt, int C,
                                                      int h, int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode_flat(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  const bool active = p < hw;
  float xn, yn;
  pixel_coords(active ? p : 0u, w, h, xn, yn);
  for (int v = 0; v < V; ++v) {
    const int i = it.b * V + v;
    Taps tp;
    make_taps(sampling + ((size_t)i * Dc + it.kk) * 9, xn, yn, h, w, tp);
    const float* fb = feat + (size_t)i * C * hw;
    float* ob = warped + ((size_t)i * C * Dc + it.kk) * hw;
    for (int c0 = 0; c0 < C; c0 += CU) {
      float val[CU];
#pragma unroll
      for (int cu = 0; cu < CU; ++cu)
        if (c0 + cu < C) val[cu] = gather(fb + (size_t)(c0 + cu) * hw, tp);
#pragma unroll
      for (int cu = 0; cu < CU; ++cu)
        if (c0 + cu < C && active) ob[(size_t)(c0 + cu) * Dc * hw + p] = val[cu];
    }
  }
}

// costvolume.py:3-16 on a materialised warped volume; M = C * D * h * w elements per image.
__global__ __launch_bounds__(kBlock) void variance_kernel(const float* __restrict__ warped,
                                                          int B, int V, size_t M,
                                                          float* __restrict__ cv) {
  const ViewDiv vd = view_div(V);
  const size_t n = (size_t)B * M;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (size_t)gridDim.x * kBlock) {
    const size_t b = e / M, m = e - b * M;
    const float* x = warped + b * V * M + m;
    float val[MVS_MAX_VIEWS];
#pragma unroll
    for (int v = 0; v < MVS_MAX_VIEWS; ++v) val[v] = v < V ? x[(size_t)v * M] : 0.0f;
    cv[e] = variance_law<MVS_MAX_VIEWS>(val, V, vd);
  }
}

}  // namespace

void launch_warp(const Geometry& g, const float* feat, const float* sampling, float* warped,
                 hipStream_t s) {
  hipLaunchKernelGGL((warp_kernel<MVS_MAX_VIEWS, false, 4>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, sampling, warped, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
}

void launch_variance(const float* warped, int B, int V, size_t M, float* cv, hipStream_t s) {
  const size_t n = (size_t)B * M;
  const size_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(variance_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(kBlock),
                     0, s, warped, B, V, M, cv);
}

}  // namespace mvs
