// common.h -- device/host helpers shared by the MVSNet cost-volume kernels (gfx950 / CDNA4).
//
// Sampling law (scripts/homography.py:83-90 -> kornia 0.6.3 warp_perspective ->
// torch grid_sample(bilinear, zeros, align_corners=False)):
//   xn = (x / (w-1) - 0.5) * 2                         kornia create_meshgrid (normalised)
//   [u, v, s] = G [xn, yn, 1]                           G = inv(Nrm H Nrm^-1), per (image, plane)
//   (u, v) *= 1 / (s + 1e-8)   where |s| > 1e-8          kornia convert_points_from_homogeneous
//   ix = (u + 1) * (w / 2) - 0.5                         grid_sample unnormalise (align_corners=False)
//   out = sum of the 4 bilinear taps, taps outside the image contribute 0
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/mvs_cost_volume.h"

namespace mvs {

constexpr int kBlock = 256;
constexpr uint32_t kInvalidTap = 0xFFFFFFFFu;

// ------------------------------------------------------------------------------------------
// sampling coordinates, one inline definition for every call site -- every view, every kernel.
// Every rounding step is the reference's torch CPU one, pinned bit for bit against torch in
// tests/test_oracle.py::test_sampling_law_is_torch_cpu_bitwise (contraction is off inside these
// helpers, and every fused step is an explicit fma, so the result never depends on what the
// compiler chooses to fuse):
//   * kornia transform_points -> torch.bmm ([h, w, 3] x [3, 3] per image; MKL sgemm, k-ordered fma
//     accumulation, for every w >= 45 -- all real feature widths; torch's own loop for 9 w < 400):
//       u = fma(yn, G1, xn * G0) + G2
//   * kornia convert_points_from_homogeneous: u * (1 / (s + 1e-8)) where |s| > 1e-8
//   * grid_sample(align_corners=False) unnormalise, ATen GridSamplerKernel.cpp (vectorised, fma):
//       ix = fma(u + 1, w / 2, -0.5)
// ------------------------------------------------------------------------------------------
__device__ inline float norm_coord(uint32_t x, int size) {
#pragma clang fp contract(off)
  return ((float)x / (float)(size - 1) - 0.5f) * 2.0f;   // kornia create_meshgrid (normalised)
}

__device__ inline void sample_coord(const float* __restrict__ G, float xn, float yn, int h, int w,
                                    float& ix, float& iy) {
#pragma clang fp contract(off)
  float u = __builtin_fmaf(yn, G[1], xn * G[0]) + G[2];
  float v = __builtin_fmaf(yn, G[4], xn * G[3]) + G[5];
  const float s = __builtin_fmaf(yn, G[7], xn * G[6]) + G[8];
  // selects, not a branch: the division runs on every lane and |s| <= 1e-8 keeps (u, v)
  const bool div = fabsf(s) > 1e-8f;
  const float sc = 1.0f / (s + 1e-8f);
  u = div ? u * sc : u;
  v = div ? v * sc : v;
  ix = __builtin_fmaf(u + 1.0f, 0.5f * (float)w, -0.5f);
  iy = __builtin_fmaf(v + 1.0f, 0.5f * (float)h, -0.5f);
}

// grid_sample's bilinear sum as torch CPU forms it: nw * t0, then fma over ne, sw, se (the
// vectorised kernel's fused multiply-adds; zero taps add exactly nothing)
__device__ inline float bilerp_sum(float t0, float t1, float t2, float t3, const float (&wt)[4]) {
#pragma clang fp contract(off)
  return __builtin_fmaf(t3, wt[3], __builtin_fmaf(t2, wt[2], __builtin_fmaf(t1, wt[1], t0 * wt[0])));
}

// ------------------------------------------------------------------------------------------
// costvolume.py:12-14 as torch CPU rounds it (pinned in tests/test_oracle.py): the view sum in view
// order, mean = sum / V and cv = (sum of (x - mean) * (x - mean) in view order) / V, every product
// and sum rounded on its own and both divisions correctly rounded.  x / V is formed as
// q = x * r, q + fma(x - q V, r) (r = RN(1 / V), the remainder exact by fma): the correctly rounded
// quotient for every normal fp32 x >= 2^-124 and V = 2..16, and for every x when V is odd or a power of
// two, checked exhaustively (tests/test_exact_division.py); one multiply and two fmas instead of the IEEE
// division sequence.  For even V = 2^k m (m odd, k, m > 1: 6, 10, 12, 14) a quotient in the subnormal
// range can be an exact tie between two subnormals, where the fma's rounding of q + e r (r inexact) falls
// on the wrong side: lanes with |x| < 2^-120 take the IEEE division then -- a wave-uniform
// launch flag, so V = 3, 5 (and every odd V) never test for it.
// ------------------------------------------------------------------------------------------
struct ViewDiv {
  float v, r;   // V and RN(1 / V)
  int tie;      // V even and not a power of two: tiny quotients take the IEEE division
};

__host__ __device__ inline ViewDiv view_div(int V) {
  return ViewDiv{(float)V, 1.0f / (float)V, (V % 2 == 0 && (V & (V - 1)) != 0) ? 1 : 0};
}

__device__ inline float div_views(float x, ViewDiv d) {
#pragma clang fp contract(off)
  const float q = x * d.r;
  float y = __builtin_fmaf(__builtin_fmaf(-q, d.v, x), d.r, q);
  if (d.tie && __builtin_expect(__builtin_fabsf(x) < 0x1p-120f, 0)) y = x / d.v;   // IEEE, correctly rounded
  return y;
}

// the variance of one element over V <= MAXV views x[0 .. V) (scalar form of packed.h variance_law4)
template <int MAXV>
__device__ inline float variance_law(const float (&x)[MAXV], int V, ViewDiv vd) {
#pragma clang fp contract(off)
  float sum = x[0];
#pragma unroll
  for (int v = 1; v < MAXV; ++v)
    if (v < V) sum += x[v];
  const float mean = div_views(sum, vd);
  float acc = 0.0f;
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) {
      const float dlt = x[v] - mean;
      acc = v == 0 ? dlt * dlt : acc + dlt * dlt;
    }
  return div_views(acc, vd);
}

// Compact tap state: integer corner (x0, y0) packed as ((y0 + 2) << 16) | (x0 + 2) plus the two
// fractions.  Positions whose 4 taps all fall outside the image (ix < -1, ix >= w, ...) are
// kInvalidTap: their sample is exactly 0.  Valid corners satisfy x0 in [-1, w-1], y0 in [-1, h-1].
__device__ inline void src_coords(const float* __restrict__ G, float xn, float yn, int h, int w,
                                  bool active, uint32_t& pos, float& wx, float& wy) {
  float ix, iy;
  sample_coord(G, xn, yn, h, w, ix, iy);
  const bool ok = active && ix >= -1.0f && ix < (float)w && iy >= -1.0f && iy < (float)h;
  const float fx = floorf(ok ? ix : 0.0f), fy = floorf(ok ? iy : 0.0f);
  wx = ok ? ix - fx : 0.0f;
  wy = ok ? iy - fy : 0.0f;
  pos = ok ? ((uint32_t)((int)fy + 2) << 16) | (uint32_t)((int)fx + 2) : kInvalidTap;
}

__device__ inline int pos_x(uint32_t p) { return (int)(p & 0xFFFFu) - 2; }
__device__ inline int pos_y(uint32_t p) { return (int)(p >> 16) - 2; }

// bilinear weights of the nw, ne, sw, se taps (torch CPU grid_sample: nw = (1-fy)(1-fx) ...)
__device__ inline void tap_weights(float wx, float wy, float (&wt)[4]) {
  const float ex = 1.0f - wx, ny = 1.0f - wy;
  wt[0] = ny * ex;
  wt[1] = ny * wx;
  wt[2] = wy * ex;
  wt[3] = wy * wx;
}

// ------------------------------------------------------------------------------------------
// per-lane taps into an NCHW plane (generic / warp / backward kernels): byte offsets + weights,
// out-of-image taps get weight 0 and offset 0
// ------------------------------------------------------------------------------------------
struct Taps {
  uint32_t off[4];
  float wt[4];
};

__device__ inline void make_taps(const float* __restrict__ G, float xn, float yn, int h, int w,
                                 Taps& tp) {
  float ix, iy;
  sample_coord(G, xn, yn, h, w, ix, iy);
  if (!(ix > -2.0f && ix < (float)w + 1.0f && iy > -2.0f && iy < (float)h + 1.0f)) {
    ix = -4.0f;  // far outside or NaN: every tap invalid, int conversion stays in range
    iy = -4.0f;
  }
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  float wt[4];
  tap_weights(ix - fx, iy - fy, wt);
  const bool vx0 = x0 >= 0 && x0 < w, vx1 = x0 + 1 >= 0 && x0 + 1 < w;
  const bool vy0 = y0 >= 0 && y0 < h, vy1 = y0 + 1 >= 0 && y0 + 1 < h;
  const uint32_t base = (uint32_t)(y0 * w + x0) * 4u;
  const bool ok[4] = {vx0 && vy0, vx1 && vy0, vx0 && vy1, vx1 && vy1};
  const uint32_t off[4] = {base, base + 4u, base + 4u * (uint32_t)w, base + 4u * (uint32_t)w + 4u};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    tp.wt[t] = ok[t] ? wt[t] : 0.0f;
    tp.off[t] = ok[t] ? off[t] : 0u;
  }
}

__device__ inline float gather(const float* __restrict__ plane, const Taps& tp) {
  const char* pb = reinterpret_cast<const char*>(plane);
  auto ld = [&](int t) { return *reinterpret_cast<const float*>(pb + tp.off[t]); };
  return bilerp_sum(ld(0), ld(1), ld(2), ld(3), tp.wt);
}

// ------------------------------------------------------------------------------------------
// buffer descriptors (cdna_hip_programming.md T8/T20): base/bytes must be workgroup-uniform
// ------------------------------------------------------------------------------------------
typedef __amdgpu_buffer_rsrc_t Rsrc;

// Workgroup-uniform values the compiler cannot prove uniform (derived from LDS loads, or computed
// in VALU): readfirstlane moves them to SGPRs, so descriptors built from them need no waterfall
// loop and branches on them are scalar.
__device__ inline int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

template <typename T>
__device__ inline T* uniform_ptr(T* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// A workgroup-uniform 3x3 sampling matrix through the constant address space: the loads become
// s_load (scalar cache, lgkmcnt only).  Read through a generic pointer they are flat loads, which
// count in vmcnt too, and every wait for them would also drain the wave's outstanding vector loads.
typedef __attribute__((address_space(4))) const float const_float;

__device__ inline void load_matrix_uniform(const float* p, float (&G)[9]) {
  const const_float* c = (const const_float*)uniform_ptr(p);
#pragma unroll
  for (int i = 0; i < 9; ++i) G[i] = c[i];
}

__device__ inline Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

__device__ inline float gather_buf(Rsrc rs, uint32_t soff, const Taps& tp) {
  const float a = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[0], soff, 0));
  const float b = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[1], soff, 0));
  const float c = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[2], soff, 0));
  const float d = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[3], soff, 0));
  return bilerp_sum(a, b, c, d, tp.wt);
}

__device__ inline void store_buf(Rsrc rs, uint32_t voff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, 0, 0);
}

// ------------------------------------------------------------------------------------------
// XCD-chunked work ids: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// §Workgroup dispatch), so w = (L % 8) * ceil(T/8) + L / 8 hands each XCD a contiguous run of work
// items -- neighbouring depth planes of one tile share source footprints through one 4 MiB L2.
// Placement only changes speed, never results.
// ------------------------------------------------------------------------------------------
__device__ inline int xcd_work_id(int L, int total) {
  const int q = (total + 7) >> 3;
  return (L & 7) * q + (L >> 3);
}

inline dim3 xcd_grid(int total) { return dim3(8u * (unsigned)((total + 7) / 8)); }

// flattened-pixel work item (generic / warp / backward kernels): 256 consecutive pixels of one
// (sample, plane)
struct WorkItem {
  int b, kk, tile;
};

__device__ inline WorkItem decode_flat(int wk, int Dc, int tiles) {
  WorkItem it;
  it.kk = wk % Dc;
  const int t = wk / Dc;
  it.tile = t % tiles;
  it.b = t / tiles;
  return it;
}

__device__ inline void pixel_coords(uint32_t p, int w, int h, float& xn, float& yn) {
  const uint32_t y = p / (uint32_t)w;
  const uint32_t x = p - y * (uint32_t)w;
  xn = norm_coord(x, w);
  yn = norm_coord(y, h);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// camera inputs of one cost-volume launch (device pointers, homography.py:6-36) and the shard's
// first plane
struct Cams {
  const float *K, *R, *T, *d_min, *d_int;
  int d_begin;
  float d_scale;
};

struct Geometry {
  int B, V, C, h, w, Dc;
  int tiles;  // flattened 256-pixel tiles per plane
  int total;  // flattened work items (B * tiles * Dc)
};

// Launch status of ONE entry point.  HIP's last-error slot is per thread and sticky.  An error left
// there before the call (a torch kernel, another library) would otherwise mask this call's own:
// comparing the slot before and after cannot tell a new failure with the same code from the old one.
// So the slot is CLEARED at entry and any error in it after the launches is this call's own:
// consumed, and reported as MVS_ERR_HIP.  The earlier error is not dropped silently: it is reported
// on stderr (once per entry) and kept in prior().  (Construct at entry, status() after the launches.)
class LaunchCheck {
 public:
  LaunchCheck() : prior_(hipGetLastError()) {
    if (prior_ != hipSuccess)
      fprintf(stderr, "mvs: a HIP error was pending before this call (cleared, not ours): %s\n",
              hipGetErrorString(prior_));
  }
  int status() const { return hipGetLastError() == hipSuccess ? MVS_OK : MVS_ERR_HIP; }
  hipError_t prior() const { return prior_; }

 private:
  hipError_t prior_;
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace mvs
