// packed.h -- the padded channel-quad feature layout shared by the fused forward and its backward.
//
//   packed[N][C4][h + 2][w + 2] float4, C4 = ceil(C / 4): channel 4q+j in component j (zero pad),
//   pixel (x, y) at padded (x + 1, y + 1); columns 0, w + 1 and rows 0, h + 1 are zero.
// Every tap corner the sampling law can produce (x0 in [-1, w-1], y0 in [-1, h-1]) then has its
// four taps inside the padded plane, and out-of-image taps read zeros: the bilinear gather needs no
// bounds test.  A sample whose taps all lie outside the image gets an out-of-range buffer offset:
// its loads return 0 without touching memory.
//   refs[B][C4][h][w] float4: the reference view resampled through its own (plane-independent)
// sampling matrix, computed once per forward launch and reused by the backward.
#pragma once

#include "common.h"

namespace mvs {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

struct PadGeom {
  int pitch;        // w + 2 slots per padded row
  uint32_t plane;   // (h + 2) * pitch slots per padded plane
};

__host__ __device__ inline PadGeom pad_geom(int h, int w) {
  PadGeom p;
  p.pitch = w + 2;
  p.plane = (uint32_t)(h + 2) * (uint32_t)(w + 2);
  return p;
}

constexpr uint32_t kOobOffset = 0x80000000u;   // >= every descriptor's num_records

// byte offset of the nw tap of a tap corner inside one padded plane
__device__ inline uint32_t tap_offset(uint32_t pos, const PadGeom& pg) {
  if (pos == kInvalidTap) return kOobOffset;
  return ((uint32_t)(pos_y(pos) + 1) * (uint32_t)pg.pitch + (uint32_t)(pos_x(pos) + 1)) * 16u;
}

__device__ inline f4v ld4(Rsrc rs, uint32_t voff, int soff) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, soff, 0));
}

__device__ inline void load_taps(Rsrc rs, uint32_t voff, int soff, int row_bytes, f4v (&t)[4]) {
  t[0] = ld4(rs, voff, soff);
  t[1] = ld4(rs, voff + 16u, soff);
  t[2] = ld4(rs, voff, soff + row_bytes);
  t[3] = ld4(rs, voff + 16u, soff + row_bytes);
}

// Bilinear sample of 4 channels: nw * t0, then fma(tap_t, weight_t, acc) over ne, sw, se -- torch CPU
// grid_sample's sum (common.h bilerp_sum; zero taps add exactly nothing).  Packed fp32 FMAs
// (v_pk_fma_f32), elementwise identical to scalar fmaf.
__device__ inline f4v bilerp(const f4v (&t)[4], float wx, float wy) {
#pragma clang fp contract(off)
  // weights {nw, ne} = (1-wy) * {1-wx, wx}, {sw, se} = wy * {1-wx, wx}: tap_weights() in pairs
  const f2v e = {1.0f - wx, wx};
  const f2v w01 = f2v{1.0f - wy, 1.0f - wy} * e;
  const f2v w23 = f2v{wy, wy} * e;
  f2v lo = t[0].xy * w01.xx, hi = t[0].zw * w01.xx;   // fma(t, w, 0) == t * w
  lo = __builtin_elementwise_fma(t[1].xy, w01.yy, lo);
  hi = __builtin_elementwise_fma(t[1].zw, w01.yy, hi);
  lo = __builtin_elementwise_fma(t[2].xy, w23.xx, lo);
  hi = __builtin_elementwise_fma(t[2].zw, w23.xx, hi);
  lo = __builtin_elementwise_fma(t[3].xy, w23.yy, lo);
  hi = __builtin_elementwise_fma(t[3].zw, w23.yy, hi);
  return f4v{lo.x, lo.y, hi.x, hi.y};
}

// x / V for 4 channels (div_views, packed: v_pk_mul_f32 + 2 v_pk_fma_f32 per channel pair)
__device__ inline f4v div_views4(const f4v& x, ViewDiv d) {
#pragma clang fp contract(off)
  const f4v r = {d.r, d.r, d.r, d.r};
  const f4v q = x * r;
  f4v y = __builtin_elementwise_fma(__builtin_elementwise_fma(-q, f4v{d.v, d.v, d.v, d.v}, x), r, q);
  if (d.tie) {   // launch-uniform: V = 6, 10, 12, 14 only (common.h div_views)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (__builtin_expect(__builtin_fabsf(x[c]) < 0x1p-120f, 0)) y[c] = x[c] / d.v;
  }
  return y;
}

// costvolume.py:12-14 for 4 channels of one voxel, in the reference's torch CPU roundings (common.h:
// view_div): mean = ((x0 + x1) + ...) / V, cv = ((d0 d0 + d1 d1) + ...) / V with d = x - mean.
// x + (-mean) == x - mean exactly (keeps v_pk_add_f32).  The one variance of every forward kernel.
template <int NS>
__device__ inline f4v variance_law4(const f4v& x0, const f4v (&xs)[NS], ViewDiv vd) {
#pragma clang fp contract(off)
#ifdef MVS_EXP_OLD_VARIANCE   // experiment only: the round-4 arithmetic (reciprocal multiply, fused squares)
  {
    const f4v iv = {vd.r, vd.r, vd.r, vd.r};
    f4v sm = x0;
    for (int s = 0; s < NS; ++s) sm += xs[s];
    const f4v nm = -(sm * iv);
    f4v dd = x0 + nm, ac = dd * dd;
    for (int s = 0; s < NS; ++s) { dd = xs[s] + nm; ac = __builtin_elementwise_fma(dd, dd, ac); }
    return ac * iv;
  }
#endif
  f4v sum = x0;
#pragma unroll
  for (int s = 0; s < NS; ++s) sum += xs[s];
  const f4v nmean = -div_views4(sum, vd);
  f4v d = x0 + nmean;
  f4v acc = d * d;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    d = xs[s] + nmean;
    acc += d * d;
  }
  return div_views4(acc, vd);
}

// workspace layout of mvs_cost_volume_fwd (and read back by mvs_cost_volume_bwd):
//   [sampling N * Dc * 9 floats, padded to 256 B][packed N * C4 * plane float4][refs B * C4 * hw float4]
__host__ __device__ inline size_t sampling_bytes_aligned(int N, int Dc) {
  return ((size_t)N * Dc * 9 * sizeof(float) + 255) & ~(size_t)255;
}

}  // namespace mvs
