// mvs_cost_volume.hip -- MI355X (gfx950 / CDNA4) kernels for the MVSNet cost-volume path.
//
// Hot path of bcollico/Deep-Multiview-Depth-Estimation:
//   scripts/homography.py:6-92   per-plane homography + kornia warp_perspective (grid_sample)
//   scripts/costvolume.py:3-16   population variance over the V views
//   scripts/depthmap.py:4-22     permutation-indexed "top-N" soft-argmin
//
// Kernels:
//   plane_sampling_kernel   fp64 per-(image, plane) sampling matrix G = inv(Nrm H Nrm^-1)
//   cost_volume_kernel      FUSED bilinear gather of every view + on-the-fly two-pass variance;
//                           writes cv[B][C][D][h][w] once, the warped volume never exists
//   warp_kernel             the same gather, writing warped[N][C][D][h][w] (API compatibility)
//   variance_kernel         costvolume.py on an already-warped volume
//   cost_volume_bwd_kernel  d cv / d feat: recompute + float-atomic scatter into grad_feat
//   soft_argmin_kernel      depthmap.py with rank counting instead of a full sort
//
// Design notes (details in DESIGN.md):
//   * one thread = one output pixel of one (sample, plane); a 256-thread workgroup covers 256
//     consecutive pixels of the flattened h*w plane, so every cv store is a 256-B coalesced
//     wave store whatever w is;
//   * the 9 floats of G per view are workgroup-uniform -> scalar loads into SGPRs;
//   * feature taps use a uniform 64-bit plane base + a 32-bit per-lane offset (saddr form:
//     no per-load VALU address arithmetic); out-of-bounds taps get weight 0 and offset 0;
//   * workgroup -> work mapping is XCD-chunked: consecutive workgroup ids are dealt round-robin
//     over the 8 XCDs, so work item w = (L % 8) * ceil(T/8) + L / 8 gives each XCD a
//     contiguous run of (tile, plane) items, planes fastest -> neighbouring depth planes of the
//     same tile (overlapping source footprints) are gathered through the same 4 MiB L2.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/mvs_cost_volume.h"

namespace {

constexpr int kBlock = 256;

// ------------------------------------------------------------------------------------------
// geometry (fp64)
// ------------------------------------------------------------------------------------------
struct Mat3 {
  double a[9];
};

__device__ inline Mat3 mat_mul(const Mat3& x, const Mat3& y) {
  Mat3 r;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      r.a[3 * i + j] = x.a[3 * i] * y.a[j] + x.a[3 * i + 1] * y.a[3 + j] + x.a[3 * i + 2] * y.a[6 + j];
  return r;
}

// Inverse by adjugate; a singular matrix yields non-finite entries (every tap then samples
// outside the image and contributes zero; the reference's torch.inverse would raise instead).
__device__ inline Mat3 mat_inv(const Mat3& m) {
  const double* a = m.a;
  double c00 = a[4] * a[8] - a[5] * a[7];
  double c01 = a[5] * a[6] - a[3] * a[8];
  double c02 = a[3] * a[7] - a[4] * a[6];
  double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
  double id = 1.0 / det;
  Mat3 r;
  r.a[0] = c00 * id;
  r.a[1] = (a[2] * a[7] - a[1] * a[8]) * id;
  r.a[2] = (a[1] * a[5] - a[2] * a[4]) * id;
  r.a[3] = c01 * id;
  r.a[4] = (a[0] * a[8] - a[2] * a[6]) * id;
  r.a[5] = (a[2] * a[3] - a[0] * a[5]) * id;
  r.a[6] = c02 * id;
  r.a[7] = (a[1] * a[6] - a[0] * a[7]) * id;
  r.a[8] = (a[0] * a[4] - a[1] * a[3]) * id;
  return r;
}

__device__ inline Mat3 load_mat(const float* p) {
  Mat3 r;
#pragma unroll
  for (int e = 0; e < 9; ++e) r.a[e] = (double)p[e];
  return r;
}

// homography.py:40-75 (H) + kornia normalize_homography / inverse, one thread per (i, kk).
__global__ void plane_sampling_kernel(const float* __restrict__ K, const float* __restrict__ R,
                                      const float* __restrict__ T, const float* __restrict__ d_min,
                                      const float* __restrict__ d_int, int B, int V, int h, int w,
                                      int d_begin, int d_count, float d_scale,
                                      float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int N = B * V;
  if (t >= N * d_count) return;
  const int i = t / d_count;
  const int kk = t - i * d_count;
  const int r = (i / V) * V;   // reference view of image i (homography.py:29-34)
  const int bq = i % B;        // d_batch = tile(d_batch_0, (V,1,1,1)): row i is sample i mod B
  // depth in fp32 exactly as homography.py:25 forms it: d_min + (D_SCALE * d_int) * k
  const float d32 = d_min[bq] + (d_scale * d_int[bq]) * (float)(d_begin + kk);
  const double d = (double)d32;

  const Mat3 Ki = load_mat(K + 9 * i), Ri = load_mat(R + 9 * i);
  const Mat3 Kr = load_mat(K + 9 * r), Rr = load_mat(R + 9 * r);
  double Ci[3], Cr[3], nr[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {  // C = -R^T T
    Ci[a] = -(Ri.a[a] * (double)T[3 * i] + Ri.a[3 + a] * (double)T[3 * i + 1] +
              Ri.a[6 + a] * (double)T[3 * i + 2]);
    Cr[a] = -(Rr.a[a] * (double)T[3 * r] + Rr.a[3 + a] * (double)T[3 * r + 1] +
              Rr.a[6 + a] * (double)T[3 * r + 2]);
    nr[a] = Rr.a[3 * a + 2];  // third column of R_ref (homography.py:49)
  }
  Mat3 P;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) P.a[3 * a + c] = (a == c ? 1.0 : 0.0) - (Ci[a] - Cr[a]) * nr[c] / d;
  Mat3 RrT;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) RrT.a[3 * a + c] = Rr.a[3 * c + a];
  const Mat3 H = mat_mul(mat_mul(Ki, Ri), mat_mul(P, mat_mul(RrT, mat_inv(Kr))));
  // kornia: dst_norm_T_src_norm = Nrm @ H @ Nrm^-1, then src_norm_T_dst_norm = inverse(.)
  const double sx = 2.0 / (double)(w - 1), sy = 2.0 / (double)(h - 1);
  Mat3 Nm = {{sx, 0.0, -1.0, 0.0, sy, -1.0, 0.0, 0.0, 1.0}};
  Mat3 Ni = {{1.0 / sx, 0.0, 1.0 / sx, 0.0, 1.0 / sy, 1.0 / sy, 0.0, 0.0, 1.0}};
  const Mat3 G = mat_inv(mat_mul(Nm, mat_mul(H, Ni)));
  float* o = out + 9 * (size_t)t;
#pragma unroll
  for (int e = 0; e < 9; ++e) o[e] = (float)G.a[e];
}

// ------------------------------------------------------------------------------------------
// sampling (fp32): kornia meshgrid/transform_points + grid_sample(bilinear, zeros,
// align_corners=False) -- SURVEY.md §8 a4
// ------------------------------------------------------------------------------------------
struct Taps {
  uint32_t off[4];  // nw, ne, sw, se BYTE offsets inside one h*w plane (0 when out of bounds)
  float wt[4];      // bilinear weights (0 when out of bounds)
};

// Source sampling position (ix, iy) of normalised reference pixel (xn, yn) under sampling matrix G
// (kornia transform_points + convert_points_from_homogeneous + grid_sample unnormalise).  Every
// rounding step is explicit (__f*_rn), so all call sites -- every view, every kernel -- produce
// bit-identical coordinates for identical inputs regardless of how the compiler contracts code.
__device__ inline void sample_coord(const float* __restrict__ G, float xn, float yn, int h, int w,
                                    float& ix, float& iy) {
  float u = __fmaf_rn(G[1], yn, __fmaf_rn(G[0], xn, G[2]));
  float v = __fmaf_rn(G[4], yn, __fmaf_rn(G[3], xn, G[5]));
  const float s = __fmaf_rn(G[7], yn, __fmaf_rn(G[6], xn, G[8]));
  if (fabsf(s) > 1e-8f) {  // kornia eps: scale = 1 / (s + eps) where |s| > eps, else 1
    const float sc = __fdiv_rn(1.0f, __fadd_rn(s, 1e-8f));
    u = __fmul_rn(u, sc);
    v = __fmul_rn(v, sc);
  }
  // grid_sample(align_corners=False) unnormalise, as torch's CPU kernel: (g + 1) * (size / 2) - 0.5
  ix = __fsub_rn(__fmul_rn(__fadd_rn(u, 1.0f), 0.5f * (float)w), 0.5f);
  iy = __fsub_rn(__fmul_rn(__fadd_rn(v, 1.0f), 0.5f * (float)h), 0.5f);
}

__device__ inline void make_taps(const float* __restrict__ G, float xn, float yn, int h, int w,
                                 Taps& tp) {
  float ix, iy;
  sample_coord(G, xn, yn, h, w, ix, iy);
  // far outside (or NaN): every tap invalid; keeps the int conversion in range
  if (!(ix > -2.0f && ix < (float)w + 1.0f && iy > -2.0f && iy < (float)h + 1.0f)) {
    ix = -4.0f;
    iy = -4.0f;
  }
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float wx = ix - fx, wy = iy - fy;
  const float ex = 1.0f - wx, ny = 1.0f - wy;
  const bool vx0 = (x0 >= 0) && (x0 < w), vx1 = (x0 + 1 >= 0) && (x0 + 1 < w);
  const bool vy0 = (y0 >= 0) && (y0 < h), vy1 = (y0 + 1 >= 0) && (y0 + 1 < h);
  const uint32_t base = (uint32_t)(y0 * w + x0) * 4u;
  tp.wt[0] = (vx0 && vy0) ? ny * ex : 0.0f;
  tp.wt[1] = (vx1 && vy0) ? ny * wx : 0.0f;
  tp.wt[2] = (vx0 && vy1) ? wy * ex : 0.0f;
  tp.wt[3] = (vx1 && vy1) ? wy * wx : 0.0f;
  tp.off[0] = (vx0 && vy0) ? base : 0u;
  tp.off[1] = (vx1 && vy0) ? base + 4u : 0u;
  tp.off[2] = (vx0 && vy1) ? base + 4u * (uint32_t)w : 0u;
  tp.off[3] = (vx1 && vy1) ? base + 4u * (uint32_t)w + 4u : 0u;
}

__device__ inline float gather(const float* __restrict__ plane, const Taps& tp) {
  const char* pb = reinterpret_cast<const char*>(plane);
  auto ld = [&](int t) { return *reinterpret_cast<const float*>(pb + tp.off[t]); };
  return ld(0) * tp.wt[0] + ld(1) * tp.wt[1] + ld(2) * tp.wt[2] + ld(3) * tp.wt[3];
}

typedef __amdgpu_buffer_rsrc_t Rsrc;

// Buffer descriptor over [base, base + bytes); base/bytes must be workgroup-uniform (kernargs
// and blockIdx-derived only) so the descriptor lives in SGPRs (cdna_hip_programming.md T8/T20).
__device__ inline Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

// Bilinear gather through a buffer descriptor: 32-bit per-lane tap offsets (voffset) plus a
// uniform channel offset in an SGPR (soffset) -- no per-load VALU address arithmetic.
__device__ inline float gather_buf(Rsrc rs, uint32_t soff, const Taps& tp) {
  const float a = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[0], soff, 0));
  const float b = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[1], soff, 0));
  const float c = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[2], soff, 0));
  const float d = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, tp.off[3], soff, 0));
  return a * tp.wt[0] + b * tp.wt[1] + c * tp.wt[2] + d * tp.wt[3];
}

__device__ inline void store_buf(Rsrc rs, uint32_t voff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, 0, 0);
}

// XCD-chunked work id (see header comment); returns >= total for surplus workgroups.
__device__ inline int xcd_work_id(int L, int total) {
  const int q = (total + 7) >> 3;
  return (L & 7) * q + (L >> 3);
}

struct WorkItem {
  int b, kk, tile;
};

__device__ inline WorkItem decode(int wk, int Dc, int tiles) {
  WorkItem it;
  it.kk = wk % Dc;
  const int t = wk / Dc;
  it.tile = t % tiles;
  it.b = t / tiles;
  return it;
}

// meshgrid of kornia (normalized_coordinates=True): (x / (w-1) - 0.5) * 2
__device__ inline float norm_coord(uint32_t x, int size) {
  return __fmul_rn(__fsub_rn(__fdiv_rn((float)x, (float)(size - 1)), 0.5f), 2.0f);
}

__device__ inline void pixel_coords(uint32_t p, int w, int h, float& xn, float& yn) {
  const uint32_t y = p / (uint32_t)w;
  const uint32_t x = p - y * (uint32_t)w;
  xn = norm_coord(x, w);
  yn = norm_coord(y, h);
}

// ------------------------------------------------------------------------------------------
// fused warp + variance.  MAXV = compile-time view bound; EXACT -> V == MAXV.
// ------------------------------------------------------------------------------------------
template <int MAXV, bool EXACT, int CU>
__global__ __launch_bounds__(kBlock) void cost_volume_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling, float* __restrict__ cv,
    int nv_rt, int C, int h, int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  const bool active = p < hw;
  float xn, yn;
  pixel_coords(active ? p : 0u, w, h, xn, yn);

  Taps tp[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) make_taps(sampling + ((size_t)(it.b * V + v) * Dc + it.kk) * 9, xn, yn, h, w, tp[v]);

  const float* fb = feat + (size_t)it.b * V * C * hw;
  float* ob = cv + ((size_t)it.b * C * Dc + it.kk) * hw;
  const size_t ostride = (size_t)Dc * hw;
  const uint32_t plane_bytes = hw * 4u;
  Rsrc rs[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) rs[v] = make_rsrc(fb + (size_t)v * C * hw, (uint32_t)C * plane_bytes);
  const float inv_v = 1.0f / (float)V;
  const uint32_t pbyte = p * 4u;

  for (int c0 = 0; c0 < C; c0 += CU) {
    float val[CU][MAXV];
#pragma unroll
    for (int cu = 0; cu < CU; ++cu) {
      if (c0 + cu < C) {
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
          if (v < V) val[cu][v] = gather_buf(rs[v], (uint32_t)(c0 + cu) * plane_bytes, tp[v]);
      }
    }
#pragma unroll
    for (int cu = 0; cu < CU; ++cu) {
      if (c0 + cu < C) {
        // costvolume.py:12-14 -- mean = sum/V, cv = sum (x - mean)^2 / V (two-pass)
        float sum = val[cu][0];
#pragma unroll
        for (int v = 1; v < MAXV; ++v)
          if (v < V) sum += val[cu][v];
        const float mean = sum * inv_v;
        float acc = 0.0f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
          if (v < V) {
            const float dlt = val[cu][v] - mean;
            acc += dlt * dlt;
          }
        if (active) store_buf(make_rsrc(ob + (size_t)(c0 + cu) * ostride, plane_bytes), pbyte, acc * inv_v);
      }
    }
  }
}

// warp only: warped[i][c][kk][p] for every image i of sample b
template <int MAXV, bool EXACT, int CU>
__global__ __launch_bounds__(kBlock) void warp_kernel(const float* __restrict__ feat,
                                                      const float* __restrict__ sampling,
                                                      float* __restrict__ warped, int nv_rt, int C,
                                                      int h, int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode(wk, Dc, tiles);
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
  const float inv_v = 1.0f / (float)V;
  const size_t n = (size_t)B * M;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (size_t)gridDim.x * kBlock) {
    const size_t b = e / M, m = e - b * M;
    const float* x = warped + b * V * M + m;
    float sum = x[0];
    for (int v = 1; v < V; ++v) sum += x[(size_t)v * M];
    const float mean = sum * inv_v;
    float acc = 0.0f;
    for (int v = 0; v < V; ++v) {
      const float dlt = x[(size_t)v * M] - mean;
      acc += dlt * dlt;
    }
    cv[e] = acc * inv_v;
  }
}

// backward: g_x_v = 2 (x_v - mean) / V * g_cv, scattered to the 4 taps with bilinear weights
template <int MAXV, bool EXACT>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling,
    const float* __restrict__ grad_cv, float* __restrict__ grad_feat, int nv_rt, int C, int h,
    int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  if (p >= hw) return;
  float xn, yn;
  pixel_coords(p, w, h, xn, yn);
  Taps tp[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) make_taps(sampling + ((size_t)(it.b * V + v) * Dc + it.kk) * 9, xn, yn, h, w, tp[v]);
  const float* fb = feat + (size_t)it.b * V * C * hw;
  float* gb = grad_feat + (size_t)it.b * V * C * hw;
  const float* gcv = grad_cv + ((size_t)it.b * C * Dc + it.kk) * hw + p;
  const float inv_v = 1.0f / (float)V;
  for (int c = 0; c < C; ++c) {
    const float g = gcv[(size_t)c * Dc * hw];
    float val[MAXV];
    float sum = 0.0f;
#pragma unroll
    for (int v = 0; v < MAXV; ++v)
      if (v < V) {
        val[v] = gather(fb + ((size_t)v * C + c) * hw, tp[v]);
        sum += val[v];
      }
    const float mean = sum * inv_v;
    const float k2 = 2.0f * inv_v * g;
#pragma unroll
    for (int v = 0; v < MAXV; ++v)
      if (v < V) {
        const float coef = k2 * (val[v] - mean);
        char* plane = reinterpret_cast<char*>(gb + ((size_t)v * C + c) * hw);
#pragma unroll
        for (int t = 0; t < 4; ++t)  // off[] are byte offsets
          if (tp[v].wt[t] != 0.0f)
            unsafeAtomicAdd(reinterpret_cast<float*>(plane + tp[v].off[t]), tp[v].wt[t] * coef);
      }
  }
}

// depthmap.py:4-22.  rank_j = #{m : P_m > P_j} + #{m < j : P_m == P_j} is the sorted position of
// plane j (descending, ties by ascending index); mask[r] = 1 exactly at r = rank_j, j < n_est.
template <int MAXE>
__global__ __launch_bounds__(kBlock) void soft_argmin_kernel(const float* __restrict__ prob,
                                                             const float* __restrict__ d_batch,
                                                             int B, int D, uint32_t hw, int n_est,
                                                             float* __restrict__ depth) {
  const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= (size_t)B * hw) return;
  const size_t b = e / hw, p = e - b * hw;
  const float* P = prob + b * D * hw + p;
  const float* db = d_batch + b * D;
  float pj[MAXE];
  int rank[MAXE];
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    pj[j] = (j < n_est) ? P[(size_t)j * hw] : 0.0f;
    rank[j] = 0;
  }
  for (int m = 0; m < D; ++m) {
    const float pm = P[(size_t)m * hw];
#pragma unroll
    for (int j = 0; j < MAXE; ++j) rank[j] += (pm > pj[j]) || (pm == pj[j] && m < j);
  }
  // sum in ascending plane order, as the masked sum over dim 2 does
#pragma unroll
  for (int a = 1; a < MAXE; ++a)
#pragma unroll
    for (int c = a; c > 0; --c)
      if (c < n_est && rank[c] < rank[c - 1]) {
        const int t = rank[c];
        rank[c] = rank[c - 1];
        rank[c - 1] = t;
      }
  float num = 0.0f, den = 0.0f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j)
    if (j < n_est) {
      const float pr = P[(size_t)rank[j] * hw];
      num += db[rank[j]] * pr;
      den += pr;
    }
  depth[e] = num / den;
}

// ------------------------------------------------------------------------------------------
// v2 fused path: features packed channel-chunk-last, source footprints staged in LDS
// ------------------------------------------------------------------------------------------
// pack: feat[N][C][h][w] -> packed[N][NCH][h][w][CH], NCH = ceil(C / CH), zero-padded channels.
template <int CH>
__global__ __launch_bounds__(kBlock) void pack_features_kernel(const float* __restrict__ feat,
                                                              float* __restrict__ packed, int N,
                                                              int C, uint32_t hw) {
  const int nch = (C + CH - 1) / CH;
  const size_t n = (size_t)N * nch * hw;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (size_t)gridDim.x * kBlock) {
    const size_t p = e % hw;
    const size_t t = e / hw;
    const int ch = (int)(t % nch);
    const size_t i = t / nch;
    float v[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = ch * CH + j;
      v[j] = c < C ? feat[(i * C + c) * hw + p] : 0.0f;
    }
    float4* o = reinterpret_cast<float4*>(packed + e * CH);
#pragma unroll
    for (int q = 0; q < CH / 4; ++q) o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
}

#ifndef MVS_EXP_TW
#define MVS_EXP_TW 16
#endif
constexpr int kTW = MVS_EXP_TW;        // tile width  (pixels)
constexpr int kTH = 256 / kTW;         // tile height (pixels): 256 threads, one pixel each
#ifndef MVS_EXP_LDS_KB
#define MVS_EXP_LDS_KB 48
#endif
constexpr int kLdsBytes = MVS_EXP_LDS_KB * 1024;   // footprint staging budget per workgroup
constexpr uint32_t kInvalidTap = 0xFFFFFFFFu;

// Source coordinates of one (pixel, view, plane): kornia sampling law as make_taps, reduced to the
// integer corner (x0, y0) and fractions; positions whose 4 taps all fall outside the image
// (ix < -1, ix >= w, ...) are marked invalid (value exactly 0).
__device__ inline void src_coords(const float* __restrict__ G, float xn, float yn, int h, int w,
                                  bool active, uint32_t& pos, float& wx, float& wy) {
  float ix, iy;
  sample_coord(G, xn, yn, h, w, ix, iy);
  const bool ok = active && ix >= -1.0f && ix < (float)w && iy >= -1.0f && iy < (float)h;
  const float fx = floorf(ok ? ix : 0.0f), fy = floorf(ok ? iy : 0.0f);
  wx = ok ? ix - fx : 0.0f;
  wy = ok ? iy - fy : 0.0f;
  // x0 in [-1, w-1], y0 in [-1, h-1]; stored +2 so both fields are positive 16-bit values
  pos = ok ? ((uint32_t)((int)fy + 2) << 16) | (uint32_t)((int)fx + 2) : kInvalidTap;
}

__device__ inline int pos_x(uint32_t p) { return (int)(p & 0xFFFFu) - 2; }
__device__ inline int pos_y(uint32_t p) { return (int)(p >> 16) - 2; }

// Workgroup-wide min of NV ints (every thread gets the result, in SGPR-uniform form).
template <int NV>
__device__ inline void block_min(int (&v)[NV], int* scratch /* >= 4 * NV ints in LDS */) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
    v[k] = x;
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[wave * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int x = scratch[k];
#pragma unroll
    for (int q = 1; q < kBlock / 64; ++q) x = min(x, scratch[q * NV + k]);
    v[k] = __builtin_amdgcn_readfirstlane(x);
  }
  __syncthreads();
}

// Footprint of one source view in LDS: region rows [y0, y0+rh), cols [x0, x0+rw), preceded by a
// zero prefix of rw + 2 pixels that invalid taps point at.  Offsets in bytes.
struct Region {
  int x0, y0, rw, rh;
  int base;  // byte offset of the prefix in the staging buffer
};

// CH == 8: pixel p occupies 16-B slots 2p + p/8 and 2p + p/8 + 1 (a 16-B pad every 8 pixels), so
// the 16 lanes of a ds_read_b128 group that read 16 consecutive pixels hit 16 distinct 4-bank groups.
// CH == 4: one 16-B slot per pixel, consecutive pixels are conflict-free as they are.
template <int CH>
__device__ inline int slot_of(int p) {
  return CH == 8 ? 2 * p + (p >> 3) : p;
}

template <int CH>
__device__ inline int region_bytes(const Region& r) {
  return r.rw > 0 ? (slot_of<CH>(r.rh * r.rw + r.rw + 2) + 2) * 16 : 0;
}

template <int CH>
__device__ inline void stage_region(char* lds, const Region& r, const float* __restrict__ src,
                                    int h, int w) {
  // src = packed[i][chunk] plane: [h][w][CH]
  constexpr int HALVES = CH / 4;
  if (r.rw <= 0) return;
  const int prefix = (r.rw + 2) * HALVES;
  const int body = r.rh * r.rw * HALVES;
  const float inv = 1.0f / (float)(r.rw * HALVES);
  for (int q = threadIdx.x; q < prefix + body; q += kBlock) {
    float4 val = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int p, half;
    if (q < prefix) {
      p = q / HALVES;
      half = q - p * HALVES;
    } else {
      const int e = q - prefix;
      const int row = (int)(((float)e + 0.5f) * inv);
      const int rem = e - row * r.rw * HALVES;
      const int col = rem / HALVES;
      half = rem - col * HALVES;
      p = r.rw + 2 + row * r.rw + col;
      const int gx = r.x0 + col, gy = r.y0 + row;
      if (gx >= 0 && gx < w && gy >= 0 && gy < h)
        val = *reinterpret_cast<const float4*>(src + ((size_t)gy * w + gx) * CH + half * 4);
    }
    *reinterpret_cast<float4*>(lds + r.base + (slot_of<CH>(p) + half) * 16) = val;
  }
}

// Bilinear sample of CH channels of one staged view: taps p, p+1, p+rw, p+rw+1.
template <int CH>
__device__ inline void gather_lds(const char* lds, const Region& r, uint32_t pos, float wx, float wy,
                                  float (&out)[CH]) {
#pragma unroll
  for (int j = 0; j < CH; ++j) out[j] = 0.0f;
  // all four taps outside the image: exactly zero (the view's region may even be empty)
  if (pos == kInvalidTap) return;
  const int p = r.rw + 2 + (pos_y(pos) - r.y0) * r.rw + (pos_x(pos) - r.x0);
  const float ex = 1.0f - wx, ny = 1.0f - wy;
  const float wt[4] = {ny * ex, ny * wx, wy * ex, wy * wx};
  const int tp[4] = {p, p + 1, p + r.rw, p + r.rw + 1};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const char* a0 = lds + r.base + slot_of<CH>(tp[t]) * 16;
#pragma unroll
    for (int q = 0; q < CH / 4; ++q) {
      const float4 a = *reinterpret_cast<const float4*>(a0 + 16 * q);
      out[4 * q + 0] += a.x * wt[t];
      out[4 * q + 1] += a.y * wt[t];
      out[4 * q + 2] += a.z * wt[t];
      out[4 * q + 3] += a.w * wt[t];
    }
  }
}

// Bilinear sample of CH channels straight from the packed global plane (ref view, and planes whose
// footprint does not fit the LDS budget).  Per-tap bounds checks; zero padding.
template <int CH>
__device__ inline void gather_global(const float* __restrict__ src, uint32_t pos, float wx, float wy,
                                     int h, int w, float (&out)[CH]) {
#pragma unroll
  for (int j = 0; j < CH; ++j) out[j] = 0.0f;
  if (pos == kInvalidTap) return;
  const int x0 = pos_x(pos), y0 = pos_y(pos);
  const float ex = 1.0f - wx, ny = 1.0f - wy;
  const float wt[4] = {ny * ex, ny * wx, wy * ex, wy * wx};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int x = x0 + (t & 1), y = y0 + (t >> 1);
    const bool ok = x >= 0 && x < w && y >= 0 && y < h;
    const float* px = src + ((size_t)(ok ? y : 0) * w + (ok ? x : 0)) * CH;
    const float wk = ok ? wt[t] : 0.0f;
#pragma unroll
    for (int q = 0; q < CH / 4; ++q) {
      const float4 a = *reinterpret_cast<const float4*>(px + 4 * q);
      out[4 * q + 0] += a.x * wk;
      out[4 * q + 1] += a.y * wk;
      out[4 * q + 2] += a.z * wk;
      out[4 * q + 3] += a.w * wk;
    }
  }
}

// One workgroup: sample b, a 16x16 pixel tile, planes [k0, k0 + npl) (npl <= kPG).
//   1. every thread computes the source corner/fractions of its pixel for every (plane, source
//      view) into registers (the ref view's sampling is plane independent: P = I exactly);
//   2. the union footprint of the whole plane group is reduced over the workgroup; if all source
//      views fit the LDS budget the group is processed as ONE sub-range, else plane by plane
//      (a plane that still does not fit gathers straight from global memory);
//   3. per sub-range and per CH-channel chunk: stage the footprints, then every thread samples
//      V views x CH channels per plane and writes CH cost-volume values (two-pass variance).
// depth planes per workgroup: the per-(plane, source view) tap state lives in registers
#ifndef MVS_EXP_PG
#define MVS_EXP_PG 8
#endif
template <int V>
constexpr int planes_per_group() { return V <= 3 ? MVS_EXP_PG : 4; }

template <int V, int CH>
__global__ __launch_bounds__(kBlock) void cost_volume_lds_kernel(
    const float* __restrict__ packed, const float* __restrict__ sampling, float* __restrict__ cv,
    int C, int h, int w, int Dc, int pg, int tiles_x, int tiles_y, int groups, int total) {
  // pg (<= kPG) planes per workgroup, chosen by the host so that small problems still fill the chip
  constexpr int NS = V - 1;
  constexpr int kPG = planes_per_group<V>();
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  __shared__ int scratch[4 * 4 * (NS > 0 ? NS : 1)];

  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int g = wk % groups;
  const int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  const int b = t / (tiles_x * tiles_y);
  const int px = (tile % tiles_x) * kTW + (threadIdx.x % kTW);
  const int py = (tile / tiles_x) * kTH + (threadIdx.x / kTW);
  const bool active = px < w && py < h;
  const int k0 = g * pg;
  const int npl = min(pg, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const int nch = (C + CH - 1) / CH;
  const float xn = norm_coord(px, w);
  const float yn = norm_coord(py, h);

  // 1. sampling coordinates
  uint32_t rpos;
  float rwx, rwy;
  src_coords(sampling + ((size_t)(b * V) * Dc + k0) * 9, xn, yn, h, w, active, rpos, rwx, rwy);
  uint32_t pos[kPG][NS > 0 ? NS : 1];
  float fwx[kPG][NS > 0 ? NS : 1], fwy[kPG][NS > 0 ? NS : 1];
#pragma unroll
  for (int pl = 0; pl < kPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pos[pl][s] = kInvalidTap;
      fwx[pl][s] = fwy[pl][s] = 0.0f;
      if (pl < npl)
        src_coords(sampling + ((size_t)(b * V + 1 + s) * Dc + k0 + pl) * 9, xn, yn, h, w, active,
                   pos[pl][s], fwx[pl][s], fwy[pl][s]);
    }

  // footprint of planes [lo, hi) per source view -> regions; returns true if all fit
  auto plan = [&](int lo, int hi, Region (&reg)[NS > 0 ? NS : 1]) -> bool {
    int bb[4 * (NS > 0 ? NS : 1)];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      int mnx = 1 << 30, mny = 1 << 30, mxx = 1 << 30, mxy = 1 << 30;  // mx* hold -max
#pragma unroll
      for (int pl = 0; pl < kPG; ++pl) {
        const uint32_t p = pos[pl][s];
        if (pl >= lo && pl < hi && p != kInvalidTap) {
          mnx = min(mnx, pos_x(p));
          mny = min(mny, pos_y(p));
          mxx = min(mxx, -(pos_x(p) + 1));
          mxy = min(mxy, -(pos_y(p) + 1));
        }
      }
      bb[4 * s + 0] = mnx;
      bb[4 * s + 1] = mny;
      bb[4 * s + 2] = mxx;
      bb[4 * s + 3] = mxy;
    }
    block_min<4 * (NS > 0 ? NS : 1)>(bb, scratch);
    int off = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      Region& r = reg[s];
      r.x0 = bb[4 * s + 0];
      r.y0 = bb[4 * s + 1];
      const int x1 = -bb[4 * s + 2], y1 = -bb[4 * s + 3];
      const bool empty = r.x0 > x1;
      r.rw = empty ? 0 : x1 - r.x0 + 1;
      r.rh = empty ? 0 : y1 - r.y0 + 1;
      r.base = off;
      off += region_bytes<CH>(r);
    }
    return off <= kLdsBytes;
  };

  const float inv_v = 1.0f / (float)V;
  // process planes [lo, hi) with the given regions (staged) or from global memory
  auto run = [&](int lo, int hi, const Region (&reg)[NS > 0 ? NS : 1], bool staged) {
    for (int ch = 0; ch < nch; ++ch) {
      const float* ref_src = packed + ((size_t)(b * V) * nch + ch) * hw * CH;
      if (staged) {
#if !defined(MVS_EXP_NO_STAGE)
#pragma unroll
        for (int s = 0; s < NS; ++s)
          stage_region<CH>(lds, reg[s], packed + ((size_t)(b * V + 1 + s) * nch + ch) * hw * CH, h, w);
#endif
        __syncthreads();
      }
      float x0v[CH];
      gather_global<CH>(ref_src, rpos, rwx, rwy, h, w, x0v);
#pragma unroll
      for (int pl = 0; pl < kPG; ++pl) {
        if (pl < lo || pl >= hi) continue;
        float sum[CH], val[NS > 0 ? NS : 1][CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) sum[j] = x0v[j];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          // opaque copies: stop the compiler from hoisting per-(plane, view) tap addresses and
          // weights out of the chunk loop (16 sets x 8 registers would not fit)
          uint32_t tpos = pos[pl][s];
          float twx = fwx[pl][s], twy = fwy[pl][s];
          asm volatile("" : "+v"(tpos), "+v"(twx), "+v"(twy));
#if defined(MVS_EXP_NO_GATHER)  // experiment: store path + staging only
          for (int j = 0; j < CH; ++j) val[s][j] = twx * (float)j + twy;
          if (false) {
          } else if (false)
#else
          if (staged)
#endif
            gather_lds<CH>(lds, reg[s], tpos, twx, twy, val[s]);
          else
            gather_global<CH>(packed + ((size_t)(b * V + 1 + s) * nch + ch) * hw * CH, tpos, twx,
                              twy, h, w, val[s]);
#pragma unroll
          for (int j = 0; j < CH; ++j) sum[j] += val[s][j];
        }
        if (active) {
          float* ob = cv + ((size_t)b * C * Dc + (size_t)(k0 + pl)) * hw + (size_t)py * w + px;
#pragma unroll
          for (int j = 0; j < CH; ++j) {
            const int c = ch * CH + j;
            if (c < C) {
              const float mean = sum[j] * inv_v;
              float d = x0v[j] - mean;
              float acc = d * d;
#pragma unroll
              for (int s = 0; s < NS; ++s) {
                d = val[s][j] - mean;
                acc += d * d;
              }
#if defined(MVS_EXP_NO_STORE)  // experiment: keep the compute, drop the traffic
              if (acc != acc) ob[(size_t)c * Dc * hw] = acc * inv_v;
#elif defined(MVS_EXP_PLAIN_STORE)
              ob[(size_t)c * Dc * hw] = acc * inv_v;
#else
              __builtin_nontemporal_store(acc * inv_v, ob + (size_t)c * Dc * hw);
#endif
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep each plane's LDS reads out of its neighbours'
      }
      if (staged) __syncthreads();
    }
  };

  Region reg[NS > 0 ? NS : 1];
  const bool whole = plan(0, npl, reg);   // whole plane group in one staging pass?
  const int nsub = whole ? 1 : npl;
  for (int sr = 0; sr < nsub; ++sr) {
    const int lo = whole ? 0 : sr, hi = whole ? npl : sr + 1;
#if defined(MVS_EXP_FORCE_GLOBAL)
    const bool staged = whole ? false : (plan(lo, hi, reg) && false);
#else
    const bool staged = whole ? true : plan(lo, hi, reg);
#endif
    run(lo, hi, reg, staged);
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
inline int hip_status() {
  return hipGetLastError() == hipSuccess ? MVS_OK : MVS_ERR_HIP;
}

struct Geometry {
  int B, V, C, h, w, Dc, tiles, total;
};

int check_geometry(int B, int V, int C, int h, int w, int d_count, Geometry& g) {
  if (B <= 0 || C <= 0 || h < 2 || w < 2 || d_count <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if (V < 1 || V > MVS_MAX_VIEWS) return MVS_ERR_UNSUPPORTED_VIEWS;
  const uint64_t hw = (uint64_t)h * (uint64_t)w;
  // per-image plane offsets are 32-bit; the work id is a 32-bit int
  if ((uint64_t)C * hw >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const uint64_t tiles = (hw + kBlock - 1) / kBlock;
  const uint64_t total = (uint64_t)B * tiles * (uint64_t)d_count;
  if (total >= (1ull << 31) - 8) return MVS_ERR_TOO_LARGE;
  g.B = B;
  g.V = V;
  g.C = C;
  g.h = h;
  g.w = w;
  g.Dc = d_count;
  g.tiles = (int)tiles;
  g.total = (int)total;
  return MVS_OK;
}

inline dim3 xcd_grid(int total) { return dim3(8u * (unsigned)((total + 7) / 8)); }

template <int MAXV, bool EXACT>
void launch_fused(const Geometry& g, const float* feat, const float* smp, float* cv,
                  hipStream_t s) {
  hipLaunchKernelGGL((cost_volume_kernel<MAXV, EXACT, 4>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, smp, cv, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

#ifndef MVS_EXP_CH3
#define MVS_EXP_CH3 8
#endif
inline int packed_chunk(int n_views) { return n_views <= 3 ? MVS_EXP_CH3 : 4; }

template <int V, int CH>
void launch_lds(const Geometry& g, const float* feat, const float* smp, float* packed, float* cv,
                hipStream_t s) {
  const uint32_t hw = (uint32_t)g.h * (uint32_t)g.w;
  const size_t n_pack = (size_t)g.B * V * ((g.C + CH - 1) / CH) * hw;
  const unsigned pgrid = (unsigned)std::min<size_t>((n_pack + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL((pack_features_kernel<CH>), dim3(pgrid), dim3(kBlock), 0, s, feat, packed,
                     g.B * V, g.C, hw);
  const int tiles_x = (g.w + kTW - 1) / kTW, tiles_y = (g.h + kTH - 1) / kTH;
  // planes per workgroup: the register maximum, lowered until the grid has >= 4 workgroups per CU
  int pg = planes_per_group<V>();
  while (pg > 1 && (long)g.B * tiles_x * tiles_y * ((g.Dc + pg - 1) / pg) < 1024) pg >>= 1;
  const int groups = (g.Dc + pg - 1) / pg;
  const int total = g.B * tiles_x * tiles_y * groups;
  hipLaunchKernelGGL((cost_volume_lds_kernel<V, CH>), xcd_grid(total), dim3(kBlock), 0, s, packed,
                     smp, cv, g.C, g.h, g.w, g.Dc, pg, tiles_x, tiles_y, groups, total);
}

template <int MAXV, bool EXACT>
void launch_bwd(const Geometry& g, const float* feat, const float* smp, const float* gcv,
                float* gf, hipStream_t s) {
  hipLaunchKernelGGL((cost_volume_bwd_kernel<MAXV, EXACT>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, smp, gcv, gf, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
}

}  // namespace

extern "C" {

int mvs_abi_version(void) { return MVS_ABI_VERSION; }

const char* mvs_status_string(int status) {
  switch (status) {
    case MVS_OK: return "ok";
    case MVS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MVS_ERR_UNSUPPORTED_VIEWS: return "n_views outside [1, MVS_MAX_VIEWS]";
    case MVS_ERR_TOO_LARGE: return "tensor exceeds the kernel's 32-bit index space";
    case MVS_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

size_t mvs_sampling_workspace_bytes(int n_images, int d_count) {
  if (n_images <= 0 || d_count <= 0) return 0;
  return (size_t)n_images * (size_t)d_count * 9 * sizeof(float);
}

int mvs_plane_sampling(const float* K, const float* R, const float* T, const float* d_min,
                       const float* d_int, int batch_size, int n_views, int h, int w, int d_begin,
                       int d_count, float d_scale, float* sampling, void* stream) {
  if (!K || !R || !T || !d_min || !d_int || !sampling) return MVS_ERR_INVALID_ARGUMENT;
  if (batch_size <= 0 || h < 2 || w < 2 || d_count <= 0 || d_begin < 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_views < 1 || n_views > MVS_MAX_VIEWS) return MVS_ERR_UNSUPPORTED_VIEWS;
  const int n = batch_size * n_views * d_count;
  hipLaunchKernelGGL(plane_sampling_kernel, dim3((n + 127) / 128), dim3(128), 0,
                     (hipStream_t)stream, K, R, T, d_min, d_int, batch_size, n_views, h, w,
                     d_begin, d_count, d_scale, sampling);
  return hip_status();
}

size_t mvs_cost_volume_workspace_bytes(int batch_size, int n_views, int channels, int h, int w,
                                       int d_count) {
  if (batch_size <= 0 || n_views <= 0 || channels <= 0 || h <= 0 || w <= 0 || d_count <= 0) return 0;
  const size_t n = (size_t)batch_size * n_views;
  const size_t ch = packed_chunk(n_views);
  const size_t nch = ((size_t)channels + ch - 1) / ch;
  return align256(mvs_sampling_workspace_bytes((int)n, d_count)) +
         n * nch * ch * (size_t)h * (size_t)w * sizeof(float);
}

int mvs_cost_volume_fwd(const float* feat, const float* K, const float* R, const float* T,
                        const float* d_min, const float* d_int, int batch_size, int n_views,
                        int channels, int h, int w, int d_begin, int d_count, float d_scale,
                        float* workspace, float* cv_out, void* stream) {
  if (!feat || !workspace || !cv_out) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g);
  if (st != MVS_OK) return st;
  st = mvs_plane_sampling(K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count,
                          d_scale, workspace, stream);
  if (st != MVS_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  if (n_views == 1) {  // variance of a single view is identically zero
    if (hipMemsetAsync(cv_out, 0, (size_t)batch_size * channels * d_count * h * w * sizeof(float), s) !=
        hipSuccess)
      return MVS_ERR_HIP;
    return hip_status();
  }
  if (n_views > 8) {  // generic path: direct gathers from the NCHW features
    launch_fused<MVS_MAX_VIEWS, false>(g, feat, workspace, cv_out, s);
    return hip_status();
  }
  float* packed = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) +
                                           align256(mvs_sampling_workspace_bytes(g.B * g.V, g.Dc)));
  switch (n_views) {
    case 2: launch_lds<2, MVS_EXP_CH3>(g, feat, workspace, packed, cv_out, s); break;
    case 3: launch_lds<3, MVS_EXP_CH3>(g, feat, workspace, packed, cv_out, s); break;
    case 4: launch_lds<4, 4>(g, feat, workspace, packed, cv_out, s); break;
    case 5: launch_lds<5, 4>(g, feat, workspace, packed, cv_out, s); break;
    case 6: launch_lds<6, 4>(g, feat, workspace, packed, cv_out, s); break;
    case 7: launch_lds<7, 4>(g, feat, workspace, packed, cv_out, s); break;
    default: launch_lds<8, 4>(g, feat, workspace, packed, cv_out, s); break;
  }
  return hip_status();
}

int mvs_homography_warp_fwd(const float* feat, const float* K, const float* R, const float* T,
                            const float* d_min, const float* d_int, int batch_size, int n_views,
                            int channels, int h, int w, int d_begin, int d_count, float d_scale,
                            float* workspace, float* warped_out, void* stream) {
  if (!feat || !workspace || !warped_out) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g);
  if (st != MVS_OK) return st;
  st = mvs_plane_sampling(K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count,
                          d_scale, workspace, stream);
  if (st != MVS_OK) return st;
  hipLaunchKernelGGL((warp_kernel<MVS_MAX_VIEWS, false, 4>), xcd_grid(g.total), dim3(kBlock), 0,
                     (hipStream_t)stream, feat, workspace, warped_out, g.V, g.C, g.h, g.w, g.Dc,
                     g.tiles, g.total);
  return hip_status();
}

int mvs_assemble_cost_volume_fwd(const float* warped, int batch_size, int n_views, int channels,
                                 int d, int h, int w, float* cv_out, void* stream) {
  if (!warped || !cv_out || batch_size <= 0 || channels <= 0 || d <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_views < 1) return MVS_ERR_UNSUPPORTED_VIEWS;
  const size_t M = (size_t)channels * d * h * w;
  const size_t n = (size_t)batch_size * M;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock < 8192 ? (n + kBlock - 1) / kBlock : 8192);
  hipLaunchKernelGGL(variance_kernel, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, warped,
                     batch_size, n_views, M, cv_out);
  return hip_status();
}

int mvs_cost_volume_bwd(const float* feat, const float* sampling, const float* grad_cv,
                        int batch_size, int n_views, int channels, int h, int w, int d_count,
                        float* grad_feat, void* stream) {
  if (!feat || !sampling || !grad_cv || !grad_feat) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  const int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g);
  if (st != MVS_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(grad_feat, 0,
                     (size_t)batch_size * n_views * channels * h * w * sizeof(float), s) !=
      hipSuccess)
    return MVS_ERR_HIP;
  switch (n_views) {
    case 1: launch_bwd<1, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 2: launch_bwd<2, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 3: launch_bwd<3, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 5: launch_bwd<5, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    default: launch_bwd<MVS_MAX_VIEWS, false>(g, feat, sampling, grad_cv, grad_feat, s); break;
  }
  return hip_status();
}

int mvs_extract_depth_map_fwd(const float* prob, const float* d_batch, int batch_size, int d,
                              int h, int w, int n_est, float* depth_out, void* stream) {
  if (!prob || !d_batch || !depth_out || batch_size <= 0 || d <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_est < 1) return MVS_ERR_INVALID_ARGUMENT;
  if (n_est > d) n_est = d;  // every plane has index < n_est: all kept
  if (n_est > 16) return MVS_ERR_INVALID_ARGUMENT;
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const size_t n = (size_t)batch_size * hw;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
  hipStream_t s = (hipStream_t)stream;
  if (n_est <= 8)
    hipLaunchKernelGGL((soft_argmin_kernel<8>), grid, dim3(kBlock), 0, s, prob, d_batch,
                       batch_size, d, hw, n_est, depth_out);
  else
    hipLaunchKernelGGL((soft_argmin_kernel<16>), grid, dim3(kBlock), 0, s, prob, d_batch,
                       batch_size, d, hw, n_est, depth_out);
  return hip_status();
}

}  // extern "C"
