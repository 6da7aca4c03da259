// conv2d_narrow.hip -- the 2-D feature encoder's and refinement net's bias-free Conv2d layers
// (model.py:22-65 FeatureEncoder, model.py:134-145 refinement), direct convolution with the eval
// BatchNorm + ReLU that follows them fused into the epilogue.  MIOpen runs these narrow layers
// (3..32 channels) at a small fraction of HBM speed (8 -> 8 at 512 x 640 x 12 images: 0.32 ms for
// 252 MB of activations); they are on the inference step's critical path.
//
// out[n][co][oy][ox] = sum_{c, ky, kx} W[co][c][ky][kx] * in[n][c][oy*S + ky - P][ox*S + kx - P]
// (zero outside the image, P = K / 2), accumulated in fp32 in the order c, ky, kx with one fma per
// term; optional epilogue max((v - mean) * scale + shift, 0).
//
// A 256-thread workgroup owns a 32 x 8 output tile of one image; one thread = one output pixel x
// COUT channels in registers (channel pairs on the packed fp32 FMA: the tap broadcast to both
// halves, the pair's weights one 64-bit scalar operand -- weights pre-transposed wt[c][ky][kx][co]
// (ops.py) and read through the constant address space, so every pair is an s_load).  The input
// halo of the tile ((8-1)*S + K rows x (32-1)*S + K columns, zero outside the image) is staged in
// LDS NC channels per pass; the next pass's elements are loaded into registers before this pass's
// arithmetic.
#include <cstdlib>

#include "launchers.h"
#include "split.h"

namespace mvs {
namespace {

constexpr int k2TX = 32, k2TY = 8;

typedef float f2v_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const f2v_t const_f2v;

constexpr int pass_channels(int cin, int cap) {
  int nc = 1;
  for (int d = 1; d <= cin && d <= cap; ++d)
    if (cin % d == 0) nc = d;
  return nc;
}

template <int CIN, int COUT, int K, int S, int SPLIT>
__global__ __launch_bounds__(kBlock) void conv2d_narrow_kernel(
    const float* __restrict__ in, const float* __restrict__ wt, float* __restrict__ out, int H, int W, int Ho,
    int Wo, int tiles_x, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, uint32_t* __restrict__ yb) {
  constexpr int P = K / 2;
  constexpr int IH = (k2TY - 1) * S + K, IW = (k2TX - 1) * S + K;
  constexpr int kPlane = IH * IW;
  // channels per staging pass: the largest divisor of CIN within about 20 KB of LDS
  constexpr int NC = pass_channels(CIN, 5120 / kPlane);
  constexpr int kStage = NC * kPlane;
  constexpr int kPer = (kStage + kBlock - 1) / kBlock;
  // SPLIT workgroups per tile (blockIdx.z) share the output channels: CO each, from co0
  constexpr int CO = COUT / SPLIT;
  constexpr int NP = CO / 2;
  __shared__ float lds[kStage];
  const int co0 = (int)blockIdx.z * CO;

  const int tile = (int)blockIdx.x;
  const int ox0 = (tile % tiles_x) * k2TX, oy0 = (tile / tiles_x) * k2TY;
  const int n = (int)blockIdx.y;
  const size_t plane = (size_t)H * W;
  const float* ib = in + (size_t)n * CIN * plane;
  const int iy0 = oy0 * S - P, ix0 = ox0 * S - P;

  // staging map: element e of one pass -> (offset inside the pass's first channel plane, valid)
  int goff[kPer];
  bool gok[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int e = (int)threadIdx.x + j * kBlock;
    const int c = e / kPlane, r = e % kPlane;
    const int gy = iy0 + r / IW, gx = ix0 + r % IW;
    gok[j] = e < kStage && gy >= 0 && gy < H && gx >= 0 && gx < W;
    goff[j] = gok[j] ? (int)((size_t)c * plane + (size_t)gy * W + gx) : 0;
  }
  float pre[kPer];
  auto fetch = [&](int q) {
    const float* src = ib + (size_t)q * NC * plane;
#pragma unroll
    for (int j = 0; j < kPer; ++j) pre[j] = gok[j] ? src[goff[j]] : 0.0f;
  };
  fetch(0);

  const int lx = (int)threadIdx.x % k2TX, ly = (int)threadIdx.x / k2TX;
  f2v_t acc2[NP > 0 ? NP : 1];
  float acc1 = 0.0f;
#pragma unroll
  for (int q = 0; q < (NP > 0 ? NP : 1); ++q) acc2[q] = f2v_t{0.0f, 0.0f};

  for (int q = 0; q < CIN / NC; ++q) {
    __syncthreads();   // the previous pass's reads are done
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int e = (int)threadIdx.x + j * kBlock;
      if (e < kStage) lds[e] = pre[j];
    }
    __syncthreads();
    if (q + 1 < CIN / NC) fetch(q + 1);   // in flight during this pass's arithmetic
#pragma unroll 1
    for (int u = 0; u < NC; ++u) {
      const int c = q * NC + u;
      const float* lc = lds + u * kPlane + (ly * S) * IW + lx * S;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float tap[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) tap[kx] = lc[ky * IW + kx];
        if constexpr (NP > 0) {
          // the K x COUT weights of (c, ky): workgroup-uniform, scalar loads
          const const_f2v* wg =
              (const const_f2v*)uniform_ptr(wt + ((size_t)(c * K + ky) * K) * COUT + co0);
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            // the memory clobber keeps the compiler from hoisting more than one tap's COUT weights
            // (they would not fit the SGPRs at COUT = 32)
            asm volatile("" ::: "memory");
#pragma unroll
            for (int p = 0; p < NP; ++p)
              acc2[p] = __builtin_elementwise_fma(f2v_t{tap[kx], tap[kx]}, wg[kx * (COUT / 2) + p], acc2[p]);
          }
        } else {
          const const_float* wg = (const const_float*)uniform_ptr(wt + (size_t)(c * K + ky) * K);
#pragma unroll
          for (int kx = 0; kx < K; ++kx) acc1 = fmaf(tap[kx], wg[kx], acc1);
        }
      }
    }
  }

  const int gx = ox0 + lx, gy = oy0 + ly;
  float vmax = 0.0f;   // the output's bound words (split-fp16 consumers: conv2d_split.hip)
  if (gx < Wo && gy < Ho) {
    const size_t oplane = (size_t)Ho * Wo;
    float* ob = out + ((size_t)n * COUT + co0) * oplane + (size_t)gy * Wo + gx;
#pragma unroll
    for (int c = 0; c < CO; ++c) {
      const int co = co0 + c;
      float v = NP > 0 ? acc2[c / 2][c & 1] : acc1;
      if (bn_scale) v = fmaxf((v - bn_mean[co]) * bn_scale[co] + bn_shift[co], 0.0f);
      vmax = fmaxf(vmax, fabsf(v));
      ob[(size_t)c * oplane] = v;
    }
  }
  if (yb) bound_update(yb, vmax);
}

// output-channel split: a small grid leaves SIMDs idle (the refinement net's 4 x 128 x 160 layers:
// 320 workgroups), so grids under kSplitTarget workgroups split COUT over up to MAXS workgroups per
// tile (the staging is repeated, the FMAs are not; each channel's sum is unchanged, bit for bit).
// Measured at cfg 2 (tools/enc_layers.py): refinement 32 -> 32 0.051 -> 0.028 ms at split 4; the
// encoder's 960-workgroup layers gain nothing from a split (32 -> 32) or lose (16 -> 32: 0.104 ->
// 0.108 / 0.132 ms at 2 / 4).  MVS_CONV2D_SPLIT forces a split (<= MAXS).
constexpr int kSplitTarget = 960;

template <int CIN, int COUT, int K, int S, int MAXS>
void launch2d(const float* in, const float* wt, float* out, int N, int H, int W, const float* sc,
              const float* sh, const float* mu, uint32_t* yb, hipStream_t s) {
  const int Ho = (H + 2 * (K / 2) - K) / S + 1, Wo = (W + 2 * (K / 2) - K) / S + 1;
  const int tiles_x = (Wo + k2TX - 1) / k2TX, tiles_y = (Ho + k2TY - 1) / k2TY;
  const long wgs = (long)tiles_x * tiles_y * N;
  int split = 1;
  while (split < MAXS && wgs * split < kSplitTarget) split *= 2;
  if (const char* e = getenv("MVS_CONV2D_SPLIT")) {
    const int f = atoi(e);
    if (f >= 1) split = f > MAXS ? MAXS : f;
  }
  const dim3 grid((unsigned)(tiles_x * tiles_y), (unsigned)N, (unsigned)split);
  if (split >= 4 && MAXS >= 4)
    hipLaunchKernelGGL((conv2d_narrow_kernel<CIN, COUT, K, S, (MAXS >= 4 ? 4 : 1)>), grid, dim3(kBlock), 0, s, in,
                       wt, out, H, W, Ho, Wo, tiles_x, sc, sh, mu, yb);
  else if (split >= 2 && MAXS >= 2)
    hipLaunchKernelGGL((conv2d_narrow_kernel<CIN, COUT, K, S, (MAXS >= 2 ? 2 : 1)>), dim3(grid.x, grid.y, 2),
                       dim3(kBlock), 0, s, in, wt, out, H, W, Ho, Wo, tiles_x, sc, sh, mu, yb);
  else
    hipLaunchKernelGGL((conv2d_narrow_kernel<CIN, COUT, K, S, 1>), dim3(grid.x, grid.y, 1), dim3(kBlock), 0, s, in,
                       wt, out, H, W, Ho, Wo, tiles_x, sc, sh, mu, yb);
}

}  // namespace

int launch_conv2d_narrow(const float* in, const float* wt, float* out, int N, int Cin, int Cout, int H, int W,
                         int K, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                         uint32_t* y_bound, hipStream_t s) {
#define MVS_CONV2D_CASE(A, C, KK, SS, MS)                                               \
  if (Cin == A && Cout == C && K == KK && stride == SS) {                               \
    launch2d<A, C, KK, SS, MS>(in, wt, out, N, H, W, bn_scale, bn_shift, bn_mean, y_bound, s); \
    return MVS_OK;                                                                      \
  }
  // FeatureEncoder (model.py:22-65) and the refinement net (model.py:134-145); the last argument
  // is the largest output-channel split (CO = COUT / split stays a multiple of 8)
  MVS_CONV2D_CASE(3, 8, 3, 1, 1) MVS_CONV2D_CASE(8, 8, 3, 1, 1) MVS_CONV2D_CASE(8, 16, 5, 2, 2)
  MVS_CONV2D_CASE(16, 16, 3, 1, 2) MVS_CONV2D_CASE(16, 32, 5, 2, 4) MVS_CONV2D_CASE(32, 32, 3, 1, 4)
  MVS_CONV2D_CASE(4, 32, 3, 1, 4) MVS_CONV2D_CASE(32, 1, 3, 1, 1)
#undef MVS_CONV2D_CASE
  return MVS_ERR_INVALID_ARGUMENT;
}

}  // namespace mvs
