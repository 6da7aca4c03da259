// conv3d_narrow.hip -- 3x3x3, stride-1, padding-1, bias-free Conv3d with few output channels
// (COUT = 1 or 8), for the regulariser's full-resolution layers that MIOpen runs far below the
// chip's fp32 rate: conv_0_0 (32 -> 8, model.py:77) and conv_out (8 -> 1, model.py:96).
//
// out[b][co][d][y][x] = sum_{c, kd, ky, kx} W[co][c][kd][ky][kx] * in[b][c][d+kd-1][y+ky-1][x+kx-1]
// (zero outside the volume), accumulated in fp32 in the order c, kd, ky, kx with one fma per term.
//
// A 256-thread workgroup owns a 32 x 8 NR (x, y) tile and DT consecutive depths of one sample; one
// thread = NR (x, y) columns of DT output voxels x COUT channels, held in registers.  Per input
// channel the workgroup stages the (DT + 2) x 10 x 34 halo block in LDS (zero-filled outside the
// volume) plus that channel's COUT x 27 weights, then every thread reads the 9 taps of each staged
// plane once (54 VGPRs) and applies them to the output depths they reach (plane p feeds depth
// p - kd).  Weights are workgroup-uniform scalar loads, 9 at a time (SGPR operands of the fmas).  The staging of channel c + 1 is loaded into registers before
// channel c is computed.  Compute-bound: COUT * 27 fmas per staged input element.
#include "launchers.h"

namespace mvs {
namespace {

constexpr int kTX = 32, kDT = 4;
constexpr int kWPad = 12;                  // one (co, kd) row of 9 weights, padded to 3 float4

// NR output rows per thread: the workgroup tile is 32 x (8 NR); a thread reads (NR + 2) x 3 taps
// per staged plane and applies each (co, kd) weight row to NR x DT outputs, so the broadcast weight
// reads (the LDS-bound part at NR = 1) are amortised over NR times the fmas.
#ifdef MVS_EXP_CONV_WPE
#define MVS_CONV_ATTR __attribute__((amdgpu_waves_per_eu(MVS_EXP_CONV_WPE)))
#else
#define MVS_CONV_ATTR
#endif
template <int COUT, int NR>
__global__ __launch_bounds__(kBlock) MVS_CONV_ATTR void conv3d_k3_narrow_kernel(
    const float* __restrict__ in, const float* __restrict__ wt, float* __restrict__ out, int Cin,
    int D, int H, int W, int tiles_x, int tiles_y, int dgroups, const float* __restrict__ bn_scale,
    const float* __restrict__ bn_shift, const float* __restrict__ bn_mean) {
  constexpr int kTY = 8 * NR;
  constexpr int kPX = kTX + 2, kPY = kTY + 2, kPD = kDT + 2;
  constexpr int kPlane = kPX * kPY;
  constexpr int kStage = kPD * kPlane;                      // floats per input channel
  constexpr int kPer = (kStage + kBlock - 1) / kBlock;      // staging elements per thread
  __shared__ float lds[kStage];
  __shared__ __attribute__((aligned(16))) float wl[COUT * 3 * kWPad];   // W[co][c][kd][.] of channel c
  int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * kTX;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * kTY;
  t /= tiles_y;
  const int d0 = (t % dgroups) * kDT;
  const int b = t / dgroups;
  const size_t plane = (size_t)H * W;
  const size_t vol = (size_t)D * plane;
  const float* ib = in + (size_t)b * Cin * vol;

  // staging map: element e of the halo block -> (global offset inside one channel, valid)
  int goff[kPer];
  bool gok[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int e = (int)threadIdx.x + j * kBlock;
    const int pd = e / kPlane, r = e % kPlane;
    const int py = r / kPX, px = r % kPX;
    const int gz = d0 + pd - 1, gy = ty0 + py - 1, gx = tx0 + px - 1;
    gok[j] = e < kStage && gz >= 0 && gz < D && gy >= 0 && gy < H && gx >= 0 && gx < W;
    goff[j] = gok[j] ? (int)((size_t)gz * plane + (size_t)gy * W + gx) : 0;
  }
  float pre[kPer];
  auto fetch = [&](int c) {
    const float* src = ib + (size_t)c * vol;
#pragma unroll
    for (int j = 0; j < kPer; ++j) pre[j] = gok[j] ? src[goff[j]] : 0.0f;
  };
  fetch(0);

  const int lx = (int)threadIdx.x % kTX, ly = ((int)threadIdx.x / kTX) * NR;
  float acc[kDT][NR][COUT];
#pragma unroll
  for (int d = 0; d < kDT; ++d)
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int co = 0; co < COUT; ++co) acc[d][r][co] = 0.0f;

  for (int c = 0; c < Cin; ++c) {
    __syncthreads();   // previous channel's reads are done
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int e = (int)threadIdx.x + j * kBlock;
      if (e < kStage) lds[e] = pre[j];
    }
#ifdef MVS_EXP_CONV_LDSW
    for (int i = (int)threadIdx.x; i < COUT * 3 * kWPad; i += kBlock) {   // weights, rows padded to 12
      const int co = i / (3 * kWPad), r = i % (3 * kWPad);
      const int kd = r / kWPad, k = r % kWPad;
      wl[i] = k < 9 ? wt[((size_t)co * Cin + c) * 27 + kd * 9 + k] : 0.0f;
    }
#endif
    __syncthreads();
    if (c + 1 < Cin) fetch(c + 1);   // in flight during this channel's arithmetic
    // the (NR + 2) x 3 taps of every staged plane, read once
    float tap[kPD][NR + 2][3];
#pragma unroll
    for (int p = 0; p < kPD; ++p)
#pragma unroll
      for (int ry = 0; ry < NR + 2; ++ry)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) tap[p][ry][kx] = lds[p * kPlane + (ly + ry) * kPX + lx + kx];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
#ifndef MVS_EXP_CONV_LDSW
        // weights as scalar loads (SGPR operands of the fmas), at most 9 live at a time: the
        // memory clobber keeps the compiler from hoisting all 216 of a channel (630 SGPR spills);
        // 3.53 ms at cfg 2 against 3.92 ms with broadcast LDS reads (-DMVS_EXP_CONV_LDSW)
        asm volatile("" ::: "memory");
        const float* wg = wt + ((size_t)co * Cin + c) * 27 + kd * 9;
        float w[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) w[k] = wg[k];
#else
        // workgroup-uniform weights: broadcast LDS reads (one address for all lanes)
        const float4* wr = reinterpret_cast<const float4*>(wl + (co * 3 + kd) * kWPad);
        const float4 w0 = wr[0], w1 = wr[1], w2 = wr[2];
        const float w[9] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x};
#endif
#pragma unroll
        for (int d = 0; d < kDT; ++d)   // output depth d reads plane d + kd through kernel depth kd
#pragma unroll
          for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx)
                acc[d][r][co] = fmaf(tap[d + kd][r + ky][kx], w[ky * 3 + kx], acc[d][r][co]);
      }
  }

  const int gx = tx0 + lx;
  if (gx >= W) return;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int gy = ty0 + ly + r;
    if (gy >= H) break;
    float* ob = out + (size_t)b * COUT * vol + (size_t)gy * W + gx;
#pragma unroll
    for (int d = 0; d < kDT; ++d) {
      if (d0 + d >= D) break;
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        float v = acc[d][r][co];
        if (bn_scale) v = fmaxf((v - bn_mean[co]) * bn_scale[co] + bn_shift[co], 0.0f);
        ob[(size_t)co * vol + (size_t)(d0 + d) * plane] = v;
      }
    }
  }
}

template <int COUT, int NR>
void launch_narrow(const float* in, const float* weight, float* out, int B, int Cin, int D, int H, int W,
                   const float* bn_scale, const float* bn_shift, const float* bn_mean, hipStream_t s) {
  const int tiles_x = (W + kTX - 1) / kTX, tiles_y = (H + 8 * NR - 1) / (8 * NR), dgroups = (D + kDT - 1) / kDT;
  const dim3 grid((unsigned)((size_t)B * dgroups * tiles_y * tiles_x));
  hipLaunchKernelGGL((conv3d_k3_narrow_kernel<COUT, NR>), grid, dim3(kBlock), 0, s, in, weight, out, Cin, D,
                     H, W, tiles_x, tiles_y, dgroups, bn_scale, bn_shift, bn_mean);
}

}  // namespace

#ifndef MVS_EXP_CONV_NR
#define MVS_EXP_CONV_NR 1   /* 2 rows per thread: 256 VGPRs, 1 wave per SIMD, 4.17 vs 3.95 ms at cfg 2 */
#endif

void launch_conv3d_k3_narrow(const float* in, const float* weight, float* out, int B, int Cin,
                             int Cout, int D, int H, int W, const float* bn_scale, const float* bn_shift,
                             const float* bn_mean, hipStream_t s) {
  if (Cout == 8)
    launch_narrow<8, MVS_EXP_CONV_NR>(in, weight, out, B, Cin, D, H, W, bn_scale, bn_shift, bn_mean, s);
  else
    launch_narrow<1, 1>(in, weight, out, B, Cin, D, H, W, bn_scale, bn_shift, bn_mean, s);
}

}  // namespace mvs
