// conv3d_narrow.hip -- 3x3x3, stride-1, padding-1, bias-free Conv3d with few output channels
// (COUT = 1 or 8), for the regulariser's full-resolution layers that MIOpen runs far below the
// chip's fp32 rate: conv_0_0 (32 -> 8, model.py:77) and conv_out (8 -> 1, model.py:96).
//
// out[b][co][d][y][x] = sum_{c, kd, ky, kx} W[co][c][kd][ky][kx] * in[b][c][d+kd-1][y+ky-1][x+kx-1]
// (zero outside the volume), accumulated in fp32 in the order c, kd, ky, kx with one fma per term.
//
// A 256-thread workgroup owns a 32 x 8 (x, y) tile and DT = 4 consecutive depths of one sample; one
// thread = DT output voxels x COUT channels, held in registers.  Per input channel the workgroup
// stages the (DT + 2) x 10 x 34 halo block in LDS (zero-filled outside the volume), and every
// thread reads the 9 taps of each staged plane once (54 VGPRs) and applies them to the output
// depths they reach (plane p feeds depth p - kd).  The staging of channel c + 1 is loaded into
// registers before channel c is computed.  Input NCDHW (C4 = 0), or channel-quad (the fused kernel's
// NC4DHW4 output): then a pass stages 4 channels with one 16-byte load per element (C4 = 1, fp32) or
// one 8-byte load widened to 4 fp32 (C4 = 2, bf16: the reduced-precision opt-in; widening is exact, so
// the arithmetic is the fp32 kernel's on the rounded values) into 4 LDS planes.
//   COUT = 8: output channels in pairs on the packed fp32 FMA (v_pk_fma_f32: the tap broadcast to
//   both halves, the two channels' weights as one 64-bit scalar operand), 2 FMAs per lane-
//   instruction -- the weights arrive pre-transposed as wt[c][kd][ky][kx][co] (ops.py), so each
//   pair is one s_load_dwordx2.  COUT = 1: scalar weights as the fmas' SGPR operand.
#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kTX = 32, kTY = 8, kDT = 4;

// WZ (COUT = 8): Winograd F(2,3) along depth.  The thread's 4 output depths are two windows of 2
// (planes 0..3 and 2..5 of the staged 6); per (channel, ky, kx) each window's 4 depth values z are
// transformed (v = B^T z: z0 - z2, z1 + z2, z2 - z1, z1 - z3, packed over the two windows) and
// multiplied position-wise with the transformed weights U = G g (g0, (g0 + g1 + g2) / 2,
// (g0 - g1 + g2) / 2, g2; formed in float64 on the host, ops.py), accumulated per position; the
// outputs are A^T m (m0 + m1 + m2, m1 - m2 - m3) at the end.  Per input channel 288 packed FMAs +
// 36 packed adds instead of 432 packed FMAs.  Weights wu[c][ky][kx][4][co].
// FOLD (COUT = 1, NCDHW: train mode's conv_out, CostVolumeReg.forward_live_train): the staged input is
// relu(BN_a(in)) + relu(BN_b(in2)) per channel, ibn = [6][Cin] (scale, shift, mean of in, then of in2)
// -- model.py:121-123's `relu(BN_0(deconv_1_0)) + y0` formed on load instead of by a pass over the
// full volume; the zero padding stays zero
template <int COUT, int C4, bool WZ = false, int DT = kDT, bool FOLD = false>
__global__ __launch_bounds__(kBlock) void conv3d_k3_narrow_kernel(
    const float* __restrict__ in, const float* __restrict__ wt, float* __restrict__ out, int Cin,
    int D, int H, int W, int tiles_x, int tiles_y, int dgroups, int n_batch, const float* __restrict__ bn_scale,
    const float* __restrict__ bn_shift, const float* __restrict__ bn_mean, const float* __restrict__ in2,
    const float* __restrict__ ibn) {
  static_assert(!FOLD || (COUT == 1 && C4 == 0), "folded input BN: conv_out on NCDHW");
  static_assert(!WZ || DT == 4, "depth Winograd: two windows of 2");
  constexpr int kPX = kTX + 2, kPY = kTY + 2, kPD = DT + 2;
  constexpr int kPlane = kPX * kPY;
  constexpr int kStage = kPD * kPlane;                      // floats per input channel
  constexpr int kPer = (kStage + kBlock - 1) / kBlock;      // staging elements per thread
  constexpr int NP = COUT / 2;                              // channel pairs (COUT = 8)
  constexpr int NQ = C4 ? 4 : 1;                            // channels staged per pass
  __shared__ float lds[NQ * kStage];
  // XCD-contiguous tiles: the halo-sharing neighbours (next x tile, next y row of tiles, next depth
  // group) run on the same XCD's L2 (common.h xcd_work_id)
  const int total = (int)gridDim.x;
  int t = xcd_work_id((int)blockIdx.x, total);
  if (t >= tiles_x * tiles_y * dgroups * n_batch) return;   // grid padding (no barrier passed yet)
  const int tx0 = (t % tiles_x) * kTX;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * kTY;
  t /= tiles_y;
  const int d0 = (t % dgroups) * DT;
  const int b = t / dgroups;
  const size_t plane = (size_t)H * W;
  const size_t vol = (size_t)D * plane;
  const float* ib = in + (size_t)b * Cin * vol;   // (channel-quad layout: the same element count)
  const uint2* ib16 = reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(in) + (size_t)b * Cin * vol * 2);

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
  // one pass = one input channel (NCDHW) or one channel quad (C4: 16-byte loads, 4 LDS planes)
  float pre[kPer][NQ];
  float pre2[FOLD ? kPer : 1];
  const float* ib2 = FOLD ? in2 + (size_t)b * Cin * vol : nullptr;
  auto fetch = [&](int q) {
    if constexpr (C4 == 2) {   // bf16 quad: the high halves of 4 fp32 words
      const uint2* src = ib16 + (size_t)q * vol;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint2 v = gok[j] ? src[goff[j]] : make_uint2(0u, 0u);
        pre[j][0] = __uint_as_float(v.x << 16);
        pre[j][1] = __uint_as_float(v.x & 0xFFFF0000u);
        pre[j][2] = __uint_as_float(v.y << 16);
        pre[j][3] = __uint_as_float(v.y & 0xFFFF0000u);
      }
    } else if constexpr (C4) {
      const float4* src = reinterpret_cast<const float4*>(ib) + (size_t)q * vol;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const float4 v = gok[j] ? src[goff[j]] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        pre[j][0] = v.x;
        pre[j][1] = v.y;
        pre[j][2] = v.z;
        pre[j][3] = v.w;
      }
    } else {
      const float* src = ib + (size_t)q * vol;
#pragma unroll
      for (int j = 0; j < kPer; ++j) pre[j][0] = gok[j] ? src[goff[j]] : 0.0f;
      if constexpr (FOLD) {
        const float* src2 = ib2 + (size_t)q * vol;
#pragma unroll
        for (int j = 0; j < kPer; ++j) pre2[j] = gok[j] ? src2[goff[j]] : 0.0f;
      }
    }
  };
  fetch(0);

  const int lx = (int)threadIdx.x % kTX, ly = (int)threadIdx.x / kTX;
  f2v acc2[DT][NP > 0 ? NP : 1];
  float acc1[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    acc1[d] = 0.0f;
#pragma unroll
    for (int q = 0; q < (NP > 0 ? NP : 1); ++q) acc2[d][q] = f2v{0.0f, 0.0f};
  }
  // WZ: per (window, position, channel pair): the Winograd-domain sums
  f2v accw[WZ ? 2 : 1][WZ ? 4 : 1][WZ ? NP : 1];
  if constexpr (WZ) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int ps = 0; ps < 4; ++ps)
#pragma unroll
        for (int q = 0; q < NP; ++q) accw[a][ps][q] = f2v{0.0f, 0.0f};
  }

  const int passes = C4 ? Cin / 4 : Cin;
  for (int q = 0; q < passes; ++q) {
    __syncthreads();   // the previous pass's reads are done
    if constexpr (FOLD) {   // channel q's two BatchNorms (workgroup-uniform)
      const float sa = ibn[q], ha = ibn[Cin + q], ma = ibn[2 * Cin + q];
      const float sb = ibn[3 * Cin + q], hb = ibn[4 * Cin + q], mb = ibn[5 * Cin + q];
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (gok[j]) pre[j][0] = fmaxf((pre[j][0] - ma) * sa + ha, 0.0f) + fmaxf((pre2[j] - mb) * sb + hb, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int e = (int)threadIdx.x + j * kBlock;
      if (e < kStage)
#pragma unroll
        for (int u = 0; u < NQ; ++u) lds[u * kStage + e] = pre[j][u];
    }
    __syncthreads();
    if (q + 1 < passes) fetch(q + 1);   // in flight during this pass's arithmetic
#pragma unroll 1
    for (int u = 0; u < NQ; ++u) {
      const int c = q * NQ + u;
      const float* lc = lds + u * kStage;
      if constexpr (WZ) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            // the tap's 6 staged planes, read as needed (not held across taps: registers);
            // windows A (planes 0..3) and B (planes 2..5) side by side in the two halves
            float t[kPD];
#pragma unroll
            for (int p = 0; p < kPD; ++p) t[p] = lc[p * kPlane + (ly + ky) * kPX + lx + kx];
            const f2v z0 = {t[0], t[2]}, z1 = {t[1], t[3]}, z2 = {t[2], t[4]}, z3 = {t[3], t[5]};
            const f2v v[4] = {z0 - z2, z1 + z2, z2 - z1, z1 - z3};
            asm volatile("" ::: "memory");
            const f2v* wg = reinterpret_cast<const f2v*>(wt + ((size_t)(c * 9 + ky * 3 + kx) * 4) * 8);
#pragma unroll
            for (int ps = 0; ps < 4; ++ps)
#pragma unroll
              for (int qq = 0; qq < NP; ++qq) {
                const f2v u = wg[ps * 4 + qq];
                accw[0][ps][qq] = __builtin_elementwise_fma(f2v{v[ps].x, v[ps].x}, u, accw[0][ps][qq]);
                accw[1][ps][qq] = __builtin_elementwise_fma(f2v{v[ps].y, v[ps].y}, u, accw[1][ps][qq]);
              }
          }
        continue;
      }
      // the 3 x 3 taps of every staged plane, read once
      float tap[kPD][3][3];
#pragma unroll
      for (int p = 0; p < kPD; ++p)
#pragma unroll
        for (int ry = 0; ry < 3; ++ry)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) tap[p][ry][kx] = lc[p * kPlane + (ly + ry) * kPX + lx + kx];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        if constexpr (COUT == 8) {
#pragma unroll
          for (int qq = 0; qq < NP; ++qq) {
            // weight pairs (co = 2qq, 2qq + 1) of the 9 (ky, kx) taps: workgroup-uniform scalar
            // loads; the memory clobber keeps the compiler from hoisting a whole channel's weights
            asm volatile("" ::: "memory");
            const f2v* wg = reinterpret_cast<const f2v*>(wt + ((size_t)(c * 3 + kd) * 9) * 8) + qq;
            f2v wp[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) wp[k] = wg[k * 4];
#pragma unroll
            for (int d = 0; d < DT; ++d)   // output depth d reads plane d + kd through kernel depth kd
#pragma unroll
              for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                  const float tv = tap[d + kd][ky][kx];
                  acc2[d][qq] = __builtin_elementwise_fma(f2v{tv, tv}, wp[ky * 3 + kx], acc2[d][qq]);
                }
          }
        } else {
          asm volatile("" ::: "memory");
          const float* wg = wt + ((size_t)c * 3 + kd) * 9;
          float w9[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) w9[k] = wg[k];
#pragma unroll
          for (int d = 0; d < DT; ++d)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) acc1[d] = fmaf(tap[d + kd][ky][kx], w9[ky * 3 + kx], acc1[d]);
        }
      }
    }
  }

  if constexpr (WZ) {   // A^T m: (m0 + m1 + m2, m1 - m2 - m3) per window
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int qq = 0; qq < NP; ++qq) {
        acc2[2 * a][qq] = accw[a][0][qq] + accw[a][1][qq] + accw[a][2][qq];
        acc2[2 * a + 1][qq] = accw[a][1][qq] - accw[a][2][qq] - accw[a][3][qq];
      }
  }
  const int gx = tx0 + lx, gy = ty0 + ly;
  if (gx >= W || gy >= H) return;
  float* ob = out + (size_t)b * COUT * vol + (size_t)gy * W + gx;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    if (d0 + d >= D) break;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float v = COUT == 8 ? acc2[d][co / 2][co & 1] : acc1[d];
      if (bn_scale) v = fmaxf((v - bn_mean[co]) * bn_scale[co] + bn_shift[co], 0.0f);
      ob[(size_t)co * vol + (size_t)(d0 + d) * plane] = v;
    }
  }
}

// COUT = 1 (conv_out): kOutDT output depths per thread -- the (DT + 2)-plane halo is re-read
// (DT + 2) / DT times (cfg 2: 4 -> 1.5x, 8 -> 1.25x of the 503 MB input)
#ifndef MVS_CONV_OUT_DT
#define MVS_CONV_OUT_DT 8
#endif
constexpr int kOutDT = MVS_CONV_OUT_DT;

template <int COUT, int C4, bool WZ = false, bool FOLD = false>
void launch_narrow(const float* in, const float* weight, float* out, int B, int Cin, int D, int H, int W,
                   const float* bn_scale, const float* bn_shift, const float* bn_mean, hipStream_t s,
                   const float* in2 = nullptr, const float* ibn = nullptr) {
  constexpr int DT = COUT == 1 ? kOutDT : kDT;
  const int tiles_x = (W + kTX - 1) / kTX, tiles_y = (H + kTY - 1) / kTY, dgroups = (D + DT - 1) / DT;
  const dim3 grid = xcd_grid(B * dgroups * tiles_y * tiles_x);
  hipLaunchKernelGGL((conv3d_k3_narrow_kernel<COUT, C4, WZ, DT, FOLD>), grid, dim3(kBlock), 0, s, in, weight, out,
                     Cin, D, H, W, tiles_x, tiles_y, dgroups, B, bn_scale, bn_shift, bn_mean, in2, ibn);
}

}  // namespace

void launch_conv3d_k3_narrow(const float* in, int in_c4, bool wino_z, const float* weight, float* out, int B,
                             int Cin, int Cout, int D, int H, int W, const float* bn_scale, const float* bn_shift,
                             const float* bn_mean, hipStream_t s, const float* in2, const float* ibn) {
  if (ibn) {   // conv_out with the folded BN + ReLU and the second input (capi checks the shape)
    launch_narrow<1, 0, false, true>(in, weight, out, B, Cin, D, H, W, bn_scale, bn_shift, bn_mean, s, in2, ibn);
    return;
  }
#define MVS_NARROW(CO, Q, WZ) launch_narrow<CO, Q, WZ>(in, weight, out, B, Cin, D, H, W, bn_scale, bn_shift, bn_mean, s)
  if (wino_z) {
    if (in_c4 == 2) MVS_NARROW(8, 2, true);
    else if (in_c4) MVS_NARROW(8, 1, true);
    else MVS_NARROW(8, 0, true);
  } else if (Cout == 8) {
    if (in_c4 == 2) MVS_NARROW(8, 2, false);
    else if (in_c4) MVS_NARROW(8, 1, false);
    else MVS_NARROW(8, 0, false);
  } else {
    if (in_c4 == 2) MVS_NARROW(1, 2, false);
    else if (in_c4) MVS_NARROW(1, 1, false);
    else MVS_NARROW(1, 0, false);
  }
#undef MVS_NARROW
}

}  // namespace mvs
