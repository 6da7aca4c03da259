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
#include <algorithm>

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
// C1 (COUT = 8, C4 = 1, WZ, Cin = 32: the fp32 eval path's conv_0_0; mvs_conv_head_fp32_fwd): conv_1_0
// (model.py:103: 32 -> 16, stride 2, padding P odd, + BN_1 + ReLU) computed from the SAME staged halo
// block on the fp32 matrix cores, so the cost volume is read once for both convolutions and the MFMA work
// co-issues with the VALU work of the other waves on the SIMD.  The tile owns the stride-2 windows whose
// start (2 o - P) is x0 - 1 + 2 j (j < 16), y0 - 1 + 2 j (j < 4), d0 - 1 + 2 j (j < 2): 8 row blocks of 16
// windows, two per wave; every window's 27 taps lie in the staged (x0 - 1 .. x0 + 32) x (y0 - 1 .. y0 + 8)
// x (d0 - 1 .. d0 + 4) block, which holds zeros outside the volume.  Per channel pass (4 channels = the
// MFMA's K of 4, lane group kq = channel kq), after the wave's conv_0_0 arithmetic: 27 taps x 2 row
// blocks of v_mfma_f32_16x16x4_f32 with A (window x, channel) and B (channel, output channel, from the
// pass's weight slice staged beside the input) read from LDS at immediate tap offsets.
struct Head1 {
  const float* w1p;            // conv_1_0 weights [Cin / 4][27][16][4] (pass, tap, c_out, channel in pass)
  const float *sc, *sh, *mu;   // BN_1 (16), all or none
  float* y1;                   // [B][on0][on1][on2][16] channels-last
  int o0[3], on[3];            // y1's region (volume output coordinates)
  int pad[3];                  // P, odd
};

// C1's waves per SIMD: 3 keeps conv_0_0's occupancy (168 registers; a few spill outside the pass loop)
#ifndef MVS_HEAD_WAVES
#define MVS_HEAD_WAVES 3
#endif

template <int COUT, int C4, bool WZ = false, int DT = kDT, bool FOLD = false, bool C1 = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(C1 ? MVS_HEAD_WAVES : 1)))
void conv3d_k3_narrow_kernel(
    const float* __restrict__ in, const float* __restrict__ wt, float* __restrict__ out, int Cin,
    int D, int H, int W, int tiles_x, int tiles_y, int dgroups, int n_batch, const float* __restrict__ bn_scale,
    const float* __restrict__ bn_shift, const float* __restrict__ bn_mean, const float* __restrict__ in2,
    const float* __restrict__ ibn, Head1 h1) {
  static_assert(!FOLD || (COUT == 1 && C4 == 0), "folded input BN: conv_out on NCDHW");
  static_assert(!WZ || DT == 4, "depth Winograd: two windows of 2");
  static_assert(!C1 || (COUT == 8 && C4 == 1 && WZ), "fused conv_1_0: the fp32 conv_0_0 kernel");
  constexpr int kPX = kTX + 2, kPY = kTY + 2, kPD = DT + 2;
  constexpr int kPlane = kPX * kPY;
  constexpr int kStage = kPD * kPlane;                      // floats per input channel
  constexpr int kPer = (kStage + kBlock - 1) / kBlock;      // staging elements per thread
  constexpr int NP = COUT / 2;                              // channel pairs (COUT = 8)
  constexpr int NQ = C4 ? 4 : 1;                            // channels staged per pass
  __shared__ float lds[NQ * kStage];
  __shared__ __attribute__((aligned(16))) float w1s[C1 ? 27 * 16 * 4 : 4];   // C1: the pass's conv_1_0 weights
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
  // C1: this wave's two conv_1_0 row blocks (wy, wz) = (rbi & 3, rbi >> 2), rbi = 2 wave + rb
  const int c1lane = (int)threadIdx.x & 63, c1wave = (int)threadIdx.x >> 6;
  const int m16 = c1lane & 15, kq = c1lane >> 4;
  f4v c1acc[2] = {f4v{0.0f, 0.0f, 0.0f, 0.0f}, f4v{0.0f, 0.0f, 0.0f, 0.0f}};
  int abase[2] = {0, 0};
  if constexpr (C1) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int rbi = 2 * c1wave + rb, wy = rbi & 3, wzz = rbi >> 2;
      abase[rb] = kq * kStage + (2 * wzz) * kPlane + (2 * wy) * kPX + 2 * m16;
    }
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
    if constexpr (C1) {   // the pass's conv_1_0 weight slice, 432 float4 (L2-resident, 55 KB in all)
      const f4v* src = reinterpret_cast<const f4v*>(h1.w1p) + (size_t)q * 432;
      f4v* dst = reinterpret_cast<f4v*>(w1s);
      for (int i = (int)threadIdx.x; i < 432; i += kBlock) dst[i] = src[i];
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
    if constexpr (C1) {
      // conv_1_0 on this pass's 4 channels: 27 taps x 2 row blocks, operands from LDS at immediate offsets
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int tz = t / 9, ty = (t / 3) % 3, tx = t % 3;
        const float bv = w1s[t * 64 + m16 * 4 + kq];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          c1acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(lds[abase[rb] + tz * kPlane + ty * kPX + tx], bv,
                                                           c1acc[rb], 0, 0, 0);
      }
    }
  }

  if constexpr (C1) {
    // conv_1_0 epilogue: c1acc[rb][r] = window x = 4 kq + r of row block rb, output channel m16
    const float sc = h1.sc ? h1.sc[m16] : 1.0f, sh = h1.sc ? h1.sh[m16] : 0.0f, mu = h1.sc ? h1.mu[m16] : 0.0f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int rbi = 2 * c1wave + rb, wy = rbi & 3, wzz = rbi >> 2;
      const int oz = (d0 - 1 + 2 * wzz + h1.pad[0]) >> 1, oy = (ty0 - 1 + 2 * wy + h1.pad[1]) >> 1;
      if (oz < h1.o0[0] || oz >= h1.o0[0] + h1.on[0] || oy < h1.o0[1] || oy >= h1.o0[1] + h1.on[1]) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ox = (tx0 - 1 + 2 * (4 * kq + r) + h1.pad[2]) >> 1;
        if (ox < h1.o0[2] || ox >= h1.o0[2] + h1.on[2]) continue;
        float v = c1acc[rb][r];
        if (h1.sc) v = fmaxf((v - mu) * sc + sh, 0.0f);
        h1.y1[((((size_t)b * h1.on[0] + (oz - h1.o0[0])) * h1.on[1] + (oy - h1.o0[1])) * h1.on[2] + (ox - h1.o0[2])) *
                  16 + m16] = v;
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

template <int COUT, int C4, bool WZ = false, bool FOLD = false, bool C1 = false>
void launch_narrow(const float* in, const float* weight, float* out, int B, int Cin, int D, int H, int W,
                   const float* bn_scale, const float* bn_shift, const float* bn_mean, hipStream_t s,
                   const float* in2 = nullptr, const float* ibn = nullptr, const Head1& h1 = Head1{}) {
  constexpr int DT = COUT == 1 ? kOutDT : kDT;
  const int tiles_x = (W + kTX - 1) / kTX, tiles_y = (H + kTY - 1) / kTY, dgroups = (D + DT - 1) / DT;
  const dim3 grid = xcd_grid(B * dgroups * tiles_y * tiles_x);
  hipLaunchKernelGGL((conv3d_k3_narrow_kernel<COUT, C4, WZ, DT, FOLD, C1>), grid, dim3(kBlock), 0, s, in, weight,
                     out, Cin, D, H, W, tiles_x, tiles_y, dgroups, B, bn_scale, bn_shift, bn_mean, in2, ibn, h1);
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

// conv_0_0 + BN_0 + ReLU over the whole volume and conv_1_0 + BN_1 + ReLU on its region from the fp32
// channel-quad cost volume in ONE kernel (C1 above); the region's outputs whose windows no tile owns --
// windows starting below -1 or past the last tile's (start >= 32 tiles_x - 1 etc.: all-padding windows
// and, when a dim is a multiple of the tile, the one at n - 1) -- by the per-lane stride-2 region kernel
// on up to six slabs, stored into y1 in place
void launch_conv_head_fp32(const float* cv4, int B, int D, int H, int W, const float* w0wz, const float* bn0_sc,
                           const float* bn0_sh, const float* bn0_mu, const float* w1, const float* w1p,
                           const float* bn1_sc, const float* bn1_sh, const float* bn1_mu, const int* pad,
                           const int* o0, const int* on, float* y0, float* y1, hipStream_t s, hipEvent_t ev0,
                           hipEvent_t ev1) {
  Head1 h1;
  h1.w1p = w1p;
  h1.sc = bn1_sc;
  h1.sh = bn1_sh;
  h1.mu = bn1_mu;
  h1.y1 = y1;
  for (int d = 0; d < 3; ++d) {
    h1.o0[d] = o0[d];
    h1.on[d] = on[d];
    h1.pad[d] = pad[d];
  }
  if (ev0) (void)hipEventRecord(ev0, s);
  launch_narrow<8, 1, true, false, true>(cv4, w0wz, y0, B, 32, D, H, W, bn0_sc, bn0_sh, bn0_mu, s, nullptr, nullptr,
                                         h1);
  if (ev1) (void)hipEventRecord(ev1, s);
  // owned windows per dim: starts -1 .. n_tiles * tile - 3 -> outputs [(P - 1) / 2, (n_tiles * tile - 3 + P) / 2]
  const int tile[3] = {kDT, kTY, kTX}, n[3] = {D, H, W};
  int clo[3], chi[3];   // core box of y1's region (inclusive), computed by the fused kernel
  for (int d = 0; d < 3; ++d) {
    const int tiles = (n[d] + tile[d] - 1) / tile[d];
    clo[d] = std::max(o0[d], (pad[d] - 1) / 2);
    chi[d] = std::min(o0[d] + on[d] - 1, (tiles * tile[d] - 3 + pad[d]) / 2);
  }
  // slabs: dim 0 lo / hi over the whole region, dim 1 within dim 0's core, dim 2 within both cores
  for (int d = 0; d < 3; ++d)
    for (int side = 0; side < 2; ++side) {
      int so[3], sn[3];
      bool empty = false;
      for (int e = 0; e < 3; ++e) {
        if (e < d) {   // inside the earlier dims' core
          so[e] = clo[e];
          sn[e] = chi[e] - clo[e] + 1;
        } else if (e > d) {   // the whole region
          so[e] = o0[e];
          sn[e] = on[e];
        } else if (side == 0) {
          so[e] = o0[e];
          sn[e] = clo[e] - o0[e];
        } else {
          so[e] = chi[e] + 1;
          sn[e] = o0[e] + on[e] - 1 - chi[e];
        }
        empty = empty || sn[e] <= 0;
      }
      if (empty) continue;
      int st0[3];
      for (int e = 0; e < 3; ++e) st0[e] = so[e] - o0[e];
      launch_conv3d_region(1 /*S2*/, false, 1, cv4, nullptr, w1, y1, B, 32, 16, n, so, sn, nullptr, nullptr, pad,
                           bn1_sc, bn1_sh, bn1_mu, s, nullptr, nullptr, false, st0, on);
    }
}

}  // namespace mvs
