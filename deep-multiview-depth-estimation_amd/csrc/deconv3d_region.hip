// deconv3d_region.hip -- stride-2, kernel-3 ConvTranspose3d of the regulariser's last up-sampling
// (deconv_1_0, 16 -> 8, model.py:87, forward at model.py:121), gather form, with the following
// BatchNorm (eval) + ReLU and the skip add `+ y0` (model.py:121-123) fused into the epilogue.
//
// y[b][co][o] = sum_{ci, k} x[b][ci][i] * W[ci][co][k],  o = 2 i + k - P  (per dim, k = 0..2)
// so output o gathers the inputs i = (o + P - k) / 2 with o + P - k even: 1 or 2 taps per dim.
// x is a REGION tensor: it holds the input only on [x0, x0 + r) per dim -- every input that
// reaches an output in [0, n) (CostVolumeReg.forward_live); inputs outside it reach no output.
// Epilogue (optional): z = max((y - mean) * rsqrt(var + eps) * gamma + beta, 0) + residual.
//
// One thread = one output voxel (x fastest: coalesced stores per channel plane) x COUT channels
// in registers; weights in LDS.  HBM-bound: the full-size output (+ residual read) dominates.
#include "launchers.h"

namespace mvs {
namespace {

constexpr int kCout = 8;

struct Taps1 {
  int n;        // 1 or 2 valid taps
  int i[2];     // input index inside the region
  int k[2];     // kernel index
};

__device__ inline Taps1 taps1(int o, int p, int x0, int r) {
  Taps1 t;
  t.n = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int q = o + p - k;
    if (q & 1) continue;
    const int i = (q >> 1) - x0;
    if (i < 0 || i >= r) continue;
    t.i[t.n] = i;
    t.k[t.n] = k;
    ++t.n;
  }
  return t;
}

__global__ __launch_bounds__(kBlock) void deconv3d_k3s2_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, int Cin, int rd, int rh, int rw,
    int x0d, int x0h, int x0w, int D, int H, int W, int pd, int ph, int pw,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ mean, const float* __restrict__ residual, float* __restrict__ y,
    size_t total) {
  extern __shared__ float wl[];   // W[ci][co][27]
  const int nw = Cin * kCout * 27;
  for (int e = (int)threadIdx.x; e < nw; e += kBlock) wl[e] = wt[e];
  __syncthreads();
  const size_t gid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (gid >= total) return;
  const int ow = (int)(gid % W);
  size_t t = gid / W;
  const int oh = (int)(t % H);
  t /= H;
  const int od = (int)(t % D);
  const int b = (int)(t / D);
  const Taps1 td = taps1(od, pd, x0d, rd), th = taps1(oh, ph, x0h, rh), tw = taps1(ow, pw, x0w, rw);
  const size_t rvol = (size_t)rd * rh * rw;
  const float* xb = x + (size_t)b * Cin * rvol;
  float acc[kCout];
#pragma unroll
  for (int co = 0; co < kCout; ++co) acc[co] = 0.0f;
  for (int ci = 0; ci < Cin; ++ci) {
    const float* xc = xb + (size_t)ci * rvol;
    const float* wc = wl + ci * kCout * 27;
    for (int a = 0; a < td.n; ++a)
      for (int c = 0; c < th.n; ++c)
        for (int e = 0; e < tw.n; ++e) {
          const float v = xc[((size_t)td.i[a] * rh + th.i[c]) * rw + tw.i[e]];
          const int k = td.k[a] * 9 + th.k[c] * 3 + tw.k[e];
#pragma unroll
          for (int co = 0; co < kCout; ++co) acc[co] = fmaf(v, wc[co * 27 + k], acc[co]);
        }
  }
  const size_t plane = (size_t)D * H * W;
  const size_t pos = ((size_t)od * H + oh) * W + ow;
  float* yb = y + (size_t)b * kCout * plane + pos;
  const float* rb = residual ? residual + (size_t)b * kCout * plane + pos : nullptr;
#pragma unroll
  for (int co = 0; co < kCout; ++co) {
    float v = acc[co];
    if (bn_scale) v = fmaxf((v - mean[co]) * bn_scale[co] + bn_shift[co], 0.0f);
    if (rb) v += rb[(size_t)co * plane];
    yb[(size_t)co * plane] = v;
  }
}

}  // namespace

void launch_deconv3d_k3s2(const float* x, int B, int Cin, int rd, int rh, int rw, int x0d, int x0h,
                          int x0w, const float* weight, int D, int H, int W, int pd, int ph, int pw,
                          const float* bn_scale, const float* bn_shift, const float* bn_mean,
                          const float* residual, float* y, hipStream_t s) {
  const size_t total = (size_t)B * D * H * W;
  const size_t blocks = (total + kBlock - 1) / kBlock;
  const size_t lds = (size_t)Cin * kCout * 27 * sizeof(float);
  hipLaunchKernelGGL(deconv3d_k3s2_kernel, dim3((unsigned)blocks), dim3(kBlock), lds, s, x, weight, Cin,
                     rd, rh, rw, x0d, x0h, x0w, D, H, W, pd, ph, pw, bn_scale, bn_shift, bn_mean, residual,
                     y, total);
}

}  // namespace mvs
