// dtu_input.hip -- the data-side neighbours of the hot path: the per-batch input
// transforms of the DTU reader, done on the device so only the decoded uint8 pixels cross PCIe.
//
//  * normalize_images_kernel: data.py:206-210 (PILToTensor -> ConvertImageDtype(float) ->
//    Normalize(mean, std)), i.e. out[n][c][y][x] = (rgb[n][y][x][c] / 255 - mean[c]) / std[c],
//    each step rounded as torch's CPU ops round it (true fp32 division, then subtraction, then
//    true division: bit-identical).  HWC uint8 in, NCHW fp32 out.
//  * depth_threshold_kernel: data.py:300-301 (cv2 THRESH_TOZERO at lo, then THRESH_TOZERO_INV at
//    hi): v = x > lo ? x : 0; v = v > hi ? 0 : v (NaN -> 0, as cv2's comparisons give).
//
// Both are HBM-bound byte/elementwise passes: no LDS, 4 pixels per thread so every uint8 load is
// a 12-byte run of whole pixels and every store a float4.
#include "launchers.h"

namespace mvs {
namespace {

__device__ inline float normalize_px(uint32_t u, float mean, float stdv) {
  return __fdiv_rn(__fsub_rn(__fdiv_rn((float)u, 255.0f), mean), stdv);
}

__global__ __launch_bounds__(kBlock) void normalize_images_kernel(
    const uint8_t* __restrict__ rgb, int n, uint32_t hw, float m0, float m1, float m2, float s0,
    float s1, float s2, float* __restrict__ out) {
  const uint32_t quads = (hw + 3) / 4;
  const size_t total = (size_t)n * quads;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < total;
       e += (size_t)gridDim.x * kBlock) {
    const size_t img = e / quads;
    const uint32_t p0 = (uint32_t)(e - img * quads) * 4u;
    const uint8_t* src = rgb + (img * hw + p0) * 3;
    float* dst = out + img * 3 * (size_t)hw + p0;
    if (p0 + 4 <= hw && (hw & 3u) == 0) {
      // 4 whole pixels = 12 bytes, 4-byte aligned (hw % 4 == 0 keeps every quad aligned)
      const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
      const uint32_t a = s32[0], b = s32[1], c = s32[2];
      uint32_t v[12];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = (a >> (8 * k)) & 0xFFu;
        v[4 + k] = (b >> (8 * k)) & 0xFFu;
        v[8 + k] = (c >> (8 * k)) & 0xFFu;
      }
      // byte j of the run is pixel j / 3, channel j % 3
      const float4 r = make_float4(normalize_px(v[0], m0, s0), normalize_px(v[3], m0, s0),
                                   normalize_px(v[6], m0, s0), normalize_px(v[9], m0, s0));
      const float4 g = make_float4(normalize_px(v[1], m1, s1), normalize_px(v[4], m1, s1),
                                   normalize_px(v[7], m1, s1), normalize_px(v[10], m1, s1));
      const float4 bl = make_float4(normalize_px(v[2], m2, s2), normalize_px(v[5], m2, s2),
                                    normalize_px(v[8], m2, s2), normalize_px(v[11], m2, s2));
      *reinterpret_cast<float4*>(dst) = r;
      *reinterpret_cast<float4*>(dst + hw) = g;
      *reinterpret_cast<float4*>(dst + 2 * (size_t)hw) = bl;
    } else {
      for (uint32_t k = 0; k < 4 && p0 + k < hw; ++k) {
        dst[k] = normalize_px(src[3 * k + 0], m0, s0);
        dst[hw + k] = normalize_px(src[3 * k + 1], m1, s1);
        dst[2 * (size_t)hw + k] = normalize_px(src[3 * k + 2], m2, s2);
      }
    }
  }
}

__device__ inline float threshold_px(float x, float lo, float hi) {
  const float v = x > lo ? x : 0.0f;   // THRESH_TOZERO
  return v > hi ? 0.0f : v;            // THRESH_TOZERO_INV
}

__global__ __launch_bounds__(kBlock) void depth_threshold_kernel(const float* __restrict__ depth,
                                                                 size_t n, float lo, float hi,
                                                                 float* __restrict__ out) {
  const size_t n4 = n / 4;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n4; e += (size_t)gridDim.x * kBlock) {
    const float4 x = reinterpret_cast<const float4*>(depth)[e];
    reinterpret_cast<float4*>(out)[e] = make_float4(threshold_px(x.x, lo, hi), threshold_px(x.y, lo, hi),
                                                    threshold_px(x.z, lo, hi), threshold_px(x.w, lo, hi));
  }
  const size_t tail = n4 * 4 + (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (tail < n) out[tail] = threshold_px(depth[tail], lo, hi);
}

unsigned grid_for(size_t items) {
  const size_t blocks = (items + kBlock - 1) / kBlock;
  return (unsigned)(blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192);
}

}  // namespace

void launch_normalize_images(const uint8_t* rgb, int n, uint32_t hw, const float* mean3,
                             const float* std3, float* out, hipStream_t s) {
  const size_t quads = (size_t)n * ((hw + 3) / 4);
  hipLaunchKernelGGL(normalize_images_kernel, dim3(grid_for(quads)), dim3(kBlock), 0, s, rgb, n, hw,
                     mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], out);
}

void launch_depth_threshold(const float* depth, size_t n, float lo, float hi, float* out,
                            hipStream_t s) {
  // the tail (n % 4 elements) is handled by block 0's first threads
  hipLaunchKernelGGL(depth_threshold_kernel, dim3(grid_for(n / 4 > 0 ? n / 4 : 1)), dim3(kBlock), 0,
                     s, depth, n, lo, hi, out);
}

}  // namespace mvs
