// soft_argmin.hip -- depthmap.py:4-22 (extract_depth_map) with the reference's permutation-indexed
// mask: plane r is kept when argsort_desc(P)[r] < n_est.  Instead of sorting D values per pixel,
// the rank of each of the first n_est planes is counted in one pass over D (ties ordered by
// ascending plane index, i.e. stable -- what torch's CPU sort does for D <= 16; above that torch's
// order for exact ties is implementation-defined).  One thread per pixel; the D reads of a pixel
// are coalesced across the wave (stride h*w), 16 planes in flight.
#include "launchers.h"

namespace mvs {
namespace {

// depthmap.py:4-22.  rank_j = #{m : P_m > P_j} + #{m < j : P_m == P_j} is the sorted position of
// plane j (descending, ties by ascending index); mask[r] = 1 exactly at r = rank_j, j < n_est.
template <int MAXE>
__global__ __launch_bounds__(64) void soft_argmin_kernel(const float* __restrict__ prob,
                                                             const float* __restrict__ d_batch,
                                                             int B, int D, uint32_t hw, int n_est,
                                                             float* __restrict__ depth) {
  const size_t e = (size_t)blockIdx.x * 64 + threadIdx.x;
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
  // 16 planes' loads in flight per round (one load at a time made the pass latency-bound: cfg 2
  // 0.090 ms for 63 MB); the counts do not depend on the order
  int m = 0;
  for (; m + 16 <= D; m += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = P[(size_t)(m + k) * hw];
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int j = 0; j < MAXE; ++j) rank[j] += (v[k] > pj[j]) || (v[k] == pj[j] && m + k < j);
  }
  for (; m < D; ++m) {
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

}  // namespace

void launch_soft_argmin(const float* prob, const float* d_batch, int B, int D, uint32_t hw,
                        int n_est, float* depth, hipStream_t s) {
  // 64-thread workgroups: the pixels of a small batch spread over every CU (cfg 2: 1,280 waves)
  const size_t n = (size_t)B * hw;
  const dim3 grid((unsigned)((n + 63) / 64));
  if (n_est <= 8)
    hipLaunchKernelGGL((soft_argmin_kernel<8>), grid, dim3(64), 0, s, prob, d_batch, B, D, hw, n_est, depth);
  else
    hipLaunchKernelGGL((soft_argmin_kernel<16>), grid, dim3(64), 0, s, prob, d_batch, B, D, hw, n_est, depth);
}

namespace {

constexpr int kSmF = 32;

// model.py:97 (CostVolumeReg.Norm = nn.Softmax(2)) over the depth planes of the regulariser's
// [B][1][D][h][w] output: per pixel m = max_d x, y_d = exp(x_d - m) / sum_d exp(x_d - m) -- the
// operation order of torch's softmax (max, then the sum of exp(x - max), then a division).  One
// thread per pixel, D reads coalesced across the wave (stride h*w), 64-thread workgroups so the
// pixels of a small batch spread over every CU.
__global__ __launch_bounds__(64) void softmax_depth_kernel(const float* __restrict__ x, int B, int D, uint32_t hw,
                                                           float* __restrict__ y) {
  const size_t e = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (e >= (size_t)B * hw) return;
  const size_t b = e / hw, p = e - b * hw;
  const float* xp = x + b * D * hw + p;
  float* yp = y + b * D * hw + p;
  // kSmF planes' loads in flight per round (the loop is latency-bound otherwise: 8 in flight
  // 0.052 ms at cfg 2); the sum keeps the sequential plane order
  float m = -INFINITY;
  int d = 0;
  for (; d + kSmF <= D; d += kSmF) {
    float v[kSmF];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) v[k] = xp[(size_t)(d + k) * hw];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) m = fmaxf(m, v[k]);
  }
  for (; d < D; ++d) m = fmaxf(m, xp[(size_t)d * hw]);
  float s = 0.0f;
  for (d = 0; d + kSmF <= D; d += kSmF) {
    float v[kSmF];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) v[k] = xp[(size_t)(d + k) * hw];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) s += expf(v[k] - m);
  }
  for (; d < D; ++d) s += expf(xp[(size_t)d * hw] - m);
  for (d = 0; d + kSmF <= D; d += kSmF) {
    float v[kSmF];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) v[k] = xp[(size_t)(d + k) * hw];
#pragma unroll
    for (int k = 0; k < kSmF; ++k) yp[(size_t)(d + k) * hw] = expf(v[k] - m) / s;
  }
  for (; d < D; ++d) yp[(size_t)d * hw] = expf(xp[(size_t)d * hw] - m) / s;
}

}  // namespace

void launch_softmax_depth(const float* x, int B, int D, uint32_t hw, float* y, hipStream_t s) {
  const size_t n = (size_t)B * hw;
  hipLaunchKernelGGL(softmax_depth_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, x, B, D, hw, y);
}

namespace {

// model.py:189-205 around the refinement net, one kernel on each side (was 9 elementwise launches of
// ~5 us each): d_span = (d_int * D) * D_SCALE, the normalised depth (ini - d_min) / d_span concatenated
// with the down-sampled reference image, and refined = ((conv + norm) * d_span) + d_min -- every
// operation a separately rounded fp32 op in the reference's order (fp contraction off in the kernels:
// the default would fuse a * b + c into an fma; the division is the correctly rounded one), so the
// results equal the torch sequence bit for bit.
__global__ __launch_bounds__(kBlock) void refine_input_kernel(const float* __restrict__ ini,
                                                              const float* __restrict__ d_min,
                                                              const float* __restrict__ d_int, float dnum,
                                                              float scale, const float* __restrict__ img,
                                                              int B, uint32_t hw, float* __restrict__ out) {
#pragma clang fp contract(off)   // separately rounded ops: no a * b + c fused into an fma
  const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= (size_t)B * hw) return;
  const size_t b = e / hw, p = e - b * hw;
  const float span = (d_int[b] * dnum) * scale;
  float* o = out + b * 4 * hw + p;
  o[0] = (ini[e] - d_min[b]) / span;
  const float* im = img + b * 3 * hw + p;
  o[hw] = im[0];
  o[2 * (size_t)hw] = im[hw];
  o[3 * (size_t)hw] = im[2 * (size_t)hw];
}

__global__ __launch_bounds__(kBlock) void refine_output_kernel(const float* __restrict__ conv,
                                                               const float* __restrict__ inp,
                                                               const float* __restrict__ d_min,
                                                               const float* __restrict__ d_int, float dnum,
                                                               float scale, int B, uint32_t hw,
                                                               float* __restrict__ out) {
#pragma clang fp contract(off)   // separately rounded ops: no a * b + c fused into an fma
  const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= (size_t)B * hw) return;
  const size_t b = e / hw, p = e - b * hw;
  const float span = (d_int[b] * dnum) * scale;
  out[e] = ((conv[e] + inp[b * 4 * hw + p]) * span) + d_min[b];
}

}  // namespace

void launch_refine_input(const float* ini, const float* d_min, const float* d_int, int d_num, float d_scale,
                         const float* img, int B, uint32_t hw, float* out, hipStream_t s) {
  const size_t n = (size_t)B * hw;
  hipLaunchKernelGGL(refine_input_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ini, d_min,
                     d_int, (float)d_num, d_scale, img, B, hw, out);
}

void launch_refine_output(const float* conv, const float* inp, const float* d_min, const float* d_int, int d_num,
                          float d_scale, int B, uint32_t hw, float* out, hipStream_t s) {
  const size_t n = (size_t)B * hw;
  hipLaunchKernelGGL(refine_output_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, conv,
                     inp, d_min, d_int, (float)d_num, d_scale, B, hw, out);
}

namespace {

// homography.py:24-26: d_batch_0[b][k] = d_min[b] + (D_SCALE * d_int[b]) * k in one launch (was 4:
// arange, two multiplies, the add), each op separately rounded in that order (contraction off), so
// the planes equal the torch expression bit for bit -- and the sampling matrices' depths
// (sampling_matrix.h forms the same expression).
__global__ __launch_bounds__(kBlock) void depth_hypotheses_kernel(const float* __restrict__ d_min,
                                                                  const float* __restrict__ d_int, float scale,
                                                                  int B, int D, float* __restrict__ out) {
#pragma clang fp contract(off)   // separately rounded ops: no a * b + c fused into an fma
  const int e = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (e >= B * D) return;
  const int b = e / D, k = e - b * D;
  out[e] = d_min[b] + (scale * d_int[b]) * (float)k;
}

}  // namespace

void launch_depth_hypotheses(const float* d_min, const float* d_int, float d_scale, int B, int D, float* out,
                             hipStream_t s) {
  hipLaunchKernelGGL(depth_hypotheses_kernel, dim3((unsigned)((B * D + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     d_min, d_int, d_scale, B, D, out);
}

}  // namespace mvs
