// channel_ops.hip -- the train-mode BatchNorm pieces of the regulariser (model.py:101-121 with every
// BatchNorm3d in training mode, test.py:53,61): per-channel batch sums of a tensor, and the
// normalisation + ReLU (+ a second normalised, rectified tensor added: model.py:121-123's
// `relu(BN_0(deconv_1_0)) + y0`, with y0 = relu(BN_0(conv_0_0)) kept un-normalised until then).
//
// Layouts: channels-last region tensors x[b][voxel][c] (CostVolumeReg.forward_live_train's conv
// outputs) or NCDHW x[b][c][voxel].  Both kernels stream the tensor once with 16-byte accesses; they
// are HBM-bound (sums: 4 B read per element; normalisation: 4 B read + 4 B written, + 4 B read for
// the addend).
//
// Sums: float64 per thread, reduced across the wave's lanes of equal channel, then across the
// workgroup's waves through LDS in a fixed order, and WRITTEN (no atomics) to the workgroup's own slot
// stats[slot][0 / 1][c] (sum / sum of squares); the caller adds the slots (mvs_channel_stats_slots of
// them) in a fixed order.  Every partial sum is formed in the same order on every run, so the batch
// statistics -- and the BatchNorm outputs and running statistics built from them -- are bit-identical
// run to run.
#include "launchers.h"
#include "split.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kWaves = kBlock / 64;
constexpr unsigned kStatsClBlocks = 1024;   // channels-last sums: at most this many workgroups (= slots)

// channels-last: float4 j holds channels 4 (j % C4) .. + 3; the grid stride is a multiple of C4
// (C4 divides kBlock), so a thread's quad never changes.  Slot = workgroup.
__global__ __launch_bounds__(kBlock) void channel_stats_cl_kernel(const float4* __restrict__ x, size_t n4, int C4,
                                                                  double* __restrict__ stats) {
  __shared__ double part[kWaves][64][8];
  double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x; j < n4; j += stride) {
    const float4 v = x[j];
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s[k] += (double)e[k];
      q[k] += (double)e[k] * (double)e[k];
    }
  }
  // lanes l and l ^ o (o >= C4) hold the same quad
  for (int o = 32; o >= C4; o >>= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s[k] += __shfl_xor(s[k], o);
      q[k] += __shfl_xor(q[k], o);
    }
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
  if (lane < C4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      part[wave][lane][k] = s[k];
      part[wave][lane][4 + k] = q[k];
    }
  }
  __syncthreads();
  if (wave == 0 && lane < C4) {
    const int C = 4 * C4;
    double* st = stats + (size_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double a = part[0][lane][k], b = part[0][lane][4 + k];
#pragma unroll
      for (int v = 1; v < kWaves; ++v) {
        a += part[v][lane][k];
        b += part[v][lane][4 + k];
      }
      st[4 * lane + k] = a;
      st[C + 4 * lane + k] = b;
    }
  }
}

// NCDHW: one (sample, channel) plane per blockIdx.y; float4 accesses when the plane is a multiple of 4.
// Slot = blockIdx.x * B + sample: every (slot, channel) is written by exactly one workgroup.
__global__ __launch_bounds__(kBlock) void channel_stats_cf_kernel(const float* __restrict__ x, size_t plane, int C,
                                                                  double* __restrict__ stats) {
  __shared__ double part[kWaves][2];
  const int c = (int)blockIdx.y % C;
  const int b = (int)blockIdx.y / C;
  const int B = (int)gridDim.y / C;
  const float* p = x + (size_t)blockIdx.y * plane;
  double s = 0.0, q = 0.0;
  const size_t stride = (size_t)gridDim.x * kBlock;
  if ((plane & 3) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x; j < plane / 4; j += stride) {
      const float4 v = p4[j];
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
      q += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
  } else {
    for (size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x; j < plane; j += stride) {
      const double v = p[j];
      s += v;
      q += v * v;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  const int wave = (int)threadIdx.x >> 6;
  if (((int)threadIdx.x & 63) == 0) {
    part[wave][0] = s;
    part[wave][1] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int v = 1; v < kWaves; ++v) {
      s += part[v][0];
      q += part[v][1];
    }
    double* st = stats + ((size_t)blockIdx.x * B + b) * 2 * C;
    st[c] = s;
    st[C + c] = q;
  }
}

__device__ inline float bn_relu(float v, float sc, float sh, float mu) { return fmaxf((v - mu) * sc + sh, 0.0f); }

// y = relu((x - mean) * scale + shift) [+ relu((r - rmean) * rscale + rshift)], channels-last
__global__ __launch_bounds__(kBlock) void bn_relu_cl_kernel(const float4* __restrict__ x, size_t n4, int C4,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ mu, const float4* __restrict__ r,
                                                            const float* __restrict__ rsc, const float* __restrict__ rsh,
                                                            const float* __restrict__ rmu, float4* __restrict__ y,
                                                            uint32_t* __restrict__ yb) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  const size_t j0 = (size_t)blockIdx.x * kBlock + threadIdx.x;
  float vmax = 0.0f;   // (outputs are >= 0)
  const int c = 4 * (int)(j0 % (size_t)C4);   // constant per thread (C4 divides the stride)
  float a[4], b[4], m[4], ra[4] = {0, 0, 0, 0}, rb[4] = {0, 0, 0, 0}, rm[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a[k] = sc[c + k];
    b[k] = sh[c + k];
    m[k] = mu[c + k];
    if (r) {
      ra[k] = rsc[c + k];
      rb[k] = rsh[c + k];
      rm[k] = rmu[c + k];
    }
  }
  for (size_t j = j0; j < n4; j += stride) {
    const float4 v = x[j];
    float4 o = make_float4(bn_relu(v.x, a[0], b[0], m[0]), bn_relu(v.y, a[1], b[1], m[1]),
                           bn_relu(v.z, a[2], b[2], m[2]), bn_relu(v.w, a[3], b[3], m[3]));
    if (r) {
      const float4 u = r[j];
      o.x += bn_relu(u.x, ra[0], rb[0], rm[0]);
      o.y += bn_relu(u.y, ra[1], rb[1], rm[1]);
      o.z += bn_relu(u.z, ra[2], rb[2], rm[2]);
      o.w += bn_relu(u.w, ra[3], rb[3], rm[3]);
    }
    vmax = fmaxf(vmax, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
    y[j] = o;
  }
  if (yb) bound_update(yb, vmax);
}

// NCDHW: one (sample, channel) plane per blockIdx.y
__global__ __launch_bounds__(kBlock) void bn_relu_cf_kernel(const float* __restrict__ x, size_t plane, int C,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ mu, const float* __restrict__ r,
                                                            const float* __restrict__ rsc, const float* __restrict__ rsh,
                                                            const float* __restrict__ rmu, float* __restrict__ y,
                                                            uint32_t* __restrict__ yb) {
  const int c = (int)blockIdx.y % C;
  float vmax = 0.0f;
  const size_t base = (size_t)blockIdx.y * plane;
  const float a = sc[c], b = sh[c], m = mu[c];
  const float ra = r ? rsc[c] : 0.0f, rb = r ? rsh[c] : 0.0f, rm = r ? rmu[c] : 0.0f;
  const size_t stride = (size_t)gridDim.x * kBlock;
  if ((plane & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x + base);
    const float4* r4 = r ? reinterpret_cast<const float4*>(r + base) : nullptr;
    float4* y4 = reinterpret_cast<float4*>(y + base);
    for (size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x; j < plane / 4; j += stride) {
      const float4 v = x4[j];
      float4 o = make_float4(bn_relu(v.x, a, b, m), bn_relu(v.y, a, b, m), bn_relu(v.z, a, b, m),
                             bn_relu(v.w, a, b, m));
      if (r4) {
        const float4 u = r4[j];
        o.x += bn_relu(u.x, ra, rb, rm);
        o.y += bn_relu(u.y, ra, rb, rm);
        o.z += bn_relu(u.z, ra, rb, rm);
        o.w += bn_relu(u.w, ra, rb, rm);
      }
      vmax = fmaxf(vmax, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
      y4[j] = o;
    }
  } else {
    for (size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x; j < plane; j += stride) {
      float o = bn_relu(x[base + j], a, b, m);
      if (r) o += bn_relu(r[base + j], ra, rb, rm);
      vmax = fmaxf(vmax, o);
      y[base + j] = o;
    }
  }
  if (yb) bound_update(yb, vmax);
}

// Train-mode BatchNorm parameters from the batch sums (mvs_bn_train_params): one workgroup, one thread
// per channel.
// Border term (conv_k_1's voxels outside its computed region, CostVolumeReg.forward_live_train): the
// previous BN's constant a_i = relu(-mean_i scale_i + shift_i), u = sum_i U[o][i][k] a_i per border
// class k, sums += (sum_k u cnt_k, sum_k u^2 cnt_k).  Then mean = s1 / n, var = max(s2 / n - mean^2, 0)
// (biased, float64), the running statistics' momentum update (unbiased variance), and
// params = (weight / sqrt(var + eps), bias, mean) in fp32 -- model.py's _bn_train / _border_class_sums /
// _bn_constant, as one launch instead of ~20 small device ops.
constexpr int kBnBorderMax = 2048;   // channels x border classes of mvs_bn_train_params

__global__ __launch_bounds__(kBlock) void bn_train_params_kernel(
    const double* __restrict__ sums, int C, double count, const double* __restrict__ bu,
    const double* __restrict__ bcnt, int Cp, int ncls, const float* __restrict__ prev, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ rmean, float* __restrict__ rvar,
    long long* __restrict__ nbt, double momentum, double eps, float* __restrict__ params) {
  __shared__ double part[2][kBnBorderMax];
  __shared__ double a[256];
  if (bu) {
    // the previous BN's constant, then u per (channel, class) in parallel; per channel the classes are
    // added in a fixed order below (bit-identical run to run)
    for (int i = (int)threadIdx.x; i < Cp; i += (int)blockDim.x)
      a[i] = (double)fmaxf(-prev[2 * Cp + i] * prev[i] + prev[Cp + i], 0.0f);
    __syncthreads();
    for (int e = (int)threadIdx.x; e < C * ncls; e += (int)blockDim.x) {
      const int o = e / ncls, k = e % ncls;
      double u = 0.0;
      for (int i = 0; i < Cp; ++i) u += bu[((size_t)o * Cp + i) * ncls + k] * a[i];
      part[0][e] = u * bcnt[k];
      part[1][e] = u * u * bcnt[k];
    }
    __syncthreads();
  }
  for (int o = (int)threadIdx.x; o < C; o += (int)blockDim.x) {
    double s1 = sums[o], s2 = sums[C + o];
    if (bu) {
      double c1 = 0.0, c2 = 0.0;
      for (int k = 0; k < ncls; ++k) {
        c1 += part[0][o * ncls + k];
        c2 += part[1][o * ncls + k];
      }
      s1 += c1;
      s2 += c2;
    }
    const double mean = s1 / count;
    const double var = fmax(s2 / count - mean * mean, 0.0);
    if (rmean) {
      const float m = (float)momentum;
      rmean[o] = rmean[o] * (1.0f - m) + m * (float)mean;
      rvar[o] = rvar[o] * (1.0f - m) + m * (float)(var * (count / fmax(count - 1.0, 1.0)));
    }
    params[o] = w[o] / sqrtf((float)var + (float)eps);
    params[C + o] = bias[o];
    params[2 * C + o] = (float)mean;
  }
  if (threadIdx.x == 0 && nbt) nbt[0] += 1;
}

unsigned grid_cl(size_t n4) {
  const size_t blocks = (n4 + kBlock - 1) / kBlock;
  return (unsigned)(blocks < 4096 ? blocks : 4096);
}

unsigned grid_cf(size_t plane, size_t planes) {
  // about 2048 workgroups in total, at least one per plane
  size_t per = (2048 + planes - 1) / planes;
  const size_t need = (plane / 4 + kBlock - 1) / kBlock;
  if (per > need) per = need;
  return (unsigned)(per > 0 ? per : 1);
}

}  // namespace

size_t channel_stats_slots(bool channels_last, int B, int C, size_t voxels) {
  if (channels_last) {
    const unsigned g = grid_cl((size_t)B * voxels * (size_t)C / 4);
    return g < kStatsClBlocks ? g : kStatsClBlocks;
  }
  return (size_t)grid_cf(voxels, (size_t)B * C) * (size_t)B;
}

void launch_channel_stats(const float* x, bool channels_last, int B, int C, size_t voxels, double* stats,
                          hipStream_t s) {
  if (channels_last) {
    const size_t n4 = (size_t)B * voxels * (size_t)C / 4;
    hipLaunchKernelGGL(channel_stats_cl_kernel, dim3((unsigned)channel_stats_slots(true, B, C, voxels)),
                       dim3(kBlock), 0, s,
                       reinterpret_cast<const float4*>(x), n4, C / 4, stats);
  } else {
    hipLaunchKernelGGL(channel_stats_cf_kernel, dim3(grid_cf(voxels, (size_t)B * C), (unsigned)(B * C)),
                       dim3(kBlock), 0, s, x, voxels, C, stats);
  }
}

void launch_bn_train_params(const double* sums, int C, double count, const double* bu, const double* bcnt, int Cp,
                            int ncls, const float* prev, const float* w, const float* bias, float* rmean, float* rvar,
                            long long* nbt, double momentum, double eps, float* params, hipStream_t s) {
  hipLaunchKernelGGL(bn_train_params_kernel, dim3(1), dim3(kBlock), 0, s, sums, C, count, bu, bcnt, Cp, ncls, prev, w,
                     bias, rmean, rvar, nbt, momentum, eps, params);
}

void launch_bn_relu(const float* x, bool channels_last, int B, int C, size_t voxels, const float* sc,
                    const float* sh, const float* mu, const float* r, const float* rsc, const float* rsh,
                    const float* rmu, float* y, uint32_t* y_bound, hipStream_t s) {
  if (channels_last) {
    const size_t n4 = (size_t)B * voxels * (size_t)C / 4;
    hipLaunchKernelGGL(bn_relu_cl_kernel, dim3(grid_cl(n4)), dim3(kBlock), 0, s, reinterpret_cast<const float4*>(x),
                       n4, C / 4, sc, sh, mu, reinterpret_cast<const float4*>(r), rsc, rsh, rmu,
                       reinterpret_cast<float4*>(y), y_bound);
  } else {
    hipLaunchKernelGGL(bn_relu_cf_kernel, dim3(grid_cf(voxels, (size_t)B * C), (unsigned)(B * C)), dim3(kBlock), 0,
                       s, x, voxels, C, sc, sh, mu, r, rsc, rsh, rmu, y, y_bound);
  }
}

}  // namespace mvs
