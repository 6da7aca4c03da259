// plane_sampling.hip -- per-(image, plane) sampling matrices (sampling_matrix.h), one thread per
// (image, plane).  The fused cost-volume launches compute the same matrices inside their prologue
// kernel (cost_volume_fwd.hip); this launcher serves mvs_plane_sampling and the generic (V > 8)
// path.
#include "launchers.h"
#include "sampling_matrix.h"

namespace mvs {
namespace {

__global__ void plane_sampling_kernel(Cams cm, int B, int V, int h, int w, int d_count,
                                      float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * V * d_count) return;
  const int i = t / d_count;
  sampling_matrix(cm, B, V, h, w, i, t - i * d_count, out + 9 * (size_t)t);
}

}  // namespace

void launch_plane_sampling(const float* K, const float* R, const float* T, const float* d_min,
                           const float* d_int, int B, int V, int h, int w, int d_begin,
                           int d_count, float d_scale, float* sampling, hipStream_t s) {
  const int n = B * V * d_count;
  const Cams cm{K, R, T, d_min, d_int, d_begin, d_scale};
  hipLaunchKernelGGL(plane_sampling_kernel, dim3((n + 127) / 128), dim3(128), 0, s, cm, B, V, h, w, d_count,
                     sampling);
}

}  // namespace mvs
