// sampling_matrix.h -- per-(image, plane) sampling matrix G in fp64 (device code).
//
// Reference: scripts/homography.py:24-26 (depth planes, d_batch tiling), :29-36 (reference index of
// image i is V*floor(i/V)), :40-75 (H = K_i R_i (I - (C_i - C_r) n_r^T / d) R_r^T K_r^-1 with
// C = -R^T T and n_r the third column of R_ref); kornia 0.6.3 normalize_homography + inverse.
// G maps kornia-normalised reference coordinates to normalised source coordinates; stored fp32 (9
// floats) and read as workgroup-uniform scalars by the sampling kernels.
#pragma once

#include "common.h"

namespace mvs {

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

// homography.py:40-75 (H) + kornia normalize_homography / inverse for image i, shard plane kk:
// G (fp64 algebra, stored fp32).  Every kernel that needs a sampling matrix calls this one
// function, so identical inputs give bit-identical matrices.
__device__ inline void sampling_matrix(const Cams& cm, int B, int V, int h, int w, int i, int kk,
                                       float* __restrict__ o) {
#pragma clang fp contract(off)   // the fp32 depth below rounds each op as torch does (no fma)
  const float* K = cm.K;
  const float* R = cm.R;
  const float* T = cm.T;
  const int r = (i / V) * V;   // reference view of image i (homography.py:29-34)
  const int bq = i % B;        // d_batch = tile(d_batch_0, (V,1,1,1)): row i is sample i mod B
  // depth in fp32 exactly as homography.py:25 forms it: d_min + (D_SCALE * d_int) * k
  const float d32 = cm.d_min[bq] + (cm.d_scale * cm.d_int[bq]) * (float)(cm.d_begin + kk);
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
#pragma unroll
  for (int e = 0; e < 9; ++e) o[e] = (float)G.a[e];
}

}  // namespace mvs
