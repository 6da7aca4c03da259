// capi.hip -- the C ABI declared in include/mvs_cost_volume.h (drop-in boundary, SURVEY.md §8 b).
//
// Validates arguments, lays out the caller-provided workspace and enqueues the launchers of the
// other translation units on the caller's stream.  No allocation, no synchronisation, no global
// mutable state: every entry point is re-entrant per stream and graph-capturable.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "launchers.h"

namespace {

using mvs::Geometry;

// store_es: output element bytes of the packed (2 <= V <= 8) fused kernel this geometry feeds (4 fp32
// NCDHW, 2 bf16, 16 channel-quad), 0 for entry points that build no cost-volume store descriptors
int check_geometry(int B, int V, int C, int h, int w, int d_count, Geometry& g, int store_es = 0) {
  if (B <= 0 || C <= 0 || h < 2 || w < 2 || d_count <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if (V < 1 || V > MVS_MAX_VIEWS) return MVS_ERR_UNSUPPORTED_VIEWS;
  const uint64_t hw = (uint64_t)h * (uint64_t)w;
  // per-image plane offsets are 32-bit; work ids are 32-bit ints; packed corners are 16-bit
  if ((uint64_t)C * hw >= (1ull << 31) || h > 32000 || w > 32000) return MVS_ERR_TOO_LARGE;
  // the packed kernels build 32-bit buffer descriptors and offsets: a sample's padded channel-quad
  // images (V * ceil(C/4) * (h+2) * (w+2) float4, byte offsets held in ints) and a plane group's
  // cost-volume run (up to 8 planes * hw * store_es bytes: the store offsets soff0 + pl * hw * es)
  const bool packed = V >= 2 && V <= 8;
  const uint64_t padded = (uint64_t)V * (uint64_t)((C + 3) / 4) * (uint64_t)(h + 2) * (uint64_t)(w + 2) * 16u;
  if (packed && (padded >= (1ull << 31) || 8ull * hw * (uint64_t)store_es >= (1ull << 32))) return MVS_ERR_TOO_LARGE;
  const uint64_t tiles = (hw + mvs::kBlock - 1) / mvs::kBlock;
  const uint64_t total = (uint64_t)B * tiles * (uint64_t)d_count;
  if (total >= (1ull << 31) - 8) return MVS_ERR_TOO_LARGE;
  g.B = B;
  g.V = V;
  g.C = C;
  g.h = h;
  g.w = w;
  g.Dc = d_count;
  g.tiles = (int)tiles;
  g.total = (int)total;
  return MVS_OK;
}

bool cams_ok(const float* K, const float* R, const float* T, const float* d_min, const float* d_int) {
  return K && R && T && d_min && d_int;
}

// Fused warp + variance into an fp32 (es = 4) or bf16 (es = 2) NCDHW cost volume, or the channel-quad
// layout in fp32 (es = 16) or bf16 (es = 8).
int cost_volume_fwd_impl(const float* feat, const float* K, const float* R, const float* T,
                         const float* d_min, const float* d_int, int batch_size, int n_views,
                         int channels, int h, int w, int d_begin, int d_count, float d_scale,
                         float* workspace, void* cv_out, int es, void* stream, void* ev0, void* ev1,
                         uint32_t* absmax = nullptr) {
  if (!feat || !workspace || !cv_out) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g, es == 17 ? 16 : es);
  if (st != MVS_OK) return st;
  if (!cams_ok(K, R, T, d_min, d_int) || d_begin < 0) return MVS_ERR_INVALID_ARGUMENT;
  const mvs::LaunchCheck lc;
  hipStream_t s = (hipStream_t)stream;
  if (n_views == 1) {  // the variance of a single view is identically zero (0 in fp32 and bf16)
    if (absmax && hipMemsetAsync(absmax, 0, 8 * sizeof(uint32_t), s) != hipSuccess) return MVS_ERR_HIP;
    st = mvs_plane_sampling(K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count,
                            d_scale, workspace, stream);
    if (st != MVS_OK) return st;
    const size_t ch = (es == 16 || es == 17 || es == 8) ? (size_t)((channels + 3) / 4) : (size_t)channels;
    if (hipMemsetAsync(cv_out, 0, (size_t)batch_size * ch * d_count * h * w * (es == 17 ? 16 : es), s) != hipSuccess)
      return MVS_ERR_HIP;
    return lc.status();
  }
  float* packed = reinterpret_cast<float*>(
      reinterpret_cast<char*>(workspace) +
      mvs::align256((size_t)batch_size * n_views * d_count * 9 * sizeof(float)));
  const mvs::Cams cm{K, R, T, d_min, d_int, d_begin, d_scale};
  if (es == 4)
    mvs::launch_cost_volume_fwd(g, feat, cm, workspace, packed, static_cast<float*>(cv_out), s,
                                (hipEvent_t)ev0, (hipEvent_t)ev1);
  else if (es == 16 || es == 17)   // 17: the split cost volume (16-byte elements)
    mvs::launch_cost_volume_fwd_c4(g, feat, cm, workspace, packed, static_cast<float*>(cv_out), s,
                                   (hipEvent_t)ev0, (hipEvent_t)ev1, absmax, es == 17);
  else if (es == 8)
    mvs::launch_cost_volume_fwd_c4_bf16(g, feat, cm, workspace, packed, cv_out, s, (hipEvent_t)ev0,
                                        (hipEvent_t)ev1);
  else
    mvs::launch_cost_volume_fwd_bf16(g, feat, cm, workspace, packed, cv_out, s, (hipEvent_t)ev0,
                                     (hipEvent_t)ev1);
  return lc.status();
}

}  // namespace

extern "C" {

int mvs_abi_version(void) { return MVS_ABI_VERSION; }

const char* mvs_status_string(int status) {
  switch (status) {
    case MVS_OK: return "ok";
    case MVS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MVS_ERR_UNSUPPORTED_VIEWS: return "n_views outside [1, MVS_MAX_VIEWS]";
    case MVS_ERR_TOO_LARGE: return "tensor exceeds the kernel's 32-bit index space";
    case MVS_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

size_t mvs_sampling_workspace_bytes(int n_images, int d_count) {
  if (n_images <= 0 || d_count <= 0) return 0;
  return (size_t)n_images * (size_t)d_count * 9 * sizeof(float);
}

size_t mvs_cost_volume_workspace_bytes(int batch_size, int n_views, int channels, int h, int w,
                                       int d_count) {
  if (batch_size <= 0 || n_views <= 0 || channels <= 0 || h <= 0 || w <= 0 || d_count <= 0) return 0;
  return mvs::align256(mvs_sampling_workspace_bytes(batch_size * n_views, d_count)) +
         mvs::packed_bytes(batch_size, n_views, channels, h, w);
}

int mvs_plane_sampling(const float* K, const float* R, const float* T, const float* d_min,
                       const float* d_int, int batch_size, int n_views, int h, int w, int d_begin,
                       int d_count, float d_scale, float* sampling, void* stream) {
  if (!cams_ok(K, R, T, d_min, d_int) || !sampling) return MVS_ERR_INVALID_ARGUMENT;
  if (batch_size <= 0 || h < 2 || w < 2 || d_count <= 0 || d_begin < 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_views < 1 || n_views > MVS_MAX_VIEWS) return MVS_ERR_UNSUPPORTED_VIEWS;
  const mvs::LaunchCheck lc;
  mvs::launch_plane_sampling(K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count,
                             d_scale, sampling, (hipStream_t)stream);
  return lc.status();
}

int mvs_cost_volume_fwd_timed(const float* feat, const float* K, const float* R, const float* T,
                              const float* d_min, const float* d_int, int batch_size, int n_views,
                              int channels, int h, int w, int d_begin, int d_count, float d_scale,
                              float* workspace, float* cv_out, void* stream,
                              void* main_begin_event, void* main_end_event) {
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 4, stream,
                              main_begin_event, main_end_event);
}

int mvs_cost_volume_fwd(const float* feat, const float* K, const float* R, const float* T,
                        const float* d_min, const float* d_int, int batch_size, int n_views,
                        int channels, int h, int w, int d_begin, int d_count, float d_scale,
                        float* workspace, float* cv_out, void* stream) {
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 4, stream, nullptr,
                              nullptr);
}

int mvs_cost_volume_fwd_bf16(const float* feat, const float* K, const float* R, const float* T,
                             const float* d_min, const float* d_int, int batch_size, int n_views,
                             int channels, int h, int w, int d_begin, int d_count, float d_scale,
                             float* workspace, void* cv_out, void* stream) {
  if (n_views > 8) return MVS_ERR_UNSUPPORTED_VIEWS;
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 2, stream, nullptr,
                              nullptr);
}

int mvs_cost_volume_fwd_c4(const float* feat, const float* K, const float* R, const float* T,
                           const float* d_min, const float* d_int, int batch_size, int n_views,
                           int channels, int h, int w, int d_begin, int d_count, float d_scale,
                           float* workspace, float* cv_out, void* stream, void* main_begin_event,
                           void* main_end_event) {
  if (n_views > 8) return MVS_ERR_UNSUPPORTED_VIEWS;
  if ((uintptr_t)cv_out & 15u) return MVS_ERR_INVALID_ARGUMENT;
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 16, stream,
                              main_begin_event, main_end_event);
}

int mvs_cost_volume_fwd_c4_absmax(const float* feat, const float* K, const float* R, const float* T,
                                  const float* d_min, const float* d_int, int batch_size, int n_views,
                                  int channels, int h, int w, int d_begin, int d_count, float d_scale,
                                  float* workspace, float* cv_out, void* stream, void* main_begin_event,
                                  void* main_end_event, unsigned* feat_absmax) {
  if (n_views > 8) return MVS_ERR_UNSUPPORTED_VIEWS;
  if (((uintptr_t)cv_out & 15u) || !feat_absmax || ((uintptr_t)feat_absmax & 3u)) return MVS_ERR_INVALID_ARGUMENT;
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 16, stream,
                              main_begin_event, main_end_event, feat_absmax);
}

int mvs_cost_volume_fwd_c4_split(const float* feat, const float* K, const float* R, const float* T,
                                 const float* d_min, const float* d_int, int batch_size, int n_views,
                                 int channels, int h, int w, int d_begin, int d_count, float d_scale,
                                 float* workspace, void* cv_out, void* stream, void* main_begin_event,
                                 void* main_end_event, unsigned* feat_absmax) {
  if (n_views > 8) return MVS_ERR_UNSUPPORTED_VIEWS;
  if (((uintptr_t)cv_out & 15u) || !feat_absmax || ((uintptr_t)feat_absmax & 3u)) return MVS_ERR_INVALID_ARGUMENT;
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 17, stream,
                              main_begin_event, main_end_event, feat_absmax);
}

int mvs_conv3d_split_weights(const float* weight, unsigned short* frag, int* weight_exp) {
  if (!weight || !frag || !weight_exp) return MVS_ERR_INVALID_ARGUMENT;
  // scale 2^ew with max|w| 2^ew < 2^14 (all-zero weights: ew = 0)
  float m = 0.0f;
  for (int k = 0; k < 8 * 32 * 27; ++k) {
    if (!std::isfinite(weight[k])) return MVS_ERR_INVALID_ARGUMENT;
    m = std::max(m, std::fabs(weight[k]));
  }
  int e = 0;
  if (m > 0.0f) (void)std::frexp(m, &e);
  const int ew = m > 0.0f ? std::min(std::max(14 - e, -120), 120) : 0;
  // frag[tap][lane][j]: lane (c = lane & 15, g = lane >> 4) holds B[k = 8g + j][col c] of the
  // 16x16x32 MFMA, column c < 8 = w_hi of output channel c, c >= 8 = w_lo of channel c - 8, k = input
  // channel; tap = (kz * 3 + ky) * 3 + kx; nn.Conv3d weight [8][32][3][3][3]
  for (int tap = 0; tap < 27; ++tap)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        const int c = lane & 15, ci = 8 * (lane >> 4) + j, co = c & 7;
        const float v = std::ldexp(weight[(co * 32 + ci) * 27 + tap], ew);
        const _Float16 hi = (_Float16)v;
        const _Float16 part = c < 8 ? hi : (_Float16)(v - (float)hi);
        uint16_t bits;
        std::memcpy(&bits, &part, 2);
        frag[(tap * 64 + lane) * 8 + j] = bits;
      }
  *weight_exp = ew;
  return MVS_OK;
}

int mvs_conv3d_s2_split_weights(const float* weight, unsigned short* frag, int* weight_exp) {
  if (!weight || !frag || !weight_exp) return MVS_ERR_INVALID_ARGUMENT;
  float m = 0.0f;
  for (int k = 0; k < 16 * 32 * 27; ++k) {
    if (!std::isfinite(weight[k])) return MVS_ERR_INVALID_ARGUMENT;
    m = std::max(m, std::fabs(weight[k]));
  }
  int e = 0;
  if (m > 0.0f) (void)std::frexp(m, &e);
  const int ew = m > 0.0f ? std::min(std::max(14 - e, -120), 120) : 0;
  // frag[tap][part][lane][j]: lane (c = lane & 15, g = lane >> 4) holds B[k = 8g + j][col c], column
  // c = output channel c, k = input channel; part 0 = hi, 1 = lo; nn.Conv3d weight [16][32][3][3][3]
  for (int tap = 0; tap < 27; ++tap)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        const int co = lane & 15, ci = 8 * (lane >> 4) + j;
        const float v = std::ldexp(weight[(co * 32 + ci) * 27 + tap], ew);
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        uint16_t bh, bl;
        std::memcpy(&bh, &hi, 2);
        std::memcpy(&bl, &lo, 2);
        frag[((tap * 2 + 0) * 64 + lane) * 8 + j] = bh;
        frag[((tap * 2 + 1) * 64 + lane) * 8 + j] = bl;
      }
  *weight_exp = ew;
  return MVS_OK;
}

int mvs_conv3d_s2_split_fwd(const void* x, int flags, const void* weight_frag, int weight_exp,
                            const unsigned* x_absmax, float* y, int batch, const int* dims,
                            const int* out_origin, const int* out_size, const int* pad, const float* bn_scale,
                            const float* bn_shift, const float* bn_mean, void* stream) {
  if (!x || !weight_frag || !y || !dims || !out_origin || !out_size || !pad || batch <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & ~MVS_CONV_IN_SPLIT) || ((flags & MVS_CONV_IN_SPLIT) && !x_absmax)) return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)x & 15u) || ((uintptr_t)weight_frag & 15u) || ((uintptr_t)x_absmax & 3u))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  if (weight_exp < -120 || weight_exp > 120) return MVS_ERR_INVALID_ARGUMENT;
  uint64_t vox = 1, ovox = 1;
  for (int d = 0; d < 3; ++d) {
    if (dims[d] <= 0 || out_size[d] <= 0 || out_origin[d] < 0 || pad[d] < 0) return MVS_ERR_INVALID_ARGUMENT;
    // outputs of conv3d(stride 2, padding pad): (n + 2 pad - 3) / 2 + 1 per dim
    if (out_origin[d] + out_size[d] > (dims[d] + 2 * pad[d] - 3) / 2 + 1) return MVS_ERR_INVALID_ARGUMENT;
    vox *= (uint64_t)dims[d];
    ovox *= (uint64_t)out_size[d];
  }
  if (128ull * vox > 0xFFFFFFF0ull || (uint64_t)batch * ovox * 16ull >= (1ull << 40)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int st = mvs::launch_conv_s2_split(x, (flags & MVS_CONV_IN_SPLIT) != 0, weight_frag, weight_exp, x_absmax,
                                           y, batch, dims, out_origin, out_size, pad, bn_scale, bn_shift, bn_mean,
                                           (hipStream_t)stream);
  return st != MVS_OK ? st : lc.status();
}

int mvs_cost_volume_head_fwd(const float* feat, const float* K, const float* R, const float* T,
                             const float* d_min, const float* d_int, int batch_size, int n_views,
                             int channels, int h, int w, int d_begin, int d_count, float d_scale,
                             const void* w0_frag, int w0_exp, const float* bn0_scale, const float* bn0_shift,
                             const float* bn0_mean, const void* w1_frag, int w1_exp, const float* bn1_scale,
                             const float* bn1_shift, const float* bn1_mean, const int* pad,
                             const int* y1_origin, const int* y1_size, const int* scv_lo, const int* scv_hi,
                             float* workspace, unsigned* feat_absmax, float* y0, float* y1, void* scv,
                             void* stream, void* main_begin_event, void* main_end_event) {
  if (!feat || !workspace || !feat_absmax || !y0 || !y1 || !w0_frag || !w1_frag || !pad || !y1_origin ||
      !y1_size || !scv_lo || !scv_hi)
    return MVS_ERR_INVALID_ARGUMENT;
  if (!cams_ok(K, R, T, d_min, d_int) || d_begin < 0) return MVS_ERR_INVALID_ARGUMENT;
  if (n_views < 2 || n_views > 3) return MVS_ERR_UNSUPPORTED_VIEWS;
  if (channels != 32 || (d_count & 1)) return MVS_ERR_INVALID_ARGUMENT;
  if ((((uintptr_t)w0_frag) | ((uintptr_t)w1_frag) | ((uintptr_t)y0) | ((uintptr_t)scv)) & 15u) return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)feat_absmax) & 3u) return MVS_ERR_INVALID_ARGUMENT;
  if ((bn0_scale != nullptr) != (bn0_shift != nullptr) || (bn0_scale != nullptr) != (bn0_mean != nullptr) ||
      (bn1_scale != nullptr) != (bn1_shift != nullptr) || (bn1_scale != nullptr) != (bn1_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  if (w0_exp < -120 || w0_exp > 120 || w1_exp < -120 || w1_exp > 120) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g, 16);
  if (st != MVS_OK) return st;
  const int n[3] = {d_count, h, w};
  uint64_t ovox = 1;
  for (int d = 0; d < 3; ++d) {
    if (pad[d] < 1 || !(pad[d] & 1)) return MVS_ERR_INVALID_ARGUMENT;
    if (y1_size[d] <= 0 || y1_origin[d] < 0 || y1_origin[d] + y1_size[d] > (n[d] + 2 * pad[d] - 3) / 2 + 1)
      return MVS_ERR_INVALID_ARGUMENT;
    if (scv_lo[d] < 0 || scv_hi[d] > n[d] || scv_lo[d] > scv_hi[d]) return MVS_ERR_INVALID_ARGUMENT;
    ovox *= (uint64_t)y1_size[d];
  }
  if (128ull * (uint64_t)(scv_hi[0] - scv_lo[0]) * (uint64_t)(scv_hi[1] - scv_lo[1]) *
          (uint64_t)(scv_hi[2] - scv_lo[2]) > 0xFFFFFFF0ull ||
      (uint64_t)batch_size * ovox * 16ull >= (1ull << 40))
    return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  hipStream_t s = (hipStream_t)stream;
  const mvs::Cams cm{K, R, T, d_min, d_int, d_begin, d_scale};
  const float* bn0[3] = {bn0_scale, bn0_shift, bn0_mean};
  const float* bn1[3] = {bn1_scale, bn1_shift, bn1_mean};
  st = mvs::launch_cv_head(g, feat, cm, workspace, reinterpret_cast<uint32_t*>(feat_absmax), w0_frag, w0_exp, w1_frag,
                           w1_exp, bn0, bn1, y0, y1, scv, pad, y1_origin, y1_size, scv_lo, scv_hi, s,
                           (hipEvent_t)main_begin_event, (hipEvent_t)main_end_event);
  if (st != MVS_OK) return st;
  return lc.status();
}

int mvs_split_head_fwd(const void* scv, const unsigned* x_absmax, int batch, int d_count, int h, int w,
                       const void* w0_frag, int w0_exp, const float* bn0_scale, const float* bn0_shift,
                       const float* bn0_mean, const void* w1_frag, int w1_exp, const float* bn1_scale,
                       const float* bn1_shift, const float* bn1_mean, const int* pad, const int* y1_origin,
                       const int* y1_size, float* y0, float* y1, unsigned* y1_bound, void* stream,
                       void* main_begin_event, void* main_end_event) {
  if (!scv || !x_absmax || !y0 || !y1 || !w0_frag || !w1_frag || !pad || !y1_origin || !y1_size)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((uintptr_t)y1_bound & 3u) return MVS_ERR_INVALID_ARGUMENT;
  if (batch <= 0 || d_count <= 0 || h <= 0 || w <= 0 || (d_count & 1)) return MVS_ERR_INVALID_ARGUMENT;
  if ((((uintptr_t)scv) | ((uintptr_t)w0_frag) | ((uintptr_t)w1_frag) | ((uintptr_t)y0)) & 15u ||
      ((uintptr_t)x_absmax & 3u))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((bn0_scale != nullptr) != (bn0_shift != nullptr) || (bn0_scale != nullptr) != (bn0_mean != nullptr) ||
      (bn1_scale != nullptr) != (bn1_shift != nullptr) || (bn1_scale != nullptr) != (bn1_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  if (w0_exp < -120 || w0_exp > 120 || w1_exp < -120 || w1_exp > 120) return MVS_ERR_INVALID_ARGUMENT;
  const int n[3] = {d_count, h, w};
  uint64_t ovox = 1;
  for (int d = 0; d < 3; ++d) {
    if (pad[d] < 1 || !(pad[d] & 1)) return MVS_ERR_INVALID_ARGUMENT;
    if (y1_size[d] <= 0 || y1_origin[d] < 0 || y1_origin[d] + y1_size[d] > (n[d] + 2 * pad[d] - 3) / 2 + 1)
      return MVS_ERR_INVALID_ARGUMENT;
    ovox *= (uint64_t)y1_size[d];
  }
  if (128ull * (uint64_t)d_count * (uint64_t)h * (uint64_t)w > 0xFFFFFFF0ull ||
      (uint64_t)batch * ovox * 16ull >= (1ull << 40))
    return MVS_ERR_TOO_LARGE;
  mvs::Geometry g;
  g.B = batch;
  g.V = 2;
  g.C = 32;
  g.h = h;
  g.w = w;
  g.Dc = d_count;
  g.tiles = 0;
  g.total = 0;
  const mvs::LaunchCheck lc;
  const float* bn0[3] = {bn0_scale, bn0_shift, bn0_mean};
  const float* bn1[3] = {bn1_scale, bn1_shift, bn1_mean};
  const int st = mvs::launch_split_head(g, scv, reinterpret_cast<const uint32_t*>(x_absmax), w0_frag, w0_exp, w1_frag,
                                        w1_exp, bn0, bn1, y0, y1, pad, y1_origin, y1_size,
                                        reinterpret_cast<uint32_t*>(y1_bound), (hipStream_t)stream,
                                        (hipEvent_t)main_begin_event, (hipEvent_t)main_end_event);
  return st != MVS_OK ? st : lc.status();
}

int mvs_conv3d_k3_split_fwd(const void* x, int flags, const void* weight_frag, int weight_exp,
                            const unsigned* x_absmax, float* y, int batch, int d, int h, int w,
                            const float* bn_scale, const float* bn_shift, const float* bn_mean, void* stream) {
  if (!x || !weight_frag || !y || batch <= 0 || d <= 0 || h <= 0 || w <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & ~MVS_CONV_IN_SPLIT) || ((flags & MVS_CONV_IN_SPLIT) && !x_absmax)) return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)x & 15u) || ((uintptr_t)weight_frag & 15u) || ((uintptr_t)x_absmax & 3u))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  if (weight_exp < -120 || weight_exp > 120) return MVS_ERR_INVALID_ARGUMENT;
  // one 32-bit buffer descriptor per sample volume (8 quads of 16 B per voxel) and 32-bit staging offsets
  if (128ull * (uint64_t)d * (uint64_t)h * (uint64_t)w > 0xFFFFFFF0ull) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int st = mvs::launch_conv3d_split(x, (flags & MVS_CONV_IN_SPLIT) != 0, weight_frag, weight_exp, x_absmax,
                                          y, batch, d, h, w, bn_scale, bn_shift, bn_mean, (hipStream_t)stream);
  return st != MVS_OK ? st : lc.status();
}

int mvs_cost_volume_fwd_c4_bf16(const float* feat, const float* K, const float* R, const float* T,
                                const float* d_min, const float* d_int, int batch_size, int n_views,
                                int channels, int h, int w, int d_begin, int d_count, float d_scale,
                                float* workspace, void* cv_out, void* stream, void* main_begin_event,
                                void* main_end_event) {
  if (n_views > 8) return MVS_ERR_UNSUPPORTED_VIEWS;
  if ((uintptr_t)cv_out & 7u) return MVS_ERR_INVALID_ARGUMENT;
  return cost_volume_fwd_impl(feat, K, R, T, d_min, d_int, batch_size, n_views, channels, h, w,
                              d_begin, d_count, d_scale, workspace, cv_out, 8, stream,
                              main_begin_event, main_end_event);
}

int mvs_homography_warp_fwd(const float* feat, const float* K, const float* R, const float* T,
                            const float* d_min, const float* d_int, int batch_size, int n_views,
                            int channels, int h, int w, int d_begin, int d_count, float d_scale,
                            float* workspace, float* warped_out, void* stream) {
  if (!feat || !workspace || !warped_out) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g);
  if (st != MVS_OK) return st;
  const mvs::LaunchCheck lc;
  st = mvs_plane_sampling(K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count,
                          d_scale, workspace, stream);
  if (st != MVS_OK) return st;
  mvs::launch_warp(g, feat, workspace, warped_out, (hipStream_t)stream);
  return lc.status();
}

int mvs_assemble_cost_volume_fwd(const float* warped, int batch_size, int n_views, int channels,
                                 int d, int h, int w, float* cv_out, void* stream) {
  if (!warped || !cv_out || batch_size <= 0 || channels <= 0 || d <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_views < 1) return MVS_ERR_UNSUPPORTED_VIEWS;
  const mvs::LaunchCheck lc;
  mvs::launch_variance(warped, batch_size, n_views, (size_t)channels * d * h * w, cv_out,
                       (hipStream_t)stream);
  return lc.status();
}

size_t mvs_cost_volume_bwd_workspace_bytes(int batch_size, int n_views, int channels, int h, int w,
                                           int d_count, int flags) {
  if (batch_size <= 0 || n_views <= 0 || channels <= 0 || h <= 0 || w <= 0 || d_count <= 0) return 0;
  if (flags & ~MVS_BWD_DETERMINISTIC) return 0;
  return mvs::cost_volume_bwd_workspace_bytes(batch_size, n_views, channels, h, w, d_count,
                                              (flags & MVS_BWD_DETERMINISTIC) != 0);
}

int mvs_cost_volume_bwd(const float* feat, const float* workspace, const float* grad_cv,
                        int batch_size, int n_views, int channels, int h, int w, int d_count,
                        int flags, void* bwd_workspace, float* grad_feat, void* stream) {
  if (!feat || !workspace || !grad_cv || !grad_feat || (n_views > 1 && !bwd_workspace))
    return MVS_ERR_INVALID_ARGUMENT;
  if (flags & ~MVS_BWD_DETERMINISTIC) return MVS_ERR_INVALID_ARGUMENT;
  Geometry g;
  const int st = check_geometry(batch_size, n_views, channels, h, w, d_count, g);
  if (st != MVS_OK) return st;
  // the packed backward reads grad_cv through a 32-bit descriptor over one 4-channel chunk
  if (n_views >= 2 && n_views <= 8 && 16ull * (uint64_t)d_count * (uint64_t)h * (uint64_t)w >= (1ull << 31))
    return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int ls = mvs::launch_cost_volume_bwd(g, feat, workspace, grad_cv, bwd_workspace, grad_feat,
                                             (flags & MVS_BWD_DETERMINISTIC) != 0, (hipStream_t)stream);
  return ls != MVS_OK ? ls : lc.status();
}

int mvs_extract_depth_map_fwd(const float* prob, const float* d_batch, int batch_size, int d,
                              int h, int w, int n_est, float* depth_out, void* stream) {
  if (!prob || !d_batch || !depth_out || batch_size <= 0 || d <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (n_est < 1) return MVS_ERR_INVALID_ARGUMENT;
  if (n_est > d) n_est = d;  // every plane index is < n_est: all planes kept
  if (n_est > 16) return MVS_ERR_INVALID_ARGUMENT;
  const mvs::LaunchCheck lc;
  mvs::launch_soft_argmin(prob, d_batch, batch_size, d, (uint32_t)h * (uint32_t)w, n_est, depth_out,
                          (hipStream_t)stream);
  return lc.status();
}

int mvs_normalize_images(const unsigned char* rgb, int n_images, int h, int w, const float* mean,
                         const float* std_dev, float* out, void* stream) {
  if (!rgb || !out || !mean || !std_dev || n_images <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)rgb & 3u) || ((uintptr_t)out & 15u)) return MVS_ERR_INVALID_ARGUMENT;
  const uint64_t hw = (uint64_t)h * (uint64_t)w;
  if (hw >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  for (int c = 0; c < 3; ++c)
    if (!(std_dev[c] != 0.0f)) return MVS_ERR_INVALID_ARGUMENT;
  const mvs::LaunchCheck lc;
  mvs::launch_normalize_images(rgb, n_images, (uint32_t)hw, mean, std_dev, out, (hipStream_t)stream);
  return lc.status();
}

int mvs_depth_threshold(const float* depth, size_t n, float lo, float hi, float* out, void* stream) {
  if (!depth || !out) return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)depth & 15u) || ((uintptr_t)out & 15u)) return MVS_ERR_INVALID_ARGUMENT;
  if (n == 0) return MVS_OK;
  const mvs::LaunchCheck lc;
  mvs::launch_depth_threshold(depth, n, lo, hi, out, (hipStream_t)stream);
  return lc.status();
}

int mvs_conv2d_fwd(const float* x, const float* weight, float* y, int n, int c_in, int c_out, int h, int w,
                   int k, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                   unsigned* y_bound, void* stream) {
  if (!x || !weight || !y || n <= 0 || n > 65535 || h <= 0 || w <= 0 || stride <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  // staging offsets inside one image are 32-bit
  if ((uint64_t)c_in * (uint64_t)h * (uint64_t)w >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int st = mvs::launch_conv2d_narrow(x, weight, y, n, c_in, c_out, h, w, k, stride, bn_scale, bn_shift,
                                           bn_mean, y_bound, (hipStream_t)stream);
  return st != MVS_OK ? st : lc.status();
}

int mvs_conv2d_split_weights(const float* weight, int c_in, int c_out, int k, unsigned short* frag, int* weight_exp) {
  if (!weight || !frag || !weight_exp || k <= 0 || k > 7) return MVS_ERR_INVALID_ARGUMENT;
  if (!(c_in == 8 || c_in == 16 || c_in == 32) || !(c_out == 8 || (c_out > 0 && c_out % 16 == 0)))
    return MVS_ERR_INVALID_ARGUMENT;
  const int taps = k * k, n = c_out * c_in * taps;
  float m = 0.0f;
  for (int i = 0; i < n; ++i) {
    if (!std::isfinite(weight[i])) return MVS_ERR_INVALID_ARGUMENT;
    m = std::max(m, std::fabs(weight[i]));
  }
  int e = 0;
  if (m > 0.0f) (void)std::frexp(m, &e);
  const int ew = m > 0.0f ? std::min(std::max(14 - e, -120), 120) : 0;
  const int kbs = mvs::conv2d_split_kblocks(c_in, k), tpb = 32 / c_in, cpt = c_in / 8;
  const bool narrow = c_out == 8;
  const int nbs = narrow ? 1 : c_out / 16;
  auto part = [&](int co, int ci, int t, int p) -> uint16_t {
    const float v = t < taps ? std::ldexp(weight[((size_t)co * c_in + ci) * taps + t], ew) : 0.0f;
    const _Float16 hi = (_Float16)v;
    const _Float16 r = p == 0 ? hi : (_Float16)(v - (float)hi);
    uint16_t b;
    std::memcpy(&b, &r, 2);
    return b;
  };
  for (int kb = 0; kb < kbs; ++kb)
    for (int nb = 0; nb < nbs; ++nb)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int c = lane & 15, g = lane >> 4;
          const int t = kb * tpb + g / cpt, ci = 8 * (g % cpt) + j;
          if (narrow) {
            frag[((size_t)kb * 64 + lane) * 8 + j] = part(c & 7, ci, t, c >> 3);
          } else {
            const size_t base = ((((size_t)kb * nbs + nb) * 2) * 64 + lane) * 8 + j;
            frag[base] = part(nb * 16 + c, ci, t, 0);
            frag[base + 64 * 8] = part(nb * 16 + c, ci, t, 1);
          }
        }
  *weight_exp = ew;
  return MVS_OK;
}

int mvs_conv2d_split_fwd(const float* x, const void* weight_frag, int weight_exp, float* y, int n, int c_in,
                         int c_out, int h, int w, int k, int stride, const float* bn_scale, const float* bn_shift,
                         const float* bn_mean, const unsigned* x_bound, unsigned* y_bound, void* stream) {
  if (!x || !weight_frag || !y || !x_bound || n <= 0 || n > 65535 || h <= 0 || w <= 0 || stride <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  if (reinterpret_cast<uintptr_t>(weight_frag) % 16) return MVS_ERR_INVALID_ARGUMENT;
  // one image's buffer resource and staging offsets are 32-bit
  if ((uint64_t)c_in * (uint64_t)h * (uint64_t)w * 4u >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int st = mvs::launch_conv2d_split(x, weight_frag, weight_exp, y, n, c_in, c_out, h, w, k, stride, bn_scale,
                                          bn_shift, bn_mean, x_bound, y_bound, (hipStream_t)stream);
  return st != MVS_OK ? st : lc.status();
}

int mvs_conv3d_k3_fwd(const float* x, int flags, const float* weight, float* y, int batch, int c_in,
                      int c_out, int d, int h, int w, const float* bn_scale, const float* bn_shift,
                      const float* bn_mean, const float* x2, const float* in_bn, void* stream) {
  if (in_bn && (c_out != 1 || flags || !x2 || bn_scale)) return MVS_ERR_INVALID_ARGUMENT;
  if (!in_bn && x2) return MVS_ERR_INVALID_ARGUMENT;
  if (!x || !weight || !y || batch <= 0 || c_in <= 0 || d <= 0 || h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (c_out != 1 && c_out != 8) return MVS_ERR_INVALID_ARGUMENT;
  if (flags & ~(MVS_CONV_IN_C4 | MVS_CONV_WINO_Z | MVS_CONV_IN_BF16)) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_IN_BF16) && (!(flags & MVS_CONV_IN_C4) || ((uintptr_t)x & 7u))) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_WINO_Z) && c_out != 8) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_IN_C4) && (c_in % 4 || (!(flags & MVS_CONV_IN_BF16) && ((uintptr_t)x & 15u))))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  // staging offsets inside one channel volume are 32-bit
  if ((uint64_t)d * (uint64_t)h * (uint64_t)w >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int quads = (flags & MVS_CONV_IN_C4) ? ((flags & MVS_CONV_IN_BF16) ? 2 : 1) : 0;
  mvs::launch_conv3d_k3_narrow(x, quads, (flags & MVS_CONV_WINO_Z) != 0, weight, y, batch,
                               c_in, c_out, d, h, w,
                               bn_scale, bn_shift, bn_mean,
                               (hipStream_t)stream, x2, in_bn);
  return lc.status();
}

size_t mvs_conv3d_k3_wgrad_workspace_bytes(int batch, int c_in, int d, int h, int w) {
  if (batch <= 0 || c_in <= 0 || d <= 0 || h <= 0 || w <= 0) return 0;
  return mvs::conv3d_wgrad_workspace_bytes(batch, c_in, d, h, w);
}

int mvs_conv3d_k3_wgrad(const float* x, const float* gy, int batch, int c_in, int c_out, int d, int h, int w,
                        float* dw, void* workspace, void* stream) {
  if (!x || !gy || !dw || !workspace || batch <= 0 || d <= 0 || h <= 0 || w <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if (!mvs::conv3d_wgrad_supported(c_in, c_out)) return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)d * (uint64_t)h * (uint64_t)w >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_conv3d_wgrad(x, gy, batch, c_in, c_out, d, h, w, static_cast<float*>(workspace), dw,
                           (hipStream_t)stream);
  return lc.status();
}

int mvs_conv_head_fp32_fwd(const float* cv4, int batch, int d, int h, int w, const float* w0_wz,
                           const float* bn0_scale, const float* bn0_shift, const float* bn0_mean, const float* w1,
                           const float* w1_pass, const float* bn1_scale, const float* bn1_shift,
                           const float* bn1_mean, const int* pad, const int* y1_origin, const int* y1_size,
                           float* y0, float* y1, void* stream, void* ev0, void* ev1) {
  if (!cv4 || !w0_wz || !w1 || !w1_pass || !y0 || !y1 || !pad || !y1_origin || !y1_size || batch <= 0 || d <= 0 ||
      h <= 0 || w <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)cv4 | (uintptr_t)w1 | (uintptr_t)w1_pass) & 15u) return MVS_ERR_INVALID_ARGUMENT;
  if ((bn0_scale != nullptr) != (bn0_shift != nullptr) || (bn0_scale != nullptr) != (bn0_mean != nullptr) ||
      (bn1_scale != nullptr) != (bn1_shift != nullptr) || (bn1_scale != nullptr) != (bn1_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  const int n[3] = {d, h, w};
  uint64_t ovox = (uint64_t)batch;
  for (int k = 0; k < 3; ++k) {
    if (pad[k] < 1 || !(pad[k] & 1)) return MVS_ERR_INVALID_ARGUMENT;   // the fused windows need P odd
    if (y1_size[k] <= 0 || y1_origin[k] < 0 || y1_origin[k] + y1_size[k] > n[k]) return MVS_ERR_INVALID_ARGUMENT;
    ovox *= (uint64_t)y1_size[k];
  }
  if ((uint64_t)d * h * w >= (1ull << 31) || ovox >= (1ull << 31) || (uint64_t)d * h * w * 64u >= 0xFFFFFFC0ull)
    return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_conv_head_fp32(cv4, batch, d, h, w, w0_wz, bn0_scale, bn0_shift, bn0_mean, w1, w1_pass, bn1_scale,
                             bn1_shift, bn1_mean, pad, y1_origin, y1_size, y0, y1, (hipStream_t)stream,
                             (hipEvent_t)ev0, (hipEvent_t)ev1);
  return lc.status();
}

int mvs_deconv3d_k3s2_fwd(const float* x, const float* x2, int flags, int batch, int c_in, int c_out,
                          int rd, int rh, int rw, int x0d, int x0h, int x0w, const float* weight, int d,
                          int h, int w, int pd, int ph, int pw, const float* bn_scale,
                          const float* bn_shift, const float* bn_mean, const float* residual, float* y,
                          void* stream) {
  if (!x || !weight || !y || batch <= 0 || c_in <= 0 || c_in > 64 || c_out != 8) return MVS_ERR_INVALID_ARGUMENT;
  if (flags & ~(MVS_LAYOUT_CHANNELS_LAST | MVS_DECONV_WEIGHT_TAPS)) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_LAYOUT_CHANNELS_LAST) && (c_in % 4 || ((uintptr_t)x & 15u) || ((uintptr_t)x2 & 15u)))
    return MVS_ERR_INVALID_ARGUMENT;   // 16-byte channel-quad loads
  if (rd <= 0 || rh <= 0 || rw <= 0 || d <= 0 || h <= 0 || w <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if (x0d < 0 || x0h < 0 || x0w < 0 || pd < 0 || ph < 0 || pw < 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  // the region input is read through 32-bit buffer descriptors over the whole batch
  if ((uint64_t)batch * c_in * rd * rh * rw * 4u >= (1ull << 31)) return MVS_ERR_TOO_LARGE;
  const int layout = (flags & MVS_LAYOUT_CHANNELS_LAST) ? ((flags & MVS_DECONV_WEIGHT_TAPS) ? 3 : 1)
                                                        : ((flags & MVS_DECONV_WEIGHT_TAPS) ? 2 : 0);
  const mvs::LaunchCheck lc;
  mvs::launch_deconv3d_k3s2(x, x2, layout, batch, c_in, rd, rh, rw, x0d, x0h,
                            x0w, weight, d, h, w, pd, ph, pw, bn_scale, bn_shift, bn_mean, residual, y,
                            (hipStream_t)stream);
  return lc.status();
}

int mvs_conv3d_region_fwd(int mode, int flags, const float* x, const float* x2, const float* weight, float* y,
                          int batch, int c_in, int c_out, const int* dims, const int* out_origin,
                          const int* out_size, const int* in_origin, const int* in_size,
                          const int* pad, const float* bn_scale, const float* bn_shift,
                          const float* bn_mean, const unsigned* x_absmax, unsigned* y_bound, void* stream) {
  if (!x || !weight || !y || !dims || !out_origin || !out_size || batch <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((uintptr_t)y_bound & 3u) return MVS_ERR_INVALID_ARGUMENT;
  if (mode < MVS_CONV_S1 || mode > MVS_CONV_T2 ||
      (flags & ~(MVS_CONV_OUT_NCDHW | MVS_CONV_IN_C4 | MVS_CONV_IN_BF16 | MVS_CONV_IN_SPLIT | MVS_CONV_PER_LANE |
                 MVS_CONV_S2_LDS)))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_S2_LDS) && (flags & MVS_CONV_PER_LANE)) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_IN_BF16) && !(flags & MVS_CONV_IN_C4)) return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_IN_SPLIT) && (!(flags & MVS_CONV_IN_C4) || (flags & MVS_CONV_IN_BF16) || !x_absmax ||
                                      ((uintptr_t)x_absmax & 3u)))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((flags & MVS_CONV_IN_C4) && (mode != MVS_CONV_S2 || c_in % 4)) return MVS_ERR_INVALID_ARGUMENT;
  if (mode != MVS_CONV_S2 && (!in_origin || !in_size)) return MVS_ERR_INVALID_ARGUMENT;
  if ((in_origin != nullptr) != (in_size != nullptr)) return MVS_ERR_INVALID_ARGUMENT;
  const bool boxed = in_origin != nullptr;   // S2: x holds the box [in_origin, + in_size) of the volume
  if (mode != MVS_CONV_S1 && !pad) return MVS_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)x | (uintptr_t)x2 | (uintptr_t)weight) & 15u) return MVS_ERR_INVALID_ARGUMENT;   // 16-byte loads
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  uint64_t ovox = (uint64_t)batch, ivox = (uint64_t)batch, nvox = (uint64_t)batch * c_in;
  for (int k = 0; k < 3; ++k) {
    if (dims[k] <= 0 || out_size[k] <= 0 || out_origin[k] < 0 || out_origin[k] + out_size[k] > dims[k])
      return MVS_ERR_INVALID_ARGUMENT;
    if (boxed && (in_size[k] <= 0 || in_origin[k] < 0 || in_origin[k] + in_size[k] > dims[k]))
      return MVS_ERR_INVALID_ARGUMENT;
    ovox *= (uint64_t)out_size[k];
    ivox *= (uint64_t)(boxed ? in_size[k] : dims[k]);
    nvox *= (uint64_t)dims[k];
  }
  // 32-bit row indices; per sample, 32-bit buffer descriptors over the input (S2: the 16 channel planes
  // or 4 channel quads of one 16-channel block, 64 B per voxel; S1 / T2: the region tensor)
  uint64_t svox = 1;
  for (int k = 0; k < 3; ++k) svox *= (uint64_t)(boxed ? in_size[k] : dims[k]);
  const uint64_t desc_bytes = mode == MVS_CONV_S2 ? svox * 64u : svox * (uint64_t)c_in * 4u;
  if (ovox >= (1ull << 31) || desc_bytes >= 0xFFFFFFC0ull || ivox * (uint64_t)c_in >= (1ull << 62) ||
      nvox >= (1ull << 62))
    return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int quads = (flags & MVS_CONV_IN_C4)
                        ? ((flags & MVS_CONV_IN_SPLIT) ? 3 : ((flags & MVS_CONV_IN_BF16) ? 2 : 1)) : 0;
  const int st = mvs::launch_conv3d_region(mode, (flags & MVS_CONV_OUT_NCDHW) != 0, quads,
                                           x, x2, weight, y, batch, c_in, c_out, dims, out_origin, out_size,
                                           in_origin, in_size, pad, bn_scale, bn_shift, bn_mean,
                                           (hipStream_t)stream, reinterpret_cast<const uint32_t*>(x_absmax),
                                           reinterpret_cast<uint32_t*>(y_bound), (flags & MVS_CONV_PER_LANE) != 0,
                                           nullptr, nullptr, (flags & MVS_CONV_S2_LDS) != 0);
  if (st != MVS_OK) return st;
  return lc.status();
}

int mvs_conv3d_region_split_weights(const float* weight, int c_in, int c_out, unsigned short* frag, int* weight_exp) {
  if (!weight || !frag || !weight_exp) return MVS_ERR_INVALID_ARGUMENT;
  if (c_out <= 0 || c_out % 16 || !(c_in == 16 || (c_in > 0 && c_in % 32 == 0))) return MVS_ERR_INVALID_ARGUMENT;
  const int n = 27 * c_out * c_in;
  float m = 0.0f;
  for (int k = 0; k < n; ++k) {
    if (!std::isfinite(weight[k])) return MVS_ERR_INVALID_ARGUMENT;
    m = std::max(m, std::fabs(weight[k]));
  }
  int e = 0;
  if (m > 0.0f) (void)std::frexp(m, &e);
  const int ew = m > 0.0f ? std::min(std::max(14 - e, -120), 120) : 0;
  // frag[kb][nb][part][lane][j]: lane (c = lane & 15, g = lane >> 4) holds B[k = 8g + j][column c] of the
  // 16x16x32 MFMA for output channel nb * 16 + c; part 0 = fp16(w 2^ew), 1 = fp16(w 2^ew - part 0).
  // K block kb: c_in >= 32: tap kb / (c_in / 32), input channel (kb % (c_in / 32)) * 32 + 8g + j;
  // c_in = 16: tap 2 kb + (g >> 1) (zero past tap 26), input channel 8 (g & 1) + j.  weight [27][c_out][c_in]
  const int kbs = mvs::conv3d_region_split_kblocks(c_in), nbs = c_out / 16;
  for (int kb = 0; kb < kbs; ++kb)
    for (int nb = 0; nb < nbs; ++nb)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int c = lane & 15, gq = lane >> 4, co = nb * 16 + c;
          int tap, ci;
          if (c_in == 16) {
            tap = 2 * kb + (gq >> 1);
            ci = 8 * (gq & 1) + j;
          } else {
            tap = kb / (c_in / 32);
            ci = (kb % (c_in / 32)) * 32 + 8 * gq + j;
          }
          const float v = tap < 27 ? std::ldexp(weight[((size_t)tap * c_out + co) * c_in + ci], ew) : 0.0f;
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (float)hi);
          uint16_t bh, bl;
          std::memcpy(&bh, &hi, 2);
          std::memcpy(&bl, &lo, 2);
          const size_t base = ((((size_t)kb * nbs + nb) * 2) * 64 + lane) * 8 + j;
          frag[base] = bh;
          frag[base + 64 * 8] = bl;
        }
  *weight_exp = ew;
  return MVS_OK;
}

int mvs_conv3d_region_split_fwd(int mode, int flags, const float* x, const float* x2, const void* weight_frag,
                                int weight_exp, float* y, int batch, int c_in, int c_out, const int* dims,
                                const int* out_origin, const int* out_size, const int* in_origin, const int* in_size,
                                const int* pad, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                                const unsigned* x_bound, const unsigned* x2_bound, unsigned* y_bound,
                                const float* y_addend, const int* store_origin, const int* store_size, double* stats,
                                float* y_mid, float* y_high, const float* in_bn, void* stream) {
  if (!x || !weight_frag || !y || !dims || !out_origin || !out_size || batch <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((store_origin != nullptr) != (store_size != nullptr) || ((uintptr_t)stats & 7u) || ((uintptr_t)in_bn & 15u))
    return MVS_ERR_INVALID_ARGUMENT;
  if (store_origin)   // the store box lies inside the output region
    for (int k = 0; k < 3; ++k)
      if (store_size[k] <= 0 || store_origin[k] < out_origin[k] ||
          store_origin[k] + store_size[k] > out_origin[k] + out_size[k])
        return MVS_ERR_INVALID_ARGUMENT;
  if (mode < MVS_CONV_S1 || mode > MVS_CONV_T2 ||
      (flags & ~(MVS_CONV_OUT_NCDHW | MVS_CONV_IN_C4 | MVS_CONV_IN_SPLIT | MVS_CONV_PER_LANE)))
    return MVS_ERR_INVALID_ARGUMENT;
  // S2 reads the split cost volume (its 8 bound words in x_bound), S1 / T2 an fp32 region tensor
  const bool s2 = mode == MVS_CONV_S2;
  const int in_flags = MVS_CONV_IN_C4 | MVS_CONV_IN_SPLIT;
  if (s2 != ((flags & in_flags) == in_flags) || (!s2 && (flags & in_flags))) return MVS_ERR_INVALID_ARGUMENT;
  if (s2 && (x2 || !x_bound || c_in != 32)) return MVS_ERR_INVALID_ARGUMENT;
  if ((in_origin != nullptr) != (in_size != nullptr) || (!s2 && !in_origin)) return MVS_ERR_INVALID_ARGUMENT;
  if (mode != MVS_CONV_S1 && !pad) return MVS_ERR_INVALID_ARGUMENT;
  int io[3] = {0, 0, 0}, is[3] = {dims[0], dims[1], dims[2]};   // S2 without a box: the whole volume
  if (in_origin)
    for (int k = 0; k < 3; ++k) {
      io[k] = in_origin[k];
      is[k] = in_size[k];
    }
  // every mode scales its input by the bound words (S2: the split volume's; S1 / T2: the region
  // tensor's, raised by the kernel that wrote it): without them the fp16 hi parts could overflow
  if (!x_bound || (x2 && !x2_bound)) return MVS_ERR_INVALID_ARGUMENT;   // a sum needs both bounds
  if (((uintptr_t)x | (uintptr_t)x2 | (uintptr_t)weight_frag) & 15u ||
      ((uintptr_t)x_bound | (uintptr_t)x2_bound | (uintptr_t)y_bound) & 3u)
    return MVS_ERR_INVALID_ARGUMENT;
  if (weight_exp < -120 || weight_exp > 120) return MVS_ERR_INVALID_ARGUMENT;
  if ((bn_scale != nullptr) != (bn_shift != nullptr) || (bn_scale != nullptr) != (bn_mean != nullptr))
    return MVS_ERR_INVALID_ARGUMENT;
  uint64_t ovox = (uint64_t)batch, svox = 1;
  for (int k = 0; k < 3; ++k) {
    if (dims[k] <= 0 || out_size[k] <= 0 || out_origin[k] < 0 || out_origin[k] + out_size[k] > dims[k])
      return MVS_ERR_INVALID_ARGUMENT;
    if (is[k] <= 0 || io[k] < 0 || io[k] + is[k] > dims[k]) return MVS_ERR_INVALID_ARGUMENT;
    ovox *= (uint64_t)out_size[k];
    svox *= (uint64_t)is[k];
  }
  if (ovox >= (1ull << 31) || svox * (uint64_t)c_in * 4u >= 0xFFFFFFC0ull) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  const int st = mvs::launch_conv3d_region_split(
      mode, (flags & MVS_CONV_OUT_NCDHW) != 0, x, x2, weight_frag, weight_exp, y, batch, c_in, c_out, dims, out_origin,
      out_size, io, is, pad, bn_scale, bn_shift, bn_mean, reinterpret_cast<const uint32_t*>(x_bound),
      reinterpret_cast<const uint32_t*>(x2_bound), reinterpret_cast<uint32_t*>(y_bound), (hipStream_t)stream,
      (flags & MVS_CONV_PER_LANE) != 0, y_addend, store_origin, store_size, stats, y_mid, y_high, in_bn);
  if (st != MVS_OK) return st;
  return lc.status();
}

long long mvs_conv3d_region_split_stats_slots(int mode, int flags, int batch, int c_in, int c_out,
                                              const int* out_size) {
  if (!out_size || batch <= 0 || mode < MVS_CONV_S1 || mode > MVS_CONV_T2) return MVS_ERR_INVALID_ARGUMENT;
  for (int k = 0; k < 3; ++k)
    if (out_size[k] <= 0) return MVS_ERR_INVALID_ARGUMENT;
  return mvs::conv3d_region_split_slots(mode, batch, c_in, c_out, out_size, (flags & MVS_CONV_PER_LANE) != 0,
                                        (flags & MVS_CONV_SUM_INPUT) != 0, (flags & MVS_CONV_IN_BN) != 0);
}


int mvs_softmax_depth_fwd(const float* x, int batch, int d_count, int h, int w, float* y, void* stream) {
  if (!x || !y || batch <= 0 || d_count <= 0 || h <= 0 || w <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)h * (uint64_t)w >= (1ull << 32) || (uint64_t)batch * h * w >= (1ull << 37)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_softmax_depth(x, batch, d_count, (uint32_t)((uint64_t)h * w), y, (hipStream_t)stream);
  return lc.status();
}

int mvs_depth_hypotheses_fwd(const float* d_min, const float* d_int, int batch, int d_num, float d_scale, float* out,
                             void* stream) {
  if (!d_min || !d_int || !out || batch <= 0 || d_num <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if ((int64_t)batch * d_num >= (1ll << 31)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_depth_hypotheses(d_min, d_int, d_scale, batch, d_num, out, (hipStream_t)stream);
  return lc.status();
}

int mvs_refine_input_fwd(const float* initial_depth, const float* d_min, const float* d_int, int batch, int h,
                         int w, int d_num, float d_scale, const float* ref_img, float* out, void* stream) {
  if (!initial_depth || !d_min || !d_int || !ref_img || !out || batch <= 0 || h <= 0 || w <= 0 || d_num <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)h * (uint64_t)w >= (1ull << 32) || (uint64_t)batch * h * w >= (1ull << 37)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_refine_input(initial_depth, d_min, d_int, d_num, d_scale, ref_img, batch, (uint32_t)((uint64_t)h * w),
                           out, (hipStream_t)stream);
  return lc.status();
}

int mvs_refine_output_fwd(const float* conv, const float* refine_in, const float* d_min, const float* d_int,
                          int batch, int h, int w, int d_num, float d_scale, float* out, void* stream) {
  if (!conv || !refine_in || !d_min || !d_int || !out || batch <= 0 || h <= 0 || w <= 0 || d_num <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)h * (uint64_t)w >= (1ull << 32) || (uint64_t)batch * h * w >= (1ull << 37)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_refine_output(conv, refine_in, d_min, d_int, d_num, d_scale, batch, (uint32_t)((uint64_t)h * w), out,
                            (hipStream_t)stream);
  return lc.status();
}

static bool channel_layout_ok(int layout, int channels, const void* a, const void* b, const void* c) {
  if (layout & ~MVS_LAYOUT_CHANNELS_LAST) return false;
  if (!(layout & MVS_LAYOUT_CHANNELS_LAST)) return true;
  const int c4 = channels / 4;
  if (channels % 4 || c4 > 64 || (c4 & (c4 - 1))) return false;   // quads per voxel: a power of two
  return ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c)) & 15u) == 0;
}

size_t mvs_channel_stats_slots(int layout, int batch, int channels, long long voxels) {
  if (batch <= 0 || channels <= 0 || voxels <= 0 || (layout & ~MVS_LAYOUT_CHANNELS_LAST)) return 0;
  return mvs::channel_stats_slots((layout & MVS_LAYOUT_CHANNELS_LAST) != 0, batch, channels, (size_t)voxels);
}

int mvs_channel_stats(const float* x, int layout, int batch, int channels, long long voxels, double* stats,
                      void* stream) {
  if (!x || !stats || batch <= 0 || channels <= 0 || voxels <= 0) return MVS_ERR_INVALID_ARGUMENT;
  if (!channel_layout_ok(layout, channels, x, nullptr, nullptr)) return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)batch * channels > 65535u && !(layout & MVS_LAYOUT_CHANNELS_LAST)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_channel_stats(x, (layout & MVS_LAYOUT_CHANNELS_LAST) != 0, batch, channels, (size_t)voxels, stats,
                            (hipStream_t)stream);
  return lc.status();
}

int mvs_bn_train_params(const double* sums, int channels, double count, const double* border_u,
                        const double* border_count, int prev_channels, int classes, const float* prev_params,
                        const float* weight, const float* bias, float* running_mean, float* running_var,
                        long long* num_batches_tracked, double momentum, double eps, float* params, void* stream) {
  if (!sums || !weight || !bias || !params || channels <= 0 || !(count > 0.0) || !(eps >= 0.0))
    return MVS_ERR_INVALID_ARGUMENT;
  if ((running_mean != nullptr) != (running_var != nullptr)) return MVS_ERR_INVALID_ARGUMENT;
  if (border_u && (!border_count || !prev_params || prev_channels <= 0 || prev_channels > 256 || classes <= 0 ||
                   (long long)channels * classes > 2048))
    return MVS_ERR_INVALID_ARGUMENT;
  const mvs::LaunchCheck lc;
  mvs::launch_bn_train_params(sums, channels, count, border_u, border_count, prev_channels, classes, prev_params,
                              weight, bias, running_mean, running_var, num_batches_tracked, momentum, eps, params,
                              (hipStream_t)stream);
  return lc.status();
}

int mvs_bn_relu(const float* x, int layout, int batch, int channels, long long voxels, const float* scale,
                const float* shift, const float* mean, const float* r, const float* r_scale,
                const float* r_shift, const float* r_mean, float* y, unsigned* y_bound, void* stream) {
  if (!x || !y || !scale || !shift || !mean || batch <= 0 || channels <= 0 || voxels <= 0)
    return MVS_ERR_INVALID_ARGUMENT;
  if ((uintptr_t)y_bound & 3u) return MVS_ERR_INVALID_ARGUMENT;
  if (r && (!r_scale || !r_shift || !r_mean)) return MVS_ERR_INVALID_ARGUMENT;
  if (!channel_layout_ok(layout, channels, x, r, y)) return MVS_ERR_INVALID_ARGUMENT;
  if ((uint64_t)batch * channels > 65535u && !(layout & MVS_LAYOUT_CHANNELS_LAST)) return MVS_ERR_TOO_LARGE;
  const mvs::LaunchCheck lc;
  mvs::launch_bn_relu(x, (layout & MVS_LAYOUT_CHANNELS_LAST) != 0, batch, channels, (size_t)voxels, scale, shift,
                      mean, r, r_scale, r_shift, r_mean, y, reinterpret_cast<uint32_t*>(y_bound),
                      (hipStream_t)stream);
  return lc.status();
}

}  // extern "C"
