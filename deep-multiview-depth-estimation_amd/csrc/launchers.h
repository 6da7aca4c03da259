// launchers.h -- host-side launchers, one per translation unit; the C ABI (capi.hip) calls these.
// Arguments are validated by the caller; launchers only enqueue work on `s` and never allocate or
// synchronise (graph-capturable).
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace mvs {

// plane_sampling.hip: sampling[N][d_count][9] (fp64 geometry, stored fp32)
void launch_plane_sampling(const float* K, const float* R, const float* T, const float* d_min,
                           const float* d_int, int B, int V, int h, int w, int d_begin,
                           int d_count, float d_scale, float* sampling, hipStream_t s);

// cost_volume_fwd.hip: fused warp + variance.  `sampling` is the workspace's matrix area (written
// by the launch: its prologue kernel forms the sampling matrices, packs the features and resamples
// the reference views in one kernel), `packed` the area after it (packed_bytes()).  ev0/ev1
// (optional) are recorded on `s` right before and after the main fused kernel (its live timing,
// bench.py).
size_t packed_bytes(int B, int V, int C, int h, int w);
void launch_cost_volume_fwd(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                            float* packed, float* cv, hipStream_t s, hipEvent_t ev0 = nullptr,
                            hipEvent_t ev1 = nullptr);
// same, channel-quad layout cv[B][C/4][Dc][h][w][4] fp32, 2 <= V <= 8
void launch_cost_volume_fwd_c4(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                               float* packed, float* cv, hipStream_t s, hipEvent_t ev0 = nullptr,
                               hipEvent_t ev1 = nullptr, uint32_t* absmax = nullptr, bool split = false);
// same, bf16 channel-quad layout cv[B][C/4][Dc][h][w][4] (RNE), 2 <= V <= 8
void launch_cost_volume_fwd_c4_bf16(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                                    float* packed, void* cv, hipStream_t s, hipEvent_t ev0 = nullptr,
                                    hipEvent_t ev1 = nullptr);
// same, bf16 cost volume (uint16 storage, RNE), 2 <= V <= 8
void launch_cost_volume_fwd_bf16(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                                 float* packed, void* cv, hipStream_t s, hipEvent_t ev0 = nullptr,
                                 hipEvent_t ev1 = nullptr);

// the fused launch's prologue alone with PIXEL-MAJOR packed features packed[N][h+2][w+2][C4] float4
// (+ refs, bound words folded into absmax[8]); ws = the area after the sampling matrices
void launch_cv_prologue_pm(const Geometry& g, const float* feat, const Cams& cm, float* sampling, float* ws,
                           uint32_t* absmax, hipStream_t s);

// cv_head.hip: the cost volume consumed where it is formed -- prologue, then ONE kernel forming the
// variance plane by plane on chip and applying conv_0_0 (+ BN_0 + ReLU, y0 [B][8][D][H][W]) and the
// stride-2 conv_1_0 (+ BN_1 + ReLU, channels-last region y1 [B][on...][16]); optionally stores the split
// cost volume on the box [r0, r1) (scv, full-size [B][8][D][H][W] x 16 B).  C = 32, V in {2, 3}, pad odd,
// D even (validated by the caller).  bn0 / bn1: {scale, shift, mean} or three nulls.
int launch_cv_head(const Geometry& g, const float* feat, const Cams& cm, float* ws, uint32_t* absmax,
                   const void* w0frag, int w_exp0, const void* w1frag, int w_exp1, const float* const* bn0,
                   const float* const* bn1, float* y0, float* y1, void* scv, const int* pad, const int* o0,
                   const int* on, const int* r0, const int* r1, hipStream_t s, hipEvent_t ev0 = nullptr,
                   hipEvent_t ev1 = nullptr);
// the same kernel on a materialised split cost volume (conv_0_0 + conv_1_0 in one pass over it)
int launch_split_head(const Geometry& g, const void* scv_in, const uint32_t* absmax, const void* w0frag, int w_exp0,
                      const void* w1frag, int w_exp1, const float* const* bn0, const float* const* bn1, float* y0,
                      float* y1, const int* pad, const int* o0, const int* on, uint32_t* y1_bound, hipStream_t s,
                      hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

// warp_variance.hip
void launch_warp(const Geometry& g, const float* feat, const float* sampling, float* warped,
                 hipStream_t s);
void launch_variance(const float* warped, int B, int V, size_t M, float* cv, hipStream_t s);

// cost_volume_bwd.hip: grad_feat (overwritten) from grad_cv, the forward's workspace (sampling
// matrices + packed features + resampled reference views) and a backward workspace of
// cost_volume_bwd_workspace_bytes(); deterministic = 64-bit fixed-point accumulation throughout
size_t cost_volume_bwd_workspace_bytes(int B, int V, int C, int h, int w, int Dc, bool deterministic);
int launch_cost_volume_bwd(const Geometry& g, const float* feat, const float* fwd_ws,
                           const float* grad_cv, void* bwd_ws, float* grad_feat, bool deterministic,
                           hipStream_t s);

// soft_argmin.hip (+ the regulariser's softmax over depth, model.py:97)
void launch_softmax_depth(const float* x, int B, int D, uint32_t hw, float* y, hipStream_t s);
void launch_depth_hypotheses(const float* d_min, const float* d_int, float d_scale, int B, int D, float* out,
                             hipStream_t s);
void launch_refine_input(const float* ini, const float* d_min, const float* d_int, int d_num, float d_scale,
                         const float* img, int B, uint32_t hw, float* out, hipStream_t s);
void launch_refine_output(const float* conv, const float* inp, const float* d_min, const float* d_int, int d_num,
                          float d_scale, int B, uint32_t hw, float* out, hipStream_t s);
void launch_soft_argmin(const float* prob, const float* d_batch, int B, int D, uint32_t hw,
                        int n_est, float* depth, hipStream_t s);

// conv3d_narrow.hip: 3x3x3 stride-1 padding-1 bias-free Conv3d, NCDHW fp32, Cout in {1, 8}
// (optional epilogue: max((v - bn_mean) * bn_scale + bn_shift, 0), all three or none); in_c4: the
// input is channel-quad in[B][Cin/4][D][H][W][4], fp32 (1) or bf16 (2)
// wino_z (Cout = 8): Winograd F(2,3) along depth, weight = the transformed wu[Cin][3][3][4][8]
// csrc/conv3d_s2_lds.hip: conv_1_0 (S2 32 -> 16) from the whole fp32 volume (channel quads or NCDHW), LDS-staged
bool conv_s2_lds_enabled();
void launch_conv_s2_lds(const float* x, int in_c4, const float* w27, float* y, int B, const int* n, const int* o0,
                        const int* on, const int* pad, const float* bn_scale, const float* bn_shift,
                        const float* bn_mean, hipStream_t s);
// csrc/conv3d_wgrad.hip: narrow Conv3d weight gradient (dw [c_out][c_in][27]); part: the workspace
size_t conv3d_wgrad_workspace_bytes(int B, int c_in, int D, int H, int W);
bool conv3d_wgrad_supported(int c_in, int c_out);
void launch_conv3d_wgrad(const float* x, const float* gy, int B, int c_in, int c_out, int D, int H, int W,
                         float* part, float* dw, hipStream_t s);
void launch_conv3d_k3_narrow(const float* in, int in_c4, bool wino_z, const float* weight, float* out, int B,
                             int Cin, int Cout, int D, int H, int W, const float* bn_scale, const float* bn_shift,
                             const float* bn_mean, hipStream_t s, const float* in2 = nullptr,
                             const float* ibn = nullptr);

// conv3d_split.hip: conv_0_0 (32 -> 8, 3x3x3, padding 1) on the f16 MFMA with split-fp16 operands;
// x channel-quad fp32 [B][8][D][H][W][4], wfrag [27][64][8] fp16 fragments (mvs_conv3d_split_weights),
// absmax 8 words bounding max|feat| of the cost volume (or NULL: unscaled); y NCDHW fp32
int launch_conv3d_split(const void* x, bool presplit, const void* wfrag, int w_exp, const uint32_t* absmax, float* y, int B,
                        int D, int H, int W, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                        hipStream_t s);

// conv3d_s2_split.hip: conv_1_0 (32 -> 16, 3x3x3, stride 2, padding pad) on an output region, split-fp16
// MFMA; x channel-quad fp32, wfrag [27][2][64][8] fp16 (mvs_conv3d_s2_split_weights), y channels-last
// region [B][on0][on1][on2][16]
int launch_conv_s2_split(const void* x, bool presplit, const void* wfrag, int w_exp, const uint32_t* absmax, float* y, int B,
                         const int* n, const int* o0, const int* on, const int* pad, const float* bn_scale,
                         const float* bn_shift, const float* bn_mean, hipStream_t s);

// conv2d_narrow.hip: bias-free Conv2d of the encoder / refinement (padding k/2), NCHW fp32, weights
// wt[c_in][k][k][c_out], optional eval BN + ReLU epilogue; MVS_ERR_INVALID_ARGUMENT for a shape
// without an instantiation
int launch_conv2d_narrow(const float* in, const float* wt, float* out, int N, int Cin, int Cout, int H, int W,
                         int K, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                         uint32_t* y_bound, hipStream_t s);

// conv2d_split.hip: the same convolutions (8..32 input channels) on the f16 matrix cores with split
// operands; x scaled by its bound words, y's bound words raised; weight fragments from
// mvs_conv2d_split_weights (conv2d_split_kblocks K-32 blocks)
int conv2d_split_kblocks(int c_in, int k);
int launch_conv2d_split(const float* x, const void* wfrag, int w_exp, float* y, int N, int Cin, int Cout, int H,
                        int W, int K, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                        const uint32_t* x_bound, uint32_t* y_bound, hipStream_t s);

// deconv3d_region.hip: stride-2 kernel-3 ConvTranspose3d (Cout 8) from a region tensor to the full
// volume, optional fused BN(eval)+ReLU and residual add
// (layout 1: x and x2 are channels-last [B][rd][rh][rw][Cin]; 0: NCDHW, weight [Cin][8][27]; 2: NCDHW,
// tap-major weight [Cin][27][8]; x2 (nullable) is added to x)
void launch_deconv3d_k3s2(const float* x, const float* x2, int layout, int B, int Cin, int rd,
                          int rh, int rw, int x0d, int x0h, int x0w, const float* weight, int D, int H,
                          int W, int pd, int ph, int pw, const float* bn_scale, const float* bn_shift,
                          const float* bn_mean, const float* residual, float* y, hipStream_t s);

// conv3d_region.hip: region convolutions of the regulariser on the fp32 MFMA (mode 0 = stride 1,
// 1 = stride 2 from the full NCDHW volume, 2 = transposed stride 2), channels-last region tensors,
// optional fused eval BN + ReLU, output channels-last or (out_cf) channels-first; in_c4 (S2): the
// volume is channel-quad, fp32 (1), bf16 (2) or the split cost volume (3, with its bound words absmax);
// MVS_ERR_INVALID_ARGUMENT for an unsupported (mode, CI, CO)
int launch_conv3d_region(int mode, bool out_cf, int in_c4, const float* x, const float* x2, const float* w,
                         float* y, int B, int CI, int CO, const int* n, const int* o0, const int* on, const int* i0,
                         const int* in,
                         const int* pad, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                         hipStream_t s, const uint32_t* absmax = nullptr, uint32_t* y_bound = nullptr,
                         bool per_lane = false, const int* st0 = nullptr, const int* stn = nullptr,
                         bool s2_lds = false);
// conv_0_0 (+ BN_0 + ReLU, whole volume) and conv_1_0 (+ BN_1 + ReLU, on its region o0 / on, channels-last)
// from the fp32 channel-quad cost volume, one fused kernel (conv3d_narrow.hip)
void launch_conv_head_fp32(const float* cv4, int B, int D, int H, int W, const float* w0wz, const float* bn0_sc,
                           const float* bn0_sh, const float* bn0_mu, const float* w1, const float* w1p,
                           const float* bn1_sc, const float* bn1_sh, const float* bn1_mu, const int* pad,
                           const int* o0, const int* on, float* y0, float* y1, hipStream_t s,
                           hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// the S1 / T2 region convolutions on split-fp16 MFMA (conv3d_region_split.hip); K-32 weight blocks
// channel_ops.hip: train-mode BatchNorm parameters (+ running statistics) from the batch sums
void launch_bn_train_params(const double* sums, int C, double count, const double* bu, const double* bcnt, int Cp,
                            int ncls, const float* prev, const float* w, const float* bias, float* rmean, float* rvar,
                            long long* nbt, double momentum, double eps, float* params, hipStream_t s);

int conv3d_region_split_kblocks(int c_in);
int launch_conv3d_region_split(int mode, bool out_cf, const float* x, const float* x2, const void* wfrag, int w_exp,
                               float* y, int B, int CI, int CO, const int* n, const int* o0, const int* on,
                               const int* i0, const int* in, const int* pad, const float* bn_scale,
                               const float* bn_shift, const float* bn_mean, const uint32_t* x_bound,
                               const uint32_t* x2_bound, uint32_t* y_bound, hipStream_t s, bool per_lane = false,
                               const float* y_addend = nullptr, const int* store_origin = nullptr,
                               const int* store_size = nullptr, double* stats = nullptr, float* y_mid = nullptr,
                               float* y_high = nullptr, const float* in_bn = nullptr);
// workgroups (= float64 sum slots) of the launch launch_conv3d_region_split makes for these arguments
long conv3d_region_split_slots(int mode, int B, int CI, int CO, const int* on, bool per_lane, bool has_x2,
                               bool in_bn = false);

// channel_ops.hip: train-mode BatchNorm pieces -- per-channel float64 sums into
// stats[slot][2][C] (64 slots) and y = relu(BN(x)) [+ relu(BN'(r))], channels-last or NCDHW
// slots (workgroups) of launch_channel_stats; stats is [slots][2][C], every entry written once
size_t channel_stats_slots(bool channels_last, int B, int C, size_t voxels);
void launch_channel_stats(const float* x, bool channels_last, int B, int C, size_t voxels, double* stats,
                          hipStream_t s);
void launch_bn_relu(const float* x, bool channels_last, int B, int C, size_t voxels, const float* sc,
                    const float* sh, const float* mu, const float* r, const float* rsc, const float* rsh,
                    const float* rmu, float* y, uint32_t* y_bound, hipStream_t s);

// dtu_input.hip: data.py:206-210 image normalisation (uint8 HWC -> fp32 NCHW), data.py:300-301
// depth thresholds
void launch_normalize_images(const uint8_t* rgb, int n, uint32_t hw, const float* mean3,
                             const float* std3, float* out, hipStream_t s);
void launch_depth_threshold(const float* depth, size_t n, float lo, float hi, float* out,
                            hipStream_t s);

}  // namespace mvs
