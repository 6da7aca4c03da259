/*
 * mvs_cost_volume.h -- C ABI of the MI355X (gfx950) MVSNet cost-volume path.
 *
 * Drop-in boundary for bcollico/Deep-Multiview-Depth-Estimation's hot path (SURVEY.md §8 b).
 * The reference boundary is three plain Python functions; each entry point below replaces one
 * of them (or a fusion of them) and is bound from Python by ctypes in
 * deep-multiview-depth-estimation_amd/mvs_amd/_lib.py (binding stub: INTEGRATION.md).
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer (HBM) except where noted; fp32 unless noted;
 *   - tensors are dense row-major (NCHW / NCDHW) exactly as the reference lays them out;
 *   - the callee allocates nothing: outputs and workspaces are caller-provided;
 *   - no global mutable state: re-entrant per stream, graph-capturable (no sync, no malloc);
 *   - `stream` is a hipStream_t (NULL = legacy default stream);
 *   - return MVS_OK (0) or a negative MVS_ERR_* code; mvs_status_string() names it.
 *
 * Shapes: B batch, V views per sample (reference view first, included in the variance),
 *         N = B*V images, C channels, h x w feature map, D planes in this call (a depth shard
 *         [d_begin, d_begin + d_count) of the full hypothesis set), plane k has depth
 *         d_min[i mod B] + d_scale * d_int[i mod B] * k for image i (homography.py:24-26 tiling).
 */
#ifndef MVS_COST_VOLUME_H
#define MVS_COST_VOLUME_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVS_ABI_VERSION 24

#define MVS_OK 0
#define MVS_ERR_INVALID_ARGUMENT (-1)  /* null pointer, non-positive or unsupported size   */
#define MVS_ERR_UNSUPPORTED_VIEWS (-2) /* n_views outside [1, MVS_MAX_VIEWS]               */
#define MVS_ERR_TOO_LARGE (-3)         /* a tensor exceeds the kernel's 32-bit index space */
#define MVS_ERR_HIP (-4)               /* a HIP launch/runtime error of THIS call (the thread's HIP
                                        last-error slot is cleared on entry, then read after the
                                        launches: an error pending from an earlier call is not
                                        reported as this call's, nor can it mask this call's)  */

#define MVS_MAX_VIEWS 16

/* ABI version of the loaded library (MVS_ABI_VERSION at build time). */
int mvs_abi_version(void);

/* Static string for a status code. */
const char* mvs_status_string(int status);

/* Bytes of the per-(image, plane) sampling workspace for n_images x d_count planes. */
size_t mvs_sampling_workspace_bytes(int n_images, int d_count);

/*
 * Per-(image, plane) sampling matrices: the 3x3 map from kornia-normalised reference
 * coordinates to normalised source coordinates, G = inv(Nrm H Nrm^-1) with
 * H = K_i R_i (I - (C_i - C_r) n_r^T / d) R_r^T K_r^-1   (homography.py:40-75, kornia
 * normalize_homography + inverse).  Computed in fp64, stored fp32 as sampling[N][d_count][9].
 *   K, R: [N][3][3]; T: [N][3]; d_min, d_int: [B].
 * Replaces homography.py:40-75 (the H_i tensor) + kornia's per-plane matrix setup.
 */
int mvs_plane_sampling(const float* K, const float* R, const float* T,
                       const float* d_min, const float* d_int,
                       int batch_size, int n_views, int h, int w,
                       int d_begin, int d_count, float d_scale,
                       float* sampling, void* stream);

/*
 * Bytes of the workspace mvs_cost_volume_fwd needs: the sampling matrices (first
 * mvs_sampling_workspace_bytes(N, d_count) bytes, rounded up to 256) followed by a copy of the
 * features packed channel-quad-last ([N][ceil(C/4)][h][w][4], zero-padded channels).
 */
size_t mvs_cost_volume_workspace_bytes(int batch_size, int n_views, int channels, int h, int w,
                                       int d_count);

/*
 * FUSED warp + variance: cv[B][C][d_count][h][w] from feat[N][C][h][w].
 * Replaces homography.py:6-92 + costvolume.py:3-16 (model.py:177-181) in one pass; the
 * warped N x C x D x h x w volume is never materialised.  `workspace` must hold
 * mvs_cost_volume_workspace_bytes(...) bytes; on return its first part holds the sampling
 * matrices (reused by mvs_cost_volume_bwd).
 */
int mvs_cost_volume_fwd(const float* feat, const float* K, const float* R, const float* T,
                        const float* d_min, const float* d_int,
                        int batch_size, int n_views, int channels, int h, int w,
                        int d_begin, int d_count, float d_scale,
                        float* workspace, float* cv_out, void* stream);

/*
 * mvs_cost_volume_fwd with live timing of its main fused kernel: main_begin_event and
 * main_end_event (hipEvent_t, either may be NULL) are recorded on `stream` immediately before
 * and after that kernel's launch (the prologue kernel -- sampling matrices, packing and
 * reference resampling in one launch -- runs before main_begin_event).  Used by bench.py for the
 * roofline's per-launch duration.
 */
int mvs_cost_volume_fwd_timed(const float* feat, const float* K, const float* R, const float* T,
                              const float* d_min, const float* d_int,
                              int batch_size, int n_views, int channels, int h, int w,
                              int d_begin, int d_count, float d_scale,
                              float* workspace, float* cv_out, void* stream,
                              void* main_begin_event, void* main_end_event);

/*
 * mvs_cost_volume_fwd with a bf16 cost volume (reduced-precision cv, opt-in;
 * halves the kernel's dominant write).  cv_out is [B][C][d_count][h][w] bf16 (uint16 storage):
 * the fp32 variance of mvs_cost_volume_fwd rounded to nearest-even, bit-identical to
 * torch's .to(torch.bfloat16) of that fp32 result.  2 <= n_views <= 8 (else
 * MVS_ERR_UNSUPPORTED_VIEWS) or n_views == 1 (zeros).  Same workspace contract.
 */
int mvs_cost_volume_fwd_bf16(const float* feat, const float* K, const float* R, const float* T,
                             const float* d_min, const float* d_int,
                             int batch_size, int n_views, int channels, int h, int w,
                             int d_begin, int d_count, float d_scale,
                             float* workspace, void* cv_out, void* stream);

/*
 * mvs_cost_volume_fwd writing the channel-quad layout cv_out[B][ceil(C/4)][d_count][h][w][4] (fp32,
 * channel 4q + j in component j, padded channels 0; 16-byte aligned): the same values, one 16-byte
 * store per (pixel, plane, 4 channels).  The layout MVSNet.forward's inference path hands to the
 * regulariser's HIP layers (mvs_conv3d_k3_fwd / mvs_conv3d_region_fwd with c4 input), which read 4
 * channels of a voxel per load.  Events as mvs_cost_volume_fwd_timed (either may be NULL).
 * 2 <= n_views <= 8 (else MVS_ERR_UNSUPPORTED_VIEWS) or n_views == 1 (zeros).
 */
int mvs_cost_volume_fwd_c4(const float* feat, const float* K, const float* R, const float* T,
                           const float* d_min, const float* d_int,
                           int batch_size, int n_views, int channels, int h, int w,
                           int d_begin, int d_count, float d_scale,
                           float* workspace, float* cv_out, void* stream,
                           void* main_begin_event, void* main_end_event);

/*
 * mvs_cost_volume_fwd_c4 that also records a bound for the split-fp16 consumers
 * (mvs_conv3d_k3_split_fwd): feat_absmax (8 uint32 words, DEVICE, 4-byte aligned) receives the
 * maximum of the |feat| bit patterns (NaN sorts above Inf above every finite value) in all 8 words:
 * the prologue's packing workgroups write per-workgroup partial maxima into the workspace and one
 * 1-workgroup kernel folds them (no memset, no atomics).  A variance over views is at most the largest squared sample, and a
 * bilinear sample (zero padding) at most max|feat|, so every element of cv_out is <= B^2 with
 * B = the float of the largest of the 8 words.  Otherwise as mvs_cost_volume_fwd_c4.
 */
int mvs_cost_volume_fwd_c4_absmax(const float* feat, const float* K, const float* R, const float* T,
                                  const float* d_min, const float* d_int,
                                  int batch_size, int n_views, int channels, int h, int w,
                                  int d_begin, int d_count, float d_scale,
                                  float* workspace, float* cv_out, void* stream,
                                  void* main_begin_event, void* main_end_event, unsigned* feat_absmax);

/*
 * mvs_cost_volume_fwd_c4_absmax writing the SPLIT cost volume: the channel-quad layout with each
 * 16-byte element {hi(c0..c3), lo(c0..c3)} fp16, hi = fp16(v 2^e), lo = fp16(v 2^e - hi) (nearest),
 * e = 14 - 2 exponent(B) with B = max of the feat_absmax words (clamped to [-120, 120]; 0 when B is 0,
 * Inf or NaN) -- the operands of the split-fp16 consumers (MVS_CONV_IN_SPLIT), which then convert
 * nothing.  hi + lo = v 2^e to 2^-22 relative.  feat_absmax required; otherwise as
 * mvs_cost_volume_fwd_c4_absmax.
 */
int mvs_cost_volume_fwd_c4_split(const float* feat, const float* K, const float* R, const float* T,
                                 const float* d_min, const float* d_int,
                                 int batch_size, int n_views, int channels, int h, int w,
                                 int d_begin, int d_count, float d_scale,
                                 float* workspace, void* cv_out, void* stream,
                                 void* main_begin_event, void* main_end_event, unsigned* feat_absmax);

/*
 * mvs_cost_volume_fwd_c4 with bf16 storage (SURVEY.md §8 f3 reduced-precision cost volume, opt-in):
 * cv_out[B][ceil(C/4)][d_count][h][w][4] bf16 (uint16 storage, 8-byte aligned), each element the fp32
 * variance of mvs_cost_volume_fwd rounded to nearest-even (bit-identical to torch's .to(torch.bfloat16)
 * of it); one 8-byte store per (pixel, plane, 4 channels), half the bytes of the fp32 layout.  Read by
 * mvs_conv3d_k3_fwd / mvs_conv3d_region_fwd with MVS_CONV_IN_C4 | MVS_CONV_IN_BF16, which widen it to
 * fp32 on load (exact) and compute in fp32.  2 <= n_views <= 8 or n_views == 1 (zeros).
 */
int mvs_cost_volume_fwd_c4_bf16(const float* feat, const float* K, const float* R, const float* T,
                                const float* d_min, const float* d_int,
                                int batch_size, int n_views, int channels, int h, int w,
                                int d_begin, int d_count, float d_scale,
                                float* workspace, void* cv_out, void* stream,
                                void* main_begin_event, void* main_end_event);

/*
 * Warp only (API-compatible homography_warping, homography.py:6-92):
 * warped[N][C][d_count][h][w].  Same workspace contract as mvs_cost_volume_fwd.
 */
int mvs_homography_warp_fwd(const float* feat, const float* K, const float* R, const float* T,
                            const float* d_min, const float* d_int,
                            int batch_size, int n_views, int channels, int h, int w,
                            int d_begin, int d_count, float d_scale,
                            float* workspace, float* warped_out, void* stream);

/*
 * Variance over views of an already-warped volume (costvolume.py:3-16):
 * warped[B*V][C][D][h][w] -> cv[B][C][D][h][w].
 */
int mvs_assemble_cost_volume_fwd(const float* warped, int batch_size, int n_views,
                                 int channels, int d, int h, int w, float* cv_out, void* stream);

/* mvs_cost_volume_bwd flags */
#define MVS_BWD_DETERMINISTIC 1

/* Bytes of the workspace mvs_cost_volume_bwd needs with these flags: three scalars, the reference
 * view's per-plane-group partial sums, and (flags = MVS_BWD_DETERMINISTIC only) 64-bit accumulators
 * for every feature element.  0 for invalid arguments or unknown flags. */
size_t mvs_cost_volume_bwd_workspace_bytes(int batch_size, int n_views, int channels, int h, int w,
                                           int d_count, int flags);

/*
 * Backward of the fused op w.r.t. the features (autograd of costvolume.py:14 + grid_sample,
 * exercised by train.py:103): grad_feat[N][C][h][w] is OVERWRITTEN with d<cv, grad_cv>/d feat.
 * `workspace` is the forward call's workspace (same geometry, not modified since): its sampling
 * matrices, packed features and resampled reference views are reused.  `bwd_workspace` holds
 * mvs_cost_volume_bwd_workspace_bytes(..., flags) bytes for the same flags.
 * flags = 0: per-tile partial sums are accumulated in fp64 on chip and added to grad_feat with
 *   fp32 atomics -- the summation order (and so the last bits) may vary between runs, like
 *   torch's grid_sample backward on GPU.
 * flags = MVS_BWD_DETERMINISTIC: 64-bit fixed point throughout (integer adds are associative),
 *   so the result is bit-identical across runs whatever the scheduling; resolution
 *   2^-61 * d_count*h*w*8*max|grad_cv|*max|feat|/n_views (about 1e-12 of the largest possible
 *   contribution at BASELINE cfg 2); one extra pass reads grad_cv for its maximum.
 *   A NaN or Inf anywhere in grad_cv or feat makes every grad_feat element NaN in this mode (fixed
 *   point cannot carry them; the default mode propagates them through the taps they reach).
 */
int mvs_cost_volume_bwd(const float* feat, const float* workspace, const float* grad_cv,
                        int batch_size, int n_views, int channels, int h, int w, int d_count,
                        int flags, void* bwd_workspace, float* grad_feat, void* stream);

/*
 * Soft-argmin with the reference's permutation-indexed mask (depthmap.py:4-22):
 * depth[b][0][y][x] = sum_r d[b][r] P[b][0][r][y][x] m_r / sum_r P m_r, with
 * m_r = (argsort_desc(P)[r] < n_est), ties broken by ascending plane index.
 *   prob: [B][1][D][h][w]; d_batch: [B][D]; depth_out: [B][1][h][w].
 */
int mvs_extract_depth_map_fwd(const float* prob, const float* d_batch, int batch_size, int d,
                              int h, int w, int n_est, float* depth_out, void* stream);

/*
 * DTU input transforms, the callers on the input side of the path.
 *
 * Image normalisation of data.py:206-210 (transforms.PILToTensor -> ConvertImageDtype(float) ->
 * Normalize(mean, std), applied per image in DtuTrainDataset.__getitem__, data.py:286-291):
 *   out[n][c][y][x] = (rgb[n][y][x][c] / 255 - mean[c]) / std_dev[c], fp32, rounded step by step
 *   exactly as torch's CPU ops (bit-identical).
 *   rgb: [n_images][h][w][3] uint8 (decoded pixels as PIL gives them), DEVICE, 4-byte aligned;
 *   mean, std_dev: 3 floats each, HOST pointers (read at launch); out: [n_images][3][h][w] fp32,
 *   DEVICE, 16-byte aligned.
 */
int mvs_normalize_images(const unsigned char* rgb, int n_images, int h, int w, const float* mean,
                         const float* std_dev, float* out, void* stream);

/*
 * Ground-truth depth clamp of data.py:300-301 (cv2.threshold THRESH_TOZERO at lo = 0, then
 * THRESH_TOZERO_INV at hi = 1000): v = x > lo ? x : 0; out = v > hi ? 0 : v.  n floats, DEVICE,
 * 16-byte aligned; out may alias depth.
 */
int mvs_depth_threshold(const float* depth, size_t n, float lo, float hi, float* out, void* stream);

/* input-layout flag of mvs_conv3d_k3_fwd / mvs_conv3d_region_fwd (MVS_CONV_S2): the volume is
 * channel-quad x[batch][c_in/4][D][H][W][4], the layout of mvs_cost_volume_fwd_c4 */
#define MVS_CONV_IN_C4 2
/* with MVS_CONV_IN_C4: the channel-quad volume is bf16 (mvs_cost_volume_fwd_c4_bf16, 8-byte aligned),
 * widened to fp32 on load (exact); the arithmetic is the fp32 path's, bit for bit */
#define MVS_CONV_IN_BF16 8
/* flag of mvs_conv3d_k3_fwd (c_out = 8): Winograd F(2,3) along depth; the weight is then the
 * transformed wu[c_in][3][3][4][8]: per (c_in, ky, kx, c_out) the depth taps g0..g2 become
 * (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2) (formed in float64, rounded once) */
#define MVS_CONV_WINO_Z 4
/* input flag of mvs_conv3d_k3_split_fwd / mvs_conv3d_s2_split_fwd / mvs_conv3d_region_fwd (MVS_CONV_S2):
 * the volume is the split cost volume of mvs_cost_volume_fwd_c4_split (the channel-quad layout, each
 * 16-byte element the fp16 hi / lo parts of 4 values scaled by 2^e, e from its bound words) */
#define MVS_CONV_IN_SPLIT 16

/* Regulariser layers conv_0_0 (32 -> 8) and conv_out (8 -> 1) of CostVolumeReg (model.py:77,96 /
 * forward at model.py:101,123): nn.Conv3d(c_in, c_out, 3, stride=1, padding=1, bias=False) over
 * x[batch][c_in][d][h][w] fp32 (flags = MVS_CONV_IN_C4: the channel-quad x[batch][c_in/4][d][h][w][4]
 * of mvs_cost_volume_fwd_c4, 16-byte aligned) into y[batch][c_out][d][h][w], with the weight TRANSPOSED to
 * weight[c_in][3][3][3][c_out] (nn.Conv3d's weight.permute(1, 2, 3, 4, 0): pairs of output channels
 * are adjacent, one 8-byte scalar load feeds a packed fp32 FMA).
 * c_out must be 1 or 8 (MVS_ERR_INVALID_ARGUMENT otherwise); d*h*w < 2^31.  Optional epilogue
 * (all three BN pointers, c_out floats each, or none): y = max((y - bn_mean) * bn_scale + bn_shift,
 * 0), the eval BN + ReLU that follows conv_0_0 (model.py:101; bn_scale = gamma / sqrt(var + eps),
 * bn_shift = beta).  Replaces the MIOpen convolution behind torch.nn.Conv3d.forward for these two
 * layers in eval-mode inference; same products per output, fp32 summation order differs.
 * x2, in_bn (both or neither; c_out 1, flags 0, no BN epilogue): train mode's conv_out input
 * relu((x - m_a) s_a + h_a) + relu((x2 - m_b) s_b + h_b) per channel formed on load (model.py:121-123,
 * `relu(BN_0(deconv_1_0)) + y0` with y0 the raw conv_0_0 output), in_bn DEVICE fp32 [6][c_in] = (s_a,
 * h_a, m_a, s_b, h_b, m_b); the zero padding stays zero. */
int mvs_conv3d_k3_fwd(const float* x, int flags, const float* weight, float* y, int batch, int c_in,
                      int c_out, int d, int h, int w, const float* bn_scale, const float* bn_shift,
                      const float* bn_mean, const float* x2, const float* in_bn, void* stream);

/* Weight gradient of a narrow full-volume Conv3d(c_in, c_out, 3, padding=1, bias=False) under autograd
 * (train.py:103's loss.backward through model.py:101 conv_0_0 and model.py:124 conv_out; csrc/conv3d_wgrad.hip):
 *   dw[c_out][c_in][3][3][3] (nn.Conv3d's weight layout) = sum over the batch and the voxels of
 *   gy[b][co][v] * x[b][ci][v + tap - 1] (zero padding), fp32 products and sums on the f32-input matrix
 *   cores, reduced in a fixed order (bit-reproducible).
 *   x[batch][c_in][d][h][w], gy[batch][c_out][d][h][w] fp32 NCDHW; (c_in, c_out) in {(32, 8), (16, 8),
 *   (8, 8), (8, 1)}, else MVS_ERR_INVALID_ARGUMENT; d*h*w < 2^31.
 *   workspace: DEVICE, mvs_conv3d_k3_wgrad_workspace_bytes(batch, c_in, d, h, w) bytes (the
 *   workgroups' partial blocks).  Replaces the weight half of torch's Conv3d backward (MIOpen's naive
 *   solver for these shapes; per-tap GEMMs in mvs_amd/tap_gemm.py). */
size_t mvs_conv3d_k3_wgrad_workspace_bytes(int batch, int c_in, int d, int h, int w);
int mvs_conv3d_k3_wgrad(const float* x, const float* gy, int batch, int c_in, int c_out, int d, int h, int w,
                        float* dw, void* workspace, void* stream);

/* conv_0_0 (model.py:77, 101: nn.Conv3d(32, 8, 3, padding=1, bias=False) + optional eval BN_0 + ReLU)
 * on the f16 matrix cores with split operands (csrc/conv3d_split.hip): every fp32 operand is scaled by
 * a power of two and carried as fp16 hi + lo parts, the four partial products of each term are exact
 * in fp32 and accumulated in fp32, so the result has fp32-level error.
 *   x: the channel-quad cost volume x[batch][8][d][h][w][4] fp32 of mvs_cost_volume_fwd_c4(_absmax)
 *      (flags 0), or the split cost volume of mvs_cost_volume_fwd_c4_split (flags MVS_CONV_IN_SPLIT:
 *      read as the kernel's own operands, no conversion), 16-byte aligned; x_absmax: its 8 bound words
 *      (every |x| <= B^2, see mvs_cost_volume_fwd_c4_absmax), DEVICE, required with
 *      MVS_CONV_IN_SPLIT, else NULL when every |x| < 2^15 is known (unscaled);
 *   weight_frag / weight_exp: from mvs_conv3d_split_weights (copied to the device, 16-byte aligned);
 *   y[batch][8][d][h][w] fp32; BN pointers as mvs_conv3d_k3_fwd (8 floats each, all or none).
 * 128*d*h*w <= 2^32 - 16 (one sample's volume bytes).  Replaces the Conv3d behind model.py:101's
 * conv_0_0 in eval inference. */
/* conv_0_0 + BN_0 + ReLU (model.py:101) and conv_1_0 + BN_1 + ReLU (model.py:103) of a MATERIALISED
 * split cost volume in ONE pass over it (the split volume of mvs_cost_volume_fwd_c4_split: read once
 * instead of once per layer; csrc/cv_head.hip's MFMA code fed by plain plane loads).
 * Bit-identical to mvs_conv3d_k3_split_fwd + mvs_conv3d_s2_split_fwd on the same volume.
 *   scv: [batch][8][d_count][h][w] x 16 B (DEVICE, 16-byte aligned), x_absmax its bound words;
 *   w0_frag / w0_exp, bn0_*, w1_frag / w1_exp, bn1_*, pad, y1_origin, y1_size, y0, y1: as
 *   mvs_cost_volume_head_fwd (d_count even, every pad odd);
 *   y1_bound: NULL, or MVS_BOUND_WORDS words (DEVICE, zeroed by the caller) raised to max|y1| (the
 *   bound words mvs_conv3d_region_split_fwd scales its input by).
 * 128 * d_count * h * w <= 2^32 - 16.  Events (either may be NULL) are recorded around the kernel. */
int mvs_split_head_fwd(const void* scv, const unsigned* x_absmax, int batch, int d_count, int h, int w,
                       const void* w0_frag, int w0_exp, const float* bn0_scale, const float* bn0_shift,
                       const float* bn0_mean, const void* w1_frag, int w1_exp, const float* bn1_scale,
                       const float* bn1_shift, const float* bn1_mean, const int* pad, const int* y1_origin,
                       const int* y1_size, float* y0, float* y1, unsigned* y1_bound, void* stream,
                       void* main_begin_event, void* main_end_event);

int mvs_conv3d_k3_split_fwd(const void* x, int flags, const void* weight_frag, int weight_exp,
                            const unsigned* x_absmax, float* y, int batch, int d, int h, int w,
                            const float* bn_scale, const float* bn_shift, const float* bn_mean, void* stream);

/* HOST function (no device work): the fp16 MFMA operand fragments of conv_0_0's weight for
 * mvs_conv3d_k3_split_fwd.  weight: nn.Conv3d layout [8][32][3][3][3] fp32, HOST, finite (else
 * MVS_ERR_INVALID_ARGUMENT); frag: HOST, 27*64*8 uint16 (fp16 bits); *weight_exp = ew with
 * max|w| * 2^ew < 2^14.  frag[tap][lane][j] (tap = (kz*3 + ky)*3 + kx): lane (c = lane & 15,
 * g = lane >> 4) holds input channel 8g + j of column c: c < 8 the hi part of output channel c,
 * c >= 8 the lo part of channel c - 8, where hi = fp16(w 2^ew), lo = fp16(w 2^ew - hi), nearest. */
int mvs_conv3d_split_weights(const float* weight, unsigned short* frag, int* weight_exp);

/* conv_1_0 (model.py:78, 103: nn.Conv3d(32, 16, 3, stride=2, padding=pad, bias=False) + optional eval
 * BN_1 + ReLU) over the channel-quad cost volume on the output region [out_origin, out_origin +
 * out_size) per dim (forward_live's halo(B)), f16 matrix cores with split operands
 * (csrc/conv3d_s2_split.hip; three partial products x_hi w_hi + x_hi w_lo + x_lo w_hi, fp32 accumulation).
 *   x: x[batch][8][dims[0]][dims[1]][dims[2]][4] fp32 (mvs_cost_volume_fwd_c4_absmax; flags 0) or the
 *   split cost volume (mvs_cost_volume_fwd_c4_split; flags MVS_CONV_IN_SPLIT), 16-byte aligned;
 *   x_absmax: its bound words (required with MVS_CONV_IN_SPLIT; else NULL: unscaled, every |x| < 2^15
 *   known); weight_frag / weight_exp:
 *   mvs_conv3d_s2_split_weights (copied to the device); y: channels-last region
 *   y[batch][out_size[0]][out_size[1]][out_size[2]][16] fp32; BN pointers 16 floats each, all or none.
 * 128 * dims[0]*dims[1]*dims[2] <= 2^32 - 16.  Replaces model.py:103's conv_1_0 in eval inference. */
int mvs_conv3d_s2_split_fwd(const void* x, int flags, const void* weight_frag, int weight_exp,
                            const unsigned* x_absmax, float* y, int batch, const int* dims,
                            const int* out_origin, const int* out_size, const int* pad, const float* bn_scale,
                            const float* bn_shift, const float* bn_mean, void* stream);

/* HOST function: the fp16 MFMA operand fragments of conv_1_0's weight for mvs_conv3d_s2_split_fwd.
 * weight [16][32][3][3][3] fp32 HOST, finite; frag HOST 27*2*64*8 uint16: frag[tap][part][lane][j] =
 * part (0 hi, 1 lo) of w[c = lane & 15][8 (lane >> 4) + j][tap] * 2^ew, *weight_exp = ew (max|w| 2^ew
 * < 2^14). */
int mvs_conv3d_s2_split_weights(const float* weight, unsigned short* frag, int* weight_exp);

/* The cost volume CONSUMED WHERE IT IS FORMED (replaces model.py:177-181 + 101-103 in
 * eval inference): homography_warping + assemble_cost_volume (homography.py:6-92, costvolume.py:3-16)
 * fused with the regulariser's two full-volume readers, conv_0_0 (model.py:101) and conv_1_0
 * (model.py:103), so the B x C x D x h x w volume is never written (csrc/cv_head.hip).
 * One prologue kernel (sampling matrices, pixel-major packed features, reference resampling, bound
 * words) and one fused kernel: per 16 x 4 x 48 tile the variance of every plane is formed on chip,
 * split into fp16 hi / lo parts (mvs_cost_volume_fwd_c4_split's arithmetic: bit-identical operands)
 * and fed to both convolutions on the f16 matrix cores (mvs_conv3d_k3_split_fwd's and
 * mvs_conv3d_s2_split_fwd's arithmetic: bit-identical outputs).
 *   feat, K, R, T, d_min, d_int, batch_size, n_views, h, w, d_begin, d_count, d_scale, workspace: as
 *     mvs_cost_volume_fwd (workspace: mvs_cost_volume_workspace_bytes); channels must be 32,
 *     n_views 2 or 3 (else MVS_ERR_UNSUPPORTED_VIEWS), d_count even;
 *   w0_frag / w0_exp: conv_0_0 (mvs_conv3d_split_weights, DEVICE); bn0_*: BN_0 eval epilogue (8 floats
 *     each, all or none); w1_frag / w1_exp: conv_1_0 (mvs_conv3d_s2_split_weights, DEVICE); bn1_*: 16
 *     floats each, all or none;
 *   pad[3] (HOST, (d, h, w) order): conv_1_0's stride-2 padding, every entry odd (n // 2 + 1 with
 *     n % 4 in {0, 1}, config.py:20);
 *   y1_origin[3], y1_size[3] (HOST): conv_1_0's output region, inside its (n + 2 pad - 3) / 2 + 1 outputs;
 *   scv_lo[3], scv_hi[3] (HOST): a box [lo, hi) of the volume whose split cost volume is also stored
 *     into scv (the input box of the regulariser's conv_2_0 / conv_3_0; scv NULL: nothing stored);
 *   feat_absmax: 8 bound words (DEVICE), written as mvs_cost_volume_fwd_c4_absmax does;
 *   y0: [batch][8][d_count][h][w] fp32 = relu(BN_0(conv_0_0(cv))); y1: channels-last region
 *     [batch][y1_size...][16] fp32 = relu(BN_1(conv_1_0(cv))); scv: the box only,
 *     [batch][8][hi0 - lo0][hi1 - lo1][hi2 - lo2] x 16 B, 16-byte aligned (read back by
 *     mvs_conv3d_region_fwd with in_origin = scv_lo, in_size = scv_hi - scv_lo).
 * 128 * d_count * h * w <= 2^32 - 16.  Events (either may be NULL) are recorded around the fused kernel. */
int mvs_cost_volume_head_fwd(const float* feat, const float* K, const float* R, const float* T,
                             const float* d_min, const float* d_int, int batch_size, int n_views,
                             int channels, int h, int w, int d_begin, int d_count, float d_scale,
                             const void* w0_frag, int w0_exp, const float* bn0_scale, const float* bn0_shift,
                             const float* bn0_mean, const void* w1_frag, int w1_exp, const float* bn1_scale,
                             const float* bn1_shift, const float* bn1_mean, const int* pad,
                             const int* y1_origin, const int* y1_size, const int* scv_lo, const int* scv_hi,
                             float* workspace, unsigned* feat_absmax, float* y0, float* y1, void* scv,
                             void* stream, void* main_begin_event, void* main_end_event);

/* Feature encoder and refinement layers (model.py:22-65 FeatureEncoder, model.py:134-145): nn.Conv2d(
 * c_in, c_out, k, stride, padding=k/2, bias=False) over x[n][c_in][h][w] fp32 into
 * y[n][c_out][ho][wo] (ho = (h + 2(k/2) - k)/stride + 1, likewise wo), with the weight TRANSPOSED to
 * weight[c_in][k][k][c_out] (nn.Conv2d's weight.permute(1, 2, 3, 0)).  Supported (c_in, c_out, k,
 * stride): the reference's layers (3,8,3,1) (8,8,3,1) (8,16,5,2) (16,16,3,1) (16,32,5,2) (32,32,3,1)
 * (4,32,3,1) (32,1,3,1); MVS_ERR_INVALID_ARGUMENT otherwise.  Optional epilogue (all three BN pointers,
 * c_out floats each, or none): y = max((y - bn_mean) * bn_scale + bn_shift, 0), the eval BN + ReLU
 * that follows these convolutions.  Replaces the MIOpen convolution behind torch.nn.Conv2d.forward
 * (and the BatchNorm2d + ReLU after it) in inference; same products, fp32 summation order differs.
 * y_bound: NULL, or MVS_BOUND_WORDS zeroed DEVICE words raised to max|y| (the input scale of a
 * following mvs_conv2d_split_fwd). */
int mvs_conv2d_fwd(const float* x, const float* weight, float* y, int n, int c_in, int c_out, int h, int w,
                   int k, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                   unsigned* y_bound, void* stream);

/* Split-fp16 weight fragments of an nn.Conv2d weight[c_out][c_in][k][k] (HOST fp32, finite) for
 * mvs_conv2d_split_fwd: frag (HOST, kb * parts * 64 * 8 uint16, kb = ceil(k^2 / (32 / c_in)) K-32
 * blocks, parts = 1 for c_out = 8 else 2 c_out / 16) and *weight_exp = ew with max|w| 2^ew < 2^14.
 * K block kb, lane (c = lane & 15, g = lane >> 4), element j: tap t = kb (32 / c_in) + g / (c_in / 8)
 * (zero past k^2), input channel 8 (g % (c_in / 8)) + j.  c_out >= 16: frag[kb][nb][part][lane][j] =
 * part (0: fp16(w 2^ew), 1: fp16(w 2^ew - part 0)) of w[16 nb + c][ci][t]; c_out = 8: frag[kb][lane][j]
 * = part 0 of w[c][ci][t] for c < 8, part 1 of w[c - 8][ci][t] for c >= 8.  c_in in {8, 16, 32},
 * c_out 8 or a multiple of 16. */
int mvs_conv2d_split_weights(const float* weight, int c_in, int c_out, int k, unsigned short* frag, int* weight_exp);

/* mvs_conv2d_fwd's convolutions with 8..32 input channels (FeatureEncoder layers 2-8, the refinement
 * net's 32 -> 32) on the f16 matrix cores with split operands (csrc/conv2d_split.hip): x scaled by
 * 2^ex from its bound words x_bound (DEVICE, required: mvs_conv2d_fwd's / this function's y_bound) and
 * split into fp16 hi + lo, the weights likewise (mvs_conv2d_split_weights: weight_frag DEVICE, 16-byte
 * aligned); per K-32 block x_hi w_hi + x_hi w_lo + x_lo w_hi in fp32 accumulation: fp32-level error,
 * not mvs_conv2d_fwd's bit pattern.  Weight in fragments, otherwise arguments as mvs_conv2d_fwd.
 * Supported (c_in, c_out, k, stride): (8,8,3,1) (8,16,5,2) (16,16,3,1) (16,32,5,2) (32,32,3,1). */
int mvs_conv2d_split_fwd(const float* x, const void* weight_frag, int weight_exp, float* y, int n, int c_in,
                         int c_out, int h, int w, int k, int stride, const float* bn_scale, const float* bn_shift,
                         const float* bn_mean, const unsigned* x_bound, unsigned* y_bound, void* stream);

/* layout flag of mvs_deconv3d_k3s2_fwd: the region input is channels-last x[batch][rd][rh][rw][c_in] */
#define MVS_LAYOUT_CHANNELS_LAST 1
/* flag of mvs_deconv3d_k3s2_fwd (either layout): the weight is tap-major weight[c_in][27][8]
 * (ConvTranspose3d's weight.reshape(c_in, 8, 27).transpose(1, 2)): output-channel pairs adjacent,
 * one 8-byte scalar operand per packed FMA */
#define MVS_DECONV_WEIGHT_TAPS 2

/* Regulariser layer deconv_1_0 (model.py:87, forward at model.py:121): nn.ConvTranspose3d(c_in, 8,
 * 3, stride=2, padding=(pd, ph, pw), output_padding, bias=False) into the full volume
 * y[batch][8][d][h][w], from a REGION input holding the input on [x0, x0 + r) per dim (it must hold
 * every input that reaches [0, n): CostVolumeReg.forward_live): x[batch][c_in][rd][rh][rw], or
 * channels-last x[batch][rd][rh][rw][c_in] with flags = MVS_LAYOUT_CHANNELS_LAST; x2 (nullable, same
 * layout) is added to x on load (model.py:121's `y2 + y1`).  weight[c_in][8][3][3][3]
 * (ConvTranspose layout), c_in <= 64.  Optional epilogue (all three BN pointers or none; residual
 * nullable): y = max((y - bn_mean) * bn_scale + bn_shift, 0) + residual, i.e. model.py:121-123's
 * ReLU(BN_0(.)) and `+ y0` (eval BN: bn_scale = gamma / sqrt(var + eps), bn_shift = beta).
 * Eval-mode inference only. */
int mvs_deconv3d_k3s2_fwd(const float* x, const float* x2, int flags, int batch, int c_in, int c_out,
                          int rd, int rh, int rw, int x0d, int x0h, int x0w, const float* weight, int d,
                          int h, int w, int pd, int ph, int pw, const float* bn_scale,
                          const float* bn_shift, const float* bn_mean, const float* residual, float* y,
                          void* stream);

/* conv_0_0 and conv_1_0 of CostVolumeReg (model.py:101 and :103, each + its eval BatchNorm + ReLU) in exact
 * fp32 from the fp32 channel-quad cost volume cv4 [batch][8][d][h][w][4] (mvs_cost_volume_fwd_c4, 16-byte
 * aligned) in ONE pass over it -- replaces mvs_conv3d_k3_fwd (MVS_CONV_IN_C4 | MVS_CONV_WINO_Z) for
 * conv_0_0 plus mvs_conv3d_region_fwd (MVS_CONV_S2, MVS_CONV_IN_C4) for conv_1_0 on its region, the
 * fp32 eval path's two layers that read the whole volume.  conv_0_0 runs on the fp32 VALU (depth-Winograd
 * F(2,3), w0_wz the transformed weights as mvs_conv3d_k3_fwd takes them) and writes y0 [batch][8][d][h][w];
 * conv_1_0 (32 -> 16, stride 2, padding pad[3], every pad odd) runs on the fp32 matrix cores from the same
 * staged tiles and writes y1 [batch][y1_size...][16] channels-last holding outputs y1_origin + [0, y1_size)
 * (w1 the region weight [27][16][32] of mvs_conv3d_region_fwd, w1_pass the same values as [8][27][16][4]:
 * channel quad, tap, output channel, channel in quad).  BN pointers: 8 / 16 floats each, all three or none
 * per layer.  Same values as the two separate kernels up to fp32 summation order (conv_1_0's channels
 * are summed per quad of the staging, not per 16).  ev0 / ev1: NULL or hipEvent_t recorded on the stream
 * right before / after the fused kernel (the slab launches for the region's unowned windows follow it). */
int mvs_conv_head_fp32_fwd(const float* cv4, int batch, int d, int h, int w, const float* w0_wz,
                           const float* bn0_scale, const float* bn0_shift, const float* bn0_mean, const float* w1,
                           const float* w1_pass, const float* bn1_scale, const float* bn1_shift,
                           const float* bn1_mean, const int* pad, const int* y1_origin, const int* y1_size,
                           float* y0, float* y1, void* stream, void* ev0, void* ev1);

/* mvs_conv3d_region_fwd modes */
#define MVS_CONV_S1 0   /* Conv3d 3x3x3, stride 1, padding 1: region -> region                     */
#define MVS_CONV_S2 1   /* Conv3d 3x3x3, stride 2, padding pad: full NCDHW volume -> region         */
#define MVS_CONV_T2 2   /* ConvTranspose3d 3x3x3, stride 2, padding pad: region (+ x2) -> region   */
/* mvs_conv3d_region_fwd flags */
#define MVS_CONV_OUT_NCDHW 1   /* output region tensor channels-first y[batch][c_out][size...]   */
/* (and MVS_CONV_IN_C4, above: an MVS_CONV_S2 input volume in the channel-quad layout) */

/* The regulariser's region convolutions (CostVolumeReg, model.py:76-95, forward at model.py:101-121,
 * evaluated on their live regions: DESIGN.md §5a) on the fp32 matrix cores, with the following eval
 * BatchNorm + ReLU fused (all three BN pointers, c_out floats each, or none):
 *   y = max((conv(x) - bn_mean) * bn_scale + bn_shift, 0).
 * The volume is dims[3] = (D, H, W); the output is the channels-last region tensor
 * y[batch][out_size[0]][out_size[1]][out_size[2]][c_out] holding voxels out_origin + [0, out_size)
 * (flags = MVS_CONV_OUT_NCDHW: channels-first y[batch][c_out][out_size...]).
 * Input: MVS_CONV_S2 the full cost volume x[batch][c_in][D][H][W] (reads 2 o - pad + t, zero outside
 * the volume) -- or, with in_origin / in_size given, only the box in_origin + [0, in_size) of it,
 * x[batch][c_in][in_size...] (the caller guarantees the box holds every in-volume voxel the outputs
 * read: voxels off the box read zero); MVS_CONV_S1 / MVS_CONV_T2 a channels-last region tensor
 * x[batch][in_size...][c_in] on in_origin + [0, in_size) (S1: o + t - 1; T2: i = (o + pad - t) / 2 for
 * t of o + pad's parity; voxels outside the volume or the input region read zero), plus x2 (same
 * geometry, nullable) added on load.  Weights transposed to weight[27][c_out][c_in] (tap =
 * (kd * 3 + kh) * 3 + kw): nn.Conv3d's weight.permute(2, 3, 4, 0, 1), nn.ConvTranspose3d's
 * weight.permute(2, 3, 4, 1, 0).  Supported (mode, c_in, c_out): S2 (32, 16|32|64), S1 (16, 16),
 * (32, 32), (64, 64), T2 (64, 32), (32, 16); else MVS_ERR_INVALID_ARGUMENT.  dims, origins, sizes and
 * pad are HOST pointers to 3 ints.  flags = MVS_CONV_S2 input MVS_CONV_IN_C4 | MVS_CONV_IN_SPLIT: the split
 * cost volume, re-formed to fp32 on load as (hi + lo) 2^-e (2^-22 of each element), x_absmax its bound
 * words (DEVICE; NULL otherwise).  y_bound: NULL, or MVS_BOUND_WORDS words (DEVICE, zeroed by the
 * caller) raised to max|y| (see mvs_conv3d_region_split_fwd).  Eval-mode inference only; products
 * summed in the order (tap, c_in) -- MIOpen sums them in other orders (fp32 rounding-level differences).
 * MVS_CONV_S1 with c_in = c_out and no x2 runs an LDS-staged kernel (each input voxel loaded once per
 * 16 x 4 x TZ output tile), bit-identical to the per-lane-operand kernel that flags MVS_CONV_PER_LANE
 * (below) selects. */
int mvs_conv3d_region_fwd(int mode, int flags, const float* x, const float* x2, const float* weight, float* y,
                          int batch, int c_in, int c_out, const int* dims, const int* out_origin,
                          const int* out_size, const int* in_origin, const int* in_size,
                          const int* pad, const float* bn_scale, const float* bn_shift,
                          const float* bn_mean, const unsigned* x_absmax, unsigned* y_bound, void* stream);

/* flag of mvs_conv3d_region_split_fwd and mvs_conv3d_region_fwd: run the per-lane-operand kernel even
 * where an LDS-staged kernel applies (the two are bit-identical; tests and A/B timing) */
#define MVS_CONV_PER_LANE 32
/* flag of mvs_conv3d_region_fwd: conv_1_0's shape (MVS_CONV_S2, c_in 32, c_out 16, the whole fp32 volume,
 * channel quads or NCDHW, channels-last output, no store box) on the LDS-staged kernel (csrc/conv3d_s2_lds.hip;
 * the default only with the environment variable MVS_S2_LDS=1: slower inside the eval step) */
#define MVS_CONV_S2_LDS 256

/* Bound words of a region tensor: MVS_BOUND_WORDS uint32 (8 KiB) holding maxima of |v| as fp32 bit
 * patterns (the tensor's bound is their maximum), raised with atomic maxima by the kernel that writes
 * the tensor into words the caller zeroed (64 slots, one per 128-byte line, so the atomics of different
 * waves do not serialise on one line; the other words stay zero). */
#define MVS_BOUND_WORDS 2048

/* HOST function: the split-fp16 MFMA fragments of a region convolution's weight for
 * mvs_conv3d_region_split_fwd.  weight [27][c_out][c_in] fp32 HOST (mvs_conv3d_region_fwd's layout),
 * finite; c_out a multiple of 16, c_in 16 or a multiple of 32; frag HOST, kb * (c_out / 16) * 2 * 64 * 8
 * uint16 with kb = 14 (c_in 16: K blocks of two taps x 16 channels) or 27 * c_in / 32;
 * *weight_exp = ew with max|w| 2^ew < 2^14.  frag[kb][nb][part][lane][j]: lane (c = lane & 15,
 * g = lane >> 4) holds K element 8g + j of output channel 16 nb + c, part 0 = fp16(w 2^ew), part 1 =
 * fp16(w 2^ew - part 0) (nearest). */
int mvs_conv3d_region_split_weights(const float* weight, int c_in, int c_out, unsigned short* frag, int* weight_exp);

/* mvs_conv3d_region_fwd's MVS_CONV_S1 and MVS_CONV_T2 convolutions (conv_k_1, model.py:104-113;
 * deconv_3_0 / deconv_2_0, model.py:117-120) on the f16 matrix cores with split operands
 * (csrc/conv3d_region_split.hip): the input v (x, or x + x2) is scaled by 2^ex -- max(bound(x) +
 * bound(x2)) 2^ex < 2^14 from its bound words -- and split into fp16 hi + lo, the weights likewise
 * (mvs_conv3d_region_split_weights: weight_frag DEVICE, 16-byte aligned, weight_exp); per K-32 block
 * x_hi w_hi + x_hi w_lo + x_lo w_hi in fp32 accumulation, output unscaled by 2^-(ex + ew): fp32-level
 * error.  Geometry, layouts, BN epilogue and flags (MVS_CONV_OUT_NCDHW) as
 * mvs_conv3d_region_fwd; in_origin / in_size required.  x_bound / x2_bound: the inputs' bound words
 * (DEVICE, required: MVS_ERR_INVALID_ARGUMENT when NULL -- unscaled values above 65504 would overflow
 * the fp16 hi part; x2_bound required with x2); y_bound: NULL or the output's bound
 * words (zeroed by the caller).  MVS_CONV_S2 (conv_k_0): flags MVS_CONV_IN_C4 | MVS_CONV_IN_SPLIT, x the
 * split cost volume (mvs_cost_volume_fwd_c4_split; its fp16 parts are the operands, no conversion) or,
 * with in_origin / in_size, a box of it, x_bound its 8 bound words, x2 NULL.  Supported (mode, c_in,
 * c_out): S1 (16, 16), (32, 32), (64, 64), T2 (64, 32), (32, 16), S2 (32, 16 | 32 | 64 | 112).  Inference
 * only (the raw outputs without the BN pointers: train-mode BN's batch statistics).  y_addend: NULL, or a
 * tensor of y's shape and layout added after BN + ReLU (deconv_3_0's output + y2, model.py:119, formed
 * once instead of on every load of deconv_2_0); the bound words then bound the sum.
 * Train-mode BatchNorm (test.py:61): store_origin / store_size (NULL, or a box inside
 * the output region, absolute voxel coordinates): y holds only that box ([batch][size...][c_out] or
 * channels-first), the rest of the region is computed but not stored; stats (NULL, or DEVICE float64,
 * 8-byte aligned, mvs_conv3d_region_split_stats_slots(...) x 2 x c_out): every workgroup writes its
 * slot stats[slot][0 / 1][c] = sum / sum of squares over the WHOLE output region of the stored value
 * (after the epilogue); the caller adds the slots in a fixed order (run-to-run bit-identical batch
 * statistics, as mvs_channel_stats).  MVS_CONV_S2 with c_out = 112 (train mode's conv_1_0, conv_2_0
 * and conv_3_0 over one region, weights concatenated along c_out): y receives channels 0-15, y_mid
 * 16-47 and y_high 48-111, each its own channels-last tensor (one launch reads the volume once for all
 * three; no addend, no MVS_CONV_OUT_NCDHW); NULL otherwise.  in_bn: NULL, or (MVS_CONV_T2 with (c_in,
 * c_out) = (64, 32) or (32, 16): the LDS-staged kernel) DEVICE fp32 [6][c_in], 16-byte aligned = (scale, shift, mean)
 * of x then of x2: the input is relu((x - mean) scale + shift) [+ the same of x2] -- train mode's BN +
 * ReLU passes folded into the staging; x_bound / x2_bound then bound the raw x / x2.  Also MVS_CONV_S1 with
 * c_in = c_out = 16 or 32 (its LDS-staged kernel), x only. */
int mvs_conv3d_region_split_fwd(int mode, int flags, const float* x, const float* x2, const void* weight_frag,
                                int weight_exp, float* y, int batch, int c_in, int c_out, const int* dims,
                                const int* out_origin, const int* out_size, const int* in_origin, const int* in_size,
                                const int* pad, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                                const unsigned* x_bound, const unsigned* x2_bound, unsigned* y_bound,
                                const float* y_addend, const int* store_origin, const int* store_size, double* stats,
                                float* y_mid, float* y_high, const float* in_bn, void* stream);

/* flags of mvs_conv3d_region_split_stats_slots: the call sums two inputs (x2 given); it passes in_bn */
#define MVS_CONV_SUM_INPUT 64
#define MVS_CONV_IN_BN 128
/* Number of float64 sum slots (workgroups) of the mvs_conv3d_region_split_fwd call with this mode,
 * flags (MVS_CONV_PER_LANE, MVS_CONV_SUM_INPUT, MVS_CONV_IN_BN), batch, channels and out_size; < 0 on invalid
 * arguments.  Host-only: no device work. */
long long mvs_conv3d_region_split_stats_slots(int mode, int flags, int batch, int c_in, int c_out,
                                              const int* out_size);

/* Softmax over the depth planes of the regulariser's output (CostVolumeReg.Norm = nn.Softmax(2),
 * model.py:97 / :125): y[b][0][d][p] = exp(x - max_d x) / sum_d exp(x - max_d x) per pixel p, in
 * torch's operation order; x, y [batch][1][d_count][h][w] fp32 (y may alias x). */
int mvs_softmax_depth_fwd(const float* x, int batch, int d_count, int h, int w, float* y, void* stream);

/* The depth planes (homography.py:24-26): out[b][k] = d_min[b] + (d_scale * d_int[b]) * k, k < d_num, each
 * op separately rounded in that order (the torch expression's result, bit for bit); d_min, d_int
 * DEVICE [batch] fp32, out DEVICE [batch][d_num]. */
int mvs_depth_hypotheses_fwd(const float* d_min, const float* d_int, int batch, int d_num, float d_scale, float* out,
                             void* stream);

/* The elementwise steps around the refinement net (model.py:189-205, MVSNet.refine), each one launch,
 * every operation a separately rounded fp32 op in the reference's order (bit-equal to the torch
 * sequence).  d_span = (d_int * d_num) * d_scale per sample; d_min, d_int DEVICE [batch] fp32.
 *   mvs_refine_input_fwd:  out [batch][4][h][w] = cat((initial_depth - d_min) / d_span, ref_img) --
 *                          torch.cat((norm_depth, ref_img), 1), model.py:197-199; initial_depth
 *                          [batch][1][h][w], ref_img [batch][3][h][w] (the down-sampled reference image).
 *   mvs_refine_output_fwd: out [batch][1][h][w] = ((conv + refine_in[:, 0]) * d_span) + d_min --
 *                          the refinement's residual add (model.py:150) and the rescale (model.py:204-205);
 *                          conv [batch][1][h][w] the refinement net's last conv, refine_in the first's input. */
int mvs_refine_input_fwd(const float* initial_depth, const float* d_min, const float* d_int, int batch, int h,
                         int w, int d_num, float d_scale, const float* ref_img, float* out, void* stream);
int mvs_refine_output_fwd(const float* conv, const float* refine_in, const float* d_min, const float* d_int,
                          int batch, int h, int w, int d_num, float d_scale, float* out, void* stream);

/* ---- train-mode BatchNorm of the regulariser (model.py:101-121 with every BatchNorm3d in training
 * mode: test.py:53,61 runs `model.train()` under no_grad; CostVolumeReg.forward_live_train) ---- */
/* Number of partial-sum slots mvs_channel_stats writes for this tensor (0 for invalid arguments). */
size_t mvs_channel_stats_slots(int layout, int batch, int channels, long long voxels);

/* Per-channel batch sums of x in float64, as partial sums: stats[slot][0][c] = a partial sum of x over
 * channel c, stats[slot][1][c] = of x^2, for slot < mvs_channel_stats_slots(...) -- every entry is
 * WRITTEN (no zeroing needed), each partial summed in a fixed order without atomics; the caller adds
 * the slots (in a fixed order: results are then bit-identical run to run).  The inputs of
 * BatchNorm3d's batch mean and biased variance.  layout: MVS_LAYOUT_CHANNELS_LAST
 * (x[batch][voxels][channels], channels / 4 a power of two <= 64, 16-byte aligned) or 0 (NCDHW
 * x[batch][channels][voxels]). */
int mvs_channel_stats(const float* x, int layout, int batch, int channels, long long voxels, double* stats,
                      void* stream);

/* Train-mode BatchNorm parameters from the batch sums (replaces torch.nn.functional.batch_norm's
 * statistics step with training=True, model.py:101-121 under test.py:61): sums (DEVICE float64
 * [2][channels]: sum, sum of squares over count elements; plus, with border_u, the border term of
 * CostVolumeReg.forward_live_train: u_k = sum_i border_u[o][i][k] a_i with the previous BN's constant
 * a_i = relu(-mean_i scale_i + shift_i) from prev_params [3][prev_channels], added as
 * (sum_k u_k border_count[k], sum_k u_k^2 border_count[k])); mean = s1 / count, var = max(s2 / count -
 * mean^2, 0) in float64; running_mean / running_var (NULL: not tracked) updated with momentum and the
 * unbiased variance var count / (count - 1); num_batches_tracked (NULL or int64) += 1; params (DEVICE
 * fp32 [3][channels]) = (weight / sqrt(var + eps), bias, mean).  One launch, one workgroup; with the
 * border term prev_channels <= 256 and channels x classes <= 2048. */
int mvs_bn_train_params(const double* sums, int channels, double count, const double* border_u,
                        const double* border_count, int prev_channels, int classes, const float* prev_params,
                        const float* weight, const float* bias, float* running_mean, float* running_var,
                        long long* num_batches_tracked, double momentum, double eps, float* params, void* stream);

/* y = max((x - mean) * scale + shift, 0) per channel (BatchNorm3d with the batch statistics:
 * scale = gamma / sqrt(var + eps), shift = beta; then ReLU), and, when r is given,
 * + max((r - r_mean) * r_scale + r_shift, 0) (model.py:121-123: relu(BN_0(deconv_1_0)) + y0).
 * Layouts as mvs_channel_stats; y may alias x.  y_bound: NULL or MVS_BOUND_WORDS zeroed words (DEVICE)
 * raised to max y (the scale a split-fp16 region convolution reads y with). */
int mvs_bn_relu(const float* x, int layout, int batch, int channels, long long voxels, const float* scale,
                const float* shift, const float* mean, const float* r, const float* r_scale,
                const float* r_shift, const float* r_mean, float* y, unsigned* y_bound, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MVS_COST_VOLUME_H */
