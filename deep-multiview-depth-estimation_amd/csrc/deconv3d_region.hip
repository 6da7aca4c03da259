// deconv3d_region.hip -- stride-2, kernel-3 ConvTranspose3d of the regulariser's last up-sampling
// (deconv_1_0, 16 -> 8, model.py:87, forward at model.py:121), gather form, with the following
// BatchNorm (eval) + ReLU and the skip add `+ y0` (model.py:121-123) fused into the epilogue.
//
// y[b][co][o] = sum_{ci, k} x[b][ci][i] * W[ci][co][k],  o = 2 i + k - P  (per dim, k = 0..2)
// so output o gathers the inputs i = (o + P - k) / 2 with o + P - k even: 1 or 2 taps per dim.
// x is a REGION tensor: it holds the input only on [x0, x0 + r) per dim -- every input that
// reaches an output in [0, n) (CostVolumeReg.forward_live); inputs outside it reach no output.
// It is NCDHW or channels-last (the MFMA region convs' layout, conv3d_region.hip), optionally the
// sum of two region tensors (model.py:121's `y2 + y1`, added on load).
// Epilogue (optional): z = max((y - mean) * scale + shift, 0) + residual (scale = gamma /
// sqrt(var + eps), shift = beta: eval BN).
//
// One thread = one 2 x 2 x 2 block of output voxels (o = 2m + s, s = 0, 1 per dim) x 8 channels.
// Per dim the block reads the two inputs L = x[m + q + c - 1], U = x[m + q + c] (P = 2q + c) and
//   c = 1:  out(s=0) = L * W1,            out(s=1) = U * W0 + L * W2
//   c = 0:  out(s=0) = U * W0 + L * W2,   out(s=1) = U * W1
// -- the tensor product over the 3 dims is the block's 27 (input, tap) pairs, so a thread does
// exactly the transposed conv's work, no lane diverges, and neighbouring lanes store adjacent
// float2 pairs.  Weights: workgroup-uniform scalar loads feeding the fmas' SGPR operand (NCDHW
// input), broadcast LDS reads of the staged 8 x 27 (padded to 28) per channel (channels-last).
// HBM-bound: the full-size output (+ residual read) dominates.
#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kCout = 8;
// the full-size output and the residual y0 stream through once: non-temporal policy for both
// (cfg 2 deconv_1_0 0.53 -> 0.43 ms alone; profiles/r03/r03z_split_conv_experiments.md)
constexpr int kNtAux = 2;
typedef float f2v_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const f2v_t const_f2v_t;
constexpr int kWRow = 28;   // 27 taps padded to 7 float4

// per dim: (input slot 0 = L, 1 = U, kernel tap k) pairs feeding output s
template <int C>
struct Stencil {
  // n[s]: number of terms for output s; in[s][t], k[s][t]
  static constexpr int n0 = C ? 1 : 2, n1 = C ? 2 : 1;
  static constexpr int in0[2] = {C ? 0 : 1, 0};
  static constexpr int k0[2] = {C ? 1 : 0, 2};
  static constexpr int in1[2] = {C ? 1 : 1, 0};
  static constexpr int k1[2] = {C ? 0 : 1, 2};
};

template <int CD, int CH, int CW, int LM>
__global__ __launch_bounds__(kBlock) void deconv3d_k3s2_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const float* __restrict__ wt, int Cin, int rd,
    int rh, int rw,
    int x0d, int x0h, int x0w, int D, int H, int W, int qd, int qh, int qw,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ mean, const float* __restrict__ residual, float* __restrict__ y,
    int md_n, int mh_n, int mw_n, size_t total, size_t total_in_bytes, size_t out_bytes) {
  constexpr bool CL = LM == 1 || LM == 3;   // channels-last input (LM 3: with tap-major weights)
  constexpr bool WT = LM == 2 || LM == 3;   // tap-major weights wt[ci][27][co]: packed FMAs, SGPR operands
  extern __shared__ float4 wl4[];   // LM 1: [ci][co][7] float4 = W[ci][co][27] padded
  if constexpr (CL && !WT) {
    float* wl = reinterpret_cast<float*>(wl4);
    const int nw = Cin * kCout * kWRow;
    for (int e = (int)threadIdx.x; e < nw; e += kBlock) {
      const int k = e % kWRow, cc = e / kWRow;
      wl[e] = k < 27 ? wt[(size_t)cc * 27 + k] : 0.0f;
    }
    __syncthreads();
  }
  // XCD-contiguous blocks (gridDim.x a multiple of 8): neighbouring output rows share input rows
  const size_t gid = (size_t)xcd_work_id((int)blockIdx.x, (int)gridDim.x) * kBlock + threadIdx.x;
  if (gid >= total) return;
  const int mw = (int)(gid % mw_n);
  size_t t = gid / mw_n;
  const int mh = (int)(t % mh_n);
  t /= mh_n;
  const int md = (int)(t % md_n);
  const int b = (int)(t / md_n);
  // region-relative indices of L (slot 0) and U (slot 1) per dim, and their validity
  const int ld = md + qd + CD - 1 - x0d, lh = mh + qh + CH - 1 - x0h, lw = mw + qw + CW - 1 - x0w;
  bool okd[2], okh[2], okw[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    okd[j] = ld + j >= 0 && ld + j < rd;
    okh[j] = lh + j >= 0 && lh + j < rh;
    okw[j] = lw + j >= 0 && lw + j < rw;
  }
  const size_t rvol = (size_t)rd * rh * rw;
  const float* xb = x + (size_t)b * Cin * rvol;
  const float* xb2 = x2 ? x2 + (size_t)b * Cin * rvol : nullptr;
  using SD = Stencil<CD>;
  using SH = Stencil<CH>;
  using SW = Stencil<CW>;
  float acc[2][2][2][kCout];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int co = 0; co < kCout; ++co) acc[a][c][e][co] = 0.0f;
  // one input channel's 8 voxel values v -> the 27 (input, tap) products of the 2x2x2 block
  auto channel = [&](int ci, const float (&v)[2][2][2]) {
#pragma unroll
    for (int co = 0; co < kCout; ++co) {
      float w[kWRow];
      if constexpr (CL) {   // broadcast LDS reads (4 channels per round keep SGPRs busy)
        const float4* wr = wl4 + (ci * kCout + co) * (kWRow / 4);
#pragma unroll
        for (int q = 0; q < kWRow / 4; ++q) {
          const float4 f = wr[q];
          w[4 * q] = f.x; w[4 * q + 1] = f.y; w[4 * q + 2] = f.z; w[4 * q + 3] = f.w;
        }
      } else {
        // workgroup-uniform scalar loads, the fmas' SGPR operand; the memory clobber keeps the
        // compiler from hoisting every channel's weights at once
        asm volatile("" ::: "memory");
        const float* wr = wt + ((size_t)ci * kCout + co) * 27;
#pragma unroll
        for (int q = 0; q < 27; ++q) w[q] = wr[q];
      }
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
#pragma unroll
        for (int td = 0; td < (sd ? SD::n1 : SD::n0); ++td)
#pragma unroll
          for (int sh = 0; sh < 2; ++sh)
#pragma unroll
            for (int th = 0; th < (sh ? SH::n1 : SH::n0); ++th)
#pragma unroll
              for (int sw = 0; sw < 2; ++sw)
#pragma unroll
                for (int tw = 0; tw < (sw ? SW::n1 : SW::n0); ++tw) {
                  const int id = sd ? SD::in1[td] : SD::in0[td], kd = sd ? SD::k1[td] : SD::k0[td];
                  const int ih = sh ? SH::in1[th] : SH::in0[th], kh = sh ? SH::k1[th] : SH::k0[th];
                  const int iw = sw ? SW::in1[tw] : SW::in0[tw], kw = sw ? SW::k1[tw] : SW::k0[tw];
                  acc[sd][sh][sw][co] = fmaf(v[id][ih][iw], w[kd * 9 + kh * 3 + kw], acc[sd][sh][sw][co]);
                }
    }
  };
  // WT: each of the 27 taps feeds exactly one output voxel of the block from one input voxel (per
  // dim, class 1: k0 -> (s1, U), k1 -> (s0, L), k2 -> (s1, L); class 0: k0 -> (s0, U),
  // k1 -> (s1, U), k2 -> (s0, L)), so a channel is 27 taps x 4 channel pairs of packed FMAs with
  // the pair's weights as one 64-bit scalar operand
  auto channel_pk = [&](int ci, const float (&v)[2][2][2]) {
    constexpr int sD[3] = {CD ? 1 : 0, CD ? 0 : 1, CD ? 1 : 0}, iD[3] = {1, CD ? 0 : 1, 0};
    constexpr int sH[3] = {CH ? 1 : 0, CH ? 0 : 1, CH ? 1 : 0}, iH[3] = {1, CH ? 0 : 1, 0};
    constexpr int sW[3] = {CW ? 1 : 0, CW ? 0 : 1, CW ? 1 : 0}, iW[3] = {1, CW ? 0 : 1, 0};
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        asm volatile("" ::: "memory");   // one (kd, kh) row of weights in SGPRs at a time
        const const_f2v_t* wg =
            (const const_f2v_t*)uniform_ptr(wt + ((size_t)ci * 27 + kd * 9 + kh * 3) * kCout);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float vv = v[iD[kd]][iH[kh]][iW[kw]];
          float* a = acc[sD[kd]][sH[kh]][sW[kw]];
#pragma unroll
          for (int p = 0; p < kCout / 2; ++p) {
            const f2v_t r = __builtin_elementwise_fma(f2v_t{vv, vv}, wg[kw * (kCout / 2) + p],
                                                      f2v_t{a[2 * p], a[2 * p + 1]});
            a[2 * p] = r.x;
            a[2 * p + 1] = r.y;
          }
        }
      }
  };
  if constexpr (CL) {
    // channels-last: 4 channels of each of the 8 input voxels per 16-byte load (Cin % 4 == 0)
    auto load_q = [&](int c0, float4 (&q)[2][2][2]) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const size_t o = (((size_t)(ld + a) * rh + (lh + c)) * rw + (lw + e)) * Cin + c0;
            float4 t = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (okd[a] && okh[c] && okw[e]) {
              t = *reinterpret_cast<const float4*>(xb + o);
              if (xb2) {
                const float4 u = *reinterpret_cast<const float4*>(xb2 + o);
                t = make_float4(t.x + u.x, t.y + u.y, t.z + u.z, t.w + u.w);
              }
            }
            q[a][c][e] = t;
          }
    };
    // (the next quad's loads issued before this quad's FMAs measured slower: 172 VGPRs, 2 waves per
    // SIMD; eval step 3.94 -> 4.04 ms)
    for (int c0 = 0; c0 < Cin; c0 += 4) {
      float4 q[2][2][2];
      load_q(c0, q);
      // one channel of the quad at a time (unrolled, the four channels' weight reads would be
      // hoisted together: 504 VGPRs); the component is picked by selects
#pragma unroll 1
      for (int j = 0; j < 4; ++j) {
        float v[2][2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const float4 t = q[a][c][e];
              v[a][c][e] = j == 0 ? t.x : (j == 1 ? t.y : (j == 2 ? t.z : t.w));
            }
        if constexpr (WT) channel_pk(c0 + j, v);
        else channel(c0 + j, v);
      }
    }
  } else {
    // channel ci + 1's 8 (or 16, with the addend) input values are loaded before channel ci's
    // 216 fmas: the loop is otherwise one exposed load latency per input channel.  Branch-free
    // buffer loads (inputs outside the region: an out-of-range offset reads 0), so the waits for
    // them are counted instead of draining every load at each branch join.
    // (descriptors over the whole batch: a workgroup's threads may span two samples, and a
    // descriptor built from a per-thread base would need a waterfall loop per load)
    const uint32_t cbytes = (uint32_t)rvol * 4u;   // batch * Cin * rvol * 4 < 2^31 (mvs_deconv3d_k3s2_fwd checks)
    const uint32_t tbytes = (uint32_t)total_in_bytes;
    const Rsrc rs = make_rsrc(x, tbytes);
    const Rsrc rs2 = make_rsrc(x2 ? x2 : x, x2 ? tbytes : 0u);
    const uint32_t sbase = (uint32_t)b * (uint32_t)Cin * cbytes;
    uint32_t voff[2][2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          voff[a][c][e] = (okd[a] && okh[c] && okw[e])
                              ? sbase + (uint32_t)((((size_t)(ld + a) * rh + (lh + c)) * rw + (lw + e)) * 4u)
                              : 0x80000000u;
    auto load = [&](int ci, float (&v)[2][2][2]) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t o = voff[a][c][e] + (uint32_t)ci * cbytes;
            float t = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)o, 0, 0));
            if (xb2) t += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs2, (int)o, 0, 0));
            v[a][c][e] = t;
          }
    };
    float vn[2][2][2];
    load(0, vn);
    for (int ci = 0; ci < Cin; ++ci) {
      float v[2][2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 2; ++e) v[a][c][e] = vn[a][c][e];
      if (ci + 1 < Cin) load(ci + 1, vn);
      if constexpr (WT) channel_pk(ci, v);
      else channel(ci, v);
    }
  }
  const size_t plane = (size_t)D * H * W;
  const int od0 = 2 * md, oh0 = 2 * mh, ow0 = 2 * mw;
  if (out_bytes) {
    // even W (every block's x pair exists and is 8-byte aligned) and an output under 2^31 bytes:
    // branch-free 8-byte buffer loads of the residual and stores (rows past D or H: out-of-range
    // offsets), a group of four channels' residual loads in flight before their stores -- the
    // branchy form waited for each residual load on its own
    const Rsrc ry = make_rsrc(y, (uint32_t)out_bytes);
    const Rsrc rr = make_rsrc(residual ? residual : y, residual ? (uint32_t)out_bytes : 0u);
    const uint32_t pb = (uint32_t)plane * 4u;
    uint32_t boff[2][2];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int od = od0 + sd, oh = oh0 + s2;
        boff[sd][s2] = (od < D && oh < H)
                           ? ((uint32_t)b * kCout * pb + (uint32_t)(((size_t)od * H + oh) * W + ow0) * 4u)
                           : 0x80000000u;
      }
#pragma unroll
    for (int c0 = 0; c0 < kCout; c0 += 4) {
      f2v r[4][2][2];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int sd = 0; sd < 2; ++sd)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            r[cc][sd][s2] = __builtin_bit_cast(
                f2v, __builtin_amdgcn_raw_buffer_load_b64(rr, (int)(boff[sd][s2] + (uint32_t)(c0 + cc) * pb), 0, kNtAux));
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const int co = c0 + cc;
        const float m = bn_scale ? mean[co] : 0.0f, sc = bn_scale ? bn_scale[co] : 0.0f,
                    sh = bn_scale ? bn_shift[co] : 0.0f;
#pragma unroll
        for (int sd = 0; sd < 2; ++sd)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            f2v o;
#pragma unroll
            for (int sw = 0; sw < 2; ++sw) {
              float v = acc[sd][s2][sw][co];
              if (bn_scale) v = fmaxf((v - m) * sc + sh, 0.0f);
              o[sw] = v + r[cc][sd][s2][sw];
            }
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o), ry,
                                                  (int)(boff[sd][s2] + (uint32_t)co * pb), 0, kNtAux);
          }
      }
    }
    return;
  }
  const bool w2 = ow0 + 1 < W;
  float* yb = y + (size_t)b * kCout * plane;
  const float* rb = residual ? residual + (size_t)b * kCout * plane : nullptr;
#pragma unroll
  for (int co = 0; co < kCout; ++co) {
    const float m = bn_scale ? mean[co] : 0.0f, sc = bn_scale ? bn_scale[co] : 0.0f,
                sh = bn_scale ? bn_shift[co] : 0.0f;
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int od = od0 + sd, oh = oh0 + s2;
        if (od >= D || oh >= H) continue;
        const size_t off = (size_t)co * plane + ((size_t)od * H + oh) * W + ow0;
        float o[2];
#pragma unroll
        for (int sw = 0; sw < 2; ++sw) {
          float v = acc[sd][s2][sw][co];
          if (bn_scale) v = fmaxf((v - m) * sc + sh, 0.0f);
          o[sw] = v;
        }
        if (w2 && !(off & 1)) {   // 8-byte aligned pair
          float2 r = rb ? *reinterpret_cast<const float2*>(rb + off) : make_float2(0.0f, 0.0f);
          *reinterpret_cast<float2*>(yb + off) = make_float2(o[0] + r.x, o[1] + r.y);
        } else {
          yb[off] = o[0] + (rb ? rb[off] : 0.0f);
          if (w2) yb[off + 1] = o[1] + (rb ? rb[off + 1] : 0.0f);
        }
      }
  }
}

template <int CD, int CH, int CW>
void launch_cls(dim3 grid, size_t lds, hipStream_t s, const float* x, const float* x2, int lm,
                const float* weight, int Cin, int rd, int rh, int rw, int x0d, int x0h, int x0w, int D, int H,
                int W, int pd, int ph, int pw, const float* bn_scale, const float* bn_shift,
                const float* bn_mean, const float* residual, float* y, int md_n, int mh_n, int mw_n,
                size_t total) {
  // bytes of the whole region input (batch x Cin x rd x rh x rw floats)
  const size_t in_bytes = total / ((size_t)md_n * mh_n * mw_n) * (size_t)Cin * rd * rh * rw * 4u;
  // the epilogue's buffer-store path: even W and the whole output under 2^31 bytes (0 = the general path)
  const size_t ob = total / ((size_t)md_n * mh_n * mw_n) * (size_t)kCout * D * H * W * 4u;
  const size_t out_bytes = (W % 2 == 0 && ob < (1ull << 31)) ? ob : 0;
  if (lm == 3)
    hipLaunchKernelGGL((deconv3d_k3s2_kernel<CD, CH, CW, 3>), grid, dim3(kBlock), 0, s, x, x2, weight, Cin,
                       rd, rh, rw, x0d, x0h, x0w, D, H, W, pd >> 1, ph >> 1, pw >> 1, bn_scale, bn_shift,
                       bn_mean, residual, y, md_n, mh_n, mw_n, total, in_bytes, out_bytes);
  else if (lm == 1)
    hipLaunchKernelGGL((deconv3d_k3s2_kernel<CD, CH, CW, 1>), grid, dim3(kBlock), lds, s, x, x2, weight, Cin,
                       rd, rh, rw, x0d, x0h, x0w, D, H, W, pd >> 1, ph >> 1, pw >> 1, bn_scale, bn_shift,
                       bn_mean, residual, y, md_n, mh_n, mw_n, total, in_bytes, out_bytes);
  else if (lm == 2)
    hipLaunchKernelGGL((deconv3d_k3s2_kernel<CD, CH, CW, 2>), grid, dim3(kBlock), lds, s, x, x2, weight, Cin,
                       rd, rh, rw, x0d, x0h, x0w, D, H, W, pd >> 1, ph >> 1, pw >> 1, bn_scale, bn_shift,
                       bn_mean, residual, y, md_n, mh_n, mw_n, total, in_bytes, out_bytes);
  else
    hipLaunchKernelGGL((deconv3d_k3s2_kernel<CD, CH, CW, 0>), grid, dim3(kBlock), lds, s, x, x2, weight, Cin,
                       rd, rh, rw, x0d, x0h, x0w, D, H, W, pd >> 1, ph >> 1, pw >> 1, bn_scale, bn_shift,
                       bn_mean, residual, y, md_n, mh_n, mw_n, total, in_bytes, out_bytes);
}

}  // namespace

void launch_deconv3d_k3s2(const float* x, const float* x2, int layout, int B, int Cin, int rd,
                          int rh, int rw, int x0d, int x0h, int x0w, const float* weight, int D, int H,
                          int W, int pd, int ph, int pw, const float* bn_scale, const float* bn_shift,
                          const float* bn_mean, const float* residual, float* y, hipStream_t s) {
  const int md_n = (D + 1) / 2, mh_n = (H + 1) / 2, mw_n = (W + 1) / 2;
  const size_t total = (size_t)B * md_n * mh_n * mw_n;
  const dim3 grid = xcd_grid((int)((total + kBlock - 1) / kBlock));
  const size_t lds = layout == 1 ? (size_t)Cin * kCout * kWRow * sizeof(float) : 0;
  const int cls = (pd & 1) * 4 + (ph & 1) * 2 + (pw & 1);
#define MVS_DECONV_CASE(c)                                                                         \
  case c:                                                                                          \
    launch_cls<(c >> 2) & 1, (c >> 1) & 1, c & 1>(grid, lds, s, x, x2, layout, weight, Cin, rd, rh, rw, x0d, x0h, \
                                                  x0w, D, H, W, pd, ph, pw, bn_scale, bn_shift,     \
                                                  bn_mean, residual, y, md_n, mh_n, mw_n, total);   \
    break;
  switch (cls) {
    MVS_DECONV_CASE(0) MVS_DECONV_CASE(1) MVS_DECONV_CASE(2) MVS_DECONV_CASE(3)
    MVS_DECONV_CASE(4) MVS_DECONV_CASE(5) MVS_DECONV_CASE(6) MVS_DECONV_CASE(7)
  }
#undef MVS_DECONV_CASE
}

}  // namespace mvs
