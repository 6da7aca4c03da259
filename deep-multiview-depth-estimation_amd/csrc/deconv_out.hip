// deconv_out.hip -- the regulariser's last two layers in one kernel (eval mode): deconv_1_0 (16 -> 8,
// 3x3x3 stride-2 transposed, from its live input region y2 + y1) + BN_0 + ReLU + the skip add y0
// (model.py:121-123), then conv_out (8 -> 1, 3x3x3, padding 1, model.py:96/125).  The 8-channel
// full-size volume between them (0.5 GB at cfg 2, written by deconv3d_region.hip and read back by
// conv3d_narrow.hip) stays on chip.
//
// A 256-thread workgroup owns a 32 x 16 (x, y) tile of conv_out's output and a chunk of kZC depths.
// It walks the depths two at a time: per step it forms one LAYER of the transposed conv -- output
// planes 2L, 2L + 1 on the tile's 34 x 18 halo, as 2 x 2 x 2 blocks, one block per thread (18 x 10
// blocks), exactly deconv3d_region.hip's block arithmetic (same products, same order: the NCDHW,
// tap-major packed-FMA form) and epilogue -- into a two-layer LDS ring, then applies conv_out to
// output planes 2L - 1 and 2L (two rows and two planes per thread, conv3d_narrow.hip's order:
// channel, kd, ky, kx).  Results are bit-identical to the two-kernel path.
// Halo cost: 36 x 20 block voxels per 32 x 16 outputs (1.41x the transposed conv's products) and
// kZC / 2 + 2 layers per kZC depths; saved: the 0.5 GB write + 0.6 GB read of the 8-channel volume.
// Measured (cfg 2): 1.87 ms with per-thread global input gathers, 3.0 ms with the LDS-staged input
// below, against 0.52 + 0.20 ms for the two kernels -- at one workgroup per CU (105 KB of LDS) the
// 144 scalar weight-row loads per layer (12 packed FMAs each) expose their latency, which the
// two-kernel path hides with 16 waves per CU.  Opt-in (MVS_DECONV_OUT=1), kept for its bit-exact
// test; the next form needs several blocks per thread per weight row.
#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kCo = 8;                       // deconv_1_0 output channels = conv_out input channels
constexpr int kTX = 32, kTY = 16;            // conv_out outputs per tile
constexpr int kHX = kTX + 2, kHY = kTY + 2;  // z halo: x0 - 1 .. x0 + 32, y0 - 1 .. y0 + 16
constexpr int kBX = kTX / 2 + 2, kBY = kTY / 2 + 2;   // 18 x 10 blocks per layer
constexpr int kZC = 32;                      // conv_out depths per workgroup
constexpr int kPlaneF = kCo * kHY * kHX;     // floats per z plane (8 channels)
constexpr int kLdsF = 2 * 2 * kPlaneF;       // two layers x two planes: 78,336 B
constexpr int kIX = kBX + 1, kIY = kBY + 1;  // input slab per region plane: 19 x 11 (blocks' L and U)
constexpr int kInF = 16 * kIY * kIX;         // floats per staged input plane (c_in = 16)
constexpr int kInPer = (kInF + kBlock - 1) / kBlock;   // staging elements per thread

typedef float f2v_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const f2v_t const_f2v_t;
constexpr int kNt = 2;   // y0 streams through once: non-temporal loads

template <int CD, int CH, int CW>
__global__ __launch_bounds__(kBlock) void deconv_out_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const float* __restrict__ wt, int Cin, int rd, int rh,
    int rw, int x0d, int x0h, int x0w, int D, int H, int W, int qd, int qh, int qw,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift, const float* __restrict__ bn_mean,
    const float* __restrict__ residual, const float* __restrict__ wout, float* __restrict__ out, int tiles_x,
    int tiles_y, int zchunks, int total, uint32_t in_bytes) {
  __shared__ float zr[kLdsF];   // [layer & 1][plane & 1][c][hy][hx]
  const int wk = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (wk >= total) return;   // workgroup-uniform, before any barrier
  int t = wk;
  const int x0 = (t % tiles_x) * kTX;
  t /= tiles_x;
  const int y0 = (t % tiles_y) * kTY;
  t /= tiles_y;
  const int z0 = (t % zchunks) * kZC;
  const int b = t / zchunks;
  const int z1 = min(z0 + kZC, D);
  const int tid = (int)threadIdx.x;
  const size_t plane = (size_t)H * W, vol = (size_t)D * plane;

  // ---- deconv block of this thread: (mw, mh) fixed, md = the layer ----
  // The region input (x + x2, summed on load as deconv3d_region.hip does) is staged in LDS one region
  // plane at a time: a block of layer md reads region planes ld, ld + 1 (ld = md + qd + CD - 1 - x0d),
  // so each layer brings one new plane (loaded a layer ahead, in registers) into a two-plane ring.
  __shared__ float xin[2 * kInF];   // [region plane & 1][ci][iy][ix]
  const bool blk = tid < kBX * kBY;
  const int bx = tid % kBX, by = tid / kBX;
  const int mw = x0 / 2 - 1 + bx, mh = y0 / 2 - 1 + by;
  const int lw0 = x0 / 2 - 1 + qw + CW - 1 - x0w, lh0 = y0 / 2 - 1 + qh + CH - 1 - x0h;   // slab origin
  const uint32_t rvol = (uint32_t)rd * rh * rw, cbytes = rvol * 4u;
  const Rsrc rs = make_rsrc(x, in_bytes);
  const Rsrc rs2 = make_rsrc(x2 ? x2 : x, x2 ? in_bytes : 0u);
  const Rsrc rres = make_rsrc(residual, (uint32_t)min<uint64_t>((uint64_t)(b + 1) * kCo * vol * 4u, 0xFFFFFFF0ull));
  // staging map: element e of a slab plane -> (region offset inside one channel plane, valid)
  uint32_t soff[kInPer];
  bool sok[kInPer];
#pragma unroll
  for (int j = 0; j < kInPer; ++j) {
    const int e = tid + j * kBlock;
    const int ci = e / (kIY * kIX), r = e % (kIY * kIX);
    const int iy = r / kIX, ix = r % kIX;
    const int gh = lh0 + iy, gw = lw0 + ix;
    sok[j] = e < kInF && ci < Cin && gh >= 0 && gh < rh && gw >= 0 && gw < rw;
    soff[j] = sok[j] ? (uint32_t)b * (uint32_t)Cin * cbytes + (uint32_t)ci * cbytes + (uint32_t)(gh * rw + gw) * 4u : 0u;
  }
  float pre[kInPer];
  auto fetch = [&](int ldp) {   // region plane ldp of the slab -> registers (0 outside the region)
    const bool pin = ldp >= 0 && ldp < rd;
#pragma unroll
    for (int j = 0; j < kInPer; ++j) {
      pre[j] = 0.0f;
      if (pin && sok[j]) {
        const uint32_t o = soff[j] + (uint32_t)ldp * (uint32_t)rh * (uint32_t)rw * 4u;
        float tv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)o, 0, 0));
        if (x2) tv += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs2, (int)o, 0, 0));
        pre[j] = tv;
      }
    }
  };
  auto stage = [&](int ldp) {   // registers -> ring slot of region plane ldp
    float* dst = xin + (ldp & 1) * kInF;
#pragma unroll
    for (int j = 0; j < kInPer; ++j) {
      const int e = tid + j * kBlock;
      if (e < kInF) dst[e] = pre[j];
    }
  };
  auto lds_drain = [&]() {   // no vector load may land in registers an outstanding LDS op still reads
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto layer = [&](int L) {   // transposed conv + BN + ReLU + y0 on planes 2L, 2L + 1 -> ring
    float* zl = zr + (L & 1) * 2 * kPlaneF;
    if (!blk) return;
    const int md = L;
    const int ld = md + qd + CD - 1 - x0d;
    float acc[2][2][2][kCo];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int co = 0; co < kCo; ++co) acc[a][c][e][co] = 0.0f;
    // the block's inputs L / U per dim: slab (by + c, bx + e) of region planes ld + a
    const float* xp[2] = {xin + (ld & 1) * kInF, xin + ((ld + 1) & 1) * kInF};
    auto load = [&](int ci, float (&v)[2][2][2]) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 2; ++e) v[a][c][e] = xp[a][(ci * kIY + by + c) * kIX + bx + e];
    };
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
              (const const_f2v_t*)uniform_ptr(wt + ((size_t)ci * 27 + kd * 9 + kh * 3) * kCo);
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const float vv = v[iD[kd]][iH[kh]][iW[kw]];
            float* ac = acc[sD[kd]][sH[kh]][sW[kw]];
#pragma unroll
            for (int p = 0; p < kCo / 2; ++p) {
              const f2v_t r = __builtin_elementwise_fma(f2v_t{vv, vv}, wg[kw * (kCo / 2) + p],
                                                        f2v_t{ac[2 * p], ac[2 * p + 1]});
              ac[2 * p] = r.x;
              ac[2 * p + 1] = r.y;
            }
          }
        }
    };
    for (int ci = 0; ci < Cin; ++ci) {
      float v[2][2][2];
      load(ci, v);
      channel_pk(ci, v);
    }
    // epilogue (deconv3d_region.hip's): max((y - mean) * scale + shift, 0) + y0; voxels outside the
    // volume are conv_out's zero padding.  Every y0 load is issued after this layer's LDS reads have
    // completed and before its first LDS write (lds_drain)
    const int od0 = 2 * md, oh0 = 2 * mh, ow0 = 2 * mw;
    lds_drain();
    float r[2][2][2][kCo];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int sw = 0; sw < 2; ++sw) {
          const int od = od0 + sd, oh = oh0 + s2, ow = ow0 + sw;
          const bool in = od >= 0 && od < D && oh >= 0 && oh < H && ow >= 0 && ow < W;
#pragma unroll
          for (int co = 0; co < kCo; ++co) {
            r[sd][s2][sw][co] = 0.0f;
            if (in && residual)
              r[sd][s2][sw][co] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  rres, (int)((((size_t)(b * kCo + co) * D + od) * plane + (size_t)oh * W + ow) * 4u), 0, kNt));
          }
        }
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int od = od0 + sd, oh = oh0 + s2;
        const int hy = oh - (y0 - 1);
        if (hy < 0 || hy >= kHY) continue;
        const bool rin = od >= 0 && od < D && oh >= 0 && oh < H;
#pragma unroll
        for (int co = 0; co < kCo; ++co) {
          const float m = bn_scale ? bn_mean[co] : 0.0f, sc = bn_scale ? bn_scale[co] : 0.0f,
                      sh = bn_scale ? bn_shift[co] : 0.0f;
#pragma unroll
          for (int sw = 0; sw < 2; ++sw) {
            const int ow = ow0 + sw, hx = ow - (x0 - 1);
            if (hx < 0 || hx >= kHX) continue;
            const bool in = rin && ow >= 0 && ow < W;
            float v = acc[sd][s2][sw][co];
            if (bn_scale) v = fmaxf((v - m) * sc + sh, 0.0f);
            zl[((sd * kCo + co) * kHY + hy) * kHX + hx] = in ? v + r[sd][s2][sw][co] : 0.0f;
          }
        }
      }
  };

  // ---- conv_out on output planes 2L - 1, 2L: thread = column (lx, ly) and (lx, ly + 8) ----
  const int lx = tid & 31, ly = tid >> 5;
  auto conv_out = [&](int L) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int p = 2 * L - 1 + pp;
      if (p < z0 || p >= z1) continue;   // uniform
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int ty = ly + 8 * rr;
        float acc = 0.0f;
#pragma unroll 1
        for (int c = 0; c < kCo; ++c) {
#pragma unroll
          for (int kd = 0; kd < 3; ++kd) {
            const int zp = p + kd - 1;
            const float* zc = zr + ((((zp >> 1) & 1) * 2 + (zp & 1)) * kCo + c) * kHY * kHX;
            asm volatile("" ::: "memory");   // scalar weight loads, one (c, kd) row at a time
            const float* wg = uniform_ptr(wout + (c * 3 + kd) * 9);
            float w9[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) w9[k] = wg[k];
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) acc = fmaf(zc[(ty + ky) * kHX + lx + kx], w9[ky * 3 + kx], acc);
          }
        }
        const int gx = x0 + lx, gy = y0 + ty;
        if (gx < W && gy < H) out[(size_t)b * vol + (size_t)p * plane + (size_t)gy * W + gx] = acc;
      }
    }
  };

  const int L0 = z0 / 2 - 1, L1 = (z1 + 1) / 2;   // layers L0 .. L1: planes z0 - 2 .. z1 + 1
  const int ld0 = L0 + qd + CD - 1 - x0d;          // region plane L of layer L0
  fetch(ld0);
  stage(ld0);
  fetch(ld0 + 1);
  for (int L = L0; L <= L1; ++L) {
    const int ldn = L + qd + CD - x0d;   // the new region plane (U) of layer L
    stage(ldn);
    __syncthreads();
    if (L < L1) fetch(ldn + 1);          // layer L + 1's, in flight during this layer
    layer(L);
    __syncthreads();
    if (L > L0) conv_out(L);
    __syncthreads();
  }
}

template <int CD, int CH, int CW>
void launch_cls(dim3 grid, hipStream_t s, const float* x, const float* x2, const float* wt, int Cin, int rd, int rh,
                int rw, int x0d, int x0h, int x0w, int D, int H, int W, int pd, int ph, int pw, const float* bs,
                const float* bh, const float* bm, const float* res, const float* wo, float* out, int tx, int ty,
                int zc, int total, uint32_t in_bytes) {
  hipLaunchKernelGGL((deconv_out_kernel<CD, CH, CW>), grid, dim3(kBlock), 0, s, x, x2, wt, Cin, rd, rh, rw, x0d,
                     x0h, x0w, D, H, W, pd >> 1, ph >> 1, pw >> 1, bs, bh, bm, res, wo, out, tx, ty, zc, total,
                     in_bytes);
}

}  // namespace

int launch_deconv_out(const float* x, const float* x2, int B, int Cin, int rd, int rh, int rw, int x0d, int x0h,
                      int x0w, const float* weight_taps, int D, int H, int W, int pd, int ph, int pw,
                      const float* bn_scale, const float* bn_shift, const float* bn_mean, const float* residual,
                      const float* conv_out_weight, float* out, hipStream_t s) {
  const uint64_t in_bytes = (uint64_t)B * Cin * rd * rh * rw * 4u;
  if (in_bytes >= (1ull << 31) || (uint64_t)B * kCo * D * H * W * 4u >= 0xFFFFFFF0ull) return MVS_ERR_TOO_LARGE;
  const int tx = (W + kTX - 1) / kTX, ty = (H + kTY - 1) / kTY, zc = (D + kZC - 1) / kZC;
  const long total = (long)B * zc * ty * tx;
  if (total >= (1L << 31) - 8) return MVS_ERR_TOO_LARGE;
  const dim3 grid = xcd_grid((int)total);
  const int cls = (pd & 1) * 4 + (ph & 1) * 2 + (pw & 1);
#define MVS_DOUT_CASE(c)                                                                                      \
  case c:                                                                                                     \
    launch_cls<(c >> 2) & 1, (c >> 1) & 1, c & 1>(grid, s, x, x2, weight_taps, Cin, rd, rh, rw, x0d, x0h, x0w, D, \
                                                  H, W, pd, ph, pw, bn_scale, bn_shift, bn_mean, residual,      \
                                                  conv_out_weight, out, tx, ty, zc, (int)total, (uint32_t)in_bytes); \
    break;
  switch (cls) {
    MVS_DOUT_CASE(0) MVS_DOUT_CASE(1) MVS_DOUT_CASE(2) MVS_DOUT_CASE(3)
    MVS_DOUT_CASE(4) MVS_DOUT_CASE(5) MVS_DOUT_CASE(6) MVS_DOUT_CASE(7)
  }
#undef MVS_DOUT_CASE
  return MVS_OK;
}

}  // namespace mvs
