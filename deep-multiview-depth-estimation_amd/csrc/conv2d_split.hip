// conv2d_split.hip -- the 2-D feature encoder's Conv2d layers past the first (model.py:35-59, 8..32
// channels) and the refinement net's 32 -> 32 layers (model.py:134-145) on the f16 matrix cores with
// split operands, eval BatchNorm + ReLU fused.  conv2d_narrow.hip computes the same convolutions
// with one fp32 FMA per term on the vector ALUs, which sets their time (8 -> 8 at 512 x 640 x 12
// images: 0.095 ms against 0.032 ms of HBM traffic).
//
// Arithmetic (split.h): the input is scaled by 2^ex, ex from its bound words (raised by the producing
// layer's epilogue), and carried as hi = fp16(v 2^ex), lo = fp16(v 2^ex - hi); the weights likewise
// with 2^ew (host, mvs_conv2d_split_weights).  One K-32 step is x_hi w_hi + x_hi w_lo + x_lo w_hi on
// v_mfma_f32_16x16x32_f16 (each product exact in fp32; the dropped x_lo w_lo is below 2^-22 of the
// product): fp32-level error, not fp32's bit pattern.
//
// GEMM mapping: rows = 16 output pixels of one image row (lane m = pixel x0 + m), columns = output
// channels, K = (tap, input channel) with 32 / CI taps per K-32 block (lane group g = lane >> 4 takes
// tap kb * (32 / CI) + g / (CI / 8), channels 8 (g % (CI / 8)) .. + 7; taps past K^2 are zeros).
// CO = 8 uses one column block holding [w_hi | w_lo] (columns 8..15 = the lo parts), so two MFMAs
// (x_hi, x_lo) give all four products and a DPP row rotation by 8 adds the halves.
//
// A workgroup (4 waves) owns a 16 XB (x) x 4 RB / XB (y) output tile: its input halo, (TX - 1) S + K x
// (TY - 1) S + K pixels with all CI channels, is loaded once from NCHW (zero outside the image),
// split and stored in LDS as one record per pixel (CI hi then CI lo fp16, 16-byte chunks
// XOR-swizzled by pixel so the 16 lanes of a row group hit 16 distinct bank groups; stride 2 stores
// even columns before odd ones so those lanes read consecutive records).  Wave w computes RB row
// blocks (RB / XB output rows of XB 16-pixel blocks) for every output channel; the weight fragments
// (L2) are fetched one K block ahead.  The epilogue unscales, applies BN + ReLU, stores NCHW (4 consecutive pixels per lane) and
// raises the output's bound words for the next layer.
#include "launchers.h"
#include "packed.h"
#include "split.h"

namespace mvs {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
constexpr uint32_t kOob2 = 0xFFFFFFC0u;   // out-of-range buffer offset: loads return 0

template <int CI, int K, int S, int RB, int XB>
struct Tile2 {
  static constexpr int TX = 16 * XB, TY = 4 * (RB / XB);
  static constexpr int IW = (TX - 1) * S + K, IH = (TY - 1) * S + K, PV = IW * IH;
  static constexpr int HALF = (IW + 1) / 2;   // S = 2: even columns at 0 .., odd ones from HALF
  static constexpr int REC = CI * 4;          // bytes per pixel record
  static constexpr int NCH = REC / 16;        // 16-byte chunks per record: 2 / 4 / 8
  static constexpr int LDS = PV * REC;
  static constexpr int TPB = 32 / CI;         // taps per K-32 block
  static constexpr int KB = (K * K + TPB - 1) / TPB;
  __device__ static int col(int px) { return S == 1 ? px : (px & 1) * HALF + (px >> 1); }
  __device__ static int chunk_off(int v, int c) { return v * REC + ((c ^ ((v / (16 / NCH)) % NCH)) << 4); }
};

__device__ inline float row_ror8(float x) {   // lane l <- lane (l + 8) mod 16 of its row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
}

template <int CI, int CO, int K, int S, int RB, int XB>
__global__ __launch_bounds__(kBlock) void conv2d_split_kernel(
    const float* __restrict__ x, const h8v* __restrict__ wf, int w_exp, float* __restrict__ y, int H, int W,
    int Ho, int Wo, int tiles_x, int tiles, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, const uint32_t* __restrict__ xb, uint32_t* __restrict__ yb) {
  using T = Tile2<CI, K, S, RB, XB>;
  static_assert(RB % XB == 0, "row blocks: XB per output row");
  static_assert(CI == 8 || CI == 16 || CI == 32, "input channels");
  static_assert(CO == 8 || CO % 16 == 0, "output channels");
  constexpr bool NARROW = CO == 8;
  constexpr int NB = NARROW ? 1 : CO / 16;
  constexpr int P = K / 2;
  __shared__ __attribute__((aligned(16))) char lds[T::LDS];

  const int t = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (t >= tiles) return;   // workgroup-uniform, before the barrier
  const int ox0 = (t % tiles_x) * T::TX, oy0 = (t / tiles_x) * T::TY;
  const int n = (int)blockIdx.y;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  const int ex = act_split_exponent(bound_read(xb));

  // ---- stage the input halo: items (channel quad, pixel), pixel fastest (coalesced rows) ----
  {
    constexpr int NQ = CI / 4, NIT = NQ * T::PV, PER = (NIT + kBlock - 1) / kBlock, BATCH = 8;
    const size_t plane = (size_t)H * W;
    const Rsrc rs = make_rsrc(x + (size_t)n * CI * plane, (uint32_t)(CI * plane * 4));
    const int iy0 = oy0 * S - P, ix0 = ox0 * S - P;
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += BATCH) {
      f4v v4[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        const int px = e % T::IW, py = (e / T::IW) % T::IH, q = e / T::PV;
        const int gx = ix0 + px, gy = iy0 + py;
        const bool ok = k0 + k < PER && e < NIT && gx >= 0 && gx < W && gy >= 0 && gy < H;
        const uint32_t off = ok ? (uint32_t)(((size_t)(4 * q) * H + gy) * W + gx) * 4u : kOob2;
        const uint32_t ps = ok ? (uint32_t)(plane * 4) : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v4[k][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + j * ps), 0, 0));
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        if (k0 + k >= PER || e >= NIT) continue;
        const int px = e % T::IW, py = (e / T::IW) % T::IH, q = e / T::PV;
        const int v = py * T::IW + T::col(px);
        uint2 hi, lo;
        split4(v4[k], ex, hi, lo);
        *reinterpret_cast<uint2*>(lds + T::chunk_off(v, q >> 1) + ((q & 1) << 3)) = hi;
        *reinterpret_cast<uint2*>(lds + T::chunk_off(v, CI / 8 + (q >> 1)) + ((q & 1) << 3)) = lo;
      }
    }
  }
  __syncthreads();

  f4v acc[RB][NB], acl[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    acl[r] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[r][nb] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  }
  // B fragments: CO >= 16 wf[kb][nb][part][lane]; CO = 8 wf[kb][lane] ([w_hi | w_lo] columns)
  struct Bf {
    h8v hi[NB], lo[NB];
  };
  auto ldb = [&](int kb, Bf& b) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (NARROW) {
        b.hi[nb] = wf[(size_t)kb * 64 + lane];
      } else {
        b.hi[nb] = wf[((size_t)(kb * NB + nb) * 2 + 0) * 64 + lane];
        b.lo[nb] = wf[((size_t)(kb * NB + nb) * 2 + 1) * 64 + lane];
      }
    }
  };
  auto kstep = [&](int kb, const Bf& b) {
    const int tap = kb * T::TPB + kq / (CI / 8), c0 = kq % (CI / 8);
    const bool tap_ok = tap < K * K;
    const int ky = tap_ok ? tap / K : 0, kx = tap_ok ? tap % K : 0;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int v = ((wave * (RB / XB) + r / XB) * S + ky) * T::IW + T::col(((r % XB) * 16 + m) * S + kx);
      h8v ahi = *reinterpret_cast<const h8v*>(lds + T::chunk_off(v, c0));
      h8v alo = *reinterpret_cast<const h8v*>(lds + T::chunk_off(v, CI / 8 + c0));
      if (!tap_ok) ahi = alo = h8v{0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (NARROW) {
        acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, b.hi[0], acc[r][0], 0, 0, 0);
        acl[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, b.hi[0], acl[r], 0, 0, 0);
      } else {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, b.hi[nb], acc[r][nb], 0, 0, 0);
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, b.lo[nb], acc[r][nb], 0, 0, 0);
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, b.hi[nb], acc[r][nb], 0, 0, 0);
        }
      }
    }
  };
  Bf b0, b1;
  ldb(0, b0);
#pragma unroll 1
  for (int kb = 0; kb < T::KB; kb += 2) {
    if (kb + 1 < T::KB) ldb(kb + 1, b1);
    kstep(kb, b0);
    if (kb + 1 < T::KB) {
      if (kb + 2 < T::KB) ldb(kb + 2, b0);
      kstep(kb + 1, b1);
    }
  }

  // ---- epilogue: acc[r][nb][i] = (pixel x0 + 4 kq + i of row r, channel nb * 16 + m) ----
  const int oexp = -(ex + w_exp);
  const size_t oplane = (size_t)Ho * Wo;
  float vmax = 0.0f;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int co = nb * 16 + m;
    const bool live = !NARROW || m < 8;
    const float sc = bn_scale && live ? bn_scale[co] : 1.0f, sh = bn_scale && live ? bn_shift[co] : 0.0f,
                mu = bn_scale && live ? bn_mean[co] : 0.0f;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int oy = oy0 + wave * (RB / XB) + r / XB, ox = ox0 + (r % XB) * 16 + 4 * kq;
      const bool vec = ox + 3 < Wo && (Wo & 3) == 0;
      f4v v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = acc[r][nb][i];
        if constexpr (NARROW) a = a + (acl[r][i] + row_ror8(a));   // hh + (lh + hl)
        a = ldexpf(a, oexp);
        if (bn_scale) a = fmaxf((a - mu) * sc + sh, 0.0f);
        v[i] = a;
      }
      if (!live || oy >= Ho) continue;
      float* dst = y + ((size_t)n * CO + co) * oplane + (size_t)oy * Wo + ox;
      if (vec) {
        *reinterpret_cast<f4v*>(dst) = v;
        vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (ox + i < Wo) {
            dst[i] = v[i];
            vmax = fmaxf(vmax, fabsf(v[i]));
          }
      }
    }
  }
  if (yb) bound_update(yb, vmax);
}

template <int CI, int CO, int K, int S, int RB, int XB>
void launch_split2d_tile(const float* x, const void* wf, int w_exp, float* y, int N, int H, int W, const float* sc,
                         const float* sh, const float* mu, const uint32_t* xb, uint32_t* yb, hipStream_t s) {
  using T = Tile2<CI, K, S, RB, XB>;
  const int Ho = (H + 2 * (K / 2) - K) / S + 1, Wo = (W + 2 * (K / 2) - K) / S + 1;
  const int tiles_x = (Wo + T::TX - 1) / T::TX, tiles_y = (Ho + T::TY - 1) / T::TY;
  const int tiles = tiles_x * tiles_y;
  const dim3 grid((unsigned)((tiles + 7) / 8 * 8), (unsigned)N);
  hipLaunchKernelGGL((conv2d_split_kernel<CI, CO, K, S, RB, XB>), grid, dim3(kBlock), 0, s, x,
                     reinterpret_cast<const h8v*>(wf), w_exp, y, H, W, Ho, Wo, tiles_x, tiles, sc, sh, mu, xb, yb);
}

// tile shapes: stride 1 32 x 8 outputs (two row blocks side by side per output row), stride 2 16 x 16.
// Measured (tools/enc_layers.py, cfg-2 encoder, 12 images of 512 x 640): 0.412 ms per encoder against
// 0.427 with 16 x 16 / 16 x 8 and 0.418 with 32 x 16 / 32 x 8 tiles (the fp32 kernels: 0.657 ms)
template <int CI, int CO, int K, int S>
void launch_split2d(const float* x, const void* wf, int w_exp, float* y, int N, int H, int W, const float* sc,
                    const float* sh, const float* mu, const uint32_t* xb, uint32_t* yb, hipStream_t s) {
  if constexpr (S == 1) launch_split2d_tile<CI, CO, K, S, 4, 2>(x, wf, w_exp, y, N, H, W, sc, sh, mu, xb, yb, s);
  else launch_split2d_tile<CI, CO, K, S, 4, 1>(x, wf, w_exp, y, N, H, W, sc, sh, mu, xb, yb, s);
}

}  // namespace

int conv2d_split_kblocks(int c_in, int k) {
  const int tpb = 32 / c_in;
  return (k * k + tpb - 1) / tpb;
}

int launch_conv2d_split(const float* x, const void* wfrag, int w_exp, float* y, int N, int Cin, int Cout, int H,
                        int W, int K, int stride, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                        const uint32_t* x_bound, uint32_t* y_bound, hipStream_t s) {
#define MVS_SPLIT2D_CASE(A, C, KK, SS)                                                                       \
  if (Cin == A && Cout == C && K == KK && stride == SS) {                                                  \
    launch_split2d<A, C, KK, SS>(x, wfrag, w_exp, y, N, H, W, bn_scale, bn_shift, bn_mean, x_bound, y_bound, s); \
    return MVS_OK;                                                                                         \
  }
  // FeatureEncoder layers 2-8 (model.py:35-59) and the refinement net's 32 -> 32 (model.py:134-145)
  MVS_SPLIT2D_CASE(8, 8, 3, 1) MVS_SPLIT2D_CASE(8, 16, 5, 2) MVS_SPLIT2D_CASE(16, 16, 3, 1)
  MVS_SPLIT2D_CASE(16, 32, 5, 2) MVS_SPLIT2D_CASE(32, 32, 3, 1)
#undef MVS_SPLIT2D_CASE
  return MVS_ERR_INVALID_ARGUMENT;
}

}  // namespace mvs
