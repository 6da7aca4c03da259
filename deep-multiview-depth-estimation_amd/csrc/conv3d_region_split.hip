// conv3d_region_split.hip -- the regulariser's stride-1 convolutions (conv_k_1, model.py:79-85,
// forward at model.py:104-113) and stride-2 transposed convolutions (deconv_3_0 / deconv_2_0,
// model.py:86-88, forward at model.py:117-120) on the f16 matrix cores with split operands, eval BN +
// ReLU fused.  Same GEMM mapping, region geometry, tap order and epilogue as conv3d_region.hip (whose
// fp32-MFMA kernel it replaces on the split-fp16 eval path); only the arithmetic differs:
//
//   * operands are split as in split.h: an activation v (fp32, channels-last region tensor, or the sum
//     of two for `y3 + y2`) is scaled by 2^ex and carried as hi = fp16(v 2^ex), lo = fp16(v 2^ex - hi),
//     the weights likewise with 2^ew (host, mvs_conv3d_region_split_weights);
//   * one K-32 step is three v_mfma_f32_16x16x32_f16 into the same accumulator: x_hi w_hi, x_hi w_lo,
//     x_lo w_hi (the dropped x_lo w_lo is below 2^-22 of the product), each product exact in fp32;
//   * ex comes from the input's BOUND WORDS: kBoundSlots partial maxima of |v| that the kernel which
//     produced the tensor wrote in its epilogue (bound_update, split.h), so max|v| 2^ex < 2^14.
//
// gfx950 runs the f16 MFMA at 16x the fp32 one's rate: the three products cost 48 cycles per
// (16 rows, 16 columns, 32 K) against 256 for the eight fp32 16x16x4 steps, on the same operand bytes
// (an fp32 K-8 lane slice is 32 B; a split one is 2 x 16 B).
//
// K blocking.  CI >= 32: one K-32 block per (tap, 32 input channels), lane (m, g) supplies channels
// 8g .. 8g + 7 of its row's tap voxel.  CI = 16 (conv_1_1, S1 only): one K-32 block per PAIR of taps
// (2j, 2j + 1; tap 27 is empty), lanes g = 0, 1 the first tap's 16 channels, g = 2, 3 the second's.
//
// S2 (conv_k_0, model.py:78-80 / :103-111): the input is the split cost volume itself (split.h's SCV,
// or a box of it), already the operands: a lane's 8 channels are the hi / lo halves of quads 2g and
// 2g + 1 (two 16-byte loads, no conversion), scaled by the volume's bound words (cv_split_exponent).
#include <cstdlib>

#include "launchers.h"
#include "packed.h"
#include "split.h"

namespace mvs {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
constexpr uint32_t kOob = 0xFFFFFFC0u;   // out-of-range buffer offset (loads return 0); +16 stays out
constexpr int kS1 = 0, kS2 = 1, kT2 = 2;

struct GeoS {
  int n[3];    // volume dims
  int o0[3];   // output region origin
  int on[3];   // output region size
  int i0[3];   // input region origin
  int in[3];   // input region size
  int pad[3];  // T2: P
  int out_cf;  // 1: output channels-first
  const float* addend;   // nullable: added to the output after BN + ReLU (same layout as y)
  int sb0[3];  // store box (absolute voxel coordinates, inside the output region): y holds these
  int sbn[3];  //   voxels only (the whole output region unless a box is given)
  double* stats;   // nullable: per-workgroup float64 (sum, sum of squares) of every output voxel's
                   // value, [slot][2][CO] (train-mode BatchNorm's batch sums; slots: split_stats_slots)
  const float* in_bn;   // nullable (LDS transposed kernel): the input is relu(BN_a(x)) [+ relu(BN_b(x2))],
                        // in_bn = [6][CI]: scale_a, shift_a, mean_a, scale_b, shift_b, mean_b (train
                        // mode's BN + ReLU passes folded into the staging)
  float* ym[2];    // S2 with CO = 112 (kS2Multi): conv_1_0 / conv_2_0 / conv_3_0 at once -- y holds
                   // channels 0-15, ym[0] 16-47, ym[1] 48-111, each its own channels-last tensor
};

// train mode's three stride-2 convolutions read the same split cost volume over the same region R2
// (CostVolumeReg.forward_live_train): one launch with their 16 + 32 + 64 output channels loads each
// A fragment once for all seven column blocks (three launches loaded it three times)
constexpr int kS2Multi = 112;
#ifndef MVS_S2M_BLDS
#define MVS_S2M_BLDS 1
#endif
// S1 64 -> 64 with the K block's weights in LDS, 2 row blocks per wave (3 waves per SIMD): train-mode
// step 12.3 -> 12.1 ms (with 4 row blocks 274 registers, one wave per SIMD: 13.4 ms)
#ifndef MVS_S1_BLDS
#define MVS_S1_BLDS 1
#endif

// per-workgroup channel sums: the wave's per-lane partial sums s / q (channel nb * 16 + (lane & 15) of
// column block nb) reduced over the lanes of equal channel, then over the waves in a fixed order, and
// written to stats[slot] (no atomics: the caller adds the slots in a fixed order -- run-to-run
// bit-identical, as channel_ops.hip's sums).  Whole workgroup (a barrier).
template <int CO, int NB, int NW>
__device__ inline void stats_write(double (&s)[NB], double (&q)[NB], int nb0, int nbs, double* __restrict__ st) {
  __shared__ double red[NW][2][CO];
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
  for (int w = (int)threadIdx.x; w < NW * 2 * CO; w += (int)blockDim.x) (&red[0][0][0])[w] = 0.0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      s[j] += __shfl_xor(s[j], o);
      q[j] += __shfl_xor(q[j], o);
    }
    if (lane < 16 && j < nbs) {
      red[wave][0][(nb0 + j) * 16 + lane] = s[j];
      red[wave][1][(nb0 + j) * 16 + lane] = q[j];
    }
  }
  __syncthreads();
  for (int t = (int)threadIdx.x; t < 2 * CO; t += (int)blockDim.x) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += (&red[w][0][0])[t];
    st[t] = a;
  }
}

__device__ inline void class_dim_s(int o0, int on, int p, int par, int& first, int& cnt) {
  first = o0 + (((o0 + p) & 1) != par ? 1 : 0);
  cnt = first < o0 + on ? (o0 + on - 1 - first) / 2 + 1 : 0;
}

template <int MODE, int CI, int CO, int RB>
__global__ __launch_bounds__(kBlock) void conv3d_region_split_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const h8v* __restrict__ wf, int w_exp,
    float* __restrict__ y, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, GeoS g, const uint32_t* __restrict__ xb, const uint32_t* __restrict__ xb2,
    uint32_t* __restrict__ yb) {
  constexpr int NB = CO / 16;
  constexpr bool PAIR = CI == 16;
  constexpr int CB = PAIR ? 1 : CI / 32;   // K-32 blocks per tap
  static_assert(CO % 16 == 0 && (PAIR || CI % 32 == 0), "channel counts");
  static_assert(!PAIR || MODE == kS1, "tap pairs: stride-1 convolutions only");
  static_assert(MODE != kS2 || CI == 32, "S2: the 32-channel split cost volume");
  const int lane = (int)threadIdx.x & 63;
  const int m = lane & 15, kq = lane >> 4;
  const int b = (int)blockIdx.z;

  int cf[3], cn[3], par[3] = {0, 0, 0};
  if constexpr (MODE == kT2) {
    const int cls = (int)blockIdx.y;
    par[0] = (cls >> 2) & 1;
    par[1] = (cls >> 1) & 1;
    par[2] = cls & 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) class_dim_s(g.o0[d], g.on[d], g.pad[d], par[d], cf[d], cn[d]);
  } else {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      cf[d] = g.o0[d];
      cn[d] = g.on[d];
    }
  }
  const int rows = cn[0] * cn[1] * cn[2];
  const int step = MODE == kT2 ? 2 : 1;
  constexpr int kRows = 16 * RB;
  const int bx = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  const int row0 = (bx * (kBlock / 64) + ((int)threadIdx.x >> 6)) * kRows;
  // wave-uniform; no barriers in this kernel unless sums are gathered (then every wave stays, the
  // ones past the rows on zeros)
  if (row0 >= rows && !g.stats && !(MODE == kS2 && CO == kS2Multi) && !(MODE == kS1 && CI == 64 && MVS_S1_BLDS)) return;

  // the input's scale: max|x| (+ max|x2|) 2^ex < 2^14; S2: the split volume's own exponent
  int ex;
  if constexpr (MODE == kS2) {
    ex = cv_split_exponent(xb);
  } else {
    float bound = bound_read(xb);
    if (x2) bound += bound_read(xb2);
    ex = act_split_exponent(bound);
  }

  int lin[RB];
  unsigned vm[RB][3];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = row0 + rb * 16 + m;
    const bool ok = r < rows;
    const int rr = ok ? r : 0;
    const int jx = rr % cn[2], t = rr / cn[2];
    const int jy = t % cn[1], jz = t / cn[1];
    const int o[3] = {cf[0] + step * jz, cf[1] + step * jy, cf[2] + step * jx};
    int bs[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      if constexpr (MODE == kS1) bs[d] = o[d] - 1 - g.i0[d];
      else if constexpr (MODE == kS2) bs[d] = 2 * o[d] - g.pad[d] - g.i0[d];   // taps off the box: off the volume
      else bs[d] = ((o[d] + g.pad[d] - par[d]) >> 1) - g.i0[d];
      unsigned mk = 0;
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        const int dl = MODE == kT2 ? -(tt >> 1) : tt;
        const bool in = ok && bs[d] + dl >= 0 && bs[d] + dl < g.in[d] && !(MODE == kT2 && ((tt & 1) != par[d]));
        mk |= in ? (1u << tt) : 0u;
      }
      vm[rb][d] = mk;
    }
    lin[rb] = (bs[0] * g.in[1] + bs[1]) * g.in[2] + bs[2];
  }

  f4v acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f4v{0.0f, 0.0f, 0.0f, 0.0f};

  const size_t rvol = (size_t)g.in[0] * g.in[1] * g.in[2];
  // S2: the sample's 8 quad planes of 16-byte elements (8 * rvol * 16 B = the same bytes as CI fp32)
  const Rsrc rs = make_rsrc(x + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
  const Rsrc rs2 = make_rsrc(x2 ? x2 + (size_t)b * rvol * CI : x, x2 ? (uint32_t)(rvol * CI * 4) : 0u);
  const int sy = g.in[2], sz = g.in[1] * g.in[2];

  // 8 channels c0 .. c0 + 7 of input voxel vx (kOob: zeros) as split fp16 parts
  auto load_split = [&](uint32_t vx, int c0, h8v& hi, h8v& lo) {
    if constexpr (MODE == kS2) {   // quads c0 / 4, c0 / 4 + 1 of the split volume: {hi x4, lo x4} each
      const uint32_t q = (uint32_t)c0 >> 2;
      const uint4 e0 = __builtin_bit_cast(uint4, ld4(rs, vx == kOob ? kOob : ((q * (uint32_t)rvol) + vx) * 16u, 0));
      const uint4 e1 = __builtin_bit_cast(uint4, ld4(rs, vx == kOob ? kOob : (((q + 1) * (uint32_t)rvol) + vx) * 16u, 0));
      hi = __builtin_bit_cast(h8v, make_uint4(e0.x, e0.y, e1.x, e1.y));
      lo = __builtin_bit_cast(h8v, make_uint4(e0.z, e0.w, e1.z, e1.w));
      return;
    }
    const uint32_t eo = vx == kOob ? kOob : (vx * (uint32_t)CI + (uint32_t)c0) * 4u;
    f4v a0 = ld4(rs, eo, 0), a1 = ld4(rs, eo + 16u, 0);
    if (x2) {
      a0 += ld4(rs2, eo, 0);
      a1 += ld4(rs2, eo + 16u, 0);
    }
    uint2 h0, l0, h1, l1;
    split4(a0, ex, h0, l0);
    split4(a1, ex, h1, l1);
    hi = __builtin_bit_cast(h8v, make_uint4(h0.x, h0.y, h1.x, h1.y));
    lo = __builtin_bit_cast(h8v, make_uint4(l0.x, l0.y, l1.x, l1.y));
  };
  // one K-32 block: the row blocks' split A fragments, the column blocks' (hi, lo) weight fragments
  // (wf[kb][nb][part][lane]), then x_hi w_hi, x_hi w_lo, x_lo w_hi per (row block, column block)
  // BL (the 3-in-1 S2: seven column blocks, 14 KB of weight fragments per K block, 378 KB in all):
  // each K block's fragments are fetched once per workgroup into an LDS double buffer (one barrier per
  // K block; the next block's global loads in flight under this block's MFMAs) instead of by every wave
  // from L2.  Every wave runs the same K sequence (taps, then channel blocks).
  constexpr bool BL = (MODE == kS2 && CO == kS2Multi && MVS_S2M_BLDS) || (MODE == kS1 && CI == 64 && MVS_S1_BLDS);
  constexpr int BFR = NB * 2 * 64;                        // h8v per K block
  constexpr int BPER = (BFR + kBlock - 1) / kBlock;
  __shared__ h8v blds[BL ? 2 : 1][BL ? BFR : 1];
  h8v bpre[BPER];
  auto bfetch = [&](int kb) {
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int e = (int)threadIdx.x + i * kBlock;
      if (e < BFR) bpre[i] = wf[(size_t)kb * BFR + e];
    }
  };
  auto bstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int e = (int)threadIdx.x + i * kBlock;
      if (e < BFR) blds[buf][e] = bpre[i];
    }
  };
  if constexpr (BL) {
    bfetch(0);
    bstore(0);
    __syncthreads();
    bfetch(1);
  }
  auto kblock = [&](int kb, const uint32_t (&vx)[RB], int c0) {
    h8v ahi[RB], alo[RB], bhi[NB], blo[NB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) load_split(vx[rb], c0, ahi[rb], alo[rb]);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if constexpr (BL) {
        bhi[nb] = blds[kb & 1][(nb * 2 + 0) * 64 + lane];
        blo[nb] = blds[kb & 1][(nb * 2 + 1) * 64 + lane];
      } else {
        bhi[nb] = wf[((size_t)(kb * NB + nb) * 2 + 0) * 64 + lane];
        blo[nb] = wf[((size_t)(kb * NB + nb) * 2 + 1) * 64 + lane];
      }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[rb], bhi[nb], acc[rb][nb], 0, 0, 0);
        acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[rb], blo[nb], acc[rb][nb], 0, 0, 0);
        acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[rb], bhi[nb], acc[rb][nb], 0, 0, 0);
      }
    if constexpr (BL) {
      constexpr int NK = 27 * CB;   // one K block per (tap, 32 channels)
      if (kb + 1 < NK) bstore((kb + 1) & 1);
      __syncthreads();
      if (kb + 2 < NK) bfetch(kb + 2);
    }
  };

  if constexpr (PAIR) {
    // tap pairs: this lane's tap 2j + (kq >> 1), channels 8 (kq & 1) .. + 7
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      const int tap = 2 * j + (kq >> 1);
      const int tz = tap / 9, ty = (tap / 3) % 3, tx = tap % 3;
      uint32_t vx[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const bool ok = tap < 27 && ((vm[rb][0] >> tz) & (vm[rb][1] >> ty) & (vm[rb][2] >> tx) & 1u) != 0;
        vx[rb] = ok ? (uint32_t)(lin[rb] + tz * sz + ty * sy + tx) : kOob;
      }
      kblock(j, vx, 8 * (kq & 1));
    }
  } else {
#pragma unroll
    for (int tz = 0; tz < 3; ++tz) {
      if (MODE == kT2 && ((tz & 1) != par[0])) continue;   // taps of o + P's parity only
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        if (MODE == kT2 && ((ty & 1) != par[1])) continue;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          if (MODE == kT2 && ((tx & 1) != par[2])) continue;
          const int dz = MODE == kT2 ? -(tz >> 1) : tz, dy = MODE == kT2 ? -(ty >> 1) : ty,
                    dx = MODE == kT2 ? -(tx >> 1) : tx;
          uint32_t vx[RB];
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            const bool ok = ((vm[rb][0] >> tz) & (vm[rb][1] >> ty) & (vm[rb][2] >> tx) & 1u) != 0;
            vx[rb] = ok ? (uint32_t)(lin[rb] + dz * sz + dy * sy + dx) : kOob;
          }
          const int tap = (tz * 3 + ty) * 3 + tx;
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) kblock(tap * CB + cb, vx, cb * 32 + 8 * kq);
        }
      }
    }
  }

  // ---- epilogue: unscale, eval BN + ReLU, store; the output's bound words.  acc[rb][nb][r] = (row
  // (lane >> 4) * 4 + r, column lane & 15)
  const int oexp = -(ex + w_exp);
  const size_t orvol = (size_t)g.sbn[0] * g.sbn[1] * g.sbn[2];
  float vmax = 0.0f;
  double ss[NB], sq[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int co = nb * 16 + m;
    const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
                mu = bn_scale ? bn_mean[co] : 0.0f;
    ss[nb] = sq[nb] = 0.0;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + rb * 16 + kq * 4 + r;
        if (row >= rows) continue;
        const int jx = row % cn[2], t = row / cn[2];
        const int jy = t % cn[1], jz = t / cn[1];
        const int vz = cf[0] + step * jz - g.sb0[0], vy = cf[1] + step * jy - g.sb0[1],
                  vxx = cf[2] + step * jx - g.sb0[2];
        float v = ldexpf(acc[rb][nb][r], oexp);
        if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
        const bool keep = vz >= 0 && vz < g.sbn[0] && vy >= 0 && vy < g.sbn[1] && vxx >= 0 && vxx < g.sbn[2];
        const size_t vox = ((size_t)vz * g.sbn[1] + vy) * g.sbn[2] + vxx;
        size_t oi;
        float* dst = y;
        if constexpr (MODE == kS2 && CO == kS2Multi) {   // (nb 0 | 1-2 | 3-6): 16 / 32 / 64 channels
          const int ck = nb == 0 ? 16 : (nb < 3 ? 32 : 64), c0 = nb == 0 ? 0 : (nb < 3 ? 16 : 48);
          dst = nb == 0 ? y : (nb < 3 ? g.ym[0] : g.ym[1]);
          oi = ((size_t)b * orvol + vox) * ck + (co - c0);
        } else {
          oi = g.out_cf ? ((size_t)b * CO + co) * orvol + vox : ((size_t)b * orvol + vox) * CO + co;
        }
        if (g.addend && keep) v += g.addend[oi];
        ss[nb] += (double)v;
        sq[nb] += (double)v * (double)v;
        if (!keep) continue;
        vmax = fmaxf(vmax, fabsf(v));
        dst[oi] = v;
      }
  }
  if (yb) bound_update(yb, vmax);
  if (g.stats) {
    const size_t slot = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    stats_write<CO, NB, kBlock / 64>(ss, sq, 0, NB, g.stats + slot * 2 * CO);
  }
}

// the per-lane kernel's grid: (row chunks of a parity class, rounded to the 8 XCDs) x classes x batch
inline dim3 split_mode_grid(int mode, int RB, int B, const int* on) {
  const int classes = mode == kT2 ? 8 : 1;
  const int rz = mode == kT2 ? (on[0] + 1) / 2 : on[0], ry = mode == kT2 ? (on[1] + 1) / 2 : on[1],
            rx = mode == kT2 ? (on[2] + 1) / 2 : on[2];
  const long rows = (long)rz * ry * rx;
  const long per_block = (kBlock / 64) * 16 * RB;
  const long blocks = (rows + per_block - 1) / per_block;
  return dim3((unsigned)((blocks + 7) / 8 * 8), (unsigned)classes, (unsigned)B);
}

template <int MODE, int CI, int CO, int RB>
void launch_split_mode(const float* x, const float* x2, const void* wf, int w_exp, float* y, const float* sc,
                       const float* sh, const float* mu, int B, const GeoS& g, const uint32_t* xb,
                       const uint32_t* xb2, uint32_t* yb, hipStream_t s) {
  const dim3 grid = split_mode_grid(MODE, RB, B, g.on);
  hipLaunchKernelGGL((conv3d_region_split_kernel<MODE, CI, CO, RB>), grid, dim3(kBlock), 0, s, x, x2,
                     reinterpret_cast<const h8v*>(wf), w_exp, y, sc, sh, mu, g, xb, xb2, yb);
}

// ---- stride-1 convolutions with LDS-staged operands (conv_k_1; model.py:104-113) ----
// The per-lane kernel above fetches every input voxel once per tap through L1 (27x): for the
// 16-channel conv_1_1 that operand traffic, not the MFMA, sets its time.  Here a workgroup (4 waves)
// owns a 16 (x) x 4 (y) x TZ (z) block of outputs; its input block, 18 x 6 x (TZ + 2) voxels with
// all CI channels, is loaded once, split into fp16 hi / lo and stored in LDS (one record per voxel:
// CI hi then CI lo values, 16-byte chunks XOR-swizzled by voxel so the 16 lanes of an MFMA row group,
// 16 consecutive voxels, hit 16 distinct bank groups).  Wave w owns column block w % NB (16 output
// channels) and 8 row blocks (16 x-voxels each, one (z, y) row of the tile): every weight fragment
// (global / L2) feeds 8 row blocks, every A fragment comes from LDS.  Same products, same K order as
// the per-lane kernel (taps, then channel blocks; tap pairs for CI = 16): bit-equal outputs.
template <int CI>
struct S1Tile {
  static constexpr int TZ = CI == 16 ? 8 : (CI == 32 ? 4 : 2);
  static constexpr int PX = 18, PY = 6, PZ = TZ + 2, PV = PX * PY * PZ;
  static constexpr int REC = CI * 4;     // bytes per voxel record (CI hi + CI lo fp16)
  static constexpr int NCH = REC / 16;   // 16-byte chunks per record: 4, 8, 16
  static constexpr int LDS = PV * REC;   // 69,120 / 82,944 / 110,592 B
};

template <int CI>
__device__ inline int s1_chunk_off(int v, int c) {
  using T = S1Tile<CI>;
  return v * T::REC + ((c ^ ((v / (16 / T::NCH)) % T::NCH)) << 4);
}

template <int CI, int CO>
__global__ __launch_bounds__(kBlock) void conv3d_s1_split_lds_kernel(
    const float* __restrict__ x, const h8v* __restrict__ wf, int w_exp, float* __restrict__ y,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift, const float* __restrict__ bn_mean,
    GeoS g, int tiles_x, int tiles_y, int tiles_z, const uint32_t* __restrict__ xb, uint32_t* __restrict__ yb) {
  using T = S1Tile<CI>;
  constexpr int NB = CO / 16;
  constexpr int RB = 8;                      // row blocks per wave: 4 y x TZ z rows / (4 / NB) row groups
  static_assert(T::TZ * NB == RB && CI == CO, "tile shapes");
  constexpr bool PAIR = CI == 16;
  constexpr int CB = PAIR ? 1 : CI / 32;
  constexpr int KB = PAIR ? 14 : 27 * CB;
  __shared__ __attribute__((aligned(16))) char lds[T::LDS];

  int t = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (t >= tiles_x * tiles_y * tiles_z) return;   // workgroup-uniform, before the barriers
  const int t0 = t;
  const int tx0 = (t % tiles_x) * 16;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * 4;
  t /= tiles_y;
  const int tz0 = t * T::TZ;
  const int b = (int)blockIdx.y;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  // the input's scale; with the folded BN + ReLU (g.in_bn: train mode's conv_k_0 outputs) a bound of
  // relu(BN(v)) over |v| <= bound(x), one channel per lane
  float bound = bound_read(xb);
  if (g.in_bn) {
    float r = 0.0f;
    if (lane < CI) {
      const float sc = g.in_bn[lane], sh = g.in_bn[CI + lane], mu = g.in_bn[2 * CI + lane];
      r = fmaxf(fmaxf((bound - mu) * sc, (-bound - mu) * sc) + sh, 0.0f);
    }
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) r = fmaxf(r, __shfl_xor(r, k));
    bound = r;
  }
  const int ex = act_split_exponent(bound);

  // ---- stage the input block: items (voxel, channel quad), quad fastest (coalesced channels-last
  // loads); voxels outside the input region are zeros (the convolution's zero padding) ----
  {
    constexpr int NQ = CI / 4, NIT = T::PV * NQ, PER = (NIT + kBlock - 1) / kBlock;
    const size_t rvol = (size_t)g.in[0] * g.in[1] * g.in[2];
    const Rsrc rs = make_rsrc(x + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
    constexpr int BATCH = 8;
    // folded BN: the thread's quad q = tid % NQ is the same for all its items (kBlock % NQ == 0)
    static_assert(kBlock % NQ == 0, "one quad per thread");
    f4v bsc, bsh, bmu;
    if (g.in_bn) {
      const int c = 4 * (tid % NQ);
      bsc = *reinterpret_cast<const f4v*>(g.in_bn + c);
      bsh = *reinterpret_cast<const f4v*>(g.in_bn + CI + c);
      bmu = *reinterpret_cast<const f4v*>(g.in_bn + 2 * CI + c);
    }
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += BATCH) {
      f4v v4[BATCH];
      bool okk[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        const int q = e % NQ, v = e / NQ;
        const int px = v % T::PX, py = (v / T::PX) % T::PY, pz = v / (T::PX * T::PY);
        const int rx = g.o0[2] + tx0 - 1 + px - g.i0[2], ry = g.o0[1] + ty0 - 1 + py - g.i0[1],
                  rz = g.o0[0] + tz0 - 1 + pz - g.i0[0];
        const bool ok = k0 + k < PER && e < NIT && rx >= 0 && rx < g.in[2] && ry >= 0 && ry < g.in[1] && rz >= 0 &&
                        rz < g.in[0];
        const uint32_t off = ok ? (uint32_t)((((size_t)rz * g.in[1] + ry) * g.in[2] + rx) * CI + 4 * q) * 4u : kOob;
        v4[k] = ld4(rs, off, 0);
        okk[k] = ok;
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        if (k0 + k >= PER || e >= NIT) continue;
        const int q = e % NQ, v = e / NQ;
        uint2 hi, lo;
        f4v a = v4[k];
        if (g.in_bn && okk[k]) {   // in-region voxels only: the zero padding stays zero
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) a[jj] = fmaxf((a[jj] - bmu[jj]) * bsc[jj] + bsh[jj], 0.0f);
        }
        split4(a, ex, hi, lo);
        *reinterpret_cast<uint2*>(lds + s1_chunk_off<CI>(v, q >> 1) + ((q & 1) << 3)) = hi;
        *reinterpret_cast<uint2*>(lds + s1_chunk_off<CI>(v, CI / 8 + (q >> 1)) + ((q & 1) << 3)) = lo;
      }
    }
  }
  __syncthreads();

  // ---- this wave: column block nb, row blocks rg * 8 .. + 7 of the tile's 4 TZ (z, y) rows ----
  const int nb = wave % NB, rg = wave / NB;
  f4v acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[r] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  // weight fragments (L2) one K block ahead: kb + 1's loads are in flight under kb's MFMAs
  auto ldb = [&](int kb, h8v& bhi, h8v& blo) {
    bhi = wf[((size_t)(kb * NB + nb) * 2 + 0) * 64 + lane];
    blo = wf[((size_t)(kb * NB + nb) * 2 + 1) * 64 + lane];
  };
  auto kstep = [&](int kb, const h8v& bhi, const h8v& blo) {
    int tap, c0;
    if constexpr (PAIR) {
      tap = 2 * kb + (kq >> 1);
      c0 = kq & 1;
    } else {
      tap = kb / CB;
      c0 = (kb % CB) * 4 + kq;
    }
    const int tz = tap / 9, ty = (tap / 3) % 3, tx = tap % 3;
    const bool tap_ok = !PAIR || tap < 27;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int rbi = rg * RB + r, zz = rbi >> 2, yy = rbi & 3;
      const int v = ((zz + tz) * T::PY + (yy + ty)) * T::PX + (m + tx);
      h8v ahi = *reinterpret_cast<const h8v*>(lds + s1_chunk_off<CI>(v, c0));
      h8v alo = *reinterpret_cast<const h8v*>(lds + s1_chunk_off<CI>(v, CI / 8 + c0));
      if (!tap_ok) ahi = alo = h8v{0, 0, 0, 0, 0, 0, 0, 0};
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bhi, acc[r], 0, 0, 0);
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc[r], 0, 0, 0);
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bhi, acc[r], 0, 0, 0);
    }
  };
  h8v bh0, bl0, bh1, bl1;
  ldb(0, bh0, bl0);
#pragma unroll 1
  for (int kb = 0; kb < KB; kb += 2) {
    if (kb + 1 < KB) ldb(kb + 1, bh1, bl1);
    kstep(kb, bh0, bl0);
    if (kb + 1 < KB) {
      if (kb + 2 < KB) ldb(kb + 2, bh0, bl0);
      kstep(kb + 1, bh1, bl1);
    }
  }

  // ---- epilogue: acc[r][i] = (x = 4 kq + i, channel nb * 16 + m) of row block r ----
  const int oexp = -(ex + w_exp);
  const int co = nb * 16 + m;
  const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
              mu = bn_scale ? bn_mean[co] : 0.0f;
  const size_t orvol = (size_t)g.sbn[0] * g.sbn[1] * g.sbn[2];
  float vmax = 0.0f;
  double ss[1] = {0.0}, sq[1] = {0.0};
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int rbi = rg * RB + r, zz = rbi >> 2, yy = rbi & 3;
    if (tz0 + zz >= g.on[0] || ty0 + yy >= g.on[1]) continue;
    // store-box-relative coordinates
    const int vz = g.o0[0] + tz0 + zz - g.sb0[0], vy = g.o0[1] + ty0 + yy - g.sb0[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (tx0 + 4 * kq + i >= g.on[2]) continue;
      const int vx = g.o0[2] + tx0 + 4 * kq + i - g.sb0[2];
      float v = ldexpf(acc[r][i], oexp);
      if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
      const bool keep = vz >= 0 && vz < g.sbn[0] && vy >= 0 && vy < g.sbn[1] && vx >= 0 && vx < g.sbn[2];
      const size_t vox = ((size_t)vz * g.sbn[1] + vy) * g.sbn[2] + vx;
      const size_t oi = g.out_cf ? ((size_t)b * CO + co) * orvol + vox : ((size_t)b * orvol + vox) * CO + co;
      if (g.addend && keep) v += g.addend[oi];
      ss[0] += (double)v;
      sq[0] += (double)v * (double)v;
      if (!keep) continue;
      vmax = fmaxf(vmax, fabsf(v));
      y[oi] = v;
    }
  }
  if (yb) bound_update(yb, vmax);
  if (g.stats) {
    const size_t slot = (size_t)b * (tiles_x * tiles_y * tiles_z) + t0;
    stats_write<CO, 1, kBlock / 64>(ss, sq, nb, 1, g.stats + slot * 2 * CO);
  }
}

template <int CI>
void s1_lds_tiles(const int* on, int& tx, int& ty, int& tz) {
  tx = (on[2] + 15) / 16;
  ty = (on[1] + 3) / 4;
  tz = (on[0] + S1Tile<CI>::TZ - 1) / S1Tile<CI>::TZ;
}

template <int CI>
void launch_s1_lds(const float* x, const void* wf, int w_exp, float* y, const float* sc, const float* sh,
                   const float* mu, int B, const GeoS& g, const uint32_t* xb, uint32_t* yb, hipStream_t s) {
  int tx, ty, tz;
  s1_lds_tiles<CI>(g.on, tx, ty, tz);
  const int per = tx * ty * tz;
  const dim3 grid((unsigned)((per + 7) / 8 * 8), (unsigned)B);
  hipLaunchKernelGGL((conv3d_s1_split_lds_kernel<CI, CI>), grid, dim3(kBlock), 0, s, x,
                     reinterpret_cast<const h8v*>(wf), w_exp, y, sc, sh, mu, g, tx, ty, tz, xb, yb);
}

// ---- transposed convolutions over large output regions with LDS-staged operands (train mode's
// deconv_3_0 / deconv_2_0 over the full volume, model.py:117-120) ----
// A workgroup owns a TX x 8 x 4 block of outputs of ALL eight parity classes; every output of it reads
// inputs i = (o + P - t) / 2 from one (TX / 2 + 1) x 5 x 3 input block, which is loaded once, split and
// stored in LDS as S1Tile's swizzled records (the per-lane kernel re-reads each input voxel through
// L1 for every (output, tap) pair: 27 times).  The four waves share each class: wave w owns row blocks
// 2 TXB w .. + 2 TXB - 1 of the class's 8 TXB (16 consecutive class outputs along x each) and all its
// column blocks; classes run one after another (taps of class (pz, py, px): 2 per dim of parity 0, 1
// of parity 1 -- 27 over the eight).  Same products and K order as the per-lane kernel (taps, then
// channel blocks): bit-equal outputs.
// (the K block's weight fragments staged in LDS once per workgroup, as the 3-in-1 S2 does: train-mode
// step 12.0 -> 12.4 ms -- a barrier per K block of a class with 1-8 taps; dropped)
// MVS_T2_TYB: class rows along y per tile / 4 (2: a 32 x 16 x 4 tile, 4 row blocks per wave, one
// workgroup per CU: train-mode step 14.1 -> 15.5 ms; the LDS kernel on eval's small regions: eval step
// 3.95 -> 4.24 ms, hence kT2LdsMinVoxels)
#ifndef MVS_T2_TYB
#define MVS_T2_TYB 1
#endif
template <int CI, int TXB, int TYB = MVS_T2_TYB>
struct T2Tile {
  static constexpr int TX = 32 * TXB, TY = 8 * TYB, TZ = 4;
  static constexpr int PX = TX / 2 + 1, PY = TY / 2 + 1, PZ = TZ / 2 + 1, PV = PX * PY * PZ;
  static constexpr int REC = CI * 4, NCH = REC / 16;
  static constexpr int LDS = PV * REC;
  __device__ static int chunk_off(int v, int c) { return v * REC + ((c ^ ((v / (16 / NCH)) % NCH)) << 4); }
};

template <int CI, int CO, int TXB>
__global__ __launch_bounds__(kBlock) void conv3d_t2_split_lds_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const h8v* __restrict__ wf, int w_exp,
    float* __restrict__ y, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, GeoS g, int tiles_x, int tiles_y, int tiles_z, const uint32_t* __restrict__ xb,
    const uint32_t* __restrict__ xb2, uint32_t* __restrict__ yb) {
  using T = T2Tile<CI, TXB>;
  constexpr int NB = CO / 16, CB = CI / 32, RB = 2 * TXB * MVS_T2_TYB;
  constexpr int NYC = 4 * MVS_T2_TYB;   // class rows along y
  static_assert(CI % 32 == 0 && CO % 16 == 0, "channel counts");
  __shared__ __attribute__((aligned(16))) char lds[T::LDS];

  int t = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (t >= tiles_x * tiles_y * tiles_z) return;   // workgroup-uniform, before the barriers
  const int t0 = t;
  // tile origin (absolute output coordinates)
  const int X0 = g.o0[2] + (t % tiles_x) * T::TX;
  t /= tiles_x;
  const int Y0 = g.o0[1] + (t % tiles_y) * T::TY;
  t /= tiles_y;
  const int Z0 = g.o0[0] + t * T::TZ;
  const int b = (int)blockIdx.y;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  // the input's scale: with the folded BN + ReLU a bound of relu(BN(v)) over |v| <= bound(x) per channel
  // (the larger of the two ends), over the channels; + the same for x2
  float bound = bound_read(xb), bound2 = x2 ? bound_read(xb2) : 0.0f;
  if (g.in_bn) {
    static_assert(CI <= 64, "one channel per lane");
    auto bn_bound = [&](float bx, int o) {   // lane c: channel c, then the wave's max (whole wave)
      float r = 0.0f;
      if (lane < CI) {
        const float sc = g.in_bn[o * CI + lane], sh = g.in_bn[(o + 1) * CI + lane], mu = g.in_bn[(o + 2) * CI + lane];
        r = fmaxf(fmaxf((bx - mu) * sc, (-bx - mu) * sc) + sh, 0.0f);
      }
#pragma unroll
      for (int k = 32; k > 0; k >>= 1) r = fmaxf(r, __shfl_xor(r, k));
      return r;
    };
    bound = bn_bound(bound, 0);
    if (x2) bound2 = bn_bound(bound2, 3);
  }
  const int ex = act_split_exponent(bound + bound2);
  // the input block's origin (absolute input coordinates): the smallest (o + P - t) / 2
  const int ilz = (Z0 + g.pad[0] - 1) >> 1, ily = (Y0 + g.pad[1] - 1) >> 1, ilx = (X0 + g.pad[2] - 1) >> 1;

  // ---- stage the input block: items (voxel, channel quad), quad fastest; outside the input region:
  // zeros (inputs that reach no output of the region) ----
  {
    constexpr int NQ = CI / 4, NIT = T::PV * NQ, PER = (NIT + kBlock - 1) / kBlock, BATCH = 8;
    const size_t rvol = (size_t)g.in[0] * g.in[1] * g.in[2];
    const Rsrc rs = make_rsrc(x + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
    const Rsrc rs2 = make_rsrc(x2 ? x2 + (size_t)b * rvol * CI : x, x2 ? (uint32_t)(rvol * CI * 4) : 0u);
    // relu(BN(v)) per channel of the thread's quad (in-region voxels only: the rest stays the zero it
    // reads as).  kBlock is a multiple of NQ, so a thread's quad q = tid % NQ is the same for all its
    // items: its 4 channels' parameters are loaded once
    static_assert(kBlock % NQ == 0, "one quad per thread");
    f4v bsc[2], bsh[2], bmu[2];
    if (g.in_bn) {
      const int c = 4 * (tid % NQ);
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        bsc[o] = *reinterpret_cast<const f4v*>(g.in_bn + (3 * o) * CI + c);
        bsh[o] = *reinterpret_cast<const f4v*>(g.in_bn + (3 * o + 1) * CI + c);
        bmu[o] = *reinterpret_cast<const f4v*>(g.in_bn + (3 * o + 2) * CI + c);
      }
    }
    auto bn4 = [&](f4v v, int, int o) {
      const int k = o / 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf((v[j] - bmu[k][j]) * bsc[k][j] + bsh[k][j], 0.0f);
      return v;
    };
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += BATCH) {
      f4v v4[BATCH], w4[BATCH];
      bool okk[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        const int q = e % NQ, v = e / NQ;
        const int px = v % T::PX, py = (v / T::PX) % T::PY, pz = v / (T::PX * T::PY);
        const int rx = ilx + px - g.i0[2], ry = ily + py - g.i0[1], rz = ilz + pz - g.i0[0];
        const bool ok = k0 + k < PER && e < NIT && rx >= 0 && rx < g.in[2] && ry >= 0 && ry < g.in[1] && rz >= 0 &&
                        rz < g.in[0];
        const uint32_t off = ok ? (uint32_t)((((size_t)rz * g.in[1] + ry) * g.in[2] + rx) * CI + 4 * q) * 4u : kOob;
        okk[k] = ok;
        v4[k] = ld4(rs, off, 0);
        if (x2) w4[k] = ld4(rs2, off, 0);
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        if (k0 + k >= PER || e >= NIT) continue;
        const int q = e % NQ, v = e / NQ;
        f4v a = v4[k];
        if (g.in_bn && okk[k]) a = bn4(a, q, 0);
        if (x2) a += (g.in_bn && okk[k]) ? bn4(w4[k], q, 3) : w4[k];
        uint2 hi, lo;
        split4(a, ex, hi, lo);
        *reinterpret_cast<uint2*>(lds + T::chunk_off(v, q >> 1) + ((q & 1) << 3)) = hi;
        *reinterpret_cast<uint2*>(lds + T::chunk_off(v, CI / 8 + (q >> 1)) + ((q & 1) << 3)) = lo;
      }
    }
  }
  __syncthreads();

  const int oexp = -(ex + w_exp);
  const size_t orvol = (size_t)g.sbn[0] * g.sbn[1] * g.sbn[2];
  float vmax = 0.0f;
  double ss[NB], sq[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) ss[nb] = sq[nb] = 0.0;
  auto ldb = [&](int kb, h8v (&bh)[NB], h8v (&bl)[NB]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      bh[nb] = wf[((size_t)(kb * NB + nb) * 2 + 0) * 64 + lane];
      bl[nb] = wf[((size_t)(kb * NB + nb) * 2 + 1) * 64 + lane];
    }
  };

#pragma unroll 1
  for (int cls = 0; cls < 8; ++cls) {
    const int pz = (cls >> 2) & 1, py = (cls >> 1) & 1, px = cls & 1;
    // the class's first output per dim inside the tile: (o + P) of parity par
    const int fz = Z0 + (((Z0 + g.pad[0]) & 1) != pz ? 1 : 0), fy = Y0 + (((Y0 + g.pad[1]) & 1) != py ? 1 : 0),
              fx = X0 + (((X0 + g.pad[2]) & 1) != px ? 1 : 0);
    // input block coordinates of (o + P - par) / 2 for the class's first output
    const int bz = ((fz + g.pad[0] - pz) >> 1) - ilz, by = ((fy + g.pad[1] - py) >> 1) - ily,
              bx = ((fx + g.pad[2] - px) >> 1) - ilx;
    const int ntz = 2 - pz, nty = 2 - py, ntx = 2 - px, nk = ntz * nty * ntx * CB;
    f4v acc[RB][NB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[r][nb] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
    // K block k of the class: taps (tz, ty, tx) with t = par + 2 j, j < nt, then channel blocks
    auto tap_of = [&](int k, int& tap, int& cb, int& dz, int& dy, int& dx) {
      cb = k % CB;
      int j = k / CB;
      const int jx = j % ntx;
      j /= ntx;
      const int jy = j % nty, jz = j / nty;
      const int tz = pz + 2 * jz, ty = py + 2 * jy, tx = px + 2 * jx;
      tap = (tz * 3 + ty) * 3 + tx;
      dz = -jz;   // input offset -(t >> 1)
      dy = -jy;
      dx = -jx;
    };
    auto kstep = [&](int k, const h8v (&bh)[NB], const h8v (&bl)[NB]) {
      int tap, cb, dz, dy, dx;
      tap_of(k, tap, cb, dz, dy, dx);
      const int c0 = cb * 4 + kq;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int rbi = wave * RB + r;                       // (z_c, y_c, xb) of the class's row blocks
        const int xbk = rbi % TXB, yc = (rbi / TXB) % NYC, zc = rbi / (NYC * TXB);
        const int v = ((bz + zc + dz) * T::PY + (by + yc + dy)) * T::PX + (bx + xbk * 16 + m + dx);
        const h8v ahi = *reinterpret_cast<const h8v*>(lds + T::chunk_off(v, c0));
        const h8v alo = *reinterpret_cast<const h8v*>(lds + T::chunk_off(v, CI / 8 + c0));
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bh[nb], acc[r][nb], 0, 0, 0);
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bl[nb], acc[r][nb], 0, 0, 0);
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[nb], acc[r][nb], 0, 0, 0);
        }
      }
    };
    h8v bh0[NB], bl0[NB], bh1[NB], bl1[NB];
    {
      int tap, cb, dz, dy, dx;
      tap_of(0, tap, cb, dz, dy, dx);
      ldb(tap * CB + cb, bh0, bl0);
    }
#pragma unroll 1
    for (int k = 0; k < nk; k += 2) {
      if (k + 1 < nk) {
        int tap, cb, dz, dy, dx;
        tap_of(k + 1, tap, cb, dz, dy, dx);
        ldb(tap * CB + cb, bh1, bl1);
      }
      kstep(k, bh0, bl0);
      if (k + 1 < nk) {
        if (k + 2 < nk) {
          int tap, cb, dz, dy, dx;
          tap_of(k + 2, tap, cb, dz, dy, dx);
          ldb(tap * CB + cb, bh0, bl0);
        }
        kstep(k + 1, bh1, bl1);
      }
    }
    // ---- the class's outputs: acc[r][nb][i] = (class output x index xbk * 16 + 4 kq + i of row r,
    // channel nb * 16 + m) ----
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co = nb * 16 + m;
      const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
                  mu = bn_scale ? bn_mean[co] : 0.0f;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int rbi = wave * RB + r;
        const int xbk = rbi % TXB, yc = (rbi / TXB) % NYC, zc = rbi / (NYC * TXB);
        const int oz = fz + 2 * zc, oy = fy + 2 * yc;
        if (oz >= min(Z0 + T::TZ, g.o0[0] + g.on[0]) || oy >= min(Y0 + T::TY, g.o0[1] + g.on[1])) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ox = fx + 2 * (xbk * 16 + 4 * kq + i);
          if (ox >= min(X0 + T::TX, g.o0[2] + g.on[2])) continue;
          float v = ldexpf(acc[r][nb][i], oexp);
          if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
          const int vz = oz - g.sb0[0], vy = oy - g.sb0[1], vx = ox - g.sb0[2];
          const bool keep = vz >= 0 && vz < g.sbn[0] && vy >= 0 && vy < g.sbn[1] && vx >= 0 && vx < g.sbn[2];
          const size_t vox = ((size_t)vz * g.sbn[1] + vy) * g.sbn[2] + vx;
          const size_t oi = g.out_cf ? ((size_t)b * CO + co) * orvol + vox : ((size_t)b * orvol + vox) * CO + co;
          if (g.addend && keep) v += g.addend[oi];
          ss[nb] += (double)v;
          sq[nb] += (double)v * (double)v;
          if (!keep) continue;
          vmax = fmaxf(vmax, fabsf(v));
          y[oi] = v;
        }
      }
    }
  }
  if (yb) bound_update(yb, vmax);
  if (g.stats) {
    const size_t slot = (size_t)b * (tiles_x * tiles_y * tiles_z) + t0;
    stats_write<CO, NB, kBlock / 64>(ss, sq, 0, NB, g.stats + slot * 2 * CO);
  }
}

template <int CI, int TXB>
void t2_lds_tiles(const int* on, int& tx, int& ty, int& tz) {
  using T = T2Tile<CI, TXB>;
  tx = (on[2] + T::TX - 1) / T::TX;
  ty = (on[1] + T::TY - 1) / T::TY;
  tz = (on[0] + T::TZ - 1) / T::TZ;
}

template <int CI, int CO, int TXB>
void launch_t2_lds(const float* x, const float* x2, const void* wf, int w_exp, float* y, const float* sc,
                   const float* sh, const float* mu, int B, const GeoS& g, const uint32_t* xb, const uint32_t* xb2,
                   uint32_t* yb, hipStream_t s) {
  int tx, ty, tz;
  t2_lds_tiles<CI, TXB>(g.on, tx, ty, tz);
  const int per = tx * ty * tz;
  const dim3 grid((unsigned)((per + 7) / 8 * 8), (unsigned)B);
  hipLaunchKernelGGL((conv3d_t2_split_lds_kernel<CI, CO, TXB>), grid, dim3(kBlock), 0, s, x, x2,
                     reinterpret_cast<const h8v*>(wf), w_exp, y, sc, sh, mu, g, tx, ty, tz, xb, xb2, yb);
}

}  // namespace

int conv3d_region_split_kblocks(int c_in) { return c_in == 16 ? 14 : 27 * (c_in / 32); }

// bit 0 / 1 / 2: the LDS-staged kernel for 16 / 32 / 64 channels.  Measured per cfg-2 step (eval /
// train mode): 16 ch 0.37 -> 0.27 / 0.35 -> 0.26 ms, 32 ch 0.18 -> 0.17 / 0.97 -> 0.93 ms; 64 ch slower
// (0.11 -> 0.13 / 2.41 -> 2.81 ms: its 110 KB tile allows one workgroup per CU).  An LDS-staged
// transposed kernel (one 17 x 5 x (TZ + 1) block per parity-class tile) measured no gain (0.31 ->
// 0.34 ms): a class reads each input voxel through 1-8 taps only.
#ifndef MVS_S1_LDS
#define MVS_S1_LDS 3
#endif
static bool split_uses_lds(int mode, int CI, int CO, bool per_lane, bool has_x2) {
  const int ci_bit = CI == 16 ? 1 : (CI == 32 ? 2 : (CI == 64 ? 4 : 0));
  return (MVS_S1_LDS & ci_bit) && !per_lane && mode == kS1 && CI == CO && !has_x2;
}

// row blocks per wave of the per-lane kernel: 4 for the stride-1 convs (each weight fragment feeds 4 row
// blocks), 2 for the transposed and stride-2 ones (measured at cfg 2, eval and train mode: S1 64 -> 64
// 2.70 -> 2.41 ms, T2 32 -> 16 2.02 against 2.36 with 4; 1 row block is slower everywhere)
// The stride-1 kernel without LDS weights drops to 2 row blocks when 4 would leave fewer than kS1WideWgs
// workgroups: eval's deep-level regions are small (conv_3_1 at cfg 2: 3.97 -> 3.87 ms per eval step with
// 2), train mode's are large (4 measured best there: 15.3 against 15.5 ms per train-mode step).  With its
// weights in LDS (64 channels, MVS_S1_BLDS) it always takes 2.  S2 with 1 / 4 row blocks: eval 4.01 /
// 4.11 ms, train 15.9 / 15.5 ms (tools/gpu_r5_bound_ab.sh r5rb).
constexpr long kS1WideWgs = 4096;
// row blocks of the 3-in-1 S2 (kS2Multi): 4 measured slower (300 registers, one wave per SIMD: train-mode
// step 12.9 -> 13.1 ms)
#ifndef MVS_S2M_RB
#define MVS_S2M_RB 2
#endif
static int split_rb(int mode, int B, const int* on, int CO) {
  if (mode == kS2 && CO == kS2Multi) return MVS_S2M_RB;
  if (mode == kS1 && CO == 64 && MVS_S1_BLDS) return 2;
  if (mode != kS1) return 2;
  const long rows = (long)B * on[0] * on[1] * on[2];
  return rows >= kS1WideWgs * (kBlock / 64) * 16 * 4 ? 4 : 2;
}

// The LDS-staged transposed kernel for large output regions (train mode's full volumes: T2 64 -> 32
// 2.41 -> 1.45 ms, 32 -> 16 1.10 -> 0.73 ms); MVS_T2_LDS=0 / 2 forces the per-lane / LDS kernel (A/B
// and tests)
constexpr long kT2LdsMinVoxels = 1l << 22;
static bool split_t2_lds(int mode, int B, int CI, int CO, const int* on, bool per_lane, bool has_x2,
                         bool in_bn = false) {
  if (mode != kT2 || !((CI == 64 && CO == 32) || (CI == 32 && CO == 16))) return false;
  if (in_bn) return true;   // the folded input BN + ReLU: this kernel only
  const char* fe = getenv("MVS_T2_LDS");   // read per call: tests switch it
  const int force = fe ? atoi(fe) : 1;
  if (per_lane || force == 0) return false;
  return force == 2 || (long)B * on[0] * on[1] * on[2] >= kT2LdsMinVoxels;
}

long conv3d_region_split_slots(int mode, int B, int CI, int CO, const int* on, bool per_lane, bool has_x2,
                               bool in_bn) {
  if (split_t2_lds(mode, B, CI, CO, on, per_lane, has_x2, in_bn)) {
    int tx, ty, tz;
    if (CI == 64) t2_lds_tiles<64, 1>(on, tx, ty, tz);
    else t2_lds_tiles<32, 2>(on, tx, ty, tz);
    return (long)B * tx * ty * tz;
  }
  if (split_uses_lds(mode, CI, CO, per_lane, has_x2)) {
    int tx, ty, tz;
    if (CI == 16) s1_lds_tiles<16>(on, tx, ty, tz);
    else if (CI == 32) s1_lds_tiles<32>(on, tx, ty, tz);
    else s1_lds_tiles<64>(on, tx, ty, tz);
    return (long)B * tx * ty * tz;
  }
  const dim3 gr = split_mode_grid(mode, split_rb(mode, B, on, CO), B, on);
  return (long)gr.x * gr.y * gr.z;
}

int launch_conv3d_region_split(int mode, bool out_cf, const float* x, const float* x2, const void* wfrag, int w_exp,
                               float* y, int B, int CI, int CO, const int* n, const int* o0, const int* on,
                               const int* i0, const int* in, const int* pad, const float* bn_scale,
                               const float* bn_shift, const float* bn_mean, const uint32_t* x_bound,
                               const uint32_t* x2_bound, uint32_t* y_bound, hipStream_t s, bool per_lane,
                               const float* y_addend, const int* store_origin, const int* store_size,
                               double* stats, float* y_mid, float* y_high, const float* in_bn) {
  GeoS g;
  g.in_bn = in_bn;
  g.ym[0] = y_mid;
  g.ym[1] = y_high;
  if ((CO == kS2Multi) != (y_mid != nullptr) || (y_mid != nullptr) != (y_high != nullptr) ||
      (CO == kS2Multi && (mode != kS2 || out_cf || y_addend)))
    return MVS_ERR_INVALID_ARGUMENT;
  g.out_cf = out_cf ? 1 : 0;
  g.addend = y_addend;
  g.stats = stats;
  for (int d = 0; d < 3; ++d) {
    g.n[d] = n[d];
    g.o0[d] = o0[d];
    g.on[d] = on[d];
    g.i0[d] = i0[d];
    g.in[d] = in[d];
    g.pad[d] = pad ? pad[d] : 1;
    g.sb0[d] = store_origin ? store_origin[d] : o0[d];
    g.sbn[d] = store_origin ? store_size[d] : on[d];
  }
#define MVS_RSPLIT_CASE(MD, A, C)                                                                          \
  if (mode == MD && CI == A && CO == C) {                                                                  \
    if (split_rb(mode, B, on, CO) == 4)                                                                    \
      launch_split_mode<MD, A, C, 4>(x, x2, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound,   \
                                     x2_bound, y_bound, s);                                                \
    else                                                                                                   \
      launch_split_mode<MD, A, C, 2>(x, x2, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound,   \
                                     x2_bound, y_bound, s);                                                \
    return MVS_OK;                                                                                         \
  }
  // S1: conv_k_1 (16 / 32 / 64 channels; LDS-staged operands per MVS_S1_LDS); T2: deconv_3_0 (64 -> 32),
  // deconv_2_0 (32 -> 16); S2: conv_k_0 from the split cost volume (32 -> 16 / 32 / 64)
  if (in_bn && !split_t2_lds(mode, B, CI, CO, on, per_lane, x2 != nullptr, true) &&
      !(split_uses_lds(mode, CI, CO, per_lane, x2 != nullptr) && CI <= 64))
    return MVS_ERR_INVALID_ARGUMENT;   // the folded input BN: the LDS-staged kernels only
  if (split_t2_lds(mode, B, CI, CO, on, per_lane, x2 != nullptr, in_bn != nullptr)) {
    if (CI == 64)
      launch_t2_lds<64, 32, 1>(x, x2, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound, x2_bound, y_bound, s);
    else
      launch_t2_lds<32, 16, 2>(x, x2, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound, x2_bound, y_bound, s);
    return MVS_OK;
  }
  if (split_uses_lds(mode, CI, CO, per_lane, x2 != nullptr)) {
    if (CI == 16) launch_s1_lds<16>(x, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound, y_bound, s);
    else if (CI == 32) launch_s1_lds<32>(x, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound, y_bound, s);
    else launch_s1_lds<64>(x, wfrag, w_exp, y, bn_scale, bn_shift, bn_mean, B, g, x_bound, y_bound, s);
    return MVS_OK;
  }
  MVS_RSPLIT_CASE(kS1, 16, 16) MVS_RSPLIT_CASE(kS1, 32, 32) MVS_RSPLIT_CASE(kS1, 64, 64)
  MVS_RSPLIT_CASE(kS2, 32, 16) MVS_RSPLIT_CASE(kS2, 32, 32) MVS_RSPLIT_CASE(kS2, 32, 64)
  MVS_RSPLIT_CASE(kS2, 32, kS2Multi)
  MVS_RSPLIT_CASE(kT2, 64, 32) MVS_RSPLIT_CASE(kT2, 32, 16)
#undef MVS_RSPLIT_CASE
  return MVS_ERR_INVALID_ARGUMENT;
}

}  // namespace mvs
