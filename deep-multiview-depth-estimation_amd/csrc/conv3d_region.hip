// conv3d_region.hip -- the regulariser's region convolutions (CostVolumeReg, model.py:76-95, forward
// at model.py:101-121) as implicit GEMMs on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact
// fp32, one rounding per product, the f32 VALU's peak rate without its operand traffic), with the
// eval-mode BatchNorm + ReLU that follows every one of them fused into the epilogue.
//
// forward_live evaluates the U-Net level k only on its live region.  The region
// tensors live channels-last, x[b][z][y][x][c] (NDHWC, the GEMM's K = channel axis contiguous),
// with their box origin (o0) in the volume; three forms:
//   S1  conv_k_1:     3x3x3, stride 1, padding 1 (zero outside the VOLUME), region -> region
//   S2  conv_k_0:     3x3x3, stride 2, padding P (config.py:20), the full cost volume (NCDHW, or
//                     the fused kernel's channel-quad NC4DHW4: 4 channels per 16-byte load) ->
//                     region: output o reads inputs 2 o - P + t, t = 0..2, per dim
//   T2  deconv_k_0:   ConvTranspose3d 3x3x3, stride 2, padding P, region -> region: output o
//                     gathers inputs i = (o + P - t) / 2 for t of o + P's parity (1 or 2 taps per
//                     dim); outputs are processed by parity class (8 launches' worth of grid.y), so
//                     every voxel of a 16-voxel MFMA row block has the same taps; the input may be
//                     the sum of two region tensors (model.py:119-121's `y3 + y2`, `y2 + y1`).
// GEMM per sample: rows = output voxels of the region (flattened z, y, x; parity class for T2),
// columns = output channels, K = (tap, input channel).  A wave owns 2 x 16 rows and every column
// block (CO / 16); per (tap, 16-channel block) each lane loads 4 consecutive channels of its row's
// input voxel (channels-last: one 16-byte load; S2 reads the NCDHW volume per channel) and of its
// column's weights, which feed 4 MFMAs (K-step s takes component s).  Weights arrive as
// w[tap][co][ci] (ops.py transposes nn.Conv3d / nn.ConvTranspose3d's layouts).  Products are summed
// per tap over channels in a fixed order -- MIOpen's kernels sum in other orders; same products,
// fp32 rounding-level differences.
#include "launchers.h"
#include "packed.h"
#include "split.h"

namespace mvs {
namespace {

typedef f4v f4v_t;
// out-of-range buffer offset for taps without input (the loads return 0); every descriptor built
// here covers less than 2^32 - 64 bytes (mvs_conv3d_region_fwd checks)
constexpr uint32_t kOob = 0xFFFFFFC0u;

// output voxels per wave: RB MFMA row blocks of 16 (template; 2 by default)

template <int MODE>
struct ConvMode {};
constexpr int kS1 = 0, kS2 = 1, kT2 = 2;

struct Geo {
  int n[3];     // volume dims (D, H, W)
  int o0[3];    // output region origin
  int on[3];    // output region size
  int i0[3];    // input region origin (S1, T2; S2: the box of the volume the input tensor holds)
  int in[3];    // input region size (S1, T2; S2: the box size, = n when the whole volume is given)
  int pad[3];   // P (S2, T2)
  int out_cf;   // 1: output region tensor channels-first y[b][co][z][y][x] (else channels-last)
  int in_c4;    // S2: the volume is channel-quad x[b][C/4][D][H][W][4], fp32 (1), bf16 (2) or the split
                //     cost volume (3, split.h: fp32 re-formed on load as (hi + lo) 2^-e); 0 NCDHW
  const uint32_t* absmax;   // in_c4 = 3: the volume's bound words (its scale)
  uint32_t* y_bound;        // optional: the output's bound words (split.h), raised in the epilogue
};

// T2 parity class: per dim, outputs o with (o + P) % 2 == par; first such o in the region and count
__device__ inline void class_dim(int o0, int on, int p, int par, int& first, int& cnt) {
  first = o0 + (((o0 + p) & 1) != par ? 1 : 0);
  cnt = first < o0 + on ? (o0 + on - 1 - first) / 2 + 1 : 0;
}

__device__ inline void store_out(float* __restrict__ y, const Geo& g, int b, int co, int vz, int vy, int vx,
                                 int CO, float v) {
  const size_t vox = ((size_t)vz * g.on[1] + vy) * g.on[2] + vx;
  const size_t rvol = (size_t)g.on[0] * g.on[1] * g.on[2];
  if (g.out_cf) y[((size_t)b * CO + co) * rvol + vox] = v;
  else y[((size_t)b * rvol + vox) * CO + co] = v;
}

// QM (S2 only): input layout of the volume -- 0 NCDHW, 1 fp32 channel quads, 2 bf16 channel quads --
// a template parameter, so the K loop has no per-load layout branches and (S1 / S2: no parity
// classes) unrolls into one basic block the scheduler can software-pipeline (loads of later taps
// issued under the MFMAs of earlier ones)
template <int MODE, int CI, int CO, int RB, int QM = 0>
__global__ __launch_bounds__(kBlock) void conv3d_region_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const float* __restrict__ w,
    float* __restrict__ y, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, Geo g) {
  constexpr int NB = CO / 16;          // column blocks
  static_assert(CI % 16 == 0 && CO % 16 == 0, "channel counts in multiples of 16");
  const int lane = (int)threadIdx.x & 63;
  const int m = lane & 15, kq = lane >> 4;   // MFMA row / K index of this lane's A value
  const int b = (int)blockIdx.z;

  // ---- rows of this wave: parity class (T2) or the whole region ----
  int cf[3], cn[3], par[3] = {0, 0, 0};
  if constexpr (MODE == kT2) {
    const int cls = (int)blockIdx.y;
    par[0] = (cls >> 2) & 1;
    par[1] = (cls >> 1) & 1;
    par[2] = cls & 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) class_dim(g.o0[d], g.on[d], g.pad[d], par[d], cf[d], cn[d]);
  } else {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      cf[d] = g.o0[d];
      cn[d] = g.on[d];
    }
  }
  const int rows = cn[0] * cn[1] * cn[2];
  const int sx = QM == 3 ? cv_split_exponent(g.absmax) : 0;
  const int step = MODE == kT2 ? 2 : 1;
  constexpr int kRows = 16 * RB;
  // XCD-contiguous row blocks (gridDim.x is a multiple of 8): workgroups are dealt round-robin over
  // the 8 XCDs, so without the remap the neighbours that share input rows / planes (the next output
  // row, the next plane ~ one row of workgroups later) sit in 8 different L2s; remapped, each XCD
  // sweeps a contiguous run of the region and re-reads them from its own L2
  const int bx = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  const int row0 = (bx * (kBlock / 64) + ((int)threadIdx.x >> 6)) * kRows;
  if (row0 >= rows) return;   // wave-uniform; no barriers in this kernel

  // per row block: this lane's input base voxel in the addressed space (the volume for S2, the
  // input region for S1 / T2) and, per dim and tap, whether the tap's input exists; input voxel of
  // tap t = base + delta(t) per dim with delta = t (S1, S2) or -(t >> 1) (T2, taps of the class's
  // parity: t = par, par + 2)
  int lim[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) lim[d] = g.in[d];
  int lin[RB];            // linear index of the base voxel (may be negative; masked)
  unsigned vm[RB][3];     // per dim: bit t = tap t's input exists
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
        const bool in = ok && bs[d] + dl >= 0 && bs[d] + dl < lim[d] && !(MODE == kT2 && ((tt & 1) != par[d]));
        mk |= in ? (1u << tt) : 0u;
      }
      vm[rb][d] = mk;
    }
    lin[rb] = (bs[0] * lim[1] + bs[1]) * lim[2] + bs[2];
  }

  f4v_t acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f4v_t{0.0f, 0.0f, 0.0f, 0.0f};

  // buffer descriptors (workgroup-uniform bases; out-of-range offsets read 0): S2 the sample's
  // volume (channel-quad: quads cb*4 .. cb*4+3 per channel block; NCDHW: 16 channel planes per
  // block), S1 / T2 the sample's region tensor (and addend)
  const size_t rvol = (size_t)g.in[0] * g.in[1] * g.in[2];
  const size_t nvol = rvol;   // S2: voxels of the (boxed) volume per channel plane / quad plane
  const int sy = lim[2], sz = lim[1] * lim[2];
  // ---- K loop: taps by rows (tz, ty); per row and 16-channel block the A values of its (up to)
  // three x taps and every row block and the matching weights are loaded together, then fed to
  // the MFMAs (3x the loads in flight of a tap-at-a-time loop) ----
#pragma unroll
  for (int tz = 0; tz < 3; ++tz) {
    if (MODE == kT2 && ((tz & 1) != par[0])) continue;   // t of o + P's parity only
#pragma unroll
    for (int ty = 0; ty < 3; ++ty) {
      if (MODE == kT2 && ((ty & 1) != par[1])) continue;
      const int dz = MODE == kT2 ? -(tz >> 1) : tz, dy = MODE == kT2 ? -(ty >> 1) : ty;
      // input voxel of this lane's row per (x tap, row block); kOob = no input (reads 0)
      uint32_t vox[3][RB];
#pragma unroll
      for (int tx = 0; tx < 3; ++tx)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const int dx = MODE == kT2 ? -(tx >> 1) : tx;
          const bool ok = ((vm[rb][0] >> tz) & (vm[rb][1] >> ty) & (vm[rb][2] >> tx) & 1u) != 0;
          vox[tx][rb] = ok ? (uint32_t)(lin[rb] + dz * sz + dy * sy + dx) : kOob;
        }
      // K = each tap's CI channels in blocks of 16: in K-step s of block cb, lane (m, kq) supplies
      // channel cb * 16 + 4 kq + s -- one 16-byte load per lane (4 consecutive channels of its row's
      // voxel, channels-last; of its column's weight row, w[tap][co][ci]) feeds 4 MFMAs
#pragma unroll
      for (int cb = 0; cb < CI / 16; ++cb) {
        const int c4 = cb * 16 + kq * 4;
        Rsrc rs, rs2;
        if constexpr (MODE == kS2) {
          if constexpr (QM == 2)   // bf16 quads: 8 bytes per voxel and quad
            rs = make_rsrc(reinterpret_cast<const char*>(x) + ((size_t)b * (CI / 4) + cb * 4) * nvol * 8,
                           (uint32_t)(nvol * 32));
          else if constexpr (QM == 1 || QM == 3)
            rs = make_rsrc(x + ((size_t)b * (CI / 4) + cb * 4) * nvol * 4, (uint32_t)(nvol * 64));
          else
            rs = make_rsrc(x + ((size_t)b * CI + cb * 16) * nvol, (uint32_t)(nvol * 64));
        } else {
          rs = make_rsrc(x + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
          if (x2) rs2 = make_rsrc(x2 + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
        }
        f4v_t a[3][RB], bw[3][NB];
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          if (MODE == kT2 && ((tx & 1) != par[2])) continue;
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            const uint32_t vx = vox[tx][rb];
            f4v_t v;
            if constexpr (MODE == kS2) {
              if constexpr (QM == 2) {   // the bf16 quad: one 8-byte load, widened (exact)
                typedef __attribute__((ext_vector_type(2))) unsigned v2u;
                const v2u p = __builtin_amdgcn_raw_buffer_load_b64(
                    rs, (int)(vx == kOob ? kOob : ((uint32_t)kq * (uint32_t)nvol + vx) * 8u), 0, 0);
                v = f4v_t{__uint_as_float(p.x << 16), __uint_as_float(p.x & 0xFFFF0000u),
                          __uint_as_float(p.y << 16), __uint_as_float(p.y & 0xFFFF0000u)};
              } else if constexpr (QM == 3) {   // split quad: 16-byte load, (hi + lo) 2^-sx (exact sum)
                v = unsplit4(__builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                 rs, (int)(vx == kOob ? kOob : ((uint32_t)kq * (uint32_t)nvol + vx) * 16u), 0, 0)),
                             sx);
              } else if constexpr (QM == 1) {   // the quad (c4 / 4) of the voxel: one 16-byte load
                v = ld4(rs, vx == kOob ? kOob : ((uint32_t)kq * (uint32_t)nvol + vx) * 16u, 0);
              } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                      rs, (int)(vx == kOob ? kOob : ((uint32_t)(kq * 4 + q) * (uint32_t)nvol + vx) * 4u), 0, 0));
              }
            } else {
              const uint32_t eo = vx == kOob ? kOob : (vx * (uint32_t)CI + (uint32_t)c4) * 4u;
              v = ld4(rs, eo, 0);
              if (x2) v += ld4(rs2, eo, 0);
            }
            a[tx][rb] = v;
          }
          const float* wt = w + (size_t)((tz * 3 + ty) * 3 + tx) * CO * CI;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            bw[tx][nb] = *reinterpret_cast<const f4v_t*>(wt + (size_t)(nb * 16 + m) * CI + c4);
        }
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          if (MODE == kT2 && ((tx & 1) != par[2])) continue;
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
              for (int nb = 0; nb < NB; ++nb)
                acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tx][rb][s], bw[tx][nb][s], acc[rb][nb], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: eval BN + ReLU, NDHWC store.  acc[rb][nb][r] = (row (lane>>4)*4 + r, col lane&15)
  float vmax = 0.0f;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int co = nb * 16 + m;
    const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
                mu = bn_scale ? bn_mean[co] : 0.0f;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + rb * 16 + kq * 4 + r;
        if (row >= rows) continue;
        const int jx = row % cn[2], t = row / cn[2];
        const int jy = t % cn[1], jz = t / cn[1];
        const int vz = cf[0] + step * jz - g.o0[0], vy = cf[1] + step * jy - g.o0[1],
                  vx = cf[2] + step * jx - g.o0[2];
        float v = acc[rb][nb][r];
        if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
        vmax = fmaxf(vmax, fabsf(v));
        store_out(y, g, b, co, vz, vy, vx, CO, v);
      }
  }
  if (g.y_bound) bound_update(g.y_bound, vmax);
}

template <int MODE, int CI, int CO, int RB, int QM = 0>
void launch_mode(const float* x, const float* x2, const float* w, float* y, const float* sc, const float* sh,
                 const float* mu, int B, const Geo& g, hipStream_t s) {
  const int classes = MODE == kT2 ? 8 : 1;
  // rows of the largest class (T2) or of the region
  const int rz = MODE == kT2 ? (g.on[0] + 1) / 2 : g.on[0], ry = MODE == kT2 ? (g.on[1] + 1) / 2 : g.on[1],
            rx = MODE == kT2 ? (g.on[2] + 1) / 2 : g.on[2];
  const int rows = rz * ry * rx;
  const int per_block = (kBlock / 64) * 16 * RB;
  const int blocks = (rows + per_block - 1) / per_block;
  const dim3 grid((unsigned)((blocks + 7) / 8 * 8), (unsigned)classes, (unsigned)B);   // XCD remap: multiple of 8
  hipLaunchKernelGGL((conv3d_region_kernel<MODE, CI, CO, RB, QM>), grid, dim3(kBlock), 0, s, x, x2, w, y, sc, sh, mu,
                     g);
}

}  // namespace

int launch_conv3d_region(int mode, bool out_cf, int in_c4, const float* x, const float* x2, const float* w,
                         float* y, int B, int CI, int CO, const int* n, const int* o0, const int* on, const int* i0,
                         const int* in, const int* pad, const float* bn_scale, const float* bn_shift,
                         const float* bn_mean, hipStream_t s, const uint32_t* absmax, uint32_t* y_bound) {
  Geo g;
  g.y_bound = y_bound;
  g.out_cf = out_cf ? 1 : 0;
  g.in_c4 = in_c4;
  g.absmax = absmax;
  for (int d = 0; d < 3; ++d) {
    g.n[d] = n[d];
    g.o0[d] = o0[d];
    g.on[d] = on[d];
    g.i0[d] = i0 ? i0[d] : 0;
    g.in[d] = in ? in[d] : n[d];
    g.pad[d] = pad ? pad[d] : 1;
  }
// two row blocks per wave (one and four measured slower on the cfg-2 eval and train-mode steps)
#define MVS_REGION_CASE(MD, A, C)                                                       \
  if (mode == MD && CI == A && CO == C) {                                               \
    launch_mode<MD, A, C, 2>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s);        \
    return MVS_OK;                                                                      \
  }
#define MVS_REGION_S2(A, C)                                                                                   \
  if (mode == kS2 && CI == A && CO == C) {                                                                    \
    if (in_c4 == 3) launch_mode<kS2, A, C, 2, 3>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s);         \
    else if (in_c4 == 2) launch_mode<kS2, A, C, 2, 2>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s);    \
    else if (in_c4) launch_mode<kS2, A, C, 2, 1>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s);         \
    else launch_mode<kS2, A, C, 2, 0>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s);                    \
    return MVS_OK;                                                                                            \
  }
  // S2: conv_1_0 / conv_2_0 / conv_3_0 (32 -> 16 / 32 / 64); S1: conv_k_1; T2: deconv_3_0 (64 -> 32),
  // deconv_2_0 (32 -> 16)
  MVS_REGION_S2(32, 16) MVS_REGION_S2(32, 32) MVS_REGION_S2(32, 64)
  MVS_REGION_CASE(kS1, 16, 16) MVS_REGION_CASE(kS1, 32, 32) MVS_REGION_CASE(kS1, 64, 64)
  MVS_REGION_CASE(kT2, 64, 32) MVS_REGION_CASE(kT2, 32, 16)
#undef MVS_REGION_CASE
#undef MVS_REGION_S2
  return MVS_ERR_INVALID_ARGUMENT;
}

}  // namespace mvs
