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
#include <cstdlib>

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
  int st0[3];   // the output region's place in the stored tensor: y holds a box of size stn whose
  int stn[3];   //   voxel st0 is the region's first (default 0 / on: y is the region)
};

// T2 parity class: per dim, outputs o with (o + P) % 2 == par; first such o in the region and count
__device__ inline void class_dim(int o0, int on, int p, int par, int& first, int& cnt) {
  first = o0 + (((o0 + p) & 1) != par ? 1 : 0);
  cnt = first < o0 + on ? (o0 + on - 1 - first) / 2 + 1 : 0;
}

__device__ inline void store_out(float* __restrict__ y, const Geo& g, int b, int co, int vz, int vy, int vx,
                                 int CO, float v) {
  const size_t vox = ((size_t)(vz + g.st0[0]) * g.stn[1] + (vy + g.st0[1])) * g.stn[2] + (vx + g.st0[2]);
  const size_t rvol = (size_t)g.stn[0] * g.stn[1] * g.stn[2];
  if (g.out_cf) y[((size_t)b * CO + co) * rvol + vox] = v;
  else y[((size_t)b * rvol + vox) * CO + co] = v;
}

// QM (S2 only): input layout of the volume -- 0 NCDHW, 1 fp32 channel quads, 2 bf16 channel quads --
// a template parameter, so the K loop has no per-load layout branches and (S1 / S2: no parity
// classes) unrolls into one basic block the scheduler can software-pipeline (loads of later taps
// issued under the MFMAs of earlier ones)
// CLS (T2 only): the parity class (pz, py, px) = bits (2, 1, 0) as a COMPILE-TIME constant, so the tap
// loops unroll to exactly the class's 1-8 taps in one basic block (the loads of every tap issued ahead of
// the MFMAs); the kernel below dispatches on blockIdx.y.  -1 (S1 / S2): no classes.
template <int MODE, int CI, int CO, int RB, int QM, int CLS>
__device__ __forceinline__ void region_conv(
    const float* __restrict__ x, const float* __restrict__ x2, const float* __restrict__ w,
    float* __restrict__ y, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, const Geo& g) {
  constexpr int NB = CO / 16;          // column blocks
  static_assert(CI % 16 == 0 && CO % 16 == 0, "channel counts in multiples of 16");
  static_assert((MODE == kT2) == (CLS >= 0), "parity classes: transposed convolutions");
  const int lane = (int)threadIdx.x & 63;
  const int m = lane & 15, kq = lane >> 4;   // MFMA row / K index of this lane's A value
  const int b = (int)blockIdx.z;

  // ---- rows of this wave: parity class (T2) or the whole region ----
  int cf[3], cn[3];
  constexpr int par[3] = {CLS >= 0 ? (CLS >> 2) & 1 : 0, CLS >= 0 ? (CLS >> 1) & 1 : 0, CLS >= 0 ? CLS & 1 : 0};
  if constexpr (MODE == kT2) {
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
__global__ __launch_bounds__(kBlock) void conv3d_region_kernel(
    const float* __restrict__ x, const float* __restrict__ x2, const float* __restrict__ w,
    float* __restrict__ y, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean, Geo g) {
  if constexpr (MODE == kT2) {
    switch (blockIdx.y) {   // workgroup-uniform
#define MVS_T2_CLASS(c) \
  case c: region_conv<MODE, CI, CO, RB, QM, c>(x, x2, w, y, bn_scale, bn_shift, bn_mean, g); break;
      MVS_T2_CLASS(0) MVS_T2_CLASS(1) MVS_T2_CLASS(2) MVS_T2_CLASS(3)
      MVS_T2_CLASS(4) MVS_T2_CLASS(5) MVS_T2_CLASS(6) MVS_T2_CLASS(7)
#undef MVS_T2_CLASS
      default: break;
    }
  } else {
    region_conv<MODE, CI, CO, RB, QM, -1>(x, x2, w, y, bn_scale, bn_shift, bn_mean, g);
  }
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

// ---- stride-1 convolutions with LDS-staged operands (conv_k_1, model.py:104-113) ----
// The per-lane kernel above fetches each input voxel once per tap through L1 / L2 (27 times) and keeps
// at most RB row blocks of loads in flight: latency-bound (conv_1_1 at ~50 TF/s in the cfg-2 step).
// Here a workgroup (4 waves) owns a 16 (x) x 4 (y) x TZ (z) block of outputs; its input block, 18 x 6 x
// (TZ + 2) voxels with all CI channels, is loaded once into LDS (one CI x 4-byte record per voxel, 16-byte
// chunks of 4 channels XOR-swizzled by voxel: the 16 lanes of an MFMA row group -- 16 consecutive
// voxels, one chunk -- and the ds_read_b128 lane groups hit distinct bank groups).  Wave w owns column
// block w % NB (16 output channels) and 8 row blocks (16 x-voxels of one (z, y) row each); every weight
// float4 (L1 / L2) feeds 8 row blocks x 4 MFMAs, every A float4 comes from LDS.  Products and their
// order per accumulator are the per-lane kernel's ((tz, ty), channel block, tx, K-step s): bit-equal.
template <int CI>
struct S1TileF {
  static constexpr int TZ = CI == 16 ? 8 : (CI == 32 ? 4 : 2);
  static constexpr int PX = 18, PY = 6, PZ = TZ + 2, PV = PX * PY * PZ;
  static constexpr int NCH = CI / 4;     // 16-byte chunks (4 channels) per voxel record
  static constexpr int REC = CI * 4;     // bytes per voxel record
  static constexpr int LDS = PV * REC;   // 69,120 / 82,944 / 110,592 B
};

template <int CI>
__device__ inline int s1f_off(int v, int c) {   // byte offset of chunk c of voxel v (swizzled)
  constexpr int NCH = CI / 4;
  return v * (CI * 4) + ((c ^ (((v * NCH) >> 3) % NCH)) << 4);
}

template <int CI, int CO>
__global__ __launch_bounds__(kBlock) void conv3d_s1_lds_kernel(
    const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift, const float* __restrict__ bn_mean, Geo g,
    int tiles_x, int tiles_y, int tiles_z) {
  using T = S1TileF<CI>;
  constexpr int NB = CO / 16;
  constexpr int RB = 8;   // row blocks per wave: 4 TZ (z, y) rows x NB column blocks / 4 waves
  static_assert(T::TZ * NB == RB && CI == CO, "tile shapes");
  __shared__ __attribute__((aligned(16))) char lds[T::LDS];

  int t = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (t >= tiles_x * tiles_y * tiles_z) return;   // workgroup-uniform, before the barrier
  const int tx0 = (t % tiles_x) * 16;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * 4;
  t /= tiles_y;
  const int tz0 = t * T::TZ;
  const int b = (int)blockIdx.y;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;

  // ---- stage the input block: items (voxel, chunk), chunk fastest (coalesced channels-last loads);
  // voxels outside the input region read 0 (the convolution's zero padding outside the volume).  Each
  // batch's loads are all complete before its LDS stores are issued (no load in flight beside an LDS
  // store: DESIGN.md §3.7) ----
  {
    constexpr int NIT = T::PV * T::NCH, PER = (NIT + kBlock - 1) / kBlock, BATCH = 8;
    const size_t rvol = (size_t)g.in[0] * g.in[1] * g.in[2];
    const Rsrc rs = make_rsrc(x + (size_t)b * rvol * CI, (uint32_t)(rvol * CI * 4));
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += BATCH) {
      f4v v4[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        const int q = e % T::NCH, v = e / T::NCH;
        const int px = v % T::PX, py = (v / T::PX) % T::PY, pz = v / (T::PX * T::PY);
        const int rx = g.o0[2] + tx0 - 1 + px - g.i0[2], ry = g.o0[1] + ty0 - 1 + py - g.i0[1],
                  rz = g.o0[0] + tz0 - 1 + pz - g.i0[0];
        const bool ok = k0 + k < PER && e < NIT && rx >= 0 && rx < g.in[2] && ry >= 0 && ry < g.in[1] && rz >= 0 &&
                        rz < g.in[0];
        v4[k] = ld4(rs, ok ? (uint32_t)((((size_t)rz * g.in[1] + ry) * g.in[2] + rx) * CI + 4 * q) * 4u : kOob, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int e = tid + kBlock * (k0 + k);
        if (k0 + k >= PER || e >= NIT) continue;
        *reinterpret_cast<f4v*>(lds + s1f_off<CI>(e / T::NCH, e % T::NCH)) = v4[k];
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();

  // ---- this wave: column block nb, row blocks rg * 8 .. + 7 of the tile's 4 TZ (z, y) rows ----
  const int nb = wave % NB, rg = wave / NB;
  f4v_t acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[r] = f4v_t{0.0f, 0.0f, 0.0f, 0.0f};
  const float* wn = w + (size_t)(nb * 16 + m) * CI + 4 * kq;   // this lane's weight row, channel offset 4 kq
  // A float4s of one (tap, channel block) for the wave's 8 row blocks (buffer tx of three), read one
  // step ahead; the weight float4s of a (tap row, channel block) one iteration ahead
  f4v_t a[3][RB];
  auto lda = [&](int tr, int tx, int cb, f4v_t (&dst)[RB]) {
    const int tz = tr / 3, ty = tr % 3;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int rbi = rg * RB + r, zz = rbi >> 2, yy = rbi & 3;
      const int v = ((zz + tz) * T::PY + (yy + ty)) * T::PX + (m + tx);
      dst[r] = *reinterpret_cast<const f4v_t*>(lds + s1f_off<CI>(v, cb * 4 + kq));
    }
  };
  auto ldw = [&](int tr, int cb, f4v_t (&bw)[3]) {
#pragma unroll
    for (int tx = 0; tx < 3; ++tx)
      bw[tx] = *reinterpret_cast<const f4v_t*>(wn + (size_t)((tr * 3 + tx) * CO) * CI + cb * 16);
  };
  constexpr int CB = CI / 16, NIT = 9 * CB;   // iterations (tap row, channel block)
  f4v_t bw[3], bn_[3];
  ldw(0, 0, bw);
  lda(0, 0, 0, a[0]);
#pragma unroll 1
  for (int it = 0; it < NIT; ++it) {
    const int tr = it / CB, cb = it % CB;
    const bool more = it + 1 < NIT;
    const int tr1 = (it + 1) / CB, cb1 = (it + 1) % CB;
    if (more) ldw(tr1, cb1, bn_);
#pragma unroll
    for (int tx = 0; tx < 3; ++tx) {
      if (tx < 2) lda(tr, tx + 1, cb, a[tx + 1]);
      else if (more) lda(tr1, 0, cb1, a[0]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < RB; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tx][r][s], bw[tx][s], acc[r], 0, 0, 0);
    }
#pragma unroll
    for (int tx = 0; tx < 3; ++tx) bw[tx] = bn_[tx];
  }

  // ---- epilogue: acc[r][i] = (x = tx0 + 4 kq + i, channel nb * 16 + m) of row block r ----
  const int co = nb * 16 + m;
  const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
              mu = bn_scale ? bn_mean[co] : 0.0f;
  float vmax = 0.0f;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int rbi = rg * RB + r, zz = rbi >> 2, yy = rbi & 3;
    if (tz0 + zz >= g.on[0] || ty0 + yy >= g.on[1]) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (tx0 + 4 * kq + i >= g.on[2]) continue;
      float v = acc[r][i];
      if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
      vmax = fmaxf(vmax, fabsf(v));
      store_out(y, g, b, co, tz0 + zz, ty0 + yy, tx0 + 4 * kq + i, CO, v);
    }
  }
  if (g.y_bound) bound_update(g.y_bound, vmax);
}

template <int CI>
void launch_s1_lds(const float* x, const float* w, float* y, const float* sc, const float* sh, const float* mu,
                   int B, const Geo& g, hipStream_t s) {
  const int tx = (g.on[2] + 15) / 16, ty = (g.on[1] + 3) / 4, tz = (g.on[0] + S1TileF<CI>::TZ - 1) / S1TileF<CI>::TZ;
  const int per = tx * ty * tz;
  const dim3 grid((unsigned)((per + 7) / 8 * 8), (unsigned)B);   // XCD remap: multiple of 8
  hipLaunchKernelGGL((conv3d_s1_lds_kernel<CI, CI>), grid, dim3(kBlock), 0, s, x, w, y, sc, sh, mu, g, tx, ty, tz);
}

}  // namespace

int launch_conv3d_region(int mode, bool out_cf, int in_c4, const float* x, const float* x2, const float* w,
                         float* y, int B, int CI, int CO, const int* n, const int* o0, const int* on, const int* i0,
                         const int* in, const int* pad, const float* bn_scale, const float* bn_shift,
                         const float* bn_mean, hipStream_t s, const uint32_t* absmax, uint32_t* y_bound,
                         bool per_lane, const int* st0, const int* stn, bool s2_lds) {
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
    g.st0[d] = st0 ? st0[d] : 0;
    g.stn[d] = stn ? stn[d] : on[d];
  }
  // stride-1 convolutions of one region tensor: the LDS-staged kernel (bit-equal) only with
  // MVS_FP32_S1_LDS=1 -- measured slower at cfg 2 (conv_1_1 0.42 against 0.34 ms alone, the fp32 eval step
  // 6.60 against 5.94 ms: its 69-110 KB tiles leave 1-2 waves per SIMD and crowd out the concurrent
  // VALU conv_0_0; gpurun_out r6e)
  static const bool s1_lds = [] {
    const char* e = getenv("MVS_FP32_S1_LDS");
    return e && e[0] == '1';
  }();
  if (mode == kS1 && !x2 && CI == CO && !per_lane && s1_lds) {
    if (CI == 16) return launch_s1_lds<16>(x, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
    if (CI == 32) return launch_s1_lds<32>(x, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
    if (CI == 64) return launch_s1_lds<64>(x, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
  }
  // conv_1_0 (S2 32 -> 16) from the whole fp32 volume: the LDS-staged kernel with MVS_S2_LDS=1 (opt-in,
  // slower in the step: conv3d_s2_lds.hip)
  if (mode == kS2 && CI == 32 && CO == 16 && (in_c4 == 0 || in_c4 == 1) && !x2 && !absmax && !y_bound &&
      !per_lane && !st0 && !stn && !i0 && !in && !out_cf && pad && (s2_lds || conv_s2_lds_enabled()) &&
      (uint64_t)n[0] * (uint64_t)n[1] * (uint64_t)n[2] * 128u < 0xFFFFFFF0ull) {   // (32-bit byte offsets)
    launch_conv_s2_lds(x, in_c4, w, y, B, n, o0, on, pad, bn_scale, bn_shift, bn_mean, s);
    return MVS_OK;
  }
  // S2 from the fp32 channel-quad volume: row blocks per wave MVS_S2_RB (2 or 4) -- A/B
  static const int s2_rb = [] {
    const char* e = getenv("MVS_S2_RB");
    return e && e[0] == '4' ? 4 : 2;
  }();
  if (mode == kS2 && in_c4 == 1 && CI == 32 && s2_rb == 4) {
    if (CO == 16) return launch_mode<kS2, 32, 16, 4, 1>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
    if (CO == 32) return launch_mode<kS2, 32, 32, 4, 1>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
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
  // transposed: four row blocks per wave for deconv_2_0 (32 -> 16: 0.323 -> 0.302 ms at cfg 2), two for
  // deconv_3_0 (64 -> 32: equal); MVS_T2_RB=2 / =4 forces one for both (A/B).  Per-output accumulation
  // order does not depend on the row blocks: bit-equal either way
  static const int t2_rb = [] {
    const char* e = getenv("MVS_T2_RB");
    return e && e[0] == '4' ? 4 : e && e[0] == '2' ? 2 : 0;
  }();
  if (mode == kT2 && CI == 64 && CO == 32 && t2_rb == 4)
    return launch_mode<kT2, 64, 32, 4>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
  if (mode == kT2 && CI == 32 && CO == 16 && t2_rb != 2)
    return launch_mode<kT2, 32, 16, 4>(x, x2, w, y, bn_scale, bn_shift, bn_mean, B, g, s), MVS_OK;
  MVS_REGION_CASE(kT2, 64, 32) MVS_REGION_CASE(kT2, 32, 16)
#undef MVS_REGION_CASE
#undef MVS_REGION_S2
  return MVS_ERR_INVALID_ARGUMENT;
}

}  // namespace mvs
