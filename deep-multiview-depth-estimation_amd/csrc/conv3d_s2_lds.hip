// conv3d_s2_lds.hip -- conv_1_0 of CostVolumeReg in exact fp32 (model.py:78, applied at model.py:103:
// Conv3d(32, 16, 3, stride 2, padding P = n//2 + 1 (config.py:20)), then BN_1 + ReLU) on the live region
// halo(B) of forward_live, from the full cost volume, on the f32-input matrix cores
// (v_mfma_f32_16x16x4_f32: every product and sum an fp32 fmaf step).
//
// Why a kernel of its own: conv3d_region.hip's S2 mode gathers every tap's operands from global memory,
// and the stride-2 windows of neighbouring outputs re-read the 2 GB volume through L2 (conv_1_0 reads the
// WHOLE volume: its halo(B) outputs reach every input).  Here each input plane is staged in LDS once per
// workgroup column and every tap reads it from there -- the structure of the split-fp16 kernel
// (conv3d_s2_split.hip) with fp32 operands:
//   * a 256-thread workgroup (4 waves) owns 16 x 2 outputs in (x, y) and walks a chunk of output depths
//     2 at a time; wave w computes the 16-output row (y = w & 1, depth = w >> 1) as one MFMA row block:
//     rows = 16 outputs along x, columns = the 16 output channels, K = 32 input channels x 27 taps;
//   * a step's two output depths read 5 input planes (2o - P .. 2o - P + 4), consecutive steps share
//     one: LDS holds a 5-plane ring of the 33 x 5 input footprint (fp32, 128 B per voxel, 21 KB per
//     plane) and the weights in MFMA-fragment order (55 KB): 160.9 KB, one workgroup per CU; the next
//     step's 4 planes are loaded into registers under the MFMAs and stored into the freed slots after;
//   * the footprint's columns are deinterleaved (even input columns first), so the 16 stride-2 taps of a
//     row block read 16 consecutive voxels, and each voxel's eight 16-byte channel quads are swizzled by
//     (voxel & 7): every ds_read_b128 lane group of the A operand hits 16 distinct bank groups (CPU model
//     of MI355X_MICROARCH.md §LDS's lane groups: 1.0-way at every slot / row / tap / channel block);
//   * per tap and 16-channel block: one ds_read_b128 of A (lane (i, kq): channels 16 cb + 4 kq .. + 3 of
//     output i's tap voxel) and one of B (lane (kq, co): the same channels of output channel co's weights)
//     feed 4 MFMAs (K-step s takes element s of both); the two channel blocks accumulate in two chains
//     (the 16x16x4 f32 MFMA's 40-cycle dependent latency under its 32-cycle issue), summed at the end.
#include <cstdlib>

#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kLX = 16, kLY = 2, kLZ = 2;                 // outputs per row block (x) / rows (y) / step (z)
constexpr int kLFX = 2 * kLX + 1, kLFY = 2 * kLY + 1;     // 33 x 5 input footprint
constexpr int kLFV = kLFX * kLFY;                         // 165 voxels per plane
constexpr int kLNew = 2 * kLZ;                            // new planes per step
constexpr int kLNPL = kLNew + 1;                          // ring slots
constexpr int kLVoxB = 128;                               // 32 fp32 channels
constexpr int kLRowB = kLFX * kLVoxB;                     // 4,224 B
constexpr int kLSlotB = kLFV * kLVoxB;                    // 21,120 B
constexpr int kLRingB = kLNPL * kLSlotB;                  // 105,600 B
constexpr int kLWB = 27 * 16 * 32 * 4;                    // 55,296 B
constexpr int kLThreads = 256;
constexpr int kLPlaneQ = kLFV * 8;                        // channel quads per plane: 1,320
constexpr int kLPre = (kLNew * kLPlaneQ + kLThreads - 1) / kLThreads;   // 21 staging quads per thread
constexpr int kLPF = 2;                                   // operand prefetch distance (tap x block items)
constexpr uint32_t kLOob = 0xFFFFFFF0u;                   // >= every descriptor's num_records

struct S2L {
  int n[3];      // volume (D, H, W)
  int o0[3];     // output region origin
  int on[3];     // output region size
  int pad[3];    // P
  int tiles_x, tiles_y, zchunks, zc;
};

// deinterleaved footprint column of input column c (0 .. 32): even columns first
__device__ inline int lcol(int c) { return (c & 1) ? (kLX + 1) + (c >> 1) : (c >> 1); }
// byte offset of channel quad q of footprint voxel v inside a plane slot
__device__ inline int lquad(int v, int q) { return v * kLVoxB + ((q ^ (v & 7)) << 4); }

template <int QM>   // input layout: 1 the fp32 channel-quad volume [B][8][D][H][W][4], 0 NCDHW [B][32][D][H][W]
__global__ __launch_bounds__(kLThreads) void conv_s2_lds_kernel(
    const float* __restrict__ x, const float* __restrict__ w27, float* __restrict__ y, S2L g, int total,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift, const float* __restrict__ bn_mean) {
  __shared__ __attribute__((aligned(16))) char lds[kLRingB + kLWB];
  const int wk = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (wk >= total) return;   // workgroup-uniform, before any barrier
  int t = wk;
  const int ox0 = g.o0[2] + (t % g.tiles_x) * kLX;
  t /= g.tiles_x;
  const int oy0 = g.o0[1] + (t % g.tiles_y) * kLY;
  t /= g.tiles_y;
  const int oz0 = g.o0[0] + (t % g.zchunks) * g.zc;
  const int b = t / g.zchunks;
  const int oz1 = min(oz0 + g.zc, g.o0[0] + g.on[0]);
  const int nsteps = (oz1 - oz0 + kLZ - 1) / kLZ;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = g.n[0], H = g.n[1], W = g.n[2];
  const size_t HW = (size_t)H * W, DHW = (size_t)D * HW;
  const uint64_t vbytes = 32ull * DHW * 4ull;   // one sample's volume
  const Rsrc rx = make_rsrc(x + (size_t)b * 32 * DHW, (uint32_t)(vbytes < kLOob ? vbytes : kLOob));
  const int ix0 = 2 * ox0 - g.pad[2], iy0 = 2 * oy0 - g.pad[1], iz0 = 2 * oz0 - g.pad[0];

  // weights: region layout w27[tap][co][ci] -> LDS [tap][cb][kq][co] x 4 channels (16 B per lane read)
  for (int e = tid; e < 27 * 16 * 8; e += kLThreads) {
    const int tap = e >> 7, co = (e >> 3) & 15, cq = e & 7;
    const f4v v = *reinterpret_cast<const f4v*>(w27 + (size_t)e * 4);
    *reinterpret_cast<f4v*>(lds + kLRingB + ((((tap * 2 + (cq >> 2)) * 4 + (cq & 3)) * 16 + co) << 4)) = v;
  }
  // staging elements (quad fastest: 8 lanes = one voxel's 8 quads): LDS offset in the slot (bits 0-14),
  // quad (15-17), plane in the group (18-20; 7 = none: outside the image or past the group), footprint
  // row (21-23), column (24-29)
  int em[kLPre];
#pragma unroll
  for (int j = 0; j < kLPre; ++j) {
    const int e = tid + kLThreads * j;
    const int q = e & 7, tt = e >> 3;
    const int pl = tt / kLFV, v = tt - pl * kLFV;
    const int yy = v / kLFX, c = v - yy * kLFX;
    const int gy = iy0 + yy, gx = ix0 + c;
    const bool ok = e < kLNew * kLPlaneQ && gy >= 0 && gy < H && gx >= 0 && gx < W;
    em[j] = lquad(yy * kLFX + lcol(c), q) | (q << 15) | ((ok ? pl : 7) << 18) | ((ok ? yy : 0) << 21) |
            ((ok ? c : 0) << 24);
  }
  f4v pre[kLPre];
  auto fetch = [&](int zg, int cnt) {   // input planes zg .. zg + cnt - 1 -> registers
#pragma unroll
    for (int j = 0; j < kLPre; ++j) {
      const int pl = (em[j] >> 18) & 7, z = zg + pl;
      const bool ok = pl < cnt && z >= 0 && z < D;
      const int q = (em[j] >> 15) & 7;
      const uint32_t vox = (uint32_t)z * (uint32_t)HW + (uint32_t)(iy0 + ((em[j] >> 21) & 7)) * (uint32_t)W +
                           (uint32_t)(ix0 + ((em[j] >> 24) & 63));
      if constexpr (QM == 1) {
        pre[j] = ld4(rx, ok ? ((uint32_t)q * (uint32_t)DHW + vox) * 16u : kLOob, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          pre[j][s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rx, (int)(ok ? ((uint32_t)(4 * q + s) * (uint32_t)DHW + vox) * 4u : kLOob), 0, 0));
      }
    }
  };
  auto stage = [&](int s0, int cnt) {   // registers -> ring slots s0 ..
#pragma unroll
    for (int j = 0; j < kLPre; ++j) {
      const int pl = (em[j] >> 18) & 7;
      if (pl >= cnt) continue;
      int s = s0 + pl;
      s = s >= kLNPL ? s - kLNPL : s;
      *reinterpret_cast<f4v*>(lds + s * kLSlotB + (em[j] & 0x7FFF)) = pre[j];
    }
  };
  // halo voxels outside the image are never staged: zero the ring once
  for (int i = tid; i < kLRingB / 16; i += kLThreads) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0u, 0u, 0u, 0u);
  fetch(iz0, kLNew);
  __syncthreads();
  stage(0, kLNew);
  fetch(iz0 + kLNew, 1);
  stage(kLNew, 1);

  const int i = lane & 15, kq = lane >> 4;
  const int wy = wave & 1, wz = wave >> 1;
  const int co = lane & 15;
  const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
              mu = bn_scale ? bn_mean[co] : 0.0f;
  asm volatile("" ::"v"(sc), "v"(sh), "v"(mu));   // consumed here: no vmcnt(0) inside the step loop
  const int oy = oy0 + wy;
  const char* wl = lds + kLRingB + ((kq * 16 + co) << 4);   // + (tap * 2 + cb) * 1024
  __syncthreads();

  for (int k = 0; k < nsteps; ++k) {
    const int zs = iz0 + kLNew * k;   // first input plane of this step's window
    if (k + 1 < nsteps) fetch(zs + kLNPL, kLNew);   // the next step's new planes, in flight under the MFMAs
    f4v acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = acc0;
    const int sb = (kLNew * k) % kLNPL;   // ring slot of plane zs
    // item it = tap * 2 + cb: A = output i's tap voxel (plane 2 wz + tz, row 2 wy + ty, column 2 i + tx),
    // channels 16 cb + 4 kq .. + 3; B = those channels of output channel co's weights
    auto ldt = [&](int it, f4v& a, f4v& bw) {
      const int tap = it >> 1, cb = it & 1;
      const int tz = tap / 9, ty = (tap / 3) % 3, tx = tap % 3;
      int s = sb + 2 * wz + tz;
      s = s >= kLNPL ? s - kLNPL : s;
      const int vox = (2 * wy + ty) * kLFX + lcol(2 * i + tx);
      a = *reinterpret_cast<const f4v*>(lds + s * kLSlotB + lquad(vox, cb * 4 + kq));
      bw = *reinterpret_cast<const f4v*>(wl + it * 1024);
    };
    f4v ra[kLPF + 1], rb[kLPF + 1];
#pragma unroll
    for (int p = 0; p < kLPF; ++p) ldt(p, ra[p], rb[p]);
#pragma unroll
    for (int it = 0; it < 54; ++it) {
      if (it + kLPF < 54) {
        const int r = (it + kLPF) % (kLPF + 1);
        ldt(it + kLPF, ra[r], rb[r]);
      }
      const int r = it % (kLPF + 1);
      if (it & 1) {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r][s], rb[r][s], acc1, 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r][s], rb[r][s], acc0, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the reads kLPF items ahead of their MFMAs
    }
    // epilogue: acc[r] = output (x = ox0 + 4 kq + r, channel co); channels-last region store
    const int oz = oz0 + kLZ * k + wz;
    if (oz < oz1 && oy < g.o0[1] + g.on[1]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ox = ox0 + 4 * kq + r;
        if (ox >= g.o0[2] + g.on[2]) continue;
        float v = acc0[r] + acc1[r];
        if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
        const size_t vx = (((size_t)(oz - g.o0[0]) * g.on[1] + (oy - g.o0[1])) * g.on[2] + (ox - g.o0[2]));
        y[((size_t)b * g.on[0] * g.on[1] * g.on[2] + vx) * 16 + co] = v;
      }
    }
    if (k + 1 < nsteps) {
      __syncthreads();          // every wave is done with planes zs .. zs + 3
      stage(sb, kLNew);         // planes zs + 5 .. zs + 8 replace them
      __syncthreads();
    }
  }
}

}  // namespace

// Opt-in (MVS_S2_LDS=1): measured slower -- conv_1_0 alone 1.42 against 1.15 ms for the per-lane region
// kernel, the fp32 eval step 6.8-6.9 against 5.9 ms: its 161 KB of LDS takes a whole CU, so the concurrent
// VALU conv_0_0 can no longer share the CUs it runs on (gpurun_out r6z)
bool conv_s2_lds_enabled() {
  static const bool on = [] {
    const char* e = getenv("MVS_S2_LDS");
    return e && e[0] == '1';
  }();
  return on;
}

void launch_conv_s2_lds(const float* x, int in_c4, const float* w27, float* y, int B, const int* n, const int* o0,
                        const int* on, const int* pad, const float* bn_scale, const float* bn_shift,
                        const float* bn_mean, hipStream_t s) {
  S2L g;
  for (int d = 0; d < 3; ++d) {
    g.n[d] = n[d];
    g.o0[d] = o0[d];
    g.on[d] = on[d];
    g.pad[d] = pad[d];
  }
  g.tiles_x = (on[2] + kLX - 1) / kLX;
  g.tiles_y = (on[1] + kLY - 1) / kLY;
  g.zc = 14;   // output depths per workgroup (7 steps): restaging its first plane costs 1/29
  g.zchunks = (on[0] + g.zc - 1) / g.zc;
  const int total = g.tiles_x * g.tiles_y * g.zchunks * B;
  if (in_c4)
    hipLaunchKernelGGL(conv_s2_lds_kernel<1>, xcd_grid(total), dim3(kLThreads), 0, s, x, w27, y, g, total, bn_scale,
                       bn_shift, bn_mean);
  else
    hipLaunchKernelGGL(conv_s2_lds_kernel<0>, xcd_grid(total), dim3(kLThreads), 0, s, x, w27, y, g, total, bn_scale,
                       bn_shift, bn_mean);
}

}  // namespace mvs
