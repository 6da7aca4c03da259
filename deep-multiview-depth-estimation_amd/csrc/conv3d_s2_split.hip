// conv3d_s2_split.hip -- conv_1_0 of CostVolumeReg (model.py:78, applied at model.py:103: 32 -> 16
// channels, 3x3x3, stride 2, padding P = n//2 + 1 (config.py:20), then eval BN_1 + ReLU) on the live
// region halo(B) of forward_live, read from the channel-quad cost volume, on the f16
// matrix cores with split operands (the arithmetic of conv3d_split.hip: power-of-two scaled hi / lo
// fp16 parts, fp32 accumulation; here three partial products x_hi w_hi + x_hi w_lo + x_lo w_hi,
// the fourth is 2^-22 of a term).
//
// Why a kernel of its own: conv3d_region.hip's S2 mode gathers every tap from global memory, and the
// stride-2 windows of neighbouring outputs re-read the 2 GB volume ~2.3x from HBM (PMC, r03e);
// conv_1_0 reads the WHOLE volume (its halo(B) outputs reach every input) and was the longest kernel
// of the eval step (1.17 ms).  Here each input plane is staged in LDS once per workgroup column and
// every tap reads it from there.
//
// Output o (per dim) reads inputs 2o - P + t, t = 0..2.  A 256-thread workgroup (4 waves) owns 16 x 2
// outputs in (x, y) and walks a chunk of output depths 2 at a time; wave w computes the 16-output row
// (y = w & 1, depth = w >> 1) as one MFMA row block: rows = 16 outputs along x, columns = the 16
// output channels, K = the 32 input channels of one tap.  A step's two output depths read 5 input
// planes (2o - P .. 2o - P + 4), consecutive steps share one: LDS holds a 5-plane ring of the
// workgroup's 33 x 5 input footprint (hi and lo parts, 21 KB per plane) and the weight fragments
// (27 taps x hi / lo, 54 KB), 160.9 KB in all; the next step's 4 planes are loaded into registers
// under the MFMAs and split into the freed slots after them.  In LDS the footprint's columns are
// deinterleaved (even input columns first, then odd), so the stride-2 taps of a row block read
// consecutive voxels, and the 16-byte channel octets are swizzled by ((voxel >> 1) & 3): every
// ds_read_b128 lane group hits 16 distinct bank groups.
#include "launchers.h"
#include "packed.h"
#include "split.h"

namespace mvs {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kOX = 16, kOY = 2, kOZ = 2;                 // outputs per workgroup row block / step
constexpr int kFX = 2 * kOX + 1, kFY = 2 * kOY + 1;       // 33 x 5 input footprint
constexpr int kFV = kFX * kFY;                            // 165 voxels per plane
constexpr int kNew = 2 * kOZ;                             // new planes per step
constexpr int kNPL = kNew + 1;                            // ring slots
constexpr int kVoxB = 64;                                 // 32 channels x fp16 per part
constexpr int kRowB = kFX * kVoxB;                        // 2,112 B
constexpr int kPartB = kFV * kVoxB;                       // 10,560 B
constexpr int kSlotB = 2 * kPartB;                        // 21,120 B
constexpr int kRingB = kNPL * kSlotB;                     // 105,600 B
constexpr int kWB = 27 * 2 * 64 * 16;                     // weight fragments: 55,296 B
constexpr int kThreads = 256;
constexpr int kPlaneQ = kFV * 8;                          // channel quads per plane: 1,320
constexpr int kPre = (kNew * kPlaneQ + kThreads - 1) / kThreads;   // 21 staging quads per thread
constexpr int kPF = 2;                                    // tap prefetch distance
constexpr uint32_t kOob = 0xFFFFFFF0u;

struct S2Geo {
  int n[3];      // volume (D, H, W)
  int o0[3];     // output region origin
  int on[3];     // output region size
  int pad[3];    // P
  int tiles_x, tiles_y, zchunks, zc;   // workgroup grid; output depths per chunk (even)
};

// deinterleaved footprint column of input column c (0 .. 32): even columns first
__device__ inline int fcol(int c) { return (c & 1) ? (kOX + 1) + (c >> 1) : (c >> 1); }

template <bool PRESPLIT>   // input: the split cost volume (SCV, split.h) or fp32 channel quads
__global__ __launch_bounds__(kThreads) void conv_s2_split_kernel(
    const f4v* __restrict__ cv, const h8v* __restrict__ wfrag, const uint32_t* __restrict__ absmax, int w_exp,
    float* __restrict__ y, S2Geo g, int total, const float* __restrict__ bn_scale, const float* __restrict__ bn_shift,
    const float* __restrict__ bn_mean) {
  __shared__ __attribute__((aligned(16))) char lds[kRingB + kWB];
  const int wk = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (wk >= total) return;   // workgroup-uniform, before any barrier
  int t = wk;
  const int ox0 = g.o0[2] + (t % g.tiles_x) * kOX;
  t /= g.tiles_x;
  const int oy0 = g.o0[1] + (t % g.tiles_y) * kOY;
  t /= g.tiles_y;
  const int oz0 = g.o0[0] + (t % g.zchunks) * g.zc;
  const int b = t / g.zchunks;
  const int oz1 = min(oz0 + g.zc, g.o0[0] + g.on[0]);
  const int nsteps = (oz1 - oz0 + kOZ - 1) / kOZ;
  const int ex = cv_split_exponent(absmax);
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = g.n[0], H = g.n[1], W = g.n[2];
  const size_t HW = (size_t)H * W, DHW = (size_t)D * HW;
  const uint64_t vbytes = 8ull * DHW * 16ull;
  const Rsrc rcv = make_rsrc(cv + (size_t)b * 8 * DHW, (uint32_t)(vbytes < kOob ? vbytes : kOob));
  // input footprint origin (x, y) and the first step's first plane
  const int ix0 = 2 * ox0 - g.pad[2], iy0 = 2 * oy0 - g.pad[1], iz0 = 2 * oz0 - g.pad[0];

  // weight fragments -> LDS (wfrag[tap][part][lane], 16 B each)
  {
    const Rsrc rw = make_rsrc(wfrag, (uint32_t)kWB);
#pragma unroll
    for (int j = 0; j < (kWB / 16 + kThreads - 1) / kThreads; ++j) {
      const int e = tid + kThreads * j;
      if (e < kWB / 16)
        *reinterpret_cast<f4v*>(lds + kRingB + e * 16) =
            __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rw, e * 16, 0, 0));
    }
  }
  // staging elements (quad fastest: 8 lanes = one voxel's 8 quads, loaded from 8 quad planes and
  // written as the voxel's 64 B of each part): packed LDS offset (bits 0-13), quad (14-16), plane in
  // the group (17-19; 7 = none: outside the image or past the group), footprint row (20-22), column
  // (23-28)
  int em[kPre];
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    const int e = tid + kThreads * j;
    const int q = e & 7, tt = e >> 3;
    const int pl = tt / kFV, v = tt - pl * kFV;
    const int yy = v / kFX, c = v - yy * kFX;
    const int gy = iy0 + yy, gx = ix0 + c;
    const bool ok = e < kNew * kPlaneQ && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const int vox = yy * kFX + fcol(c);
    const int loff = vox * kVoxB + (((q >> 1) ^ ((vox >> 1) & 3)) << 4) + ((q & 1) << 3);
    em[j] = loff | (q << 14) | ((ok ? pl : 7) << 17) | ((ok ? yy : 0) << 20) | ((ok ? c : 0) << 23);
  }
  f4v pre[kPre];
  auto fetch = [&](int zg, int cnt) {   // input planes zg .. zg + cnt - 1 -> registers
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int pl = (em[j] >> 17) & 7, z = zg + pl;
      const bool ok = pl < cnt && z >= 0 && z < D;
      const uint32_t goff = (uint32_t)((em[j] >> 14) & 7) * (uint32_t)DHW +
                            (uint32_t)(iy0 + ((em[j] >> 20) & 7)) * (uint32_t)W + (uint32_t)(ix0 + ((em[j] >> 23) & 63));
      pre[j] = ld4(rcv, ok ? (goff + (uint32_t)z * (uint32_t)HW) * 16u : kOob, 0);
    }
  };
  auto stage = [&](int s0, int cnt) {   // registers -> ring slots s0 .. (split into hi / lo parts)
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int pl = (em[j] >> 17) & 7;
      if (pl >= cnt) continue;
      int s = s0 + pl;
      s = s >= kNPL ? s - kNPL : s;
      uint2 hi, lo;
      if constexpr (PRESPLIT) {   // already the consumer's operands: two 8-byte halves
        const uint4 w = __builtin_bit_cast(uint4, pre[j]);
        hi = make_uint2(w.x, w.y);
        lo = make_uint2(w.z, w.w);
      } else {
        split4(pre[j], ex, hi, lo);
      }
      char* p = lds + s * kSlotB + (em[j] & 0x3FFF);
      *reinterpret_cast<uint2*>(p) = hi;
      *reinterpret_cast<uint2*>(p + kPartB) = lo;
    }
  };
  // halo voxels outside the image are never staged: zero the ring once
  for (int i = tid; i < kRingB / 16; i += kThreads) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0u, 0u, 0u, 0u);
  fetch(iz0, kNew);
  __syncthreads();
  stage(0, kNew);
  fetch(iz0 + kNew, 1);
  stage(kNew, 1);

  // per-lane constants: row i = output x ox0 + i, octet gq = input channels 8 gq .. 8 gq + 7
  const int i = lane & 15, gq = lane >> 4;
  const int wy = wave & 1, wz = wave >> 1;
  int aoff[3];   // byte offset of tap column tx in the footprint row (deinterleaved, swizzled)
#pragma unroll
  for (int tx = 0; tx < 3; ++tx) {
    const int c = 2 * i + tx;
    aoff[tx] = fcol(c) * kVoxB;   // + row * kRowB below; swizzle uses the whole voxel index
  }
  const int co = lane & 15;
  const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
              mu = bn_scale ? bn_mean[co] : 0.0f;
  // consume the BN loads here: first used inside the step loop, their wait would be a vmcnt(0) there
  // that also drains every step's plane prefetch
  asm volatile("" ::"v"(sc), "v"(sh), "v"(mu));
  const int oexp = -(ex + w_exp);
  const int oy = oy0 + wy;
  const char* wl = lds + kRingB + lane * 16;
  __syncthreads();

  for (int k = 0; k < nsteps; ++k) {
    const int zs = iz0 + kNew * k;   // first input plane of this step's window
    if (k + 1 < nsteps) fetch(zs + kNPL, kNew);   // the next step's new planes, in flight under the MFMAs
    f4 aa = {0.0f, 0.0f, 0.0f, 0.0f}, ab = aa, ac = aa;
    const int sb = (kNew * k) % kNPL;   // ring slot of plane zs
    // 27 taps (tz, ty, tx): A = the row block's inputs (plane 2 wz + tz, row 2 wy + ty, columns
    // 2 i + tx), B = the tap's hi / lo weight fragments
    auto ldt = [&](int tap, h8v& xh, h8v& xl, h8v& bh, h8v& bl) {
      const int tz = tap / 9, ty = (tap / 3) % 3, tx = tap % 3;
      int s = sb + 2 * wz + tz;
      s = s >= kNPL ? s - kNPL : s;
      const int vox = (2 * wy + ty) * kFX + fcol(2 * i + tx);
      const char* base = lds + s * kSlotB + (2 * wy + ty) * kRowB + aoff[tx] + ((gq ^ ((vox >> 1) & 3)) << 4);
      xh = *reinterpret_cast<const h8v*>(base);
      xl = *reinterpret_cast<const h8v*>(base + kPartB);
      bh = *reinterpret_cast<const h8v*>(wl + (tap * 2) * 1024);
      bl = *reinterpret_cast<const h8v*>(wl + (tap * 2 + 1) * 1024);
    };
    h8v rxh[kPF + 1], rxl[kPF + 1], rbh[kPF + 1], rbl[kPF + 1];
#pragma unroll
    for (int tp = 0; tp < kPF; ++tp) ldt(tp, rxh[tp], rxl[tp], rbh[tp], rbl[tp]);
#pragma unroll
    for (int tp = 0; tp < 27; ++tp) {
      if (tp + kPF < 27) {
        const int r = (tp + kPF) % (kPF + 1);
        ldt(tp + kPF, rxh[r], rxl[r], rbh[r], rbl[r]);
      }
      const int r = tp % (kPF + 1);
      aa = __builtin_amdgcn_mfma_f32_16x16x32_f16(rxh[r], rbh[r], aa, 0, 0, 0);
      ab = __builtin_amdgcn_mfma_f32_16x16x32_f16(rxh[r], rbl[r], ab, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(rxl[r], rbh[r], ac, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads kPF taps ahead of their MFMAs
    }
    // epilogue: acc[r] = output (x = ox0 + 4 (lane >> 4) + r, channel co); channels-last region store
    const int oz = oz0 + kOZ * k + wz;
    if (oz < oz1 && oy < g.o0[1] + g.on[1]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ox = ox0 + 4 * gq + r;
        if (ox >= g.o0[2] + g.on[2]) continue;
        float v = ldexpf(aa[r] + (ab[r] + ac[r]), oexp);
        if (bn_scale) v = fmaxf((v - mu) * sc + sh, 0.0f);
        const size_t vx = (((size_t)(oz - g.o0[0]) * g.on[1] + (oy - g.o0[1])) * g.on[2] + (ox - g.o0[2]));
        y[((size_t)b * g.on[0] * g.on[1] * g.on[2] + vx) * 16 + co] = v;
      }
    }
    if (k + 1 < nsteps) {
      __syncthreads();          // every wave is done with planes zs .. zs + 3
      stage(sb, kNew);          // planes zs + 5 .. zs + 8 replace them
      __syncthreads();
    }
  }
}

}  // namespace

int launch_conv_s2_split(const void* x, bool presplit, const void* wfrag, int w_exp, const uint32_t* absmax, float* y, int B,
                         const int* n, const int* o0, const int* on, const int* pad, const float* bn_scale,
                         const float* bn_shift, const float* bn_mean, hipStream_t s) {
  S2Geo g;
  for (int d = 0; d < 3; ++d) {
    g.n[d] = n[d];
    g.o0[d] = o0[d];
    g.on[d] = on[d];
    g.pad[d] = pad[d];
  }
  g.tiles_x = (on[2] + kOX - 1) / kOX;
  g.tiles_y = (on[1] + kOY - 1) / kOY;
  g.zc = 14;   // output depths per workgroup (7 steps): restaging its first plane costs 1/29
  g.zchunks = (on[0] + g.zc - 1) / g.zc;
  const long total = (long)g.tiles_x * g.tiles_y * g.zchunks * B;
  if (total >= (1L << 31) - 8) return MVS_ERR_TOO_LARGE;
  hipLaunchKernelGGL(presplit ? conv_s2_split_kernel<true> : conv_s2_split_kernel<false>, xcd_grid((int)total),
                     dim3(kThreads), 0, s, reinterpret_cast<const f4v*>(x),
                     reinterpret_cast<const h8v*>(wfrag), absmax, w_exp, y, g, (int)total, bn_scale, bn_shift, bn_mean);
  return MVS_OK;
}

}  // namespace mvs
