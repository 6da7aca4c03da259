// conv3d_split.hip -- conv_0_0 of CostVolumeReg (model.py:77, applied at model.py:101: 32 -> 8
// channels, 3x3x3, stride 1, padding 1, then the eval BN_0 + ReLU) on the f16 matrix cores, with
// fp32-level accuracy through split operands.
//
// Why: gfx950's fp32 MFMA runs at the fp32 VALU rate, 1/16 of the f16 MFMA.  conv_0_0 is 2.2e11
// FLOP per cfg-2 step and compute-bound in fp32 (conv3d_narrow.hip: ~1.9 ms, VALU ~91 % busy).
//
// Split arithmetic.  Every fp32 operand v is scaled by a power of two (exact) and written as
// v = hi + lo + r with hi = fp16(v), lo = fp16(v - hi) (round to nearest): |r| <= 2^-22 |v| for
// v in fp16's normal range (lo below it is a subnormal with absolute error <= 2^-25, ~2^-39 of the
// scaled maximum 2^14).  One 16x16x32 f16 MFMA with the weight operand's 16 columns laid out as
// [8 output channels of w_hi | the same 8 of w_lo] gives x_hi*w_hi and x_hi*w_lo, a second one with
// x_lo gives x_lo*w_hi and x_lo*w_lo: all four partial products, each exact in fp32 (11-bit x 11-bit
// significands), accumulated by the MFMA in fp32.  Per product the error is that of the operand
// residuals (~2^-21 relative) -- small against the fp32 accumulation error of the 864-term sums,
// so the outputs carry fp32-level error (measured against float64 and the fp32 kernels in
// tests/test_split_conv.py).  The scales: weights 2^ew with max|w| 2^ew < 2^14 (host, with the
// fragments); the cost volume 2^ex with (max|feat|)^2 2^ex < 2^14 -- a variance over views is at
// most max|x_v|^2, and mvs_cost_volume_fwd_c4 records max|feat| (per-XCD words) when asked.  The
// output is the fp32 sum times 2^-(ex + ew), exact.
//
// GEMM mapping.  Rows = 16 consecutive x voxels of one output row (MFMA M), columns = 8 channels
// x {hi, lo} weights (N = 16), K = the 32 input channels of one tap (one K-32 MFMA per tap and
// split part).  Lane (i = l & 15, g = l >> 4) supplies channels 8g .. 8g + 7 of voxel i's tap
// input: one ds_read_b128 per (tap, part).
//
// Tiling.  A 256-thread workgroup (4 waves) owns a 16 x 4 (x, y) column of outputs, one y row per
// wave, and walks kZC depths in steps of 3.  LDS holds 5 input planes (the 18 x 6 halo of the
// column, 32 channels, hi and lo parts: 13.5 KB per plane, 69 KB in all) as a ring, so two
// workgroups share a CU and one's staging overlaps the other's MFMAs; a
// step reads planes zs-1 .. zs+3, and each (plane, ky, kx) A fragment feeds every output depth it
// reaches (up to 3): 90 LDS reads for 162 MFMAs per wave and step.  The weight fragments stay in
// registers (108 VGPRs), so the step's only vector-memory loads are the next step's 3 planes,
// issued at its start (in flight under the MFMAs) and split into the freed ring slots after it.  Octets are swizzled by voxel column ((x >> 1) & 3), which makes
// every ds_read_b128 lane group hit 16 distinct 16-byte bank groups for all three kx shifts.
#include "launchers.h"
#include "packed.h"
#include "split.h"

namespace mvs {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));

constexpr int kSX = 16, kSY = 4, kZS = 2, kZC = 48;
constexpr int kPX = kSX + 2, kPY = kSY + 2, kPV = kPX * kPY;   // 18 x 6 voxels per staged plane
constexpr int kNPL = kZS + 2;                                   // resident planes (ring slots)
constexpr int kVoxB = 64;                                       // 32 channels x fp16 per part
constexpr int kRowB = kPX * kVoxB;                              // 1,152 B
constexpr int kPartB = kPV * kVoxB;                             // 6,912 B
constexpr int kSlotB = 2 * kPartB;                              // hi + lo parts
constexpr int kLdsB = kNPL * kSlotB;                            // 55,296 B: 2 workgroups per CU
constexpr int kThreads = 256;
constexpr int kPlaneQ = kPV * 8;                                // channel quads per plane: 1,440
constexpr int kPre = (kZS * kPlaneQ + kThreads - 1) / kThreads;  // 7 staging quads per thread
constexpr int kPF = 3;                                           // A-fragment prefetch distance (items)
constexpr uint32_t kOob = 0xFFFFFFF0u;                          // buffer offset past every descriptor

__device__ inline float ror8(float v) {   // value of lane (l ^ 8) inside each 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
}

template <bool PRESPLIT>   // input: the split cost volume (SCV, split.h) or fp32 channel quads
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void conv0_split_kernel(
    const f4v* __restrict__ cv, const h8v* __restrict__ wfrag, const uint32_t* __restrict__ absmax, int w_exp,
    float* __restrict__ out, int D, int H, int W, int tiles_x, int tiles_y, int zchunks, int total,
    const float* __restrict__ bn_scale, const float* __restrict__ bn_shift, const float* __restrict__ bn_mean) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsB];
  const int wk = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (wk >= total) return;   // workgroup-uniform, before any barrier
  int t = wk;
  const int x0 = (t % tiles_x) * kSX;
  t /= tiles_x;
  const int y0 = (t % tiles_y) * kSY;
  t /= tiles_y;
  const int z0 = (t % zchunks) * kZC;
  const int b = t / zchunks;
  const int z1 = min(z0 + kZC, D);
  const int nsteps = (z1 - z0 + kZS - 1) / kZS;
  const int ex = cv_split_exponent(absmax);
  const int tid = (int)threadIdx.x;
  const size_t HW = (size_t)H * W, DHW = (size_t)D * HW;
  // the sample's volume through one buffer descriptor (8 D H W quads of 16 B <= 2^32 - 16, checked by
  // the C ABI); out-of-range offsets read 0: halo outside the image and planes outside the volume
  const uint64_t vbytes = 8ull * DHW * 16ull;
  const Rsrc rcv = make_rsrc(cv + (size_t)b * 8 * DHW, (uint32_t)(vbytes < kOob ? vbytes : kOob));
  const Rsrc rwf = make_rsrc(wfrag, 27u * 64u * 16u);

  // ---- staging map: quad e = tid + 512 j of a kZS-plane group -> (plane in group, global offset
  // inside that plane's (quad) volume, LDS byte offset inside a ring slot) ----
  // B fragments (wfrag[tap][lane], 27 x 1 KB): held in registers for the whole kernel, so the MFMA
  // loop issues no vector-memory load that a wait could make the plane prefetch drain for.  Loaded
  // before the first planes, whose staging waits retire them: none is outstanding in the step loop
  // (the loop's counted waits would otherwise drain each step's prefetch)
  const int lane = tid & 63;
  h8v bw[27];
#pragma unroll
  for (int t = 0; t < 27; ++t)
    bw[t] = __builtin_bit_cast(h8v, __builtin_amdgcn_raw_buffer_load_b128(rwf, lane * 16, t * 1024, 0));
  // per staging element, one packed word: LDS byte offset inside a ring slot (bits 0-12), quad q
  // (13-15), plane in the group (16-17; 3 = no element: outside the image or past the group), halo
  // row yy (18-20) and column xx (21-25); the global offset is re-formed at each fetch (registers)
  int em[kPre];
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    // quad fastest: 8 lanes write one voxel's 64 B (a 16-lane ds_write_b64 group two whole voxels,
    // conflict-free) and load its 8 quads; 8 voxels of a row per wave-instruction and quad
    const int e = tid + kThreads * j;
    const int q = e & 7, t = e >> 3;
    const int pl = t / kPV, v = t - pl * kPV;
    const int yy = v / kPX, xx = v - yy * kPX;
    const int gy = y0 - 1 + yy, gx = x0 - 1 + xx;
    const bool ok = e < kZS * kPlaneQ && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const int loff = v * kVoxB + (((q >> 1) ^ ((xx >> 1) & 3)) << 4) + ((q & 1) << 3);
    em[j] = loff | (q << 13) | ((ok ? pl : 3) << 16) | ((ok ? yy : 0) << 18) | ((ok ? xx : 0) << 21);
  }
  f4v pre[kPre];
  const uint32_t gbase = (uint32_t)(y0 - 1) * (uint32_t)W + (uint32_t)(x0 - 1);   // (may wrap: re-added)
  // planes zg .. zg + cnt - 1 -> registers (zero outside the volume)
  auto fetch = [&](int zg, int cnt) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int pl = (em[j] >> 16) & 3, z = zg + pl;
      const bool ok = pl < cnt && z >= 0 && z < D;
      const uint32_t goff = (uint32_t)((em[j] >> 13) & 7) * (uint32_t)DHW + gbase +
                            (uint32_t)((em[j] >> 18) & 7) * (uint32_t)W + (uint32_t)((em[j] >> 21) & 31);
      pre[j] = ld4(rcv, ok ? (goff + (uint32_t)z * (uint32_t)HW) * 16u : kOob, 0);
    }
  };
  // registers -> ring slots (slot of the group's first plane: s0), split into hi / lo parts
  auto stage = [&](int s0, int cnt) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int pl = (em[j] >> 16) & 3;
      if (pl >= cnt) continue;   // 3: outside the image, the slot keeps the zeros written first
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
      char* p = lds + s * kSlotB + (em[j] & 0x1FFF);
      *reinterpret_cast<uint2*>(p) = hi;
      *reinterpret_cast<uint2*>(p + kPartB) = lo;
    }
  };
  // halo voxels outside the image are never written by stage(): zero the whole ring once
  for (int i = tid; i < kLdsB / 16; i += kThreads) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0u, 0u, 0u, 0u);
  fetch(z0 - 1, kZS);
  __syncthreads();
  stage(0, kZS);
  fetch(z0 - 1 + kZS, kNPL - kZS);
  stage(kZS, kNPL - kZS);

  // ---- per-lane constants ----
  const int wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  int aoff[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) aoff[kx] = wave * kRowB + (i + kx) * kVoxB + ((g ^ (((i + kx) >> 1) & 3)) << 4);
  const int co = lane & 7;
  const float sc = bn_scale ? bn_scale[co] : 1.0f, sh = bn_scale ? bn_shift[co] : 0.0f,
              mu = bn_scale ? bn_mean[co] : 0.0f;
  // consume the BN loads here: first used inside the step loop, their wait would be a vmcnt(0) there
  // that also drains every step's plane prefetch
  asm volatile("" ::"v"(sc), "v"(sh), "v"(mu));
  const int oexp = -(ex + w_exp);
  const int gy = y0 + wave;
  const int gx0 = x0 + 4 * g;
  const bool store_lane = (lane & 15) < 8 && gy < H;
  const bool vec_store = (W & 3) == 0 && gx0 + 3 < W;
  __syncthreads();

  for (int k = 0; k < nsteps; ++k) {
    const int zs = z0 + kZS * k;
    if (k + 1 < nsteps) fetch(zs + kNPL - 1, kZS);   // the next step's new planes, in flight under the MFMAs
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 ah[kZS], al[kZS];
#pragma unroll
    for (int d = 0; d < kZS; ++d) {
      ah[d] = f4{0.0f, 0.0f, 0.0f, 0.0f};
      al[d] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const int sb = (kZS * k) % kNPL;   // ring slot of plane zs - 1
    const char* base[kNPL];
#pragma unroll
    for (int p = 0; p < kNPL; ++p) base[p] = lds + (sb + p >= kNPL ? sb + p - kNPL : sb + p) * kSlotB;
    // 45 items (ky, kx, p) in order; per item the A fragments (hi, lo) of plane p at tap (ky, kx)
    // feed every output depth they reach (d = p - kz).  Software pipeline: item it + kPF's A is read
    // from LDS before item it's MFMAs issue
    constexpr int kItems = 9 * kNPL;
    auto lda = [&](int it, h8v& hi, h8v& lo) {
      const int grp = it / kNPL, p = it % kNPL, ky = grp / 3, kx = grp % 3;
      hi = *reinterpret_cast<const h8v*>(base[p] + ky * kRowB + aoff[kx]);
      lo = *reinterpret_cast<const h8v*>(base[p] + kPartB + ky * kRowB + aoff[kx]);
    };
    // register ring of kPF + 1 A-fragment pairs: item it + kPF is read while item it's MFMAs issue
    h8v rh[kPF + 1], rl[kPF + 1];
#pragma unroll
    for (int it = 0; it < kPF; ++it) lda(it, rh[it], rl[it]);
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
      const int p = it % kNPL, grp = it / kNPL;
      if (it + kPF < kItems) lda(it + kPF, rh[(it + kPF) % (kPF + 1)], rl[(it + kPF) % (kPF + 1)]);
      const h8v ch = rh[it % (kPF + 1)], cl = rl[it % (kPF + 1)];
#pragma unroll
      for (int kz = 0; kz < 3; ++kz) {
        const int d = p - kz;   // output depth zs + d reads plane zs - 1 + p through tap kz
        if (d < 0 || d >= kZS) continue;
        ah[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch, bw[kz * 9 + grp], ah[d], 0, 0, 0);
        al[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cl, bw[kz * 9 + grp], al[d], 0, 0, 0);
      }
      // pin the schedule: the scheduler would otherwise sink each read next to its first use
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: lane (j < 8) of each row group adds its partner's (j + 8) w_lo columns;
    // acc[r] = output (x = 4 g + r, channel j) ----
#pragma unroll
    for (int d = 0; d < kZS; ++d) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float hh = ah[d][r], lh = al[d][r];
        const float hl = ror8(hh), ll = ror8(lh);
        float s = ldexpf(hh + ((lh + hl) + ll), oexp);
        if (bn_scale) s = fmaxf((s - mu) * sc + sh, 0.0f);
        v[r] = s;
      }
      const int z = zs + d;
      if (store_lane && z < z1) {
        float* o = out + ((size_t)(b * 8 + co) * D + z) * HW + (size_t)gy * W + gx0;
        if (vec_store) {
          // non-temporal: the 0.5 GB output is read once, by deconv_1_0 much later in the step
          // (1.10 -> 1.07 ms alone; profiles/r03/r03z_split_conv_experiments.md)
          __builtin_nontemporal_store(f4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<f4v*>(o));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (gx0 + r < W) o[r] = v[r];
        }
      }
    }
    if (k + 1 < nsteps) {
      __syncthreads();   // every wave is done with planes zs - 1 .. zs + kZS - 2
      stage(sb, kZS);    // planes zs + kNPL - 1 .. replace them
      __syncthreads();
    }
  }
}

}  // namespace

int launch_conv3d_split(const void* x, bool presplit, const void* wfrag, int w_exp, const uint32_t* absmax, float* y,
                        int B, int D, int H, int W, const float* bn_scale, const float* bn_shift, const float* bn_mean,
                        hipStream_t s) {
  const int tiles_x = (W + kSX - 1) / kSX, tiles_y = (H + kSY - 1) / kSY, zchunks = (D + kZC - 1) / kZC;
  const long total = (long)tiles_x * tiles_y * zchunks * B;
  if (total >= (1L << 31) - 8) return MVS_ERR_TOO_LARGE;
  hipLaunchKernelGGL(presplit ? conv0_split_kernel<true> : conv0_split_kernel<false>, xcd_grid((int)total),
                     dim3(kThreads), 0, s,
                     reinterpret_cast<const f4v*>(x), reinterpret_cast<const h8v*>(wfrag), absmax, w_exp, y, D, H,
                     W, tiles_x, tiles_y, zchunks, (int)total, bn_scale, bn_shift, bn_mean);
  return MVS_OK;
}

}  // namespace mvs
