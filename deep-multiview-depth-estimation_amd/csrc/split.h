// split.h -- split-fp16 operands of the f16 matrix-core kernels (conv3d_split.hip, conv3d_s2_split.hip)
// and of the cost volume that feeds them (cost_volume_fwd.hip, ES = kQuadSplit).
//
// A fp32 value v is scaled by 2^e (exact) and carried as hi = fp16(v 2^e), lo = fp16(v 2^e - hi), both
// rounded to nearest: hi + lo is v 2^e to 2^-22 relative (fp16's normal range; below it lo is a
// subnormal with absolute error <= 2^-25 of the 2^14 scale).  For a cost volume the scale comes from
// the bound words (max |feat|: the prologue's per-workgroup partial maxima, folded into 8 words by
// absmax_reduce_kernel; cost_volume_fwd.hip): every variance over views is at most
// max|feat|^2, so e = 14 - 2 exponent(max|feat|) keeps every scaled element below 2^14 (fp16 max 65504).
//
// Split cost-volume layout ("SCV"): the channel-quad layout cv[B][C/4][D][h][w] with each 16-byte
// element {hi(c0) hi(c1) hi(c2) hi(c3) lo(c0) lo(c1) lo(c2) lo(c3)} (fp16), scaled by 2^e.
#pragma once
#include "common.h"
#include "packed.h"

namespace mvs {

__device__ inline int cv_split_exponent(const uint32_t* __restrict__ absmax) {
  if (!absmax) return 0;
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) m = max(m, absmax[i]);
  if (m == 0u || m >= 0x7F800000u) return 0;   // all zero, or Inf/NaN present: unscaled
  int e;
  (void)frexpf(__uint_as_float(m), &e);   // max|feat| < 2^e
  return min(max(14 - 2 * e, -120), 120);
}

// hi / lo fp16 parts of 4 fp32 values times 2^e, packed 2 per dword.  Packed arithmetic: the scale as
// one fp32 multiply by 2^e (exact, e in [-120, 120]), v_cvt_pk_f16_f32 (nearest) for the parts, and
// the remainder v 2^e - hi as one packed fma (exact: hi holds the leading 11 bits)
__device__ inline void split4(const f4v v, int e, uint2& hi, uint2& lo) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const float sc = __builtin_ldexpf(1.0f, e);
  const f2 a = f2{v[0], v[1]} * sc, b = f2{v[2], v[3]} * sc;
  const h2 ha = __builtin_convertvector(a, h2), hb = __builtin_convertvector(b, h2);
  const h2 la = __builtin_convertvector(a - __builtin_convertvector(ha, f2), h2);
  const h2 lb = __builtin_convertvector(b - __builtin_convertvector(hb, f2), h2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, ha), __builtin_bit_cast(uint32_t, hb));
  lo = make_uint2(__builtin_bit_cast(uint32_t, la), __builtin_bit_cast(uint32_t, lb));
}

// fp32 of one split element (4 channels): (hi + lo) 2^-e, exact sum of the parts
__device__ inline f4v unsplit4(const uint4 p, int e) {
  auto h = [](uint32_t w, int k) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> (16 * k))); };
  return f4v{ldexpf(h(p.x, 0) + h(p.z, 0), -e), ldexpf(h(p.x, 1) + h(p.z, 1), -e),
             ldexpf(h(p.y, 0) + h(p.w, 0), -e), ldexpf(h(p.y, 1) + h(p.w, 1), -e)};
}

// Activation bounds of a region tensor ("bound words"): kBoundSlots partial maxima of |v| as fp32 bits
// (non-negative floats order like their bit patterns), raised by the producing kernel's epilogue into
// words the caller zeroed; the split-fp16 consumers scale the tensor by 2^act_split_exponent(bound).
// Each slot sits on its own 128-byte line (kBoundStride words apart) and a wave picks slot (global wave
// index mod kBoundSlots): device-scope atomics on one line serialise at the memory side, and with all
// slots on 2 lines the encoder's 61k-wave layers spent 0.2 ms in them (tools/enc_layers.py).  A wave
// whose max does not exceed its slot's current value skips the atomic (the slot only grows, so a stale
// read can only cause an unneeded atomic, never a missed one).
constexpr int kBoundSlots = 64, kBoundStride = 32, kBoundWords = kBoundSlots * kBoundStride;

// the tensor's bound: the max over its slots (whole wave; 0 without words)
__device__ inline float bound_read(const uint32_t* __restrict__ words) {
  if (!words) return 0.0f;
  uint32_t v = words[(threadIdx.x & 63) * kBoundStride];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return __uint_as_float(v);
}

// e with bound 2^e < 2^14 (fp16 max 65504); 0 for a zero or non-finite bound
__device__ inline int act_split_exponent(float bound) {
  if (!(bound > 0.0f) || !(bound <= 3.0e38f)) return 0;
  int e;
  (void)frexpf(bound, &e);   // bound < 2^e
  return min(max(14 - e, -120), 120);
}

// raise the bound words by this wave's max |v| (m >= 0 per lane; whole wave).  kCheck: read the slot
// first (the read's round trip holds the wave: for epilogues at a kernel's end; a persistent kernel's
// mid-loop update, cv_head.hip, sends the atomic unconditionally)
#ifndef MVS_BOUND_CHECK
#define MVS_BOUND_CHECK 1
#endif
template <bool kCheck = (MVS_BOUND_CHECK != 0)>
__device__ inline void bound_update(uint32_t* __restrict__ words, float m) {
  uint32_t v = __float_as_uint(m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  if ((threadIdx.x & 63) == 0) {
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    uint32_t* w = words + (wave % kBoundSlots) * kBoundStride;
    if (!kCheck || v > __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(w, v);
  }
}

}  // namespace mvs
