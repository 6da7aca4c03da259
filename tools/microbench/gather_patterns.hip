// Gather-pattern microbenchmark: cost of one 64-lane 16-byte load instruction on gfx950 for the
// access shapes of the cost-volume gather (L2-resident source, 8 waves per SIMD).
// Each kernel issues ITERS x 8 buffer_load_dwordx4 per wave; we report ns per wave-instruction
// per CU (chip time x CUs / instructions) and effective B/clk/CU at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int ITERS = 256;
constexpr int W = 162;   // padded row pitch in 16-B slots (w = 160)

__device__ inline f4v ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// mode 0: coalesced (lane l reads slot base + l)
// mode 1: tile gather: lanes = 2 rows x 32 px, slot = (row + y) * W + x + shift (tap pattern)
// mode 2: like 1 but odd lanes OOB (50 % invalid, interleaved)
// mode 3: like 1 but lanes 32..63 OOB (50 % invalid, whole half)
// mode 4: all lanes OOB
// mode 5: like 1, exec-masked half (lanes >= 32 skip the load)
// mode 6: broadcast (all lanes same slot)
// mode 7: dword loads coalesced (4 B per lane)
// mode 8: tile gather 4 rows x 16 px (square-ish)
template <int MODE>
__global__ __launch_bounds__(256) void k(const float4* src, uint32_t n_slots, float* out, int spread) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(n_slots * 16u), 0x00020000);
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  uint32_t slot;
  if (MODE == 0 || MODE == 6 || MODE == 7) slot = (MODE == 6) ? 0 : lane;
  else if (MODE == 8) slot = (lane >> 4) * W + (lane & 15);
  else slot = (lane >> 5) * W + (lane & 31);
  uint32_t base = spread ? (uint32_t)(wave * 37 % 97) * 2 * W : 0u;   // spread: ~200 rows (L2); else L1
  uint32_t off = (base + slot) * 16u;
  if (MODE == 2 && (lane & 1)) off = 0x80000000u;
  if (MODE == 3 && lane >= 32) off = 0x80000000u;
  if (MODE == 4) off = 0x80000000u;
  f4v acc = {0, 0, 0, 0};
  for (int it = 0; it < ITERS; ++it) {
    const uint32_t step = (uint32_t)(it & 7) * W * 16u;   // walk down rows, stays in L2
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t o = off + step + (uint32_t)((t & 1) * 16 + (t >> 1) * W * 16);
      if (MODE == 7) {
        acc.x += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)((base * 16u) + lane * 4u + step + t * 256u), 0, 0));
      } else if (MODE == 5) {
        if (lane < 32) acc += ld(r, o);
      } else {
        acc += ld(r, o);
      }
    }
  }
  if (acc.x + acc.y + acc.z + acc.w == 123.456f) out[0] = acc.x;
}

template <int MODE>
void run(const char* name, const float4* src, uint32_t n, float* out, int cus, int spread) {
  const int blocks = cus * 8;   // 8 WGs x 4 waves per CU = 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) k<MODE><<<blocks, 256>>>(src, n, out, spread);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) k<MODE><<<blocks, 256>>>(src, n, out, spread);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  const double instr_per_cu = (double)blocks * 4 * ITERS * 8 / cus;
  const double cyc = ms * 1e-3 * 2.4e9 / instr_per_cu;
  printf("%s %-34s %8.4f ms  %6.2f cyc/instr/CU  %6.1f B/clk/CU (16B x 64 lanes)\n", spread ? "L2" : "L1", name, ms, cyc,
         1024.0 / cyc);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const uint32_t n = 300 * W;   // 300 padded rows = 777 KB
  float4* src;
  float* out;
  hipMalloc(&src, (size_t)n * 16);
  hipMemset(src, 0, (size_t)n * 16);
  hipMalloc(&out, 64);
  printf("CUs %d\n", cus);
  for (int spread = 0; spread < 2; ++spread) {
    run<0>("coalesced 1KB", src, n, out, cus, spread);
    run<1>("tile 2x32 taps", src, n, out, cus, spread);
    run<2>("tile 2x32, odd lanes OOB", src, n, out, cus, spread);
    run<3>("tile 2x32, upper half OOB", src, n, out, cus, spread);
    run<4>("all lanes OOB", src, n, out, cus, spread);
    run<5>("tile 2x32, upper half exec-off", src, n, out, cus, spread);
    run<6>("broadcast", src, n, out, cus, spread);
    run<7>("dword coalesced (256B)", src, n, out, cus, spread);
    run<8>("tile 4x16 taps", src, n, out, cus, spread);
  }
  hipFree(src);
  hipFree(out);
  return 0;
}
