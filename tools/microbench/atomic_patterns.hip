// Atomic-throughput microbenchmark for the cost-volume backward's scatter (grad_feat, cfg 2:
// 12 x 32 x 128 x 160 fp32 = 31 MB).  Measures, per second:
//   (a) global float atomic adds (no return), each wave adding to 64 consecutive floats of a
//       pseudo-random row of the target (the footprint-flush pattern);
//   (b) the same with 64-bit integer atomic adds (fixed-point deterministic accumulation);
//   (c) LDS ds_add_f32, lanes on consecutive dwords (conflict-free);
//   (d) LDS 64-bit integer adds, lanes on consecutive qwords.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t kTarget = 12ull * 32 * 128 * 160;   // floats
constexpr int kIters = 64;

__device__ inline uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <typename T>
__global__ void k_global(T* t, uint32_t rows) {
  const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  for (int i = 0; i < kIters; ++i) {
    const uint32_t row = hash(wave * kIters + i) % rows;
    T* p = t + (size_t)row * 64 + lane;
    if constexpr (sizeof(T) == 4) unsafeAtomicAdd(p, (T)1.0f);
    else if constexpr (__is_same(T, double)) unsafeAtomicAdd(p, 1.0);
    else atomicAdd((unsigned long long*)p, 1ull);
  }
}

template <typename T>
__global__ void k_lds(T* out) {
  __shared__ T s[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) s[i] = 0;
  __syncthreads();
  for (int i = 0; i < 1024; ++i) {
    const int a = (threadIdx.x + i * 256) & 8191;
    if constexpr (__is_same(T, float)) atomicAdd(&s[a], 1.0f);
    else if constexpr (__is_same(T, unsigned)) atomicAdd(&s[a], 1u);
    else if constexpr (__is_same(T, int)) s[a] = i;   // plain ds_write baseline
    else if constexpr (__is_same(T, double)) unsafeAtomicAdd(&s[a], 1.0);
    else atomicAdd((unsigned long long*)&s[a], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[blockIdx.x & 8191];
}

template <typename F>
float time_ms(F f, int reps = 5) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  float* tf;
  unsigned long long* ti;
  hipMalloc(&tf, kTarget * 4);
  hipMalloc(&ti, kTarget * 8);
  hipMemset(tf, 0, kTarget * 4);
  hipMemset(ti, 0, kTarget * 8);
  const int blocks = 8192;
  const double n = (double)blocks * 256 * kIters;
  float ms = time_ms([&] { k_global<float><<<blocks, 256>>>(tf, (uint32_t)(kTarget / 64)); });
  printf("(a) global f32 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, n / 1e6, n / ms / 1e6);
  ms = time_ms([&] { k_global<unsigned long long><<<blocks, 256>>>((unsigned long long*)ti, (uint32_t)(kTarget / 64)); });
  printf("(b) global u64 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, n / 1e6, n / ms / 1e6);
  const double nl = 2048.0 * 256 * 1024;
  ms = time_ms([&] { k_lds<float><<<2048, 256>>>(tf); });
  printf("(c) LDS f32 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, nl / 1e6, nl / ms / 1e6);
  ms = time_ms([&] { k_lds<unsigned long long><<<2048, 256>>>(ti); });
  printf("(d) LDS u64 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, nl / 1e6, nl / ms / 1e6);
  ms = time_ms([&] { k_lds<unsigned><<<2048, 256>>>((unsigned*)ti); });
  printf("(e) LDS u32 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, nl / 1e6, nl / ms / 1e6);
  ms = time_ms([&] { k_lds<int><<<2048, 256>>>((int*)ti); });
  printf("(f) LDS plain b32 write: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, nl / 1e6, nl / ms / 1e6);
  ms = time_ms([&] { k_lds<double><<<2048, 256>>>((double*)ti); });
  printf("(g) LDS f64 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, nl / 1e6, nl / ms / 1e6);
  ms = time_ms([&] { k_global<double><<<blocks, 256>>>((double*)ti, (uint32_t)(kTarget / 64)); });
  printf("(h) global f64 atomic add: %.3f ms for %.0f M lanes = %.1f G/s\n", ms, n / 1e6, n / ms / 1e6);
  return 0;
}
