// Store-pattern microbenchmark for the cost-volume write: cv[B][C][D][h][w] fp32 (cfg 2: 2 GB).
// Every kernel writes every element exactly once; only the work->thread mapping differs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int B = 4, C = 32, D = 192, H = 128, W = 160, HW = H * W;

__device__ inline int xcd(int L, int total) { int q = (total + 7) >> 3; return (L & 7) * q + (L >> 3); }

// (a) linear float4 stream
__global__ void k_linear(float4* o, size_t n4) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(f4{1, 2, 3, 4}, (f4*)(o + i));
}
// (b) block = (b, k, 256 flattened px): 32 channel runs of 1 KB (dword per lane)
template <bool NT>
__global__ void k_flat256(float* o, int total) {
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tiles = HW / 256; int k = wk % D; int t = wk / D; int tile = t % tiles; int b = t / tiles;
  int p = tile * 256 + threadIdx.x;
  for (int c = 0; c < C; ++c) {
    float* dst = o + (((size_t)b * C + c) * D + k) * HW + p;
    if (NT) __builtin_nontemporal_store((float)c, dst); else *dst = (float)c;
  }
}
// (c) block = (b, k, 1024 px): float4 per lane, 32 channel runs of 4 KB
template <bool NT>
__global__ void k_flat1024v4(float* o, int total) {
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tiles = HW / 1024; int k = wk % D; int t = wk / D; int tile = t % tiles; int b = t / tiles;
  int p = tile * 1024 + threadIdx.x * 4;
  for (int c = 0; c < C; ++c) {
    float4* dst = (float4*)(o + (((size_t)b * C + c) * D + k) * HW + p);
    f4 v = {(float)c, (float)c, (float)c, (float)c}; if (NT) __builtin_nontemporal_store(v, (f4*)dst); else *(f4*)dst = v;
  }
}
// (d) v2: block = (b, 16x16 tile, 8 planes): 256 (c,k) planes x 16 rows x 64 B
template <int TW, int PG, bool NT>
__global__ void k_tile(float* o, int total) {
  constexpr int TH = 256 / TW;
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tx = W / TW, ty = H / TH, groups = D / PG;
  int g = wk % groups; int t = wk / groups; int tile = t % (tx * ty); int b = t / (tx * ty);
  int px = (tile % tx) * TW + threadIdx.x % TW, py = (tile / tx) * TH + threadIdx.x / TW;
  for (int ch = 0; ch < C / 8; ++ch)
    for (int pl = 0; pl < PG; ++pl)
      for (int j = 0; j < 8; ++j) {
        float* dst = o + (((size_t)b * C + ch * 8 + j) * D + g * PG + pl) * HW + py * W + px;
        if (NT) __builtin_nontemporal_store((float)j, dst); else *dst = (float)j;
      }
}
// (e) flat 256 px, 8 planes per block (planes inner), 32 channels
template <int PG, bool NT>
__global__ void k_flat256pg(float* o, int total) {
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tiles = HW / 256, groups = D / PG;
  int g = wk % groups; int t = wk / groups; int tile = t % tiles; int b = t / tiles;
  int p = tile * 256 + threadIdx.x;
  for (int ch = 0; ch < C / 8; ++ch)
    for (int pl = 0; pl < PG; ++pl)
      for (int j = 0; j < 8; ++j) {
        float* dst = o + (((size_t)b * C + ch * 8 + j) * D + g * PG + pl) * HW + p;
        if (NT) __builtin_nontemporal_store((float)j, dst); else *dst = (float)j;
      }
}

// (f) 32x8 tile, 8 planes: after a 4x4 quad transpose each lane owns 4 consecutive pixels of ONE
// channel -> one float4 store per (plane, 4-channel chunk) instead of four dword stores
template <bool NT>
__global__ void k_tile32q(float* o, int total) {
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tx = W / 32, ty = H / 8, groups = D / 8;
  int g = wk % groups; int t = wk / groups; int tile = t % (tx * ty); int b = t / (tx * ty);
  int lane = threadIdx.x;
  int j = lane & 3;                       // channel within the chunk
  int q = lane >> 2;                      // quad id: 64 quads = 8 per row x 8 rows
  int px = (tile % tx) * 32 + (q & 7) * 4, py = (tile / tx) * 8 + (q >> 3);
  for (int ch = 0; ch < C / 4; ++ch)
    for (int pl = 0; pl < 8; ++pl) {
      float* dst = o + (((size_t)b * C + ch * 4 + j) * D + g * 8 + pl) * HW + py * W + px;
      f4 v = {(float)j, 1, 2, 3};
      if (NT) __builtin_nontemporal_store(v, (f4*)dst); else *(f4*)dst = v;
    }
}
// (g) 64x4 tile, 8 planes, dword per lane, 4 channels per chunk (rows of 256 B)
template <bool NT>
__global__ void k_tile64(float* o, int total) {
  int wk = xcd(blockIdx.x, total); if (wk >= total) return;
  int tx = W / 32, ty = H / 4, groups = D / 8;   // W = 160 = 2.5 x 64: half-used tiles at the edge
  int g = wk % groups; int t = wk / groups; int tile = t % (tx * ty); int b = t / (tx * ty);
  (void)tile; (void)b; (void)g;
  int px = (tile % tx) * 32 + (int)(threadIdx.x % 64) / 2 * 0 + (int)(threadIdx.x % 32);
  int py = (tile / tx) * 4 + (int)(threadIdx.x / 64);
  // 32x4 per 128 threads: each tile is covered twice over two 8-plane halves to keep 256 threads
  int half = (threadIdx.x / 32) & 1;
  py = (tile / tx) * 4 + (int)(threadIdx.x / 64);
  for (int ch = 0; ch < C / 4; ++ch)
    for (int pl = 0; pl < 4; ++pl)
      for (int jj = 0; jj < 4; ++jj) {
        float* dst = o + (((size_t)b * C + ch * 4 + jj) * D + g * 8 + half * 4 + pl) * HW + py * W + px;
        if (NT) __builtin_nontemporal_store((float)jj, dst); else *dst = (float)jj;
      }
}

template <typename F>
void timeit(const char* name, F launch, size_t bytes) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(a);
  const int it = 10;
  for (int i = 0; i < it; ++i) launch();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= it;
  printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
}

int main() {
  size_t n = (size_t)B * C * D * HW, bytes = n * 4;
  float* o; hipMalloc(&o, bytes);
  int t256 = B * D * (HW / 256), t1024 = B * D * (HW / 1024);
  auto g = [](int total) { return dim3(8 * ((total + 7) / 8)); };
  timeit("linear float4 nt", [&] { k_linear<<<4096, 256>>>((float4*)o, n / 4); }, bytes);
  timeit("flat256 nt", [&] { k_flat256<true><<<g(t256), 256>>>(o, t256); }, bytes);
  timeit("flat256 plain", [&] { k_flat256<false><<<g(t256), 256>>>(o, t256); }, bytes);
  timeit("flat1024 v4 nt", [&] { k_flat1024v4<true><<<g(t1024), 256>>>(o, t1024); }, bytes);
  timeit("flat1024 v4 plain", [&] { k_flat1024v4<false><<<g(t1024), 256>>>(o, t1024); }, bytes);
  int tt = B * (W / 16) * (H / 16) * (D / 8);
  timeit("tile16 pg8 nt", [&] { k_tile<16, 8, true><<<g(tt), 256>>>(o, tt); }, bytes);
  timeit("tile16 pg8 plain", [&] { k_tile<16, 8, false><<<g(tt), 256>>>(o, tt); }, bytes);
  int tt1 = B * (W / 16) * (H / 16) * D;
  timeit("tile16 pg1 nt", [&] { k_tile<16, 1, true><<<g(tt1), 256>>>(o, tt1); }, bytes);
  int t32 = B * (W / 32) * (H / 8) * (D / 8);
  timeit("tile32 pg8 nt", [&] { k_tile<32, 8, true><<<g(t32), 256>>>(o, t32); }, bytes);
  int tf = B * (HW / 256) * (D / 8);
  timeit("flat256 pg8 nt", [&] { k_flat256pg<8, true><<<g(tf), 256>>>(o, tf); }, bytes);
  int tf2 = B * (HW / 256) * (D / 2);
  timeit("flat256 pg2 nt", [&] { k_flat256pg<2, true><<<g(tf2), 256>>>(o, tf2); }, bytes);
  timeit("tile32 pg8 plain", [&] { k_tile<32, 8, false><<<g(t32), 256>>>(o, t32); }, bytes);
  timeit("tile32 quad-f4 nt", [&] { k_tile32q<true><<<g(t32), 256>>>(o, t32); }, bytes);
  timeit("tile32 quad-f4 plain", [&] { k_tile32q<false><<<g(t32), 256>>>(o, t32); }, bytes);
  int t64 = B * (W / 32) * (H / 4) * (D / 8);
  timeit("tile32x4 halves nt", [&] { k_tile64<true><<<g(t64), 256>>>(o, t64); }, bytes);
  hipFree(o);
  return 0;
}
