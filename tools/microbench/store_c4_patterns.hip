// Store-pattern microbenchmark for the CHANNEL-QUAD cost volume cv[B][C/4][D][h][w][4] (16 B per
// voxel quad; cfg 2: 2 GB), the layout the inference step's fused kernel writes.  Every kernel writes
// every 16-byte element exactly once (nt stores, like the fused kernel); only the work -> lane mapping
// and the order of the stores differ.  Question: which mapping reaches the chip's plain-store rate
// (MI355X_MICROARCH.md: 6.0-6.2 TB/s) -- the fused kernel's 32 x 8-tile x 8-plane pattern measured
// 0.41 ms = 4.9 TB/s store-only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int B = 4, C4 = 8, D = 192, H = 128, W = 160, HW = H * W;

__device__ inline int xcd(int L, int total) {
  int q = (total + 7) >> 3;
  return (L & 7) * q + (L >> 3);
}
__device__ inline void st(f4* p, f4 v) { __builtin_nontemporal_store(v, p); }

// (a) linear float4 stream (the ceiling)
__global__ void k_linear(f4* o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st(o + i, f4{1, 2, 3, 4});
}

// (b) the fused kernel's mapping: WG = (b, 32x8 tile, group of PG planes); chunk-outer, plane-inner
template <int TW, int PG, bool PLANE_OUTER>
__global__ void k_tile(f4* o, int total) {
  constexpr int TH = 256 / TW;
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tx = W / TW, ty = H / TH, groups = D / PG;
  const int g = wk % groups, t = wk / groups, tile = t % (tx * ty), b = t / (tx * ty);
  const int px = (tile % tx) * TW + threadIdx.x % TW, py = (tile / tx) * TH + threadIdx.x / TW;
  const size_t pix = (size_t)py * W + px;
  if (PLANE_OUTER) {
    for (int pl = 0; pl < PG; ++pl)
      for (int ch = 0; ch < C4; ++ch) st(o + (((size_t)b * C4 + ch) * D + g * PG + pl) * HW + pix, f4{1, 2, 3, 4});
  } else {
    for (int ch = 0; ch < C4; ++ch)
      for (int pl = 0; pl < PG; ++pl) st(o + (((size_t)b * C4 + ch) * D + g * PG + pl) * HW + pix, f4{1, 2, 3, 4});
  }
}

// (c) flat: WG = (b, 256 consecutive pixels, PG planes): a wave's stores are 1 KB contiguous, the
// WG's 4 KB
template <int PG, bool PLANE_OUTER>
__global__ void k_flat(f4* o, int total) {
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tiles = HW / 256, groups = D / PG;
  const int g = wk % groups, t = wk / groups, tile = t % tiles, b = t / tiles;
  const size_t pix = (size_t)tile * 256 + threadIdx.x;
  if (PLANE_OUTER) {
    for (int pl = 0; pl < PG; ++pl)
      for (int ch = 0; ch < C4; ++ch) st(o + (((size_t)b * C4 + ch) * D + g * PG + pl) * HW + pix, f4{1, 2, 3, 4});
  } else {
    for (int ch = 0; ch < C4; ++ch)
      for (int pl = 0; pl < PG; ++pl) st(o + (((size_t)b * C4 + ch) * D + g * PG + pl) * HW + pix, f4{1, 2, 3, 4});
  }
}

// (d) tile mapping, but XCD-blocked by chunk: consecutive work ids walk the planes of ONE chunk first
// (the WG loops over planes only; the chunk comes from the work id) -- each XCD then streams into a
// few long runs instead of 64 distinct regions per WG
template <int PG>
__global__ void k_tile_chunkwise(f4* o, int total) {
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tx = W / 32, ty = H / 8, groups = D / PG;
  const int g = wk % groups, t0 = wk / groups, tile = t0 % (tx * ty), t1 = t0 / (tx * ty), ch = t1 % C4,
            b = t1 / C4;
  const int px = (tile % tx) * 32 + threadIdx.x % 32, py = (tile / tx) * 8 + threadIdx.x / 32;
  const size_t pix = (size_t)py * W + px;
  for (int pl = 0; pl < PG; ++pl) st(o + (((size_t)b * C4 + ch) * D + g * PG + pl) * HW + pix, f4{1, 2, 3, 4});
}

// (e) VOXEL-MAJOR layout cv[B][D][h][w][C/4] (a voxel's 8 quads = one 128-B line): the fused
// kernel's mapping (lane = pixel, chunk-outer), so one wave-store writes 64 lines 16 B each and the
// 8 chunk passes complete them; (f) the same layout with lane = (pixel, quad): 8 lanes fill a line
template <int PG>
__global__ void k_vox_chunk_outer(f4* o, int total) {
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tx = W / 32, ty = H / 8, groups = D / PG;
  const int g = wk % groups, t = wk / groups, tile = t % (tx * ty), b = t / (tx * ty);
  const int px = (tile % tx) * 32 + threadIdx.x % 32, py = (tile / tx) * 8 + threadIdx.x / 32;
  const size_t pix = (size_t)py * W + px;
  for (int ch = 0; ch < C4; ++ch)
    for (int pl = 0; pl < PG; ++pl) st(o + (((size_t)b * D + g * PG + pl) * HW + pix) * C4 + ch, f4{1, 2, 3, 4});
}
template <int PG>
__global__ void k_vox_chunk_outer_plain(f4* o, int total) {   // (e) with plain (L2-allocating) stores
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tx = W / 32, ty = H / 8, groups = D / PG;
  const int g = wk % groups, t = wk / groups, tile = t % (tx * ty), b = t / (tx * ty);
  const int px = (tile % tx) * 32 + threadIdx.x % 32, py = (tile / tx) * 8 + threadIdx.x / 32;
  const size_t pix = (size_t)py * W + px;
  for (int ch = 0; ch < C4; ++ch)
    for (int pl = 0; pl < PG; ++pl) o[(((size_t)b * D + g * PG + pl) * HW + pix) * C4 + ch] = f4{1, 2, 3, 4};
}
template <int PG>
__global__ void k_vox_lane_quad(f4* o, int total) {
  int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  const int tx = W / 32, ty = H / 8, groups = D / PG;
  const int g = wk % groups, t = wk / groups, tile = t % (tx * ty), b = t / (tx * ty);
  for (int pass = 0; pass < C4; ++pass) {   // 8 passes of 32 pixels x 8 quads per 256 lanes
    const int e = pass * 256 + threadIdx.x, ch = e & 7, p = e >> 3;
    const int px = (tile % tx) * 32 + p % 32, py = (tile / tx) * 8 + p / 32;
    const size_t pix = (size_t)py * W + px;
    for (int pl = 0; pl < PG; ++pl) st(o + (((size_t)b * D + g * PG + pl) * HW + pix) * C4 + ch, f4{1, 2, 3, 4});
  }
}

template <typename F>
void timeit(const char* name, F launch, size_t bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(a);
  const int it = 10;
  for (int i = 0; i < it; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= it;
  printf("%-34s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  const size_t n = (size_t)B * C4 * D * HW, bytes = n * 16;
  f4* o;
  if (hipMalloc(&o, bytes) != hipSuccess) return 1;
  auto g = [](int total) { return dim3(8 * ((total + 7) / 8)); };
  timeit("linear f4 nt", [&] { k_linear<<<8192, 256>>>(o, n); }, bytes);
  const int t32_8 = B * (W / 32) * (H / 8) * (D / 8);
  timeit("tile32x8 pg8 chunk-outer (fused)", [&] { k_tile<32, 8, false><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  timeit("tile32x8 pg8 plane-outer", [&] { k_tile<32, 8, true><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  const int t32_4 = B * (W / 32) * (H / 8) * (D / 4);
  timeit("tile32x8 pg4 chunk-outer", [&] { k_tile<32, 4, false><<<g(t32_4), 256>>>(o, t32_4); }, bytes);
  const int t32_16 = B * (W / 32) * (H / 8) * (D / 16);
  timeit("tile32x8 pg16 chunk-outer", [&] { k_tile<32, 16, false><<<g(t32_16), 256>>>(o, t32_16); }, bytes);
  const int t64 = B * (W / 32) * (H / 4) * (D / 8);   // 64x4 would not divide W = 160: 32x8 vs 16x16 below
  const int t16 = B * (W / 16) * (H / 16) * (D / 8);
  timeit("tile16x16 pg8 chunk-outer", [&] { k_tile<16, 8, false><<<g(t16), 256>>>(o, t16); }, bytes);
  (void)t64;
  const int tf8 = B * (HW / 256) * (D / 8);
  timeit("flat256 pg8 chunk-outer", [&] { k_flat<8, false><<<g(tf8), 256>>>(o, tf8); }, bytes);
  timeit("flat256 pg8 plane-outer", [&] { k_flat<8, true><<<g(tf8), 256>>>(o, tf8); }, bytes);
  const int tf2 = B * (HW / 256) * (D / 2);
  timeit("flat256 pg2 chunk-outer", [&] { k_flat<2, false><<<g(tf2), 256>>>(o, tf2); }, bytes);
  const int tc = B * C4 * (W / 32) * (H / 8) * (D / 8);
  timeit("tile32x8 pg8 chunk per WG", [&] { k_tile_chunkwise<8><<<g(tc), 256>>>(o, tc); }, bytes);
  const int tc2 = B * C4 * (W / 32) * (H / 8) * (D / 32);
  timeit("tile32x8 pg32 chunk per WG", [&] { k_tile_chunkwise<32><<<g(tc2), 256>>>(o, tc2); }, bytes);
  timeit("voxel-major, lane=pixel chunk-outer", [&] { k_vox_chunk_outer<8><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  timeit("voxel-major, lane=pixel chunk-outer, plain", [&] { k_vox_chunk_outer_plain<8><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  timeit("voxel-major, lane=(pixel,quad)", [&] { k_vox_lane_quad<8><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  timeit("tile32x8 pg8 chunk-outer (fused)", [&] { k_tile<32, 8, false><<<g(t32_8), 256>>>(o, t32_8); }, bytes);
  hipFree(o);
  return 0;
}
