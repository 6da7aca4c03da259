// Read-pattern microbenchmark for the consumers of the split cost volume (SCV, 16-B channel quads,
// cfg 2: 2 GB).  The stride-2 conv_1_0 (conv3d_s2_split.hip) stages, per workgroup and step, the
// 33 x 5 input footprint of 4 planes; in today's quad-major layout [B][8][D][H][W] x 16 B every
// footprint row is 8 separate 528-B runs (one per quad plane, 252 MB apart).  In a voxel-major
// layout [B][D][H][W][8] x 16 B the same row is one 4,224-B run.  Same bytes, same workgroup grid,
// same loads per thread; only the address of each 16-B element differs.  Question: is the consumers'
// ~2.5 TB/s the access pattern's DRAM rate?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int B = 4, Q = 8, D = 192, H = 128, W = 160, HW = H * W;
constexpr int OX = 16, OY = 2, FX = 2 * OX + 1, FY = 2 * OY + 1, FV = FX * FY;   // S2 footprint 33 x 5
constexpr int NEW = 4, ZC = 14;                                                // planes per step, outputs per chunk
constexpr int PRE = (NEW * FV * Q + 255) / 256;

__device__ inline int xcd(int L, int total) {
  int q = (total + 7) >> 3;
  return (L & 7) * q + (L >> 3);
}

// VOXEL_MAJOR: element (b, q, z, y, x) at ((b D + z) HW + y W + x) 8 + q, else ((b 8 + q) D + z) HW + y W + x
template <bool VOXEL_MAJOR>
__global__ __launch_bounds__(256) void k_s2(const f4* __restrict__ v, float* __restrict__ out, int total, int tx, int ty,
                                            int zch) {
  const int wk = xcd(blockIdx.x, total);
  if (wk >= total) return;
  int t = wk;
  const int ix0 = (t % tx) * 2 * OX - 1;
  t /= tx;
  const int iy0 = (t % ty) * 2 * OY - 1;
  t /= ty;
  const int iz0 = (t % zch) * 2 * ZC - 1;
  const int b = t / zch;
  f4 acc = {0, 0, 0, 0};
  for (int step = 0; step < ZC / 2 + 1; ++step) {
    f4 pre[PRE];
#pragma unroll
    for (int j = 0; j < PRE; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int q = e & 7, tt = e >> 3;
      const int pl = tt / FV, vv = tt - pl * FV;
      const int yy = vv / FX, xx = vv - yy * FX;
      const int z = iz0 + NEW * step + pl, y = iy0 + yy, x = ix0 + xx;
      const bool ok = e < NEW * FV * Q && z >= 0 && z < D && y >= 0 && y < H && x >= 0 && x < W;
      size_t idx = VOXEL_MAJOR ? ((((size_t)b * D + z) * HW + (size_t)y * W + x) * Q + q)
                               : ((((size_t)b * Q + q) * D + z) * HW + (size_t)y * W + x);
      pre[j] = ok ? v[idx] : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < PRE; ++j) acc += pre[j];
    __syncthreads();
  }
  out[(size_t)wk * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

__global__ void k_linear(const f4* __restrict__ v, float* __restrict__ out, size_t n) {
  f4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

template <typename F>
void timeit(const char* name, F launch, double bytes) {
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
  printf("%-40s %8.4f ms  %7.1f GB/s (volume bytes / time)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  const size_t n = (size_t)B * Q * D * HW, bytes = n * 16;
  f4* v;
  float* out;
  if (hipMalloc(&v, bytes) != hipSuccess) return 1;
  if (hipMalloc(&out, 64ull << 20) != hipSuccess) return 1;
  hipMemset(v, 0, bytes);
  const int tx = (W / 2 + OX - 1) / OX, ty = (H / 2 + OY - 1) / OY, zch = (D / 2 + ZC - 1) / ZC;
  const int total = tx * ty * zch * B;
  const int grid = 8 * ((total + 7) / 8);
  timeit("linear f4 read", [&] { k_linear<<<8192, 256>>>(v, out, n); }, (double)bytes);
  timeit("S2 footprint, quad-major (today)", [&] { k_s2<false><<<grid, 256>>>(v, out, total, tx, ty, zch); },
         (double)bytes);
  timeit("S2 footprint, voxel-major", [&] { k_s2<true><<<grid, 256>>>(v, out, total, tx, ty, zch); },
         (double)bytes);
  timeit("S2 footprint, quad-major (today)", [&] { k_s2<false><<<grid, 256>>>(v, out, total, tx, ty, zch); },
         (double)bytes);
  timeit("S2 footprint, voxel-major", [&] { k_s2<true><<<grid, 256>>>(v, out, total, tx, ty, zch); },
         (double)bytes);
  hipFree(v);
  hipFree(out);
  return 0;
}
