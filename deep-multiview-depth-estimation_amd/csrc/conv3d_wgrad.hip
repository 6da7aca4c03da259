// conv3d_wgrad.hip -- weight gradient of the narrow full-volume convolutions under autograd
// (train.py:97-104 through CostVolumeReg: conv_0_0 Conv3d(32, 8, 3, padding 1), model.py:101, and
// conv_out Conv3d(8, 1, 3, padding 1), model.py:124), on the f32-input matrix cores.
//
//   dW[co][ci][t] = sum over the batch and every voxel v of gy[co][v] * x[ci][v + t - 1]
//
// is a GEMM with M = 27 taps (two 16-row blocks; rows 27..31 are dropped), N = c_out (<= 16 columns)
// and K = the voxels.  A persistent workgroup walks 32 x 8 x 4-voxel tiles: the tile's output
// gradient (c_out x 1024 values) is staged in LDS once, then per pass four input channels' halo
// blocks (6 x 10 x 34, zero padded), one channel per wave; a wave runs the tile's 256 K-steps of 4
// consecutive voxels as v_mfma_f32_16x16x4_f32 (A: the 16 taps x 4 voxels of its channel, read from
// LDS at per-lane tap offsets; B: 4 voxels x the c_out gradients), its accumulators per channel in
// registers across every tile it visits.  Each workgroup stores its partial [c_in][32][16] block;
// conv3d_wgrad_reduce_kernel sums the partials in a fixed order (deterministic).  Products and sums
// are fp32 (each MFMA step an fmaf chain), as a GEMM-based autograd would form them.
#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kWTX = 32, kWTY = 8, kWDT = 4;
constexpr int kWPX = kWTX + 2, kWPY = kWTY + 2, kWPD = kWDT + 2;
constexpr int kWPlane = kWPX * kWPY;         // 340
constexpr int kWStage = kWPD * kWPlane;      // 2040 floats per staged channel
constexpr int kWVox = kWTX * kWTY * kWDT;    // 1024 voxels per tile
constexpr int kGyPitch = kWVox + 2;          // B-operand rows: lanes (kq, co) on banks 2 co + kq
constexpr int kWgradBlocks = 512;            // persistent workgroups (2 per CU: 65 KB of LDS each)

template <int CIN, int COUT>
__global__ __launch_bounds__(kBlock) void conv3d_wgrad_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ gy,
                                                             float* __restrict__ part, int B, int D, int H,
                                                             int W, int tiles_x, int tiles_y, int dgroups) {
  static_assert(CIN % 4 == 0 && COUT >= 1 && COUT <= 16, "c_in in quads, c_out <= 16");
  constexpr int NP = CIN / 4;   // passes of 4 channels, one per wave
  __shared__ float xs[4 * kWStage];
  __shared__ float gys[COUT * kGyPitch];
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
  const int m16 = lane & 15, kq = lane >> 4;
  // A operand: lane (m16, kq) supplies tap rb * 16 + m16 (clamped: rows >= 27 are dropped) of voxel
  // 4 xg + kq of its wave's channel
  int toff[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int t = min(rb * 16 + m16, 26);
    toff[rb] = wave * kWStage + (t / 9) * kWPlane + ((t / 3) % 3) * kWPX + (t % 3) + kq;
  }
  // B operand: lane (kq, m16) supplies gy[co = m16][voxel 4 xg + kq] (0 for m16 >= c_out)
  const bool bon = m16 < COUT;
  const int boff = (bon ? m16 : 0) * kGyPitch + kq;
  f4v acc[NP][2];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  const size_t plane = (size_t)H * W, vol = (size_t)D * plane;
  const int total = B * dgroups * tiles_y * tiles_x;
  for (int tile = (int)blockIdx.x; tile < total; tile += (int)gridDim.x) {   // workgroup-uniform
    int t = tile;
    const int tx0 = (t % tiles_x) * kWTX;
    t /= tiles_x;
    const int ty0 = (t % tiles_y) * kWTY;
    t /= tiles_y;
    const int d0 = (t % dgroups) * kWDT;
    const int b = t / dgroups;
    __syncthreads();   // the previous tile's reads are done
    const float* gb = gy + (size_t)b * COUT * vol;
    for (int e = (int)threadIdx.x; e < COUT * kWVox; e += kBlock) {
      const int co = e / kWVox, v = e % kWVox;
      const int gx = tx0 + v % kWTX, gyy = ty0 + (v / kWTX) % kWTY, gz = d0 + v / (kWTX * kWTY);
      gys[co * kGyPitch + v] =
          (gx < W && gyy < H && gz < D) ? gb[(size_t)co * vol + (size_t)gz * plane + (size_t)gyy * W + gx] : 0.0f;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (p > 0) __syncthreads();   // the previous pass's A reads are done
      const float* xb = x + ((size_t)b * CIN + 4 * p) * vol;
      for (int e = (int)threadIdx.x; e < 4 * kWStage; e += kBlock) {
        const int u = e / kWStage, r = e % kWStage;
        const int pd = r / kWPlane, q = r % kWPlane;
        const int gz = d0 + pd - 1, gyy = ty0 + q / kWPX - 1, gx = tx0 + q % kWPX - 1;
        xs[e] = (gz >= 0 && gz < D && gyy >= 0 && gyy < H && gx >= 0 && gx < W)
                    ? xb[(size_t)u * vol + (size_t)gz * plane + (size_t)gyy * W + gx]
                    : 0.0f;
      }
      __syncthreads();
#pragma unroll 2
      for (int zy = 0; zy < kWDT * kWTY; ++zy) {
        const int lz = zy / kWTY, ly = zy % kWTY;
        const int abase = lz * kWPlane + ly * kWPX, bbase = zy * kWTX;
#pragma unroll
        for (int xg = 0; xg < kWTX / 4; ++xg) {
          float bv = gys[boff + bbase + 4 * xg];
          bv = bon ? bv : 0.0f;
          const float a0 = xs[toff[0] + abase + 4 * xg], a1 = xs[toff[1] + abase + 4 * xg];
          acc[p][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv, acc[p][0], 0, 0, 0);
          acc[p][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bv, acc[p][1], 0, 0, 0);
        }
      }
    }
  }
  // partial [c_in][32 rows][16 cols]: acc[p][rb][r] = D[row rb * 16 + 4 kq + r][col m16], channel 4 p + wave
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        part[(((size_t)blockIdx.x * CIN + 4 * p + wave) * 32 + rb * 16 + 4 * kq + r) * 16 + m16] = acc[p][rb][r];
}

// dW[co][ci][t] = sum over the partials in workgroup order (fixed: deterministic)
__global__ __launch_bounds__(kBlock) void conv3d_wgrad_reduce_kernel(const float* __restrict__ part, int nblocks,
                                                                    int cin, int cout, float* __restrict__ dw) {
  const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (i >= cout * cin * 27) return;
  const int t = i % 27, ci = (i / 27) % cin, co = i / (27 * cin);
  float s = 0.0f;
  for (int g = 0; g < nblocks; ++g) s += part[(((size_t)g * cin + ci) * 32 + t) * 16 + co];
  dw[i] = s;
}

int wgrad_blocks(int B, int D, int H, int W) {
  const long tiles = (long)B * ((D + kWDT - 1) / kWDT) * ((H + kWTY - 1) / kWTY) * ((W + kWTX - 1) / kWTX);
  return (int)(tiles < kWgradBlocks ? tiles : kWgradBlocks);
}

}  // namespace

size_t conv3d_wgrad_workspace_bytes(int B, int c_in, int D, int H, int W) {
  return (size_t)wgrad_blocks(B, D, H, W) * c_in * 32 * 16 * sizeof(float);
}

bool conv3d_wgrad_supported(int c_in, int c_out) {
  return (c_in == 32 && c_out == 8) || (c_in == 8 && c_out == 1) || (c_in == 8 && c_out == 8) ||
         (c_in == 16 && c_out == 8);
}

void launch_conv3d_wgrad(const float* x, const float* gy, int B, int c_in, int c_out, int D, int H, int W,
                         float* part, float* dw, hipStream_t s) {
  const int tiles_x = (W + kWTX - 1) / kWTX, tiles_y = (H + kWTY - 1) / kWTY, dgroups = (D + kWDT - 1) / kWDT;
  const int nb = wgrad_blocks(B, D, H, W);
#define MVS_WGRAD(CI, CO)                                                                                \
  hipLaunchKernelGGL((conv3d_wgrad_kernel<CI, CO>), dim3(nb), dim3(kBlock), 0, s, x, gy, part, B, D, H, W, \
                     tiles_x, tiles_y, dgroups)
  if (c_in == 32 && c_out == 8) MVS_WGRAD(32, 8);
  else if (c_in == 16 && c_out == 8) MVS_WGRAD(16, 8);
  else if (c_in == 8 && c_out == 8) MVS_WGRAD(8, 8);
  else MVS_WGRAD(8, 1);
#undef MVS_WGRAD
  const int n = c_out * c_in * 27;
  hipLaunchKernelGGL(conv3d_wgrad_reduce_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, part, nb, c_in,
                     c_out, dw);
}

}  // namespace mvs
