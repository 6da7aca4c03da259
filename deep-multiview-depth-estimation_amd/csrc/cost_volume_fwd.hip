// cost_volume_fwd.hip -- FUSED homography warp + variance cost volume (the north-star kernel).
//
// Reference: scripts/homography.py:6-92 (warp every view onto D planes, kornia warp_perspective)
// followed by scripts/costvolume.py:3-16 (cv = sum_v (x_v - mean)^2 / V), model.py:177-181.
// Here both are one pass: every view is sampled and the two-pass variance is formed in registers,
// so the B*V x C x D x h x w warped volume never exists; cv[B][C][D][h][w] is written once.
//
// Structure of cost_volume_tile_kernel (V = 2..8 views):
//   * features are first packed channel-quad-last, packed[N][C/4][h][w][4] (one float4 per pixel
//     and 4-channel chunk), so one LDS slot / one 16-B load carries 4 channels of a tap;
//   * a 256-thread workgroup owns a 32 x 8 pixel tile of one sample and a group of `pg` depth
//     planes; 32-pixel rows make every cost-volume store a 128-B line segment (a 16-wide tile
//     measured 3.2 TB/s store-only vs 5.0 TB/s at 32 wide, tools/microbench/store_patterns.hip);
//   * each thread keeps, in registers, the tap corner + fractions of its pixel for every
//     (plane, source view); the reference view's sampling is plane independent (C_i = C_r gives
//     P = I exactly), so it is sampled once per channel chunk and reused for every plane;
//   * the union footprint of the tile over the plane group is reduced across the workgroup for
//     every view and staged in LDS, 4 channels at a time.  Staging of chunk c+1 is issued into
//     registers BEFORE chunk c's cost-volume stores (vmcnt counts loads and stores in order, so
//     the loads are then waited for without waiting for the stores), and written to LDS after;
//   * a plane group whose union footprint does not fit the 40 KB LDS budget is processed plane by
//     plane; a plane that still does not fit samples straight from the packed global features.
// Workgroup ids are remapped so each XCD walks consecutive (tile, plane group) items.
#include "launchers.h"

namespace mvs {
namespace {

// Generic fused kernel for 9..16 views: one thread per pixel of one (sample, plane), direct dword
// gathers from the NCHW features through buffer descriptors.
template <int MAXV, bool EXACT, int CU>
__global__ __launch_bounds__(kBlock) void cost_volume_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling, float* __restrict__ cv,
    int nv_rt, int C, int h, int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode_flat(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  const bool active = p < hw;
  float xn, yn;
  pixel_coords(active ? p : 0u, w, h, xn, yn);

  Taps tp[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) make_taps(sampling + ((size_t)(it.b * V + v) * Dc + it.kk) * 9, xn, yn, h, w, tp[v]);

  const float* fb = feat + (size_t)it.b * V * C * hw;
  float* ob = cv + ((size_t)it.b * C * Dc + it.kk) * hw;
  const size_t ostride = (size_t)Dc * hw;
  const uint32_t plane_bytes = hw * 4u;
  Rsrc rs[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) rs[v] = make_rsrc(fb + (size_t)v * C * hw, (uint32_t)C * plane_bytes);
  const float inv_v = 1.0f / (float)V;
  const uint32_t pbyte = p * 4u;

  for (int c0 = 0; c0 < C; c0 += CU) {
    float val[CU][MAXV];
#pragma unroll
    for (int cu = 0; cu < CU; ++cu) {
      if (c0 + cu < C) {
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
          if (v < V) val[cu][v] = gather_buf(rs[v], (uint32_t)(c0 + cu) * plane_bytes, tp[v]);
      }
    }
#pragma unroll
    for (int cu = 0; cu < CU; ++cu) {
      if (c0 + cu < C) {
        // costvolume.py:12-14 -- mean = sum/V, cv = sum (x - mean)^2 / V (two-pass)
        float sum = val[cu][0];
#pragma unroll
        for (int v = 1; v < MAXV; ++v)
          if (v < V) sum += val[cu][v];
        const float mean = sum * inv_v;
        float acc = 0.0f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
          if (v < V) {
            const float dlt = val[cu][v] - mean;
            acc += dlt * dlt;
          }
        if (active) store_buf(make_rsrc(ob + (size_t)(c0 + cu) * ostride, plane_bytes), pbyte, acc * inv_v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// packing: feat[N][C][h][w] -> packed[N][C4][h][w] float4, C4 = ceil(C / 4), zero-padded channels
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void pack4_kernel(const float* __restrict__ feat,
                                                       float4* __restrict__ packed, int N, int C,
                                                       uint32_t hw) {
  const int c4 = (C + 3) / 4;
  const size_t n = (size_t)N * c4 * hw;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (size_t)gridDim.x * kBlock) {
    const size_t p = e % hw;
    const size_t t = e / hw;
    const int ch = (int)(t % c4);
    const size_t i = t / c4;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = ch * 4 + j;
      v[j] = c < C ? feat[(i * C + c) * hw + p] : 0.0f;
    }
    packed[e] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// ------------------------------------------------------------------------------------------
// tile kernel
// ------------------------------------------------------------------------------------------
constexpr int kTileW = 32;
constexpr int kTileH = kBlock / kTileW;   // 8
constexpr int kLdsSlots = 2560;           // 40 KB of float4 slots -> 4 workgroups per CU
constexpr int kPrefetch = 4;              // staging pieces per thread carried in registers

template <int V>
#ifndef MVS_EXP_PG
#define MVS_EXP_PG 4
#endif
constexpr int group_planes() { return V <= 3 ? MVS_EXP_PG : (V <= 5 ? 4 : 2); }

// Footprint of one view in LDS: pixels [x0, x0+rw) x [y0, y0+rh), row-major from slot `base`.
struct Region {
  int x0, y0, rw, rh, base;
};

__device__ inline float4 f4zero() { return make_float4(0.0f, 0.0f, 0.0f, 0.0f); }

__device__ inline void fma4(float4& acc, const float4& a, float w) {
  acc.x = __fmaf_rn(a.x, w, acc.x);
  acc.y = __fmaf_rn(a.y, w, acc.y);
  acc.z = __fmaf_rn(a.z, w, acc.z);
  acc.w = __fmaf_rn(a.w, w, acc.w);
}

// bilinear sample of 4 channels from a staged region
__device__ inline float4 gather_lds4(const float4* lds, const Region& r, uint32_t pos, float wx,
                                     float wy) {
  float4 acc = f4zero();
  if (pos == kInvalidTap) return acc;
  const int p = r.base + (pos_y(pos) - r.y0) * r.rw + (pos_x(pos) - r.x0);
  float wt[4];
  tap_weights(wx, wy, wt);
  fma4(acc, lds[p], wt[0]);
  fma4(acc, lds[p + 1], wt[1]);
  fma4(acc, lds[p + r.rw], wt[2]);
  fma4(acc, lds[p + r.rw + 1], wt[3]);
  return acc;
}

// bilinear sample of 4 channels straight from a packed global plane (fallback path)
__device__ inline float4 gather_glb4(const float4* __restrict__ src, uint32_t pos, float wx, float wy,
                                     int h, int w) {
  float4 acc = f4zero();
  if (pos == kInvalidTap) return acc;
  const int x0 = pos_x(pos), y0 = pos_y(pos);
  float wt[4];
  tap_weights(wx, wy, wt);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int x = x0 + (t & 1), y = y0 + (t >> 1);
    const bool ok = x >= 0 && x < w && y >= 0 && y < h;
    const float4 a = src[ok ? (size_t)y * w + x : 0];
    fma4(acc, a, ok ? wt[t] : 0.0f);
  }
  return acc;
}

// Workgroup-wide min of NV ints; every thread gets the result as a wave-uniform value.
template <int NV>
__device__ inline void block_min(int (&v)[NV], int* scratch /* >= 4 * NV ints of LDS */) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
    v[k] = x;
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[wave * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int x = scratch[k];
#pragma unroll
    for (int q = 1; q < kBlock / 64; ++q) x = min(x, scratch[q * NV + k]);
    v[k] = __builtin_amdgcn_readfirstlane(x);
  }
  __syncthreads();
}

template <int V>
struct Plan {
  Region reg[V];
  int cum[V + 1];    // prefix sums of region sizes (pieces = pixels)
  float inv_rw[V];   // 1 / rw for the piece -> (row, col) split
  bool fits;
};

// One staging piece = one pixel (float4) of one view's region.  Regions are selected with an
// unrolled compare chain (static indices only: a runtime-indexed Region array would live in scratch).
template <int V>
__device__ inline int piece_slot(const Plan<V>& pl, int q, int& view, int& gx, int& gy) {
  int v = 0, x0 = pl.reg[0].x0, y0 = pl.reg[0].y0, rw = pl.reg[0].rw, base = pl.reg[0].base, cum = 0;
  float inv = pl.inv_rw[0];
#pragma unroll
  for (int k = 1; k < V; ++k)
    if (q >= pl.cum[k]) {
      v = k;
      x0 = pl.reg[k].x0;
      y0 = pl.reg[k].y0;
      rw = pl.reg[k].rw;
      base = pl.reg[k].base;
      cum = pl.cum[k];
      inv = pl.inv_rw[k];
    }
  view = v;
  const int e = q - cum;
  const int row = (int)(((float)e + 0.5f) * inv);
  const int col = e - row * rw;
  gx = x0 + col;
  gy = y0 + row;
  return base + e;
}

template <int V, int KPG>
__global__ __launch_bounds__(kBlock) void cost_volume_tile_kernel(
    const float4* __restrict__ packed, const float* __restrict__ sampling, float* __restrict__ cv,
    int C, int h, int w, int Dc, int pg, int tiles_x, int tiles_y, int groups, int total) {
  constexpr int NS = V - 1;
  __shared__ float4 lds[kLdsSlots];
  __shared__ int scratch[4 * 4 * V];

  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int g = wk % groups;
  const int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  const int b = t / (tiles_x * tiles_y);
  const int px = (tile % tiles_x) * kTileW + (int)(threadIdx.x % kTileW);
  const int py = (tile / tiles_x) * kTileH + (int)(threadIdx.x / kTileW);
  const bool active = px < w && py < h;
  const int k0 = g * pg;
  const int npl = min(pg, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const int c4 = (C + 3) / 4;
  const float xn = norm_coord(active ? px : 0, w);
  const float yn = norm_coord(active ? py : 0, h);

  // tap state: view 0 (plane independent), then (plane, source view)
  uint32_t rpos;
  float rwx, rwy;
  src_coords(sampling + ((size_t)(b * V) * Dc + k0) * 9, xn, yn, h, w, active, rpos, rwx, rwy);
  uint32_t pos[KPG][NS];
  float fwx[KPG][NS], fwy[KPG][NS];
#pragma unroll
  for (int pl = 0; pl < KPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pos[pl][s] = kInvalidTap;
      fwx[pl][s] = fwy[pl][s] = 0.0f;
      if (pl < npl)
        src_coords(sampling + ((size_t)(b * V + 1 + s) * Dc + k0 + pl) * 9, xn, yn, h, w, active,
                   pos[pl][s], fwx[pl][s], fwy[pl][s]);
    }

  // footprints of planes [lo, hi): view 0 from rpos, source views from pos[lo..hi)
  auto make_plan = [&](int lo, int hi, Plan<V>& P) {
    int bb[4 * V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      int mnx = 1 << 30, mny = 1 << 30, mxx = 1 << 30, mxy = 1 << 30;  // mx*: -(max + 1)
      auto take = [&](uint32_t p) {
        if (p != kInvalidTap) {
          mnx = min(mnx, pos_x(p));
          mny = min(mny, pos_y(p));
          mxx = min(mxx, -(pos_x(p) + 1));
          mxy = min(mxy, -(pos_y(p) + 1));
        }
      };
      if (v == 0) {
        take(rpos);
      } else {
#pragma unroll
        for (int pl = 0; pl < KPG; ++pl)
          if (pl >= lo && pl < hi) take(pos[pl][v - 1]);
      }
      bb[4 * v + 0] = mnx;
      bb[4 * v + 1] = mny;
      bb[4 * v + 2] = mxx;
      bb[4 * v + 3] = mxy;
    }
    block_min<4 * V>(bb, scratch);
    int off = 0;
    P.cum[0] = 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      Region& r = P.reg[v];
      r.x0 = bb[4 * v + 0];
      r.y0 = bb[4 * v + 1];
      const int x1 = -bb[4 * v + 2], y1 = -bb[4 * v + 3];
      const bool empty = r.x0 > x1;
      r.rw = empty ? 0 : x1 - r.x0 + 1;
      r.rh = empty ? 0 : y1 - r.y0 + 1;
      r.base = off;
      off += r.rw * r.rh;
      P.cum[v + 1] = off;
      P.inv_rw[v] = r.rw > 0 ? 1.0f / (float)r.rw : 0.0f;
    }
    P.fits = off <= kLdsSlots;
  };

  const float inv_v = 1.0f / (float)V;

  // staging: pieces q = threadIdx.x + kBlock * j; the first kPrefetch per thread go through
  // registers (issued early), the rest are copied synchronously
  float4 pre[kPrefetch];
  int pslot[kPrefetch];
  auto src_of = [&](int v, int ch) {
    return packed + ((size_t)(b * V + v) * c4 + ch) * hw;
  };
  auto prefetch = [&](const Plan<V>& P, int ch) {
#pragma unroll
    for (int j = 0; j < kPrefetch; ++j) {
      const int q = (int)threadIdx.x + kBlock * j;
      pslot[j] = -1;
      pre[j] = f4zero();
      if (q < P.cum[V]) {
        int v, gx, gy;
        pslot[j] = piece_slot<V>(P, q, v, gx, gy);
        if (gx >= 0 && gx < w && gy >= 0 && gy < h) pre[j] = src_of(v, ch)[(size_t)gy * w + gx];
      }
    }
  };
  auto commit = [&](const Plan<V>& P, int ch) {
#pragma unroll
    for (int j = 0; j < kPrefetch; ++j)
      if (pslot[j] >= 0) lds[pslot[j]] = pre[j];
    for (int q = (int)threadIdx.x + kBlock * kPrefetch; q < P.cum[V]; q += kBlock) {
      int v, gx, gy;
      const int slot = piece_slot<V>(P, q, v, gx, gy);
      lds[slot] = (gx >= 0 && gx < w && gy >= 0 && gy < h) ? src_of(v, ch)[(size_t)gy * w + gx]
                                                           : f4zero();
    }
  };

  // one plane's 4 channels: sample every view, two-pass variance, store
  auto emit = [&](int pl, int ch, const float4& x0, const float4 (&xs)[NS > 0 ? NS : 1]) {
    if (!active) return;
    float* ob = cv + ((size_t)b * C * Dc + (size_t)(k0 + pl)) * hw + (size_t)py * w + px;
    const float* xv0 = &x0.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = ch * 4 + j;
      if (c < C) {
        float sum = xv0[j];
#pragma unroll
        for (int s = 0; s < NS; ++s) sum += (&xs[s].x)[j];
        const float mean = sum * inv_v;
        float d = xv0[j] - mean;
        float acc = d * d;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          d = (&xs[s].x)[j] - mean;
          acc += d * d;
        }
        __builtin_nontemporal_store(acc * inv_v, ob + (size_t)c * Dc * hw);
      }
    }
  };

  Plan<V> P;
  make_plan(0, npl, P);
  const bool whole = P.fits;
  const int nsub = whole ? 1 : npl;
  for (int sr = 0; sr < nsub; ++sr) {
    const int lo = whole ? 0 : sr, hi = whole ? npl : sr + 1;
    if (!whole) make_plan(lo, hi, P);
    if (P.fits) {
      prefetch(P, 0);
      for (int ch = 0; ch < c4; ++ch) {
        __syncthreads();   // every wave is done reading the previous chunk
        commit(P, ch);
        __syncthreads();   // chunk ch is in LDS
        if (ch + 1 < c4) prefetch(P, ch + 1);   // in flight during this chunk's stores
        const float4 x0 = gather_lds4(lds, P.reg[0], rpos, rwx, rwy);
#pragma unroll
        for (int pl = 0; pl < KPG; ++pl) {
          if (pl < lo || pl >= hi) continue;
          float4 xs[NS > 0 ? NS : 1];
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            // opaque copies: keep per-(plane, view) address/weight math inside the chunk loop
            uint32_t tpos = pos[pl][s];
            float twx = fwx[pl][s], twy = fwy[pl][s];
            asm volatile("" : "+v"(tpos), "+v"(twx), "+v"(twy));
            xs[s] = gather_lds4(lds, P.reg[1 + s], tpos, twx, twy);
          }
          emit(pl, ch, x0, xs);
          __builtin_amdgcn_sched_barrier(0);  // one plane's LDS reads in flight at a time
        }
      }
      __syncthreads();   // LDS reused by the next sub-range's staging
    } else {
      // footprint too large even for one plane (extreme zoom): sample the packed global features.
      // Rare, so kept register-light: runtime plane loop, taps recomputed from G.
      for (int ch = 0; ch < c4; ++ch) {
        const float4 x0 = gather_glb4(src_of(0, ch), rpos, rwx, rwy, h, w);
#pragma unroll 1
        for (int pl = lo; pl < hi; ++pl) {
          float4 xs[NS > 0 ? NS : 1];
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            uint32_t tpos;
            float twx, twy;
            src_coords(sampling + ((size_t)(b * V + 1 + s) * Dc + k0 + pl) * 9, xn, yn, h, w,
                       active, tpos, twx, twy);
            xs[s] = gather_glb4(src_of(1 + s, ch), tpos, twx, twy, h, w);
          }
          emit(pl, ch, x0, xs);
        }
      }
    }
  }
}

// Direct-gather variant: same tiling, tap state and stores as the LDS kernel, but every view is
// sampled straight from the packed global features (one 16-B load per tap and 4-channel chunk);
// no LDS, no barriers, so occupancy is set by registers alone.
template <int V, int KPG>
__global__ __launch_bounds__(kBlock) void cost_volume_direct_tile_kernel(
    const float4* __restrict__ packed, const float* __restrict__ sampling, float* __restrict__ cv,
    int C, int h, int w, int Dc, int pg, int tiles_x, int tiles_y, int groups, int total) {
  constexpr int NS = V - 1;
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int g = wk % groups;
  const int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  const int b = t / (tiles_x * tiles_y);
  const int px = (tile % tiles_x) * kTileW + (int)(threadIdx.x % kTileW);
  const int py = (tile / tiles_x) * kTileH + (int)(threadIdx.x / kTileW);
  const bool active = px < w && py < h;
  if (!active) return;   // no barriers in this kernel
  const int k0 = g * pg;
  const int npl = min(pg, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const int c4 = (C + 3) / 4;
  const float xn = norm_coord(px, w);
  const float yn = norm_coord(py, h);
  uint32_t rpos;
  float rwx, rwy;
  src_coords(sampling + ((size_t)(b * V) * Dc + k0) * 9, xn, yn, h, w, true, rpos, rwx, rwy);
  uint32_t pos[KPG][NS];
  float fwx[KPG][NS], fwy[KPG][NS];
#pragma unroll
  for (int pl = 0; pl < KPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pos[pl][s] = kInvalidTap;
      fwx[pl][s] = fwy[pl][s] = 0.0f;
      if (pl < npl)
        src_coords(sampling + ((size_t)(b * V + 1 + s) * Dc + k0 + pl) * 9, xn, yn, h, w, true,
                   pos[pl][s], fwx[pl][s], fwy[pl][s]);
    }
  const float inv_v = 1.0f / (float)V;
  float* obase = cv + ((size_t)b * C * Dc + (size_t)k0) * hw + (size_t)py * w + px;
  for (int ch = 0; ch < c4; ++ch) {
    const float4* src0 = packed + ((size_t)(b * V) * c4 + ch) * hw;
    const float4 x0 = gather_glb4(src0, rpos, rwx, rwy, h, w);
#pragma unroll
    for (int pl = 0; pl < KPG; ++pl) {
      if (pl >= npl) continue;
      float4 xs[NS > 0 ? NS : 1];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        uint32_t tpos = pos[pl][s];
        float twx = fwx[pl][s], twy = fwy[pl][s];
        asm volatile("" : "+v"(tpos), "+v"(twx), "+v"(twy));
        xs[s] = gather_glb4(packed + ((size_t)(b * V + 1 + s) * c4 + ch) * hw, tpos, twx, twy, h, w);
      }
      float* ob = obase + (size_t)pl * hw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ch * 4 + j;
        if (c < C) {
          const float a0 = (&x0.x)[j];
          float sum = a0;
#pragma unroll
          for (int s = 0; s < NS; ++s) sum += (&xs[s].x)[j];
          const float mean = sum * inv_v;
          float d = a0 - mean;
          float acc = d * d;
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            d = (&xs[s].x)[j] - mean;
            acc += d * d;
          }
          __builtin_nontemporal_store(acc * inv_v, ob + (size_t)c * Dc * hw);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <int V>
void launch_tile(const Geometry& g, const float* feat, const float* smp, float* packed, float* cv,
                 hipStream_t s) {
  const uint32_t hw = (uint32_t)g.h * (uint32_t)g.w;
  const size_t n_pack = (size_t)g.B * V * ((g.C + 3) / 4) * hw;
  const size_t pblocks = (n_pack + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(pack4_kernel, dim3((unsigned)(pblocks < 4096 ? pblocks : 4096)), dim3(kBlock), 0,
                     s, feat, reinterpret_cast<float4*>(packed), g.B * V, g.C, hw);
  const int tiles_x = (g.w + kTileW - 1) / kTileW, tiles_y = (g.h + kTileH - 1) / kTileH;
  // planes per workgroup: the register maximum, halved until the grid has >= 8 workgroups per CU
  int pg = group_planes<V>();
  while (pg > 1 && (long)g.B * tiles_x * tiles_y * ((g.Dc + pg - 1) / pg) < 2048) pg >>= 1;
  const int groups = (g.Dc + pg - 1) / pg;
  const int total = g.B * tiles_x * tiles_y * groups;
#if !defined(MVS_FWD_LDS)
  hipLaunchKernelGGL((cost_volume_direct_tile_kernel<V, group_planes<V>()>), xcd_grid(total),
                     dim3(kBlock), 0, s, reinterpret_cast<const float4*>(packed), smp, cv, g.C, g.h,
                     g.w, g.Dc, pg, tiles_x, tiles_y, groups, total);
#else
  hipLaunchKernelGGL((cost_volume_tile_kernel<V, group_planes<V>()>), xcd_grid(total), dim3(kBlock), 0,
                     s, reinterpret_cast<const float4*>(packed), smp, cv, g.C, g.h, g.w, g.Dc, pg,
                     tiles_x, tiles_y, groups, total);
#endif
}

template <int MAXV, bool EXACT>
void launch_direct(const Geometry& g, const float* feat, const float* smp, float* cv, hipStream_t s) {
  hipLaunchKernelGGL((cost_volume_kernel<MAXV, EXACT, 4>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, smp, cv, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
}

}  // namespace

size_t packed_bytes(int B, int V, int C, int h, int w) {
  return (size_t)B * V * ((C + 3) / 4) * (size_t)h * (size_t)w * sizeof(float4);
}

void launch_cost_volume_fwd(const Geometry& g, const float* feat, const float* sampling,
                            float* packed, float* cv, hipStream_t s) {
  switch (g.V) {
    case 2: launch_tile<2>(g, feat, sampling, packed, cv, s); break;
    case 3: launch_tile<3>(g, feat, sampling, packed, cv, s); break;
    case 4: launch_tile<4>(g, feat, sampling, packed, cv, s); break;
    case 5: launch_tile<5>(g, feat, sampling, packed, cv, s); break;
    case 6: launch_tile<6>(g, feat, sampling, packed, cv, s); break;
    case 7: launch_tile<7>(g, feat, sampling, packed, cv, s); break;
    case 8: launch_tile<8>(g, feat, sampling, packed, cv, s); break;
    default: launch_direct<MVS_MAX_VIEWS, false>(g, feat, sampling, cv, s); break;
  }
}

}  // namespace mvs
