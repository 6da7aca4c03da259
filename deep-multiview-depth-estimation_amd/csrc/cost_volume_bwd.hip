// cost_volume_bwd.hip -- gradient of the fused warp + variance w.r.t. the features.
//
// Autograd of costvolume.py:14 (d cv / d x_v = 2 (x_v - mean) / V) composed with the
// grid_sample backward of homography.py:86 (each sample's gradient is scattered to its 4 bilinear
// taps), as train.py:103 exercises it.  One thread per output pixel of one (sample, plane): the
// samples are recomputed (no warped volume is stored) and scattered with float atomics into
// grad_feat[N][C][h][w] -- like torch's grid_sample backward on GPU, the summation order is not
// deterministic.
#include "launchers.h"

namespace mvs {
namespace {

// backward: g_x_v = 2 (x_v - mean) / V * g_cv, scattered to the 4 taps with bilinear weights
template <int MAXV, bool EXACT>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling,
    const float* __restrict__ grad_cv, float* __restrict__ grad_feat, int nv_rt, int C, int h,
    int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int V = EXACT ? MAXV : nv_rt;
  const WorkItem it = decode_flat(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  if (p >= hw) return;
  float xn, yn;
  pixel_coords(p, w, h, xn, yn);
  Taps tp[MAXV];
#pragma unroll
  for (int v = 0; v < MAXV; ++v)
    if (v < V) make_taps(sampling + ((size_t)(it.b * V + v) * Dc + it.kk) * 9, xn, yn, h, w, tp[v]);
  const float* fb = feat + (size_t)it.b * V * C * hw;
  float* gb = grad_feat + (size_t)it.b * V * C * hw;
  const float* gcv = grad_cv + ((size_t)it.b * C * Dc + it.kk) * hw + p;
  const float inv_v = 1.0f / (float)V;
  for (int c = 0; c < C; ++c) {
    const float g = gcv[(size_t)c * Dc * hw];
    float val[MAXV];
    float sum = 0.0f;
#pragma unroll
    for (int v = 0; v < MAXV; ++v)
      if (v < V) {
        val[v] = gather(fb + ((size_t)v * C + c) * hw, tp[v]);
        sum += val[v];
      }
    const float mean = sum * inv_v;
    const float k2 = 2.0f * inv_v * g;
#pragma unroll
    for (int v = 0; v < MAXV; ++v)
      if (v < V) {
        const float coef = k2 * (val[v] - mean);
        char* plane = reinterpret_cast<char*>(gb + ((size_t)v * C + c) * hw);
#pragma unroll
        for (int t = 0; t < 4; ++t)  // off[] are byte offsets
          if (tp[v].wt[t] != 0.0f)
            unsafeAtomicAdd(reinterpret_cast<float*>(plane + tp[v].off[t]), tp[v].wt[t] * coef);
      }
  }
}

// Grouped form (V = 2..8, the default): one thread per pixel of one (sample, group of PG planes).
// The reference view's sampling is plane independent (C_i = C_r gives P = I exactly; the forward
// resamples it once per launch), so its gradient coefficients are summed over the group's planes
// in registers and scattered once per group: PG times fewer reference-view atomics, and PG times
// less same-address contention (all planes of a pixel hit the same 4 reference taps).  Channels
// run in chunks of CC so the per-channel reference values and sums stay in registers.
constexpr int kBwdPG = 8, kBwdCC = 8;

template <int V>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_grouped_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling,
    const float* __restrict__ grad_cv, float* __restrict__ grad_feat, int C, int h, int w, int Dc,
    int tiles, int groups, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const int grp = wk % groups;
  const int t = wk / groups;
  const int tile = t % tiles;
  const int b = t / tiles;
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)tile * kBlock + threadIdx.x;
  if (p >= hw) return;
  const int k0 = grp * kBwdPG;
  const int npl = min(kBwdPG, Dc - k0);
  float xn, yn;
  pixel_coords(p, w, h, xn, yn);
  Taps tref;
  make_taps(sampling + ((size_t)(b * V) * Dc + k0) * 9, xn, yn, h, w, tref);
  const float* fb = feat + (size_t)b * V * C * hw;
  float* gb = grad_feat + (size_t)b * V * C * hw;
  const float* gcv = grad_cv + (size_t)b * C * Dc * hw + p;
  const float inv_v = 1.0f / (float)V;
  for (int c0 = 0; c0 < C; c0 += kBwdCC) {
    float rval[kBwdCC], racc[kBwdCC];
#pragma unroll
    for (int cc = 0; cc < kBwdCC; ++cc) {
      racc[cc] = 0.0f;
      rval[cc] = c0 + cc < C ? gather(fb + (size_t)(c0 + cc) * hw, tref) : 0.0f;
    }
    for (int kk = 0; kk < npl; ++kk) {
      const int k = k0 + kk;
      Taps tp[V - 1];
#pragma unroll
      for (int v = 1; v < V; ++v)
        make_taps(sampling + ((size_t)(b * V + v) * Dc + k) * 9, xn, yn, h, w, tp[v - 1]);
#pragma unroll
      for (int cc = 0; cc < kBwdCC; ++cc) {
        const int c = c0 + cc;
        if (c >= C) break;
        const float g = gcv[((size_t)c * Dc + k) * hw];
        float val[V];
        val[0] = rval[cc];
        float sum = val[0];
#pragma unroll
        for (int v = 1; v < V; ++v) {
          val[v] = gather(fb + ((size_t)v * C + c) * hw, tp[v - 1]);
          sum += val[v];
        }
        const float mean = sum * inv_v;
        const float k2 = 2.0f * inv_v * g;
        racc[cc] += k2 * (val[0] - mean);
#pragma unroll
        for (int v = 1; v < V; ++v) {
          const float coef = k2 * (val[v] - mean);
          char* plane = reinterpret_cast<char*>(gb + ((size_t)v * C + c) * hw);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (tp[v - 1].wt[q] != 0.0f)
              unsafeAtomicAdd(reinterpret_cast<float*>(plane + tp[v - 1].off[q]), tp[v - 1].wt[q] * coef);
        }
      }
    }
#pragma unroll
    for (int cc = 0; cc < kBwdCC; ++cc) {
      if (c0 + cc >= C) break;
      char* plane = reinterpret_cast<char*>(gb + (size_t)(c0 + cc) * hw);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (tref.wt[q] != 0.0f)
          unsafeAtomicAdd(reinterpret_cast<float*>(plane + tref.off[q]), tref.wt[q] * racc[cc]);
    }
  }
}

// LDS-accumulated form (V = 2..8, the default): a workgroup owns a 32 x 8 pixel tile of one sample
// and a group of 8 planes, like the forward's staged kernel.  Per channel, every source view's
// gradient taps land in an LDS image of that view's footprint over the group (bounding box of the
// tile's tap corners, ds_add_f32), which is then flushed with one global atomic per nonzero slot
// (instead of 4 per (pixel, plane)); the reference view is summed over the group's planes in
// registers as in the grouped form.  A tile whose footprints exceed the LDS budget scatters
// straight to global memory.
constexpr int kBwdTW = 32, kBwdTH = 8, kBwdSlots = 8192;   // 32 KB of fp32 accumulators

template <int V>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_lds_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling,
    const float* __restrict__ grad_cv, float* __restrict__ grad_feat, int C, int h, int w, int Dc,
    int tiles_x, int tiles_y, int groups, int total) {
  constexpr int NS = V - 1;
  __shared__ float acc_l[kBwdSlots];
  __shared__ int bb[4 * NS];
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;   // workgroup-uniform
  const int grp = wk % groups;
  const int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  const int b = t / (tiles_x * tiles_y);
  const int px = (tile % tiles_x) * kBwdTW + (int)(threadIdx.x % kBwdTW);
  const int py = (tile / tiles_x) * kBwdTH + (int)(threadIdx.x / kBwdTW);
  const bool active = px < w && py < h;
  const int k0 = grp * kBwdPG;
  const int npl = min(kBwdPG, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const float xn = norm_coord(active ? px : 0, w), yn = norm_coord(active ? py : 0, h);

  uint32_t pos[kBwdPG][NS];
  float fwx[kBwdPG][NS], fwy[kBwdPG][NS];
#pragma unroll
  for (int pl = 0; pl < kBwdPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int kk = k0 + (pl < npl ? pl : npl - 1);
      src_coords(sampling + ((size_t)(b * V + 1 + s) * Dc + kk) * 9, xn, yn, h, w, active, pos[pl][s],
                 fwx[pl][s], fwy[pl][s]);
      if (pl >= npl) pos[pl][s] = kInvalidTap;
    }
  if (threadIdx.x < 4 * NS) bb[threadIdx.x] = 1 << 30;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int mnx = 1 << 30, mny = 1 << 30, mxx = 1 << 30, mxy = 1 << 30;   // mx*: -(max corner)
#pragma unroll
    for (int pl = 0; pl < kBwdPG; ++pl) {
      const uint32_t p = pos[pl][s];
      if (p == kInvalidTap) continue;
      mnx = min(mnx, pos_x(p));
      mny = min(mny, pos_y(p));
      mxx = min(mxx, -pos_x(p));
      mxy = min(mxy, -pos_y(p));
    }
    if (mnx != (1 << 30)) {
      atomicMin(&bb[4 * s], mnx);
      atomicMin(&bb[4 * s + 1], mny);
      atomicMin(&bb[4 * s + 2], mxx);
      atomicMin(&bb[4 * s + 3], mxy);
    }
  }
  __syncthreads();
  int rx0[NS], ry0[NS], rw[NS], rh[NS], base[NS + 1];
  base[0] = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const bool empty = bb[4 * s] == (1 << 30);
    rx0[s] = empty ? 0 : bb[4 * s];
    ry0[s] = empty ? 0 : bb[4 * s + 1];
    rw[s] = empty ? 0 : -bb[4 * s + 2] - rx0[s] + 2;   // taps x0 .. x0 + 1
    rh[s] = empty ? 0 : -bb[4 * s + 3] - ry0[s] + 2;
    base[s + 1] = base[s] + rw[s] * rh[s];
  }
  const int nslots = base[NS];
  const bool use_lds = nslots <= kBwdSlots;

  Taps tref;
  make_taps(sampling + ((size_t)(b * V) * Dc + k0) * 9, xn, yn, h, w, tref);
  const float* fb = feat + (size_t)b * V * C * hw;
  float* gb = grad_feat + (size_t)b * V * C * hw;
  const uint32_t pix = (uint32_t)(active ? py : 0) * (uint32_t)w + (uint32_t)(active ? px : 0);
  const float* gcv = grad_cv + (size_t)b * C * Dc * hw + pix;
  const float inv_v = 1.0f / (float)V;

  for (int c = 0; c < C; ++c) {
    if (use_lds) {
      __syncthreads();   // the previous channel's flush has read every slot
      for (int q = (int)threadIdx.x; q < nslots; q += kBlock) acc_l[q] = 0.0f;
      __syncthreads();
    }
    if (active) {
      const float rv = gather(fb + (size_t)c * hw, tref);
      float racc = 0.0f;
      for (int pl = 0; pl < npl; ++pl) {
        const float g = gcv[((size_t)c * Dc + k0 + pl) * hw];
        float val[V], wt[NS][4];
        val[0] = rv;
        float sum = rv;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          float x = 0.0f;
          uint32_t p = kInvalidTap;
          float wx = 0.0f, wy = 0.0f;
#pragma unroll
          for (int q = 0; q < kBwdPG; ++q)   // static register indexing
            if (q == pl) {
              p = pos[q][s];
              wx = fwx[q][s];
              wy = fwy[q][s];
            }
          tap_weights(wx, wy, wt[s]);
          if (p != kInvalidTap) {
            const int x0 = pos_x(p), y0 = pos_y(p);
            const float* fp = fb + ((size_t)(1 + s) * C + c) * hw;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int xx = x0 + (q & 1), yy = y0 + (q >> 1);
              if (xx >= 0 && xx < w && yy >= 0 && yy < h) x += fp[(size_t)yy * w + xx] * wt[s][q];
              else wt[s][q] = 0.0f;
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) wt[s][q] = 0.0f;
          }
          val[1 + s] = x;
          sum += x;
        }
        const float mean = sum * inv_v;
        const float k2 = 2.0f * inv_v * g;
        racc += k2 * (val[0] - mean);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const float coef = k2 * (val[1 + s] - mean);
          uint32_t p = kInvalidTap;
#pragma unroll
          for (int q = 0; q < kBwdPG; ++q)
            if (q == pl) p = pos[q][s];
          if (p == kInvalidTap) continue;
          const int x0 = pos_x(p), y0 = pos_y(p);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (wt[s][q] == 0.0f) continue;
            const int xx = x0 + (q & 1), yy = y0 + (q >> 1);
            if (use_lds) {
              const int slot = base[s] + (yy - ry0[s]) * rw[s] + (xx - rx0[s]);
              atomicAdd(&acc_l[slot], wt[s][q] * coef);
            } else {
              unsafeAtomicAdd(gb + ((size_t)(1 + s) * C + c) * hw + (size_t)yy * w + xx, wt[s][q] * coef);
            }
          }
        }
      }
      char* rplane = reinterpret_cast<char*>(gb + (size_t)c * hw);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (tref.wt[q] != 0.0f)
          unsafeAtomicAdd(reinterpret_cast<float*>(rplane + tref.off[q]), tref.wt[q] * racc);
    }
    if (use_lds) {
      __syncthreads();   // every tap of this channel is in LDS
      for (int q = (int)threadIdx.x; q < nslots; q += kBlock) {
        const float v = acc_l[q];
        if (v == 0.0f) continue;
        int s = 0;
#pragma unroll
        for (int k = 1; k < NS; ++k)
          if (q >= base[k]) s = k;
        int ww = rw[0], xo = rx0[0], yo = ry0[0], bs = base[0];
#pragma unroll
        for (int k = 1; k < NS; ++k)
          if (s == k) {
            ww = rw[k];
            xo = rx0[k];
            yo = ry0[k];
            bs = base[k];
          }
        const int e = q - bs;
        const int yy = yo + e / ww, xx = xo + e % ww;
        if (xx >= 0 && xx < w && yy >= 0 && yy < h)   // always: only in-image taps were added
          unsafeAtomicAdd(gb + ((size_t)(1 + s) * C + c) * hw + (size_t)yy * w + xx, v);
      }
    }
  }
}

template <int V>
void launch_bwd_lds(const Geometry& g, const float* feat, const float* smp, const float* gcv, float* gf,
                    hipStream_t s) {
  const int tiles_x = (g.w + kBwdTW - 1) / kBwdTW, tiles_y = (g.h + kBwdTH - 1) / kBwdTH;
  const int groups = (g.Dc + kBwdPG - 1) / kBwdPG;
  const int total = g.B * tiles_x * tiles_y * groups;
  hipLaunchKernelGGL((cost_volume_bwd_lds_kernel<V>), xcd_grid(total), dim3(kBlock), 0, s, feat, smp, gcv,
                     gf, g.C, g.h, g.w, g.Dc, tiles_x, tiles_y, groups, total);
}

template <int V>
void launch_bwd_grouped(const Geometry& g, const float* feat, const float* smp, const float* gcv,
                        float* gf, hipStream_t s) {
  const int groups = (g.Dc + kBwdPG - 1) / kBwdPG;
  const int total = g.B * g.tiles * groups;
  hipLaunchKernelGGL((cost_volume_bwd_grouped_kernel<V>), xcd_grid(total), dim3(kBlock), 0, s, feat, smp,
                     gcv, gf, g.C, g.h, g.w, g.Dc, g.tiles, groups, total);
}

template <int MAXV, bool EXACT>
void launch_bwd(const Geometry& g, const float* feat, const float* smp, const float* gcv,
                float* gf, hipStream_t s) {
  hipLaunchKernelGGL((cost_volume_bwd_kernel<MAXV, EXACT>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, smp, gcv, gf, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
}

}  // namespace

void launch_cost_volume_bwd(const Geometry& g, const float* feat, const float* sampling,
                            const float* grad_cv, float* grad_feat, hipStream_t s) {
  switch (g.V) {
    case 1: launch_bwd<1, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
#ifdef MVS_EXP_BWD_FLAT
    case 2: launch_bwd<2, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 3: launch_bwd<3, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 5: launch_bwd<5, true>(g, feat, sampling, grad_cv, grad_feat, s); break;
#elif defined(MVS_EXP_BWD_GROUPED)
    case 2: launch_bwd_grouped<2>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 3: launch_bwd_grouped<3>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 4: launch_bwd_grouped<4>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 5: launch_bwd_grouped<5>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 6: launch_bwd_grouped<6>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 7: launch_bwd_grouped<7>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 8: launch_bwd_grouped<8>(g, feat, sampling, grad_cv, grad_feat, s); break;
#else
    case 2: launch_bwd_lds<2>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 3: launch_bwd_lds<3>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 4: launch_bwd_lds<4>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 5: launch_bwd_lds<5>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 6: launch_bwd_lds<6>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 7: launch_bwd_lds<7>(g, feat, sampling, grad_cv, grad_feat, s); break;
    case 8: launch_bwd_lds<8>(g, feat, sampling, grad_cv, grad_feat, s); break;
#endif
    default: launch_bwd<MVS_MAX_VIEWS, false>(g, feat, sampling, grad_cv, grad_feat, s); break;
  }
}

}  // namespace mvs
