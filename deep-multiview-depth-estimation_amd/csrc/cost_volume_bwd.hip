// cost_volume_bwd.hip -- gradient of the fused warp + variance w.r.t. the features.
//
// Autograd of costvolume.py:14 (d cv / d x_v = 2 (x_v - mean) / V) composed with the grid_sample
// backward of homography.py:86 (each sample's gradient is scattered to its 4 bilinear taps), as
// train.py:103 exercises it.  No warped volume is stored: the samples are recomputed from the
// forward's packed features (packed.h), exactly as the forward computed them.
//
// LDS accumulation never uses fp32 atomics: on gfx950 ds_add_f32 runs at 0.20 T lanes/s against
// 4.3 T for ds_add_f64 and 5.1 T for ds_add_u64 (tools/microbench/atomic_patterns.hip).  Two modes:
//   default        footprint images in fp64 LDS (each contribution an fp32 product widened once),
//                  flushed with fp32 global atomics (summation order varies, like torch's
//                  grid_sample backward on GPU);
//   deterministic  (MVS_BWD_DETERMINISTIC; torch.use_deterministic_algorithms) 64-bit FIXED POINT
//                  everywhere: every contribution v is added as llrint(v * 2^S), with one shift S
//                  per launch derived on the device from max|grad_cv| and max|feat| so that no
//                  gradient element can exceed 2^62 (bound: d_count * h * w contributions of at most
//                  4 max|g| max|feat| / V each).  Integer addition is associative, so the result is
//                  bit-identical whatever the order in which workgroups and lanes add.  Resolution:
//                  2^-S = d_count*h*w*8*max|g|*max|feat|/V * 2^-61, about 1e-12 of the largest
//                  possible contribution at BASELINE cfg 2.
//
// Kernels (V = 2..8 views):
//   abs_max_kernel        (deterministic) max|grad_cv|, max|feat| (device scalars, atomicMax)
//   cost_volume_bwd_kernel  a 256-thread workgroup owns a 32 x 8 pixel tile of one sample, a
//                         group of 32 planes and one 4-channel chunk.  Per plane, every thread
//                         recomputes its pixel's samples of all views (packed float4 gathers),
//                         forms the per-view coefficients 2/V g (x_v - mean), keeps the reference
//                         view's sum over planes in registers (its taps do not depend on the
//                         plane), and adds each source view's 4 tap contributions into an LDS
//                         image of the tile's footprint (ds_add_f64 / ds_add_u64).  Footprints: the
//                         tile's 4 corners per (plane, view) (a homography maps the tile to a
//                         convex quad); consecutive planes share one LDS image while the union
//                         fits the budget, which is then flushed with one global atomic
//                         per slot and channel.  Taps outside the image box (rounding) or a plane
//                         whose footprint alone exceeds the budget go straight to global atomics.
//   ref_scatter_kernel    sums the reference view's per-group partials in a fixed order and
//                         scatters them to its (plane-independent) taps
//   fixed_to_float_kernel (deterministic) grad_feat = acc * 2^-S
// More than 8 views: one thread per (sample, plane, pixel) with NCHW gathers and global atomics.
#include "launchers.h"
#include "packed.h"

namespace mvs {
namespace {

constexpr int kBwdTW = 32, kBwdTH = 8;
constexpr int kBwdKPG = 32;              // planes per workgroup
// LDS accumulator image: slot-major, one slot = the 4 channels of one footprint pixel at a stride of
// kSlotWords = 5 8-byte words: consecutive slots then fall on distinct bank pairs of a 16-lane
// ds_add group (a stride of 4 words is a 4-way conflict: cfg 2 3.30 against 2.57 ms), and a tap's
// 4 channels are immediate offsets of one address.  48 KB per workgroup (1228 slots, 3 workgroups
// per CU): at V = 3 a single plane's footprint (both source views) fits, so no plane takes the
// global-atomic path, and a 32-plane group needs 2.2 passes on average (tools/bwd_plan.py); 36 KB
// at 4 workgroups per CU measured the same at cfg 2 and slower at cfg 1 and 3, 30 KB at 5 waves per
// SIMD 1.6x slower (5 % of the planes overflow to global atomics).
constexpr int kSlotWords = 5;
template <int V>
constexpr int bwd_slots() {
  return 49152 / (8 * kSlotWords);
}
typedef unsigned long long u64;

// ---- fixed point ------------------------------------------------------------------------------
struct Fixed {
  float to_fixed;    // 2^S
  double to_float;   // 2^-S
};

__device__ inline Fixed fixed_scale(const unsigned* __restrict__ mx, int V, int Dc, uint32_t hw) {
  const double gmax = (double)__uint_as_float(mx[0]), fmax = (double)__uint_as_float(mx[1]);
  // mx[2] != 0 (a NaN / Inf input): any finite scale; fixed_to_float_kernel writes NaN
  // |2/V g (x - mean)| <= 4 gmax fmax / V per contribution; a gradient element collects at most
  // Dc * hw of them (tap weights of one sample sum to 1); x2 margin for fp32 rounding
  const double bound = 8.0 * gmax * fmax / (double)V * (double)Dc * (double)hw;
  int S = 0;
  if (bound > 0.0 && bound < 1e300) {
    int e;
    frexp(bound, &e);   // bound < 2^e
    S = 61 - e;
  }
  S = S < -100 ? -100 : (S > 120 ? 120 : S);
  Fixed f;
  f.to_fixed = ldexpf(1.0f, S);
  f.to_float = ldexp(1.0, -S);
  return f;
}

__device__ inline u64 to_fixed(float v, float sc) { return (u64)(long long)__builtin_rintf(v * sc); }

__device__ inline void gadd(u64* p, u64 v) { atomicAdd(p, v); }

// ---- max|x| pre-pass ---------------------------------------------------------------------------
// out: the maximum as float bits; nonfinite: set to 1 when any element is NaN or +-Inf (the gradient
// is then NaN, fixed_to_float_kernel: fixed point cannot carry non-finite values)
__global__ __launch_bounds__(kBlock) void abs_max_kernel(const float* __restrict__ a, size_t n,
                                                         unsigned* __restrict__ out,
                                                         unsigned* __restrict__ nonfinite) {
  float m = 0.0f;
  bool bad = false;
  const size_t stride = (size_t)gridDim.x * kBlock;
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (((uintptr_t)a & 15u) == 0) {
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const size_t n4 = n / 4;
    for (size_t j = i; j < n4; j += stride) {
      const float4 v = a4[j];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    i += n4 * 4;
  }
  for (; i < n; i += stride) {
    m = fmaxf(m, fabsf(a[i]));
    bad |= !isfinite(a[i]);
  }
  // fmaxf drops NaN (it returns the other operand): NaN and Inf are tracked by `bad` instead
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));   // m >= 0: uint order = float order
  if (__builtin_amdgcn_ballot_w64(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(nonfinite, 1u);
}

// ---- per-(plane, view) footprint boxes -----------------------------------------------------------
// Box of the taps of a tile for one (plane, view), from the tile's 4 corner pixels: with the
// homogeneous coordinate s of one sign and |s| > 1e-8 at the corners (s is affine in the pixel, so
// then everywhere in the tile) the tile maps to a convex quad whose bounding box is the corners'
// bounding box (taps x0 .. x0 + 1).  Boxes are clipped to the image plus its one-pixel zero border
// ([-1, w] x [-1, h], where every tap of a valid sample lies): border slots collect the taps the
// zero padding drops, and are never flushed, so the accumulation needs no per-tap bounds test.  A
// sample whose taps fp32 rounding of an interior pixel puts just outside goes straight to the
// global accumulators.  Otherwise (pole in the tile): the whole bordered image.
struct Box {
  int x0, y0, x1, y1;   // inclusive, clipped to the image; x1 < x0 = empty
};

__device__ inline int box_area(const Box& b) {
  return (b.x1 < b.x0 || b.y1 < b.y0) ? 0 : (b.x1 - b.x0 + 1) * (b.y1 - b.y0 + 1);
}

__device__ inline Box box_union(const Box& a, const Box& b) {
  if (a.x1 < a.x0 || a.y1 < a.y0) return b;
  if (b.x1 < b.x0 || b.y1 < b.y0) return a;
  return Box{min(a.x0, b.x0), min(a.y0, b.y0), max(a.x1, b.x1), max(a.y1, b.y1)};
}

__device__ Box tile_box(const float* __restrict__ G, int px0, int py0, int px1, int py1, int h, int w) {
  float mnx = 1e30f, mny = 1e30f, mxx = -1e30f, mxy = -1e30f;
  bool pos = false, neg = false, bad = false;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float xn = norm_coord((c & 1) ? px1 : px0, w), yn = norm_coord((c & 2) ? py1 : py0, h);
    float u = __fmaf_rn(G[1], yn, __fmaf_rn(G[0], xn, G[2]));
    float v = __fmaf_rn(G[4], yn, __fmaf_rn(G[3], xn, G[5]));
    const float s = __fmaf_rn(G[7], yn, __fmaf_rn(G[6], xn, G[8]));
    if (!(fabsf(s) > 1e-8f)) bad = true;
    pos |= s > 0.0f;
    neg |= s < 0.0f;
    const float sc = __fdiv_rn(1.0f, __fadd_rn(s, 1e-8f));
    u = __fmul_rn(u, sc);
    v = __fmul_rn(v, sc);
    const float ix = __fsub_rn(__fmul_rn(__fadd_rn(u, 1.0f), 0.5f * (float)w), 0.5f);
    const float iy = __fsub_rn(__fmul_rn(__fadd_rn(v, 1.0f), 0.5f * (float)h), 0.5f);
    if (!(fabsf(ix) < 1e7f && fabsf(iy) < 1e7f)) bad = true;   // also NaN
    mnx = fminf(mnx, ix);
    mny = fminf(mny, iy);
    mxx = fmaxf(mxx, ix);
    mxy = fmaxf(mxy, iy);
  }
  if (bad || (pos && neg)) return Box{-1, -1, w, h};
  Box b;
  b.x0 = max((int)floorf(mnx), -1);
  b.y0 = max((int)floorf(mny), -1);
  b.x1 = min((int)floorf(mxx) + 1, w);
  b.y1 = min((int)floorf(mxy) + 1, h);
  return b;
}

// ---- main kernel (2 <= V <= 8) -----------------------------------------------------------------
// DET = false (default): the LDS footprint images accumulate in fp64 (ds_add_f64, ~4.3 T lanes/s;
// each contribution is an exact fp32 product widened once) and are flushed to grad_feat with fp32
// global atomics.  DET = true: 64-bit fixed point in LDS and in the global accumulators (see top).
template <bool DET>
struct Acc;
template <>
struct Acc<false> {
  typedef double lds_t;
  __device__ static lds_t conv(float v, float) { return (double)v; }
};
template <>
struct Acc<true> {
  typedef u64 lds_t;
  __device__ static lds_t conv(float v, float sc) { return to_fixed(v, sc); }
};

template <int V, bool DET>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_kernel(
    const float4* __restrict__ packed, const float4* __restrict__ refs,
    const float* __restrict__ sampling, const float* __restrict__ grad_cv, u64* __restrict__ acc,
    float* __restrict__ grad_feat, float4* __restrict__ ref_part, const unsigned* __restrict__ mx, int B,
    int C, int h, int w, int Dc, int tiles_x, int tiles_y, int groups, int total) {
  constexpr int NS = V - 1;
  typedef typename Acc<DET>::lds_t lds_t;
  constexpr int kBwdSlots = bwd_slots<V>();
  __shared__ lds_t lds[kSlotWords * kBwdSlots];
  __shared__ Box boxes[kBwdKPG][NS];

  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;   // workgroup-uniform
  const int c4 = (C + 3) / 4;
  const int grp = wk % groups;
  int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  t /= tiles_x * tiles_y;
  const int ch = t % c4;
  const int b = t / c4;
  const int tx0 = (tile % tiles_x) * kBwdTW, ty0 = (tile / tiles_x) * kBwdTH;
  const int px = tx0 + (int)(threadIdx.x % kBwdTW), py = ty0 + (int)(threadIdx.x / kBwdTW);
  const bool active = px < w && py < h;
  const int k0 = grp * kBwdKPG;
  const int npl = min(kBwdKPG, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const PadGeom pg = pad_geom(h, w);
  const float sc = DET ? fixed_scale(mx, V, Dc, hw).to_fixed : 1.0f;

  // footprint box of every (plane, view): one (plane, view) per thread
  if ((int)threadIdx.x < npl * NS) {
    const int pl = (int)threadIdx.x / NS, s = (int)threadIdx.x % NS;
    boxes[pl][s] = tile_box(sampling + ((size_t)(b * V + 1 + s) * Dc + k0 + pl) * 9, tx0, ty0,
                            min(tx0 + kBwdTW, w) - 1, min(ty0 + kBwdTH, h) - 1, h, w);
  }

  const float xn = norm_coord(active ? px : 0, w), yn = norm_coord(active ? py : 0, h);
  const uint32_t pix = (uint32_t)(active ? py : 0) * (uint32_t)w + (uint32_t)(active ? px : 0);
  const float4 r4 = refs[((size_t)b * c4 + ch) * hw + pix];
  const f4v x0 = {r4.x, r4.y, r4.z, r4.w};
  const f4v inv_v = {1.0f / (float)V, 1.0f / (float)V, 1.0f / (float)V, 1.0f / (float)V};
  const f4v two_inv_v = inv_v + inv_v;
  const ViewDiv vd = view_div(V);   // the forward's mean (packed.h variance_law4)
  const int soff = (int)((uint32_t)ch * pg.plane * 16u);
  const int row_bytes = pg.pitch * 16;
  // grad_cv of channel 4 ch + j, plane k0 + pl at this pixel: byte j * cst_bytes + (pl * hw + pix) * 4
  const int nch = min(C - ch * 4, 4);
  const uint32_t cst_bytes = (uint32_t)Dc * hw * 4u;   // < 2^29 (mvs_cost_volume_bwd checks 16 Dc hw)
  const Rsrc grs = make_rsrc(uniform_ptr(grad_cv + (((size_t)b * C + (size_t)ch * 4) * Dc + k0) * hw),
                             (uint32_t)uniform((int)((uint32_t)(nch - 1) * cst_bytes + (uint32_t)(Dc - k0) * hw * 4u)));
  // per-image planes of this chunk's channels (global accumulators / gradient)
  auto gidx = [&](int n, int j, int yy, int xx) -> size_t {
    return ((size_t)n * C + (size_t)ch * 4 + j) * hw + (size_t)yy * w + xx;
  };
  auto gadd_out = [&](int n, int j, int yy, int xx, lds_t v) {
    if constexpr (DET) gadd(acc + gidx(n, j, yy, xx), v);
    else unsafeAtomicAdd(grad_feat + gidx(n, j, yy, xx), (float)v);
  };
  // per source view: sampling matrices of the group's planes, packed-feature descriptor (uniform)
  const float* smat[NS];
  Rsrc prs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    smat[s] = uniform_ptr(sampling + ((size_t)(b * V + 1 + s) * Dc + k0) * 9);
    prs[s] = make_rsrc(uniform_ptr(packed + (size_t)(b * V + 1 + s) * c4 * pg.plane), (uint32_t)c4 * pg.plane * 16u);
  }
  f4v racc = {0.0f, 0.0f, 0.0f, 0.0f};
  __syncthreads();   // boxes

  // view subsets: consecutive source views whose largest single-plane footprints fit the budget
  // together (all views at once unless the views are many or the footprints large); every subset
  // recomputes the samples, the reference view's sum is kept in the first subset's passes only
  int amax[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int m = 0;
    for (int pl = 0; pl < npl; ++pl) m = max(m, box_area(boxes[pl][s]));
    amax[s] = uniform(m);
  }
  for (int s0 = 0; s0 < NS;) {
    int s1 = s0 + 1, sub_area = amax[s0];
#pragma unroll
    for (int s = 1; s < NS; ++s)
      if (s == s1 && s1 < NS && sub_area + amax[s] <= kBwdSlots) {
        sub_area += amax[s];
        ++s1;
      }
  for (int kp = 0; kp < npl;) {
    // ---- plan a pass: consecutive planes whose union footprint fits the LDS budget (uniform) ----
    Box ub[NS];
    int area = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const Box bx = boxes[kp][s];
      ub[s] = (s >= s0 && s < s1) ? Box{uniform(bx.x0), uniform(bx.y0), uniform(bx.x1), uniform(bx.y1)}
                                  : Box{0, 0, -1, -1};
      area += box_area(ub[s]);
    }
    int ke = kp + 1;
    if (area <= kBwdSlots) {
      for (; ke < npl; ++ke) {
        Box nb[NS];
        int na = 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const Box bx = boxes[ke][s];
          nb[s] = (s >= s0 && s < s1)
                      ? box_union(ub[s], Box{uniform(bx.x0), uniform(bx.y0), uniform(bx.x1), uniform(bx.y1)})
                      : ub[s];
          na += box_area(nb[s]);
        }
        if (na > kBwdSlots) break;
#pragma unroll
        for (int s = 0; s < NS; ++s) ub[s] = nb[s];
        area = na;
      }
    }
    const bool use_lds = area <= kBwdSlots;
    const int T = use_lds ? area : 0;   // slots of the LDS image
    int base[NS], bw[NS];
    {
      int o = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        base[s] = o;
        bw[s] = ub[s].x1 - ub[s].x0 + 1;
        o += box_area(ub[s]);
      }
    }
    if (use_lds) {
      for (int q = (int)threadIdx.x; q < kSlotWords * T; q += kBlock) lds[q] = (lds_t)0;
      __syncthreads();
    }

    // ---- the pass's planes (every lane runs them; inactive lanes have g = 0 and no taps) ----
    // grad_cv of the chunk's 4 channels at this pixel, one plane ahead (the HBM read of the loop)
    // (buffer loads, no branches or selects: channels >= C lie past the descriptor's range and read
    // 0; inactive lanes read pixel 0 and have no taps.  Every plane issues the same 4 loads, so the
    // waits on them are counted exactly)
    auto load_g = [&](int pl) {
      f4v g;
      const uint32_t o = ((uint32_t)pl * hw + pix) * 4u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        g[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, o + (uint32_t)j * cst_bytes, 0, 0));
      return g;
    };
    // Run-length accumulation in registers (V <= 3).  A sample's tap corner moves slowly with
    // the plane (it repeats from one plane to the next for ~70 % of the samples at cfg 2, for every
    // lane of the wave ~50 % of the time), so each lane sums its 16 tap x channel contributions in
    // fp32 registers while its corner stays put and adds them to the LDS image (16 ds_add_f64) only
    // when the corner moves and at the end of the pass; a wave with no moved corner skips the adds
    // with one scalar branch.  More than 3 views add every contribution directly (the accumulators
    // would cost the third wave per SIMD), as does the deterministic mode (fixed point per
    // contribution: register sums converted at the flush measured 3.16 against 3.05 ms at cfg 2).
    constexpr bool RL = !DET && V <= 3;
    uint32_t apos[NS];
    f4v acc[NS][4];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      apos[s] = kInvalidTap;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[s][q] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    // the lanes in `flush` add acc[s] at corner apos[s] to the LDS image and clear it
    auto flush_acc = [&](int s, bool flush) {
      if (__builtin_amdgcn_ballot_w64(flush) == 0) return;   // uniform
      if (flush) {
        const int cx = pos_x(apos[s]), cy = pos_y(apos[s]);
        lds_t* a0 = lds + (base[s] + (cy - ub[s].y0) * bw[s] + (cx - ub[s].x0)) * kSlotWords;
        lds_t* a1 = a0 + bw[s] * kSlotWords;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          atomicAdd(a0 + j, (lds_t)acc[s][0][j]);
          atomicAdd(a0 + kSlotWords + j, (lds_t)acc[s][1][j]);
          atomicAdd(a1 + j, (lds_t)acc[s][2][j]);
          atomicAdd(a1 + kSlotWords + j, (lds_t)acc[s][3][j]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[s][q] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
      }
    };
    // grad_cv one plane ahead, issued after the plane's tap gathers (vmcnt retires loads in issue
    // order: waiting for the gathers then leaves the next plane's grad_cv loads in flight)
    f4v g_next = load_g(kp);
    for (int pl = kp; pl < ke; ++pl) {
      const f4v g = g_next;
      uint32_t pos[NS];
      float wx[NS], wy[NS];
      f4v tp[NS][4];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        // the sampling matrix is workgroup-uniform: scalar loads (load_matrix_uniform)
        float G[9];
        load_matrix_uniform(smat[s] + pl * 9, G);
        src_coords(G, xn, yn, h, w, active, pos[s], wx[s], wy[s]);
        load_taps(prs[s], tap_offset(pos[s], pg), soff, row_bytes, tp[s]);
      }
      g_next = load_g(min(pl + 1, ke - 1));
      f4v xs[NS];
      f4v sum = x0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        xs[s] = bilerp(tp[s], wx[s], wy[s]);
        sum += xs[s];
      }
      const f4v nmean = -div_views4(sum, vd);
      const f4v k2 = two_inv_v * g;
      if (s0 == 0) racc += k2 * (x0 + nmean);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s < s0 || s >= s1) continue;   // uniform
        const f4v cs = k2 * (xs[s] + nmean);
        const float ex = 1.0f - wx[s], ny = 1.0f - wy[s];
        const float wt[4] = {ny * ex, ny * wx[s], wy[s] * ex, wy[s] * wx[s]};
        const int cx = pos_x(pos[s]), cy = pos_y(pos[s]);
        const bool valid = pos[s] != kInvalidTap;
        const bool inb = use_lds && valid && cx >= ub[s].x0 && cx < ub[s].x1 && cy >= ub[s].y0 && cy < ub[s].y1;
        if constexpr (!RL) {
          // all 4 taps inside the pass's box: 16 LDS adds at immediate offsets of two addresses
          if (inb) {
            lds_t* a0 = lds + (base[s] + (cy - ub[s].y0) * bw[s] + (cx - ub[s].x0)) * kSlotWords;
            lds_t* a1 = a0 + bw[s] * kSlotWords;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              atomicAdd(a0 + j, Acc<DET>::conv(wt[0] * cs[j], sc));
              atomicAdd(a0 + kSlotWords + j, Acc<DET>::conv(wt[1] * cs[j], sc));
              atomicAdd(a1 + j, Acc<DET>::conv(wt[2] * cs[j], sc));
              atomicAdd(a1 + kSlotWords + j, Acc<DET>::conv(wt[3] * cs[j], sc));
            }
          }
        } else {
          // a corner inside the box that differs from the accumulated one flushes the registers
          flush_acc(s, inb && apos[s] != kInvalidTap && apos[s] != pos[s]);
          if (inb) {
            apos[s] = pos[s];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[s][q] = __builtin_elementwise_fma(f4v{wt[q], wt[q], wt[q], wt[q]}, cs, acc[s][q]);
          }
        }
        // no LDS image for this pass, or a rounding outlier: in-image taps to the accumulators
        // (a wave-uniform test first: the common wave skips the whole path with one scalar branch)
        if (__builtin_amdgcn_ballot_w64(valid && !inb) != 0 && valid && !inb) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int xx = cx + (q & 1), yy = cy + (q >> 1);
            if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;   // zero padding: no gradient
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < nch) gadd_out(b * V + 1 + s, j, yy, xx, Acc<DET>::conv(wt[q] * cs[j], sc));
          }
        }
      }
    }

    if constexpr (RL) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s < s0 || s >= s1) continue;   // uniform
        flush_acc(s, apos[s] != kInvalidTap);
      }
    }

    // ---- flush the pass's LDS image: one global atomic per nonzero (slot, channel) ----
    if (use_lds) {
      __syncthreads();
      for (int e = (int)threadIdx.x; e < T; e += kBlock) {
        int s = 0;
#pragma unroll
        for (int q = 1; q < NS; ++q)
          if (e >= base[q]) s = q;
        int o = 0, ww = 1, bx = 0, by = 0;
#pragma unroll
        for (int q = 0; q < NS; ++q)
          if (q == s) {
            o = base[q];
            ww = bw[q];
            bx = ub[q].x0;
            by = ub[q].y0;
          }
        const int r = (e - o) / ww, c = (e - o) - r * ww;
        const int yy = by + r, xx = bx + c;
        if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;   // border slot: padding taps
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j >= nch) break;
          const lds_t v = lds[e * kSlotWords + j];
          if (v != (lds_t)0) gadd_out(b * V + 1 + s, j, yy, xx, v);
        }
      }
      __syncthreads();   // the next pass re-zeroes the image
    }
    kp = ke;
  }
    s0 = s1;
  }
  if (active) ref_part[(((size_t)grp * B + b) * c4 + ch) * hw + pix] = make_float4(racc.x, racc.y, racc.z, racc.w);
}

// Reference view: S = sum over plane groups of the partials (fixed order), scattered to the
// reference view's plane-independent taps (its sampling matrix, plane 0 of the shard).
template <bool DET>
__global__ __launch_bounds__(kBlock) void ref_scatter_kernel(const float4* __restrict__ ref_part,
                                                            const float* __restrict__ sampling,
                                                            u64* __restrict__ acc, float* __restrict__ grad_feat,
                                                            const unsigned* __restrict__ mx, int B,
                                                            int V, int C, int h, int w, int Dc,
                                                            int groups) {
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const int c4 = (C + 3) / 4;
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const int ch = (int)blockIdx.y % c4;
  const int b = (int)blockIdx.y / c4;
  if (p >= hw) return;
  const float sc = DET ? fixed_scale(mx, V, Dc, hw).to_fixed : 1.0f;
  f4v S = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int g = 0; g < groups; ++g) {
    const float4 v = ref_part[(((size_t)g * B + b) * c4 + ch) * hw + p];
    S += f4v{v.x, v.y, v.z, v.w};
  }
  const int y = (int)(p / (uint32_t)w), x = (int)(p % (uint32_t)w);
  uint32_t pos;
  float wx, wy;
  src_coords(sampling + (size_t)(b * V) * Dc * 9, norm_coord(x, w), norm_coord(y, h), h, w, true, pos,
             wx, wy);
  if (pos == kInvalidTap) return;
  const float ex = 1.0f - wx, ny = 1.0f - wy;
  const float wt[4] = {ny * ex, ny * wx, wy * ex, wy * wx};
  const int cx = pos_x(pos), cy = pos_y(pos);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int xx = cx + (q & 1), yy = cy + (q >> 1);
    if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = ch * 4 + j;
      if (c >= C) break;
      const size_t o = ((size_t)(b * V) * C + c) * hw + (size_t)yy * w + xx;
      if constexpr (DET) gadd(acc + o, to_fixed(wt[q] * S[j], sc));
      else unsafeAtomicAdd(grad_feat + o, wt[q] * S[j]);
    }
  }
}

// More than 8 views (no packed workspace): one thread per (sample, plane, pixel), NCHW gathers,
// every view's taps straight to the global accumulators.
template <bool DET>
__global__ __launch_bounds__(kBlock) void cost_volume_bwd_generic_kernel(
    const float* __restrict__ feat, const float* __restrict__ sampling,
    const float* __restrict__ grad_cv, u64* __restrict__ acc, float* __restrict__ grad_feat,
    const unsigned* __restrict__ mx, int V, int C, int h, int w, int Dc, int tiles, int total) {
  const int wk = xcd_work_id(blockIdx.x, total);
  if (wk >= total) return;
  const WorkItem it = decode_flat(wk, Dc, tiles);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const uint32_t p = (uint32_t)it.tile * kBlock + threadIdx.x;
  if (p >= hw) return;
  const float sc = DET ? fixed_scale(mx, V, Dc, hw).to_fixed : 1.0f;
  float xn, yn;
  pixel_coords(p, w, h, xn, yn);
  Taps tp[MVS_MAX_VIEWS];
  for (int v = 0; v < V; ++v) make_taps(sampling + ((size_t)(it.b * V + v) * Dc + it.kk) * 9, xn, yn, h, w, tp[v]);
  const float* fb = feat + (size_t)it.b * V * C * hw;
  const float inv_v = 1.0f / (float)V;
  const ViewDiv vd = view_div(V);
  for (int c = 0; c < C; ++c) {
    const float g = grad_cv[(((size_t)it.b * C + c) * Dc + it.kk) * hw + p];
    float val[MVS_MAX_VIEWS];
    float sum = 0.0f;
    for (int v = 0; v < V; ++v) {
      val[v] = gather(fb + ((size_t)v * C + c) * hw, tp[v]);
      sum += val[v];
    }
    const float nmean = -div_views(sum, vd);   // the forward's mean (common.h variance_law)
    const float k2 = (inv_v + inv_v) * g;
    for (int v = 0; v < V; ++v) {
      const float coef = k2 * (val[v] + nmean);
      const size_t plane = ((size_t)(it.b * V + v) * C + c) * hw;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (tp[v].wt[q] == 0.0f) continue;
        const size_t o = plane + tp[v].off[q] / 4u;
        if constexpr (DET) gadd(acc + o, to_fixed(tp[v].wt[q] * coef, sc));
        else unsafeAtomicAdd(grad_feat + o, tp[v].wt[q] * coef);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void fixed_to_float_kernel(const u64* __restrict__ acc, size_t n,
                                                               const unsigned* __restrict__ mx, int V,
                                                               int Dc, uint32_t hw, float* __restrict__ out) {
  const Fixed fx = fixed_scale(mx, V, Dc, hw);
  // a non-finite grad_cv or feature element: the float path would propagate it (NaN * weight into
  // some taps); fixed point cannot carry it, so the whole gradient is NaN -- what torch's NaN checks
  // and GradScaler's inf/NaN skip look for
  const bool nonfinite = mx[2] != 0u;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = nonfinite ? __builtin_nanf("") : (float)((double)(long long)acc[i] * fx.to_float);
}

template <int V, bool DET>
void launch_main(const Geometry& g, const float4* packed, const float4* refs, const float* smp,
                 const float* gcv, u64* acc, float* grad_feat, float4* ref_part, const unsigned* mx,
                 hipStream_t s) {
  const int tiles_x = (g.w + kBwdTW - 1) / kBwdTW, tiles_y = (g.h + kBwdTH - 1) / kBwdTH;
  const int groups = (g.Dc + kBwdKPG - 1) / kBwdKPG;
  const int c4 = (g.C + 3) / 4;
  const int total = g.B * c4 * tiles_x * tiles_y * groups;
  hipLaunchKernelGGL((cost_volume_bwd_kernel<V, DET>), xcd_grid(total), dim3(kBlock), 0, s, packed, refs, smp,
                     gcv, acc, grad_feat, ref_part, mx, g.B, g.C, g.h, g.w, g.Dc, tiles_x, tiles_y, groups, total);
}

template <bool DET>
void launch_views(const Geometry& g, const float4* packed, const float4* refs, const float* smp,
                  const float* gcv, u64* acc, float* grad_feat, float4* ref_part, const unsigned* mx,
                  hipStream_t s) {
  switch (g.V) {
    case 2: launch_main<2, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    case 3: launch_main<3, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    case 4: launch_main<4, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    case 5: launch_main<5, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    case 6: launch_main<6, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    case 7: launch_main<7, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
    default: launch_main<8, DET>(g, packed, refs, smp, gcv, acc, grad_feat, ref_part, mx, s); break;
  }
}

// backward workspace: [3 uints: max|grad_cv|, max|feat|, non-finite flag (deterministic mode)]
// [ref partials groups*B*C4*hw float4 (2 <= V <= 8)][acc u64 N*C*hw (deterministic mode only)]
struct BwdLayout {
  size_t mx, ref_part, acc, total;
};

BwdLayout bwd_layout(int B, int V, int C, int h, int w, int Dc, bool deterministic) {
  BwdLayout L;
  const size_t hw = (size_t)h * w;
  const size_t groups = (size_t)(Dc + kBwdKPG - 1) / kBwdKPG;
  L.mx = 0;
  L.ref_part = 256;
  L.acc = L.ref_part + (V >= 2 && V <= 8 ? align256(groups * B * ((C + 3) / 4) * hw * 16) : 0);
  L.total = L.acc + (deterministic ? align256((size_t)B * V * C * hw * 8) : 0);
  return L;
}

}  // namespace

size_t cost_volume_bwd_workspace_bytes(int B, int V, int C, int h, int w, int Dc, bool deterministic) {
  return bwd_layout(B, V, C, h, w, Dc, deterministic).total;
}

int launch_cost_volume_bwd(const Geometry& g, const float* feat, const float* fwd_ws,
                           const float* grad_cv, void* bwd_ws, float* grad_feat, bool deterministic,
                           hipStream_t s) {
  const size_t n_feat = (size_t)g.B * g.V * g.C * g.h * g.w;
  if (!deterministic || g.V == 1)   // V == 1: the variance of one view is identically 0, so is its gradient
    if (hipMemsetAsync(grad_feat, 0, n_feat * sizeof(float), s) != hipSuccess) return MVS_ERR_HIP;
  if (g.V == 1) return MVS_OK;
  const BwdLayout L = bwd_layout(g.B, g.V, g.C, g.h, g.w, g.Dc, deterministic);
  char* ws = static_cast<char*>(bwd_ws);
  u64* acc = reinterpret_cast<u64*>(ws + L.acc);
  float4* ref_part = reinterpret_cast<float4*>(ws + L.ref_part);
  unsigned* mx = reinterpret_cast<unsigned*>(ws + L.mx);
  if (deterministic) {
    if (hipMemsetAsync(acc, 0, n_feat * 8, s) != hipSuccess) return MVS_ERR_HIP;
    if (hipMemsetAsync(mx, 0, 12, s) != hipSuccess) return MVS_ERR_HIP;
    const size_t n_gcv = (size_t)g.B * g.C * g.Dc * g.h * g.w;
    hipLaunchKernelGGL(abs_max_kernel, dim3(2048), dim3(kBlock), 0, s, grad_cv, n_gcv, mx, mx + 2);
    hipLaunchKernelGGL(abs_max_kernel, dim3(256), dim3(kBlock), 0, s, feat, n_feat, mx + 1, mx + 2);
  }
  const float* smp = fwd_ws;
  if (g.V <= 8) {
    const float4* packed = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(fwd_ws) +
                                                           sampling_bytes_aligned(g.B * g.V, g.Dc));
    const int c4 = (g.C + 3) / 4;
    const float4* refs = packed + (size_t)g.B * g.V * c4 * pad_geom(g.h, g.w).plane;
    if (deterministic) launch_views<true>(g, packed, refs, smp, grad_cv, acc, grad_feat, ref_part, mx, s);
    else launch_views<false>(g, packed, refs, smp, grad_cv, acc, grad_feat, ref_part, mx, s);
    const uint32_t hw = (uint32_t)g.h * (uint32_t)g.w;
    const int groups = (g.Dc + kBwdKPG - 1) / kBwdKPG;
    const dim3 grid((hw + kBlock - 1) / kBlock, (unsigned)(g.B * c4));
    if (deterministic)
      hipLaunchKernelGGL(ref_scatter_kernel<true>, grid, dim3(kBlock), 0, s, ref_part, smp, acc, grad_feat, mx,
                         g.B, g.V, g.C, g.h, g.w, g.Dc, groups);
    else
      hipLaunchKernelGGL(ref_scatter_kernel<false>, grid, dim3(kBlock), 0, s, ref_part, smp, acc, grad_feat, mx,
                         g.B, g.V, g.C, g.h, g.w, g.Dc, groups);
  } else if (deterministic) {
    hipLaunchKernelGGL(cost_volume_bwd_generic_kernel<true>, xcd_grid(g.total), dim3(kBlock), 0, s, feat, smp,
                       grad_cv, acc, grad_feat, mx, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
  } else {
    hipLaunchKernelGGL(cost_volume_bwd_generic_kernel<false>, xcd_grid(g.total), dim3(kBlock), 0, s, feat, smp,
                       grad_cv, acc, grad_feat, mx, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
  }
  if (deterministic) {
    const size_t blocks = (n_feat + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(fixed_to_float_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(kBlock), 0,
                       s, acc, n_feat, mx, g.V, g.Dc, (uint32_t)((size_t)g.h * g.w), grad_feat);
  }
  return MVS_OK;
}

}  // namespace mvs
