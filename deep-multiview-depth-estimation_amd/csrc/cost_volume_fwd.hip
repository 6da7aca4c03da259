// cost_volume_fwd.hip -- FUSED homography warp + variance cost volume (the north-star kernel).
//
// Reference: scripts/homography.py:6-92 (warp every view onto D planes, kornia warp_perspective)
// followed by scripts/costvolume.py:3-16 (cv = sum_v (x_v - mean)^2 / V), model.py:177-181.
// Here both are one pass: every view is sampled and the two-pass variance is formed in registers,
// so the B*V x C x D x h x w warped volume never exists; cv[B][C][D][h][w] is written once.
//
// Structure of cost_volume_staged_kernel (V = 2..8 views):
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
#include <cstdlib>

#include "launchers.h"
#include "split.h"
#include "packed.h"
#include "sampling_matrix.h"

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
  const ViewDiv vd = view_div(V);
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
        if (active)
          store_buf(make_rsrc(ob + (size_t)(c0 + cu) * ostride, plane_bytes), pbyte, variance_law<MAXV>(val[cu], V, vd));
      }
    }
  }
}


// Prologue of the fused launch: ONE kernel, three independent jobs by workgroup range (they used
// to be three dependent launches; cfg 4's 32-plane shard is launch-bound):
//   [0, nb_smp)                sampling matrices G[N][Dc][9] (sampling_matrix.h), one per thread;
//   [nb_smp, nb_smp + nb_pack) padded channel-quad features (packed.h), grid-stride;
//   the rest                   refs[b][ch][p]: the reference image b*V bilinearly sampled through its
//                              own G (shard plane 0, computed here by the same function, so it is
//                              the matrix the sampling job stores), read from the NCHW features
//                              with the packed layout's rules (taps outside the image are 0; same
//                              taps, weights and fma order as bilerp): bit-identical to sampling the
//                              packed image.
//   pixel_major: the pack job writes packed[N][h + 2][w + 2][C4] instead (cv_head.hip: one tap's C4
//                quads are one contiguous run), same values, same zero border.
__global__ __launch_bounds__(kBlock) void prologue_kernel(const float* __restrict__ feat, Cams cm,
                                                          float* __restrict__ sampling,
                                                          float4* __restrict__ packed, float4* __restrict__ refs,
                                                          int B, int V, int C, int h, int w, int Dc, int nb_smp,
                                                          int nb_pack, uint32_t* __restrict__ absmax,
                                                          int pixel_major) {
  const int N = B * V;
  const int c4 = (C + 3) / 4;
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  int blk = (int)blockIdx.x;
  if (blk < nb_smp) {
    const int t = blk * kBlock + (int)threadIdx.x;
    if (t < N * Dc) {
      const int i = t / Dc;
      sampling_matrix(cm, B, V, h, w, i, t - i * Dc, sampling + 9 * (size_t)t);
    }
    return;
  }
  blk -= nb_smp;
  if (blk < nb_pack) {
    const PadGeom pg = pad_geom(h, w);
    const size_t n = (size_t)N * c4 * pg.plane;
    uint32_t am = 0;   // max |feature| bits (absmax requested): bounds every variance by am^2
    for (size_t e = (size_t)blk * kBlock + threadIdx.x; e < n; e += (size_t)nb_pack * kBlock) {
      uint32_t q;
      int ch;
      size_t i;
      if (pixel_major) {   // e = (i * plane + q) * c4 + ch
        ch = (int)(e % c4);
        const size_t t = e / c4;
        q = (uint32_t)(t % pg.plane);
        i = t / pg.plane;
      } else {             // e = (i * c4 + ch) * plane + q
        q = (uint32_t)(e % pg.plane);
        const size_t t = e / pg.plane;
        ch = (int)(t % c4);
        i = t / c4;
      }
      const int y = (int)(q / (uint32_t)pg.pitch) - 1;
      const int x = (int)(q % (uint32_t)pg.pitch) - 1;
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (x >= 0 && x < w && y >= 0 && y < h) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = ch * 4 + j;
          if (c < C) v[j] = feat[(i * C + c) * hw + (size_t)y * w + x];
        }
      }
      packed[e] = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
      for (int j = 0; j < 4; ++j) am = max(am, __float_as_uint(v[j]) & 0x7FFFFFFFu);   // NaN > Inf > finite
    }
    if (absmax) {   // this workgroup's maximum -> its own partial slot (absmax_reduce_kernel folds them)
      __shared__ uint32_t wmax[kBlock / 64];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o));
      if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = am;
      __syncthreads();   // the pack job is workgroup-uniform: every thread of the block is here
      if (threadIdx.x == 0) {
        uint32_t m = wmax[0];
#pragma unroll
        for (int i = 1; i < kBlock / 64; ++i) m = max(m, wmax[i]);
        absmax[blk] = m;
      }
    }
    return;
  }
  blk -= nb_pack;
  const int pblocks = (int)((hw + kBlock - 1) / kBlock);
  const int bc = blk / pblocks;   // b * c4 + ch
  const uint32_t p = (uint32_t)(blk - bc * pblocks) * kBlock + threadIdx.x;
  const int ch = bc % c4, b = bc / c4;
  // the reference image's matrix once per workgroup (fp64, ~1k instructions: per thread it set the
  // prologue's duration -- cfg 2 34 us, cfg 3 63 us)
  __shared__ float Gs[9];
  if (threadIdx.x == 0) sampling_matrix(cm, B, V, h, w, b * V, 0, Gs);
  __syncthreads();   // (before the pixel-range exit: every thread of the workgroup reaches it)
  if (p >= hw) return;
  float G[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) G[e] = Gs[e];
  const int y = (int)(p / (uint32_t)w), x = (int)(p % (uint32_t)w);
  uint32_t pos;
  float wx, wy;
  src_coords(G, norm_coord(x, w), norm_coord(y, h), h, w, true, pos, wx, wy);
  f4v t[4] = {};
  if (pos != kInvalidTap) {
    const float* fb = feat + ((size_t)(b * V) * C + (size_t)ch * 4) * hw;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int xx = pos_x(pos) + (q & 1), yy = pos_y(pos) + (q >> 1);
      if (xx < 0 || xx >= w || yy < 0 || yy >= h) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ch * 4 + j < C) t[q][j] = fb[(size_t)j * hw + (size_t)yy * w + xx];
    }
  }
  const f4v r = bilerp(t, wx, wy);
  refs[(size_t)bc * hw + p] = make_float4(r.x, r.y, r.z, r.w);
}

// max|feat| bound words: one workgroup folds the pack workgroups' partial maxima (no atomics, no
// memset: every word is written) into the caller's 8 words
__global__ __launch_bounds__(kBlock) void absmax_reduce_kernel(const uint32_t* __restrict__ partial, int n,
                                                               uint32_t* __restrict__ absmax) {
  __shared__ uint32_t wmax[kBlock / 64];
  uint32_t m = 0;
  for (int i = (int)threadIdx.x; i < n; i += kBlock) m = max(m, partial[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x < 8) {
    uint32_t r = wmax[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; ++i) r = max(r, wmax[i]);
    absmax[threadIdx.x] = r;
  }
}

// pack workgroups with the bound words requested (one partial maximum each): enough for one element per
// thread at cfg 2 (7,898 workgroups); 1,024 made every thread walk 8 grid-stride steps, each waiting
// on its strided loads (the head prologue 28 us)
constexpr int kPackPartials = 8192;
constexpr int kTileW = 32;                // pixels per tile row: every cost-volume store is a 128-B row
constexpr int kTileH = kBlock / kTileW;   // 8

// planes per workgroup: the tap state of every (plane, source view) lives in registers
template <int V>
constexpr int group_planes() {
  return V <= 3 ? 8 : (V <= 5 ? 4 : 2);
}

// ------------------------------------------------------------------------------------------
// LDS-staged kernel (2 <= V <= 8).  A 256-thread workgroup owns a 32 x 8 pixel tile of one sample
// and a group of up to KPG consecutive depth planes; one thread = one pixel.  Per thread, the tap
// state of every (plane, source view) is computed once and kept in registers (3 VGPRs each).  The
// source views are read from LDS: per 4-channel chunk the workgroup stages,
// for every source view, the bounding box of all tap corners of its tile over its plane group
// (the footprint, about 1.8 slots per pixel at P = 4 on DTU geometry) with one coalesced 16-byte
// load per slot, and every bilinear tap is then a conflict-light ds_read_b128 (4 LDS cycles per
// wave-instruction against about 12 texture-path cycles for a 16-byte global gather, measured
// in tools/microbench/gather_patterns.hip).  A zero area at the front of LDS serves the samples
// with every tap outside the image (exactly 0).  A workgroup whose footprint exceeds the LDS
// budget samples the packed features straight from global memory (16-byte buffer gathers).
// ------------------------------------------------------------------------------------------
template <int V>
constexpr int staged_slots() {
  return V <= 3 ? 2560 : (V <= 5 ? 3072 : 4096);   // 40 / 48 / 64 KB: 4 / 3 / 2 workgroups per CU
}
// 3 waves per SIMD (at most 168 VGPRs): without the hint the V = 3 kernel lands at 169 VGPRs and 2
// waves; with it, 153 VGPRs and no VGPR spill.
#define MVS_STAGED_ATTR __attribute__((amdgpu_waves_per_eu(3)))

// Wave-wide min on the DPP network (no LDS traffic): xor-1 and xor-2 quad permutes, half-row and
// row mirrors (min over 16 lanes), then the row broadcasts of lanes 15 and 31; lane 63 ends with the
// minimum of the wave.  Lanes of rows a broadcast does not write keep their value (old = x).
__device__ inline int wave_min_to_lane63(int x) {
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false));  // row_half_mirror
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x140, 0xF, 0xF, false));  // row_mirror
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x142, 0xA, 0xF, false));  // row_bcast15 -> rows 1, 3
  x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x143, 0xC, 0xF, false));  // row_bcast31 -> rows 2, 3
  return x;
}

// Workgroup-wide min of NV ints; every thread gets the result as a wave-uniform value.  The scratch
// may alias LDS that the caller writes next (the staged kernel's staging slots): the closing barrier
// orders every wave's scratch reads before any such write.
template <int NV>
__device__ inline void block_min(int (&v)[NV], int* scratch /* >= 4 * NV ints of LDS */) {
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int m = __builtin_amdgcn_readlane(wave_min_to_lane63(v[k]), 63);
    if ((threadIdx.x & 63) == 0) scratch[wave * NV + k] = m;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int x = scratch[k];
#pragma unroll
    for (int q = 1; q < kBlock / 64; ++q) x = min(x, scratch[q * NV + k]);
    v[k] = __builtin_amdgcn_readfirstlane(x);
  }
  __syncthreads();   // scratch reads done before the caller's next LDS writes (WAR)
}

// Cost-volume stores through a buffer descriptor per (channel, plane group): planes past the group's
// end, channels past C and inactive lanes get out-of-range offsets and are dropped by the hardware,
// so every wave issues the same, statically known number of stores per chunk (the waits for the
// next chunk's staging loads then never wait for this chunk's stores).
constexpr int kStoreAux = 2;   // nt: 0.52 ms at cfg 2 against 0.66 ms with the default policy
__device__ inline void store_cv(Rsrc rs, uint32_t voff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)voff, 0, kStoreAux);
}

// bf16 output (opt-in): the fp32 variance rounded to nearest-even exactly as
// torch's float -> bfloat16 conversion (c10::BFloat16 round_to_nearest_even; NaN -> 0x7FC0).
__device__ inline uint32_t bf16_rne(float v) {
  const uint32_t u = __float_as_uint(v);
  if (v != v) return 0x7FC0u;
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

template <int ES>
__device__ inline void store_out(Rsrc rs, uint32_t voff, float v) {
  if constexpr (ES == 4) {
    store_cv(rs, voff, v);
  } else {
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bf16_rne(v), rs, (int)voff, 0, kStoreAux);
  }
}

// Output element bytes / layout of the staged kernel:
//   ES = 4   fp32 cv[B][C][D][h][w] (the reference layout)
//   ES = 2   bf16, same layout (SURVEY.md §8 f3 opt-in)
//   ES = 16  fp32 channel-quad cv[B][C/4][D][h][w][4] ("NC4DHW4"): each (pixel, plane, chunk) is one
//            16-byte store, a wave's 64 pixels one contiguous 1 KB run; the regulariser's HIP layers
//            read 4 channels of a voxel per load from it (MVSNet.forward's inference path)
//   ES = 8   bf16 channel-quad (SURVEY.md §8 f3 reduced-precision opt-in): the same layout with each
//            fp32 variance rounded to nearest-even bf16, one 8-byte store per (pixel, plane, chunk), a
//            wave's 64 pixels one contiguous 512-B run; the regulariser's HIP layers widen it on load
//   ES = kQuadSplit  the split cost volume (split.h "SCV", the split-fp16 consumers' operands): the
//            channel-quad layout with each 16-byte element the fp16 hi / lo parts of the 4 fp32
//            variances scaled by 2^e, e from the prologue's max|feat| bound words
constexpr int kQuad = 16;
constexpr int kQuadBf16 = 8;
constexpr int kQuadSplit = 32;   // a tag: 16-byte elements
template <int ES>
constexpr bool quad_layout() {
  return ES == kQuad || ES == kQuadBf16 || ES == kQuadSplit;
}
template <int ES>
constexpr uint32_t elem_bytes() {
  return ES == kQuadSplit ? 16u : (uint32_t)ES;
}

// staging pieces per thread carried in registers across a chunk: 4 covers the V = 3 footprints
// (about 3.5 pieces per thread and chunk at cfg 2); 4 views of 4-plane groups average 6 (cfg 3)
template <int V>
constexpr int prefetch_pieces() {
  return V <= 3 ? 4 : 8;
}

template <int V, int KPG, int ES /* output layout: 4 fp32, 2 bf16, 16 / 8 / kQuadSplit channel quads */>
__global__ __launch_bounds__(kBlock) MVS_STAGED_ATTR void cost_volume_staged_kernel(
    const float4* __restrict__ packed, const float4* __restrict__ refs,
    const float* __restrict__ sampling, void* __restrict__ cv, int C, int h, int w, int Dc, int pg_n,
    int tiles_x, int tiles_y, int groups, int total, const uint32_t* __restrict__ absmax, int csplit) {
  constexpr int NS = V - 1;
  constexpr int SLOTS = staged_slots<V>();
  __shared__ f4v lds[SLOTS];
  // block_min's scratch lives in the last slots of the staging area (which include the dummy slot
  // SLOTS - 1 and, near the budget, real staging slots): block_min ends with a barrier after its
  // scratch reads, so the zero-area writes and stage(0) that follow cannot overwrite scratch another
  // wave still reads.  Keeping the whole workgroup at exactly SLOTS * 16 B (40 KB at V = 3) fits 4
  // workgroups per CU.
  int* scratch = reinterpret_cast<int*>(&lds[SLOTS - (4 * 4 * NS + 3) / 4]);

  const int wk0 = xcd_work_id(blockIdx.x, total);
  if (wk0 >= total) return;   // workgroup-uniform
  // csplit > 1 (small plane shards): the channel chunks split over csplit workgroups per (tile, group)
  const int cpart = wk0 % csplit;
  const int wk = wk0 / csplit;
  const int g = wk % groups;
  const int t = wk / groups;
  const int tile = t % (tiles_x * tiles_y);
  const int b = t / (tiles_x * tiles_y);
  constexpr int TW = kTileW, TH = kTileH;
  const int px = (tile % tiles_x) * TW + (int)(threadIdx.x % TW);
  const int py = (tile / tiles_x) * TH + (int)(threadIdx.x / TW);
  const bool active = px < w && py < h;
  const int k0 = g * pg_n;
  const int npl = min(pg_n, Dc - k0);
  const uint32_t hw = (uint32_t)h * (uint32_t)w;
  const int c4 = (C + 3) / 4;
  const int ch_lo = (int)(((long)c4 * cpart) / csplit), ch_hi = (int)(((long)c4 * (cpart + 1)) / csplit);
  const PadGeom pg = pad_geom(h, w);
  const float xn = norm_coord(active ? px : 0, w);
  const float yn = norm_coord(active ? py : 0, h);

  uint32_t pos[KPG][NS];
  float fwx[KPG][NS], fwy[KPG][NS];
#pragma unroll
  for (int pl = 0; pl < KPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // planes past the group's end (last group only) compute a clamped plane, then drop it
      const int kk = k0 + (pl < npl ? pl : npl - 1);
      float G[9];
      load_matrix_uniform(sampling + ((size_t)(b * V + 1 + s) * Dc + kk) * 9, G);
      src_coords(G, xn, yn, h, w, active, pos[pl][s], fwx[pl][s], fwy[pl][s]);
      if (pl >= npl) {
        pos[pl][s] = kInvalidTap;
        fwx[pl][s] = fwy[pl][s] = 0.0f;
      }
    }

  // footprint of every source view: bounding box of the valid tap corners over the plane group
  int bb[4 * NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int mnx = 1 << 30, mny = 1 << 30, mxx = 1 << 30, mxy = 1 << 30;   // mx*: -(max corner)
#pragma unroll
    for (int pl = 0; pl < KPG; ++pl) {   // branch-free: invalid taps contribute 1 << 30
      const uint32_t p = pos[pl][s];
      const bool ok = p != kInvalidTap;
      const int x = pos_x(p), y = pos_y(p);
      mnx = min(mnx, ok ? x : 1 << 30);
      mny = min(mny, ok ? y : 1 << 30);
      mxx = min(mxx, ok ? -x : 1 << 30);
      mxy = min(mxy, ok ? -y : 1 << 30);
    }
    bb[4 * s + 0] = mnx;
    bb[4 * s + 1] = mny;
    bb[4 * s + 2] = mxx;
    bb[4 * s + 3] = mxy;
  }
  block_min<4 * NS>(bb, scratch);
  // LDS image: [zero area][view 1 footprint][view 2 footprint] ...; footprint rows are padded to a
  // pitch rp = 16k slots, so a row change inside a 16-lane ds_read_b128 group shifts every address
  // of that group by a multiple of the 16 four-bank groups: no bank conflict from row crossings.
  // The zero area (max rp + 2 slots) holds the taps of samples outside the image.
  int rx0[NS], ry0[NS], rw[NS], rp[NS], pcum[NS + 1], scum[NS + 1];
  int zero_slots = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const bool empty = bb[4 * s] == (1 << 30);
    rx0[s] = bb[4 * s];
    ry0[s] = bb[4 * s + 1];
    rw[s] = empty ? 0 : -bb[4 * s + 2] - rx0[s] + 2;   // taps x0 .. x0 + 1
    rp[s] = (rw[s] + 15) & ~15;
    zero_slots = max(zero_slots, rp[s] + 2);
  }
  zero_slots = (zero_slots + 15) & ~15;
  int rh[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) rh[s] = rw[s] == 0 ? 0 : -bb[4 * s + 3] - ry0[s] + 2;
  auto layout = [&]() {
    pcum[0] = 0;
    scum[0] = zero_slots;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pcum[s + 1] = pcum[s] + rw[s] * rh[s];   // staging pieces (real pixels)
      scum[s + 1] = scum[s] + rp[s] * rh[s];   // LDS slots (padded rows)
    }
  };
  layout();
  // Over budget with 16-slot row pitches: retry with unpadded rows (pitch = width).  Row crossings
  // inside a 16-lane ds_read_b128 group may then conflict, but the workgroup stays on LDS instead of
  // the global-gather path (unpadded, 97.1 % of V = 5 footprints fit instead of 92.3 %,
  // tools/footprint_stats.py).
  if (scum[NS] > SLOTS - 1) {
    zero_slots = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      rp[s] = rw[s];
      zero_slots = max(zero_slots, rp[s] + 2);
    }
    zero_slots = (zero_slots + 15) & ~15;
    layout();
  }

  const ViewDiv vd = view_div(V);
  const uint32_t pix = (uint32_t)(active ? py : 0) * (uint32_t)w + (uint32_t)(active ? px : 0);
  const float4* rbase = refs + (size_t)b * c4 * hw + pix;
  // store byte offset of (plane 0, this pixel) inside a (channel, group) descriptor
  constexpr uint32_t EB = elem_bytes<ES>();
  const uint32_t soff0 = active ? pix * EB : kOobOffset;
  const uint32_t grp_bytes = (uint32_t)npl * hw * EB;
  const int sx = ES == kQuadSplit ? cv_split_exponent(absmax) : 0;   // split scale 2^sx (split.h)

  // store descriptors of chunk ch's four channels (planes k0 .. k0 + npl of this sample); the
  // channel-quad layout has one descriptor for the chunk's quad plane
  auto chunk_rsrc = [&](int ch, Rsrc (&rs)[4]) {
    if constexpr (quad_layout<ES>()) {
      rs[0] = make_rsrc(static_cast<char*>(cv) + (((size_t)b * c4 + ch) * Dc + k0) * hw * EB, grp_bytes);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ch * 4 + j;
        rs[j] = make_rsrc(static_cast<char*>(cv) + (((size_t)b * C + (c < C ? c : 0)) * Dc + k0) * hw * ES,
                          c < C ? grp_bytes : 0u);
      }
    }
  };
  auto emit = [&](int pl, const Rsrc (&rs)[4], const f4v& x0, const f4v (&xs)[NS]) {
    const f4v acc = variance_law4<NS>(x0, xs, vd);
    if constexpr (ES == kQuad) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, acc),
                                             rs[0], (int)(soff0 + (uint32_t)pl * hw * (uint32_t)kQuad), 0, kStoreAux);
    } else if constexpr (ES == kQuadSplit) {
      uint2 hi, lo;
      split4(acc, sx, hi, lo);
      typedef __attribute__((ext_vector_type(4))) unsigned v4u;
      __builtin_amdgcn_raw_buffer_store_b128(v4u{hi.x, hi.y, lo.x, lo.y}, rs[0],
                                             (int)(soff0 + (uint32_t)pl * hw * EB), 0, kStoreAux);
    } else if constexpr (ES == kQuadBf16) {
      typedef __attribute__((ext_vector_type(2))) unsigned v2u;
      const v2u pk = {bf16_rne(acc[0]) | (bf16_rne(acc[1]) << 16), bf16_rne(acc[2]) | (bf16_rne(acc[3]) << 16)};
      __builtin_amdgcn_raw_buffer_store_b64(pk, rs[0], (int)(soff0 + (uint32_t)pl * hw * (uint32_t)kQuadBf16), 0,
                                            kStoreAux);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) store_out<ES>(rs[j], soff0 + (uint32_t)pl * hw * (uint32_t)ES, acc[j]);
    }
  };

  // the last slot is the dummy target of prefetch registers that carry no piece (kDummy below)
  if (scum[NS] > SLOTS - 1) {
    // footprint beyond the LDS budget (extreme zoom / long epipolar sweep): global gathers
    if (!active) return;   // no barriers below
    Rsrc rs[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s)
      rs[s] = make_rsrc(packed + (size_t)(b * V + 1 + s) * c4 * pg.plane, (uint32_t)c4 * pg.plane * 16u);
    for (int ch = ch_lo; ch < ch_hi; ++ch) {
      const float4 r4 = rbase[(size_t)ch * hw];
      const f4v x0 = {r4.x, r4.y, r4.z, r4.w};
      const int soff = (int)((uint32_t)ch * pg.plane * 16u);
      Rsrc ors[4];
      chunk_rsrc(ch, ors);
#pragma unroll 1
      for (int pl = 0; pl < npl; ++pl) {
        f4v xs[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          uint32_t p = kInvalidTap;
          float wx = 0.0f, wy = 0.0f;
#pragma unroll
          for (int q = 0; q < KPG; ++q)   // static register indexing
            if (q == pl) {
              p = pos[q][s];
              wx = fwx[q][s];
              wy = fwy[q][s];
            }
          f4v tp[4];
          load_taps(rs[s], tap_offset(p, pg), soff, pg.pitch * 16, tp);
          xs[s] = bilerp(tp, wx, wy);
        }
        emit(pl, ors, x0, xs);
      }
    }
    return;
  }

  // LDS index of every (plane, view) nw tap; 0 (zero area) for samples outside the image: its
  // other taps (1, rp, rp + 1) lie in the zero area too
  uint32_t li[KPG][NS];
#pragma unroll
  for (int pl = 0; pl < KPG; ++pl)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t p = pos[pl][s];
      li[pl][s] = p == kInvalidTap ? 0u
                                   : (uint32_t)(scum[s] + (pos_y(p) - ry0[s]) * rp[s] + (pos_x(p) - rx0[s]));
    }
  float inv_rw[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) inv_rw[s] = rw[s] > 0 ? 1.0f / (float)rw[s] : 0.0f;
  for (int q = (int)threadIdx.x; q < zero_slots; q += kBlock) lds[q] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  const int n_pieces = pcum[NS];

  // staging piece q -> (LDS slot, element of the padded packed source planes of chunk 0)
  auto piece = [&](int q, uint32_t& slot) -> uint32_t {   // element index relative to this sample
    int s = 0;
#pragma unroll
    for (int k = 1; k < NS; ++k)
      if (q >= pcum[k]) s = k;
    int p0 = pcum[0], s0 = scum[0], x0 = rx0[0], y0 = ry0[0], ww = rw[0], pp = rp[0];
    float iw = inv_rw[0];
#pragma unroll
    for (int k = 1; k < NS; ++k)
      if (s == k) {
        p0 = pcum[k];
        s0 = scum[k];
        x0 = rx0[k];
        y0 = ry0[k];
        ww = rw[k];
        pp = rp[k];
        iw = inv_rw[k];
      }
    const int e = q - p0;
    const int row = (int)(((float)e + 0.5f) * iw);
    const int col = e - row * ww;
    slot = (uint32_t)(s0 + row * pp + col);
    return (uint32_t)(1 + s) * (uint32_t)c4 * pg.plane + (uint32_t)((y0 + row + 1) * pg.pitch + (x0 + col + 1));
  };
  const float4* pbase = packed + (size_t)b * V * c4 * pg.plane;
  constexpr int kPrefetch = prefetch_pieces<V>();
  uint32_t psrc[kPrefetch], pslot[kPrefetch];
#pragma unroll
  for (int j = 0; j < kPrefetch; ++j) {
    const int q = (int)threadIdx.x + kBlock * j;
    pslot[j] = SLOTS - 1;   // dummy slot: never read
    psrc[j] = q < n_pieces ? piece(q, pslot[j]) : 0;
  }
  float4 pre[kPrefetch];
  float4 rpre;
  auto prefetch = [&](int ch) {   // chunk ch's first kBlock * kPrefetch pieces + reference -> registers
    rpre = rbase[(size_t)ch * hw];
#pragma unroll
    for (int j = 0; j < kPrefetch; ++j)
      pre[j] = pbase[psrc[j] + (uint32_t)ch * pg.plane];
  };
  prefetch(ch_lo);

  // Staging of chunk ch from the prefetch registers (and the pieces beyond them) into LDS.  It runs
  // right after the previous chunk's stores, and consumes only loads issued BEFORE those stores:
  // vmcnt retires in issue order, so its waits are counted (vmcnt(36) ...) and never wait for the
  // stores.  (With the staging at the top of the loop, the loop-header merge of the first
  // iteration's counts made every wait there drain all of the previous chunk's stores.)
  f4v x0;
  auto stage = [&](int ch) {
    x0 = f4v{rpre.x, rpre.y, rpre.z, rpre.w};
    // branch-free: registers without a piece go to the dummy slot, so every wait here is executed
    // by the whole wave and stays counted (a skipped conditional wait would leave the loads
    // formally pending at the loop head and force a full vmcnt drain there)
#pragma unroll
    for (int j = 0; j < kPrefetch; ++j) lds[pslot[j]] = f4v{pre[j].x, pre[j].y, pre[j].z, pre[j].w};
    // pieces beyond the prefetch registers (rare at V <= 3): one at a time there; with more views
    // four loads in flight per round (a load-store loop waits for every load; cfg 3 1.92 -> 1.85
    // ms), rounds past the end targeting the dummy slot
    if constexpr (V <= 3) {
      for (int q = (int)threadIdx.x + kBlock * kPrefetch; q < n_pieces; q += kBlock) {
        uint32_t slot;
        const float4 v = pbase[piece(q, slot) + (uint32_t)ch * pg.plane];
        lds[slot] = f4v{v.x, v.y, v.z, v.w};
      }
      return;
    }
    for (int q0 = (int)threadIdx.x + kBlock * kPrefetch; q0 < n_pieces; q0 += 4 * kBlock) {
      uint32_t slot[4];
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + u * kBlock;
        slot[u] = SLOTS - 1;
        const uint32_t src = q < n_pieces ? piece(q, slot[u]) : 0u;
        v[u] = pbase[src + (uint32_t)ch * pg.plane];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) lds[slot[u]] = f4v{v[u].x, v[u].y, v[u].z, v[u].w};
    }
  };
  stage(ch_lo);

  for (int ch = ch_lo; ch < ch_hi; ++ch) {
    __syncthreads();   // chunk ch is in LDS
    const f4v xr = x0;
    if (ch + 1 < ch_hi) prefetch(ch + 1);   // in flight during this chunk's stores
    Rsrc ors[4];
    chunk_rsrc(ch, ors);
#pragma unroll
    for (int pl = 0; pl < KPG; ++pl) {
      f4v xs[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t i0 = li[pl][s];
        f4v tp[4];
        tp[0] = lds[i0];
        tp[1] = lds[i0 + 1];
        tp[2] = lds[i0 + rp[s]];
        tp[3] = lds[i0 + rp[s] + 1];
        // opaque copies: the weights are rebuilt per chunk (3 VALU) instead of being held in 8
        // VGPRs per (plane, view) across the chunk loop
        float twx = fwx[pl][s], twy = fwy[pl][s];
        asm volatile("" : "+v"(twx), "+v"(twy));
        xs[s] = bilerp(tp, twx, twy);
      }
      emit(pl, ors, xr, xs);
    }
    if (ch + 1 < ch_hi) {
      __syncthreads();   // every wave is done reading chunk ch
      stage(ch + 1);
    }
  }
}

// The staged kernel instantiated with KPG = pg: its per-plane tap state, staging and store loop are
// unrolled over KPG planes, so a group narrower than the template (small plane shards, where pg is
// halved to fill the chip) would still compute and drop KPG - pg planes.
template <int V, int KPG, int ES>
void launch_staged(int pg, dim3 grid, hipStream_t s, const float4* packed, const float4* refs,
                   const float* smp, void* cv, const Geometry& g, int tiles_x, int tiles_y, int groups,
                   int total, const uint32_t* absmax, int csplit) {
  if constexpr (KPG > 1) {
    if (pg < KPG) {
      launch_staged<V, KPG / 2, ES>(pg, grid, s, packed, refs, smp, cv, g, tiles_x, tiles_y, groups, total, absmax,
                                    csplit);
      return;
    }
  }
  hipLaunchKernelGGL((cost_volume_staged_kernel<V, KPG, ES>), grid, dim3(kBlock), 0, s, packed, refs, smp, cv,
                     g.C, g.h, g.w, g.Dc, pg, tiles_x, tiles_y, groups, total, absmax, csplit);
}

template <int V, int ES>
void launch_gather(const Geometry& g, const float* feat, const Cams& cm, float* smp, float* ws, void* cv,
                   hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, uint32_t* absmax = nullptr) {
  const int c4 = (g.C + 3) / 4;
  const PadGeom pgeo = pad_geom(g.h, g.w);
  float4* packed = reinterpret_cast<float4*>(ws);
  float4* refs = packed + (size_t)g.B * V * c4 * pgeo.plane;
  const size_t n_pack = (size_t)g.B * V * c4 * pgeo.plane;
  const size_t pblocks = (n_pack + kBlock - 1) / kBlock;
  const int nb_smp = (g.B * V * g.Dc + kBlock - 1) / kBlock;
  // with the bound words requested, at most kPackPartials pack workgroups (grid-stride loops): one
  // partial maximum each (8192 atomicMax on 8 words serialised at L2 for ~0.3 ms)
  const size_t max_pack = absmax ? (size_t)kPackPartials : 8192;
  const int nb_pack = (int)(pblocks < max_pack ? pblocks : max_pack);
  const uint32_t hw = (uint32_t)g.h * (uint32_t)g.w;
  const int nb_ref = (int)((hw + kBlock - 1) / kBlock) * g.B * c4;
  // partial maxima of the pack workgroups: the 4 KB after the reference views (packed_bytes)
  uint32_t* partial = absmax ? reinterpret_cast<uint32_t*>(refs + (size_t)g.B * c4 * ((size_t)g.h * g.w)) : nullptr;
  hipLaunchKernelGGL(prologue_kernel, dim3((unsigned)(nb_smp + nb_pack + nb_ref)), dim3(kBlock), 0, s, feat, cm,
                     smp, packed, refs, g.B, V, g.C, g.h, g.w, g.Dc, nb_smp, nb_pack, partial, 0);
  if (absmax) hipLaunchKernelGGL(absmax_reduce_kernel, dim3(1), dim3(kBlock), 0, s, partial, nb_pack, absmax);
  constexpr int TW = kTileW, TH = kTileH;
  const int tiles_x = (g.w + TW - 1) / TW, tiles_y = (g.h + TH - 1) / TH;
  // planes per workgroup: the register maximum, halved until the grid has >= 4 workgroups per CU
  // (cfg 4, 32-plane shards: 0.128 ms with the 8-plane template at pg = 1, 0.044 ms at pg = 2)
  constexpr long kMinWorkgroups = 1024;
  int pg = group_planes<V>();
  // small shards: the channel chunks split over 2 workgroups per (tile, plane group) (MVS_CV_CSPLIT, 1..8),
  // then the plane group halved until the grid has the workgroups -- cfg 4's 32-plane shard: 4-plane
  // groups, 2 chunk halves, 43 us against 47 us for 2-plane groups (4: 51, 8: 57 us; gpurun_out r6s)
  static const int csplit_env = [] {
    const char* e = getenv("MVS_CV_CSPLIT");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : (v > 8 ? 8 : v);
  }();
  const int csplit = (long)g.B * tiles_x * tiles_y * ((g.Dc + pg - 1) / pg) < kMinWorkgroups ? csplit_env : 1;
  while (pg > 1 && (long)g.B * tiles_x * tiles_y * ((g.Dc + pg - 1) / pg) * csplit < kMinWorkgroups) pg >>= 1;
  const int groups = (g.Dc + pg - 1) / pg;
  const int total = g.B * tiles_x * tiles_y * groups * csplit;
  if (ev0) (void)hipEventRecord(ev0, s);
  launch_staged<V, group_planes<V>(), ES>(pg, xcd_grid(total), s, packed, refs, smp, cv, g, tiles_x, tiles_y,
                                         groups, total, absmax, csplit);
  if (ev1) (void)hipEventRecord(ev1, s);
}

template <int MAXV, bool EXACT>
void launch_direct(const Geometry& g, const float* feat, const float* smp, float* cv, hipStream_t s,
                   hipEvent_t ev0, hipEvent_t ev1) {
  if (ev0) (void)hipEventRecord(ev0, s);
  hipLaunchKernelGGL((cost_volume_kernel<MAXV, EXACT, 4>), xcd_grid(g.total), dim3(kBlock), 0, s,
                     feat, smp, cv, g.V, g.C, g.h, g.w, g.Dc, g.tiles, g.total);
  if (ev1) (void)hipEventRecord(ev1, s);
}

}  // namespace

// The prologue alone, for the fused consumer (cv_head.hip): sampling matrices, PIXEL-MAJOR padded
// features packed[N][h + 2][w + 2][C4] float4, the resampled reference views refs[B][C4][h][w] and the
// bound words (max |feat|, folded into absmax[8]); same workspace layout as launch_gather.
void launch_cv_prologue_pm(const Geometry& g, const float* feat, const Cams& cm, float* smp, float* ws,
                           uint32_t* absmax, hipStream_t s) {
  const int V = g.V;
  const int c4 = (g.C + 3) / 4;
  const PadGeom pgeo = pad_geom(g.h, g.w);
  float4* packed = reinterpret_cast<float4*>(ws);
  float4* refs = packed + (size_t)g.B * V * c4 * pgeo.plane;
  const size_t n_pack = (size_t)g.B * V * c4 * pgeo.plane;
  const size_t pblocks = (n_pack + kBlock - 1) / kBlock;
  const int nb_smp = (g.B * V * g.Dc + kBlock - 1) / kBlock;
  const int nb_pack = (int)(pblocks < (size_t)kPackPartials ? pblocks : (size_t)kPackPartials);
  const uint32_t hw = (uint32_t)g.h * (uint32_t)g.w;
  const int nb_ref = (int)((hw + kBlock - 1) / kBlock) * g.B * c4;
  uint32_t* partial = reinterpret_cast<uint32_t*>(refs + (size_t)g.B * c4 * ((size_t)g.h * g.w));
  hipLaunchKernelGGL(prologue_kernel, dim3((unsigned)(nb_smp + nb_pack + nb_ref)), dim3(kBlock), 0, s, feat, cm,
                     smp, packed, refs, g.B, V, g.C, g.h, g.w, g.Dc, nb_smp, nb_pack, partial, 1);
  hipLaunchKernelGGL(absmax_reduce_kernel, dim3(1), dim3(kBlock), 0, s, partial, nb_pack, absmax);
}

size_t packed_bytes(int B, int V, int C, int h, int w) {
  if (V < 2 || V > 8)  // generic kernel: reads the NCHW features directly
    return 0;
  const size_t c4 = (size_t)((C + 3) / 4);
  // + the pack workgroups' partial maxima of the bound words (kPackPartials uint32)
  return ((size_t)B * V * c4 * pad_geom(h, w).plane + (size_t)B * c4 * h * w) * sizeof(float4) +
         kPackPartials * sizeof(uint32_t);
}

void launch_cost_volume_fwd_bf16(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                                 float* packed, void* cv, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  switch (g.V) {
    case 2: launch_gather<2, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 3: launch_gather<3, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 4: launch_gather<4, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 5: launch_gather<5, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 6: launch_gather<6, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 7: launch_gather<7, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 8: launch_gather<8, 2>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    default: break;   // rejected by the C ABI (2 <= V <= 8 only)
  }
}

void launch_cost_volume_fwd_c4(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                               float* packed, float* cv, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                               uint32_t* absmax, bool split) {
  if (split) {   // the split cost volume (split.h): absmax required (its bound sets the scale)
    switch (g.V) {
      case 2: launch_gather<2, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 3: launch_gather<3, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 4: launch_gather<4, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 5: launch_gather<5, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 6: launch_gather<6, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 7: launch_gather<7, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      case 8: launch_gather<8, kQuadSplit>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
      default: break;
    }
    return;
  }
  switch (g.V) {
    case 2: launch_gather<2, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 3: launch_gather<3, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 4: launch_gather<4, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 5: launch_gather<5, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 6: launch_gather<6, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 7: launch_gather<7, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    case 8: launch_gather<8, kQuad>(g, feat, cm, sampling, packed, cv, s, ev0, ev1, absmax); break;
    default: break;   // rejected by the C ABI (2 <= V <= 8 only)
  }
}

void launch_cost_volume_fwd_c4_bf16(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                                    float* packed, void* cv, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  switch (g.V) {
    case 2: launch_gather<2, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 3: launch_gather<3, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 4: launch_gather<4, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 5: launch_gather<5, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 6: launch_gather<6, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 7: launch_gather<7, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 8: launch_gather<8, kQuadBf16>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    default: break;   // rejected by the C ABI (2 <= V <= 8 only)
  }
}

void launch_cost_volume_fwd(const Geometry& g, const float* feat, const Cams& cm, float* sampling,
                            float* packed, float* cv, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  switch (g.V) {
    case 2: launch_gather<2, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 3: launch_gather<3, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 4: launch_gather<4, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 5: launch_gather<5, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 6: launch_gather<6, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 7: launch_gather<7, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    case 8: launch_gather<8, 4>(g, feat, cm, sampling, packed, cv, s, ev0, ev1); break;
    default:   // generic kernel (9..16 views): sampling matrices first, then the direct gathers
      launch_plane_sampling(cm.K, cm.R, cm.T, cm.d_min, cm.d_int, g.B, g.V, g.h, g.w, cm.d_begin, g.Dc, cm.d_scale,
                            sampling, s);
      launch_direct<MVS_MAX_VIEWS, false>(g, feat, sampling, cv, s, ev0, ev1);
      break;
  }
}

}  // namespace mvs
