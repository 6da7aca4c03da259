// cv_head.hip -- the cost volume consumed where it is formed (north_star: "the
// B x C x D x H x W volume is never materialised before it is consumed").
//
// Reference: scripts/homography.py:6-92 + scripts/costvolume.py:3-16 (warp every source view onto D
// planes, variance over views) feeding scripts/model.py:101-103 (conv_0_0 + BN_0 + ReLU and conv_1_0 +
// BN_1 + ReLU both read cv in full).  One kernel forms the variance of a tile's voxels plane by plane
// on chip and applies both convolutions to it; nothing of the 2 GB volume reaches HBM except the
// middle region that conv_2_0 / conv_3_0 read.
//
// Workgroup: 512 threads = 4 CONSUMER waves (0-3, matrix cores) + 4 PRODUCER waves (4-7, gathers +
// variance).  It owns a 16 x 4 (x, y) column of conv_0_0 outputs and a chunk of kZC output depths;
// per step of two depths:
//   * producers compute the variance of the column's 18 x 6 halo on the next two planes -- the
//     fused forward's arithmetic exactly (same sampling coordinates, bilinear taps, two-pass variance,
//     split4 into fp16 hi / lo): taps are 16-byte gathers from PIXEL-MAJOR padded features (one tap
//     pixel's 8 channel quads are one 128-B line; L2 / MALL resident), per-(voxel, view) sampling
//     state computed one step ahead into an LDS table -- and write the split operands into a 6-plane
//     LDS ring in the layout conv3d_split.hip stages (so the conv_0_0 MFMA loop below is that kernel's);
//   * consumers run conv_0_0 (split-fp16 f16 MFMA, 2 per (16 voxels, tap), conv3d_split.hip's order)
//     on the 4 resident planes, and conv_1_0 (stride 2, padding P odd in every dim): the tile owns the
//     8 x 2 stride-2 windows starting at (x0 - 1 + 2 jx, y0 - 1 + 2 jy) -- one 16-row MFMA block -- and
//     the depth windows starting at z0 - 1 + 2k; consumer wave w < 3 accumulates product w of the
//     three split products (x_hi w_hi, x_hi w_lo, x_lo w_hi, conv3d_s2_split.hip's), tap by tap in
//     that kernel's order, and wave 3 combines a completed window's three partials (aa + (ab + ac)) one
//     step later and applies BN_1 + ReLU; then all four form the sampling state of the batch after next
//     and copy the tile's voxels inside conv_2_0's input box from the ring to the split cost volume
//     (SCV, split.h).  The producers issue nothing but in-range gathers (see items()).
// Per step: producers ~6.6k cycles of gathers + variance, consumers ~4k of MFMA (stamps,
// tools/dbg/stamps.py): the producers' gather latency is the critical path.
// Results are bit-identical to the materialising path (fused forward -> SCV -> conv3d_split /
// conv3d_s2_split): the same operands meet the same MFMAs in the same order.
#include "launchers.h"
#include "packed.h"
#include "split.h"

#include <algorithm>
#ifdef MVS_HEAD_STAMP
#include <cstdio>
#include <cstdlib>
#include <vector>
#endif

namespace mvs {
namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kC4 = 8;                                   // 32 channels = 8 quads (fixed: conv_0_0 / conv_1_0)
constexpr int kTX = 16, kTY = 4;                         // conv_0_0 outputs per tile
constexpr int kHX = kTX + 2, kHY = kTY + 2, kHV = kHX * kHY;   // 18 x 6 halo voxels
constexpr int kVoxB = 64;                                // 32 channels x fp16 per part
constexpr int kRowB = kHX * kVoxB;                       // 1,152 B
constexpr int kPartB = kHY * kRowB;                      // 6,912 B
constexpr int kSlotB = 2 * kPartB;                       // hi + lo: 13,824 B per plane
constexpr int kRing = 6;                                 // 4 planes read + 2 being written
constexpr int kRingB = kRing * kSlotB;                   // 82,944 B
// PRESPLIT: the producers run AHEAD batches ahead of the step they fill for (2 more slots each), so
// a slow load batch does not stall the consumers at the next barrier
#ifndef MVS_HEAD_PRE_AHEAD
#define MVS_HEAD_PRE_AHEAD 1
#endif
constexpr int kPreAhead = MVS_HEAD_PRE_AHEAD;
template <bool PRE>
constexpr int ring_slots() {
  return PRE ? kRing + 2 * kPreAhead : kRing;
}
constexpr int kW1B = 27 * 2 * 64 * 16;                   // conv_1_0 fragments: 55,296 B
constexpr int kScrB = 2 * 3 * 64 * 16;                   // conv_1_0 partials, double buffered
#ifndef MVS_HEAD_ZC
#define MVS_HEAD_ZC 48
#endif
constexpr int kZC = MVS_HEAD_ZC;                         // output depths per workgroup (even)
constexpr int kThreads = 512;
constexpr int kPlaneItems = kHV * kC4;                   // 864 (voxel, quad) items per plane
constexpr int kBatchItems = 2 * kPlaneItems;             // two planes per step
constexpr int kItems = (kBatchItems + 255) / 256;        // 7 per producer thread
#ifndef MVS_HEAD_KPF
#define MVS_HEAD_KPF 3
#endif
constexpr int kPF = MVS_HEAD_KPF;                        // conv_0_0 A-fragment prefetch (items)
#ifndef MVS_HEAD_PD
#define MVS_HEAD_PD 1
#endif
constexpr int kPD = MVS_HEAD_PD;                         // PRESPLIT: batches of loads in flight
#ifndef MVS_HEAD_VFAST
#define MVS_HEAD_VFAST 1
#endif
constexpr bool kPreVoxelFast = MVS_HEAD_VFAST;
// the sampling state of a batch is formed by the CONSUMER waves after their matrix work (they wait at
// the step barrier otherwise; the producers' gathers are the step's critical path: cfg 2 2.28 -> 2.19 ms)
#ifdef MVS_HEAD_COORDS_BY_PRODUCERS   // experiment (DESIGN.md §3.7 residual): the producers form their own sampling state
constexpr bool kCoordsByConsumers = false;
#else
constexpr bool kCoordsByConsumers = true;
#endif

template <int NS, bool PRE = false>
constexpr int coord_bytes() {   // [2 buffers][2 planes][NS views][108 voxels] x {off, wx, wy, -}
  return PRE ? 0 : 2 * 2 * NS * kHV * 16;
}
template <bool PRE>
constexpr int w1_lds_bytes() {   // PRE: the conv_1_0 product waves hold their fragments in registers
  return PRE ? 0 : kW1B;
}
template <int NS, bool PRE = false>
constexpr int lds_bytes() {
  return ring_slots<PRE>() * kSlotB + w1_lds_bytes<PRE>() + coord_bytes<NS, PRE>() + kScrB;
}

struct HeadArgs {
  const float4* packed;       // pixel-major padded features [N][h + 2][w + 2][8] float4
  const float4* refs;         // resampled reference views [B][8][h][w] float4
  const float* sampling;      // [N][D][9]
  const uint32_t* absmax;     // bound words (split scale)
  const h8v* w0;              // conv_0_0 fragments [27][64]
  const h8v* w1;              // conv_1_0 fragments [27][2][64]
  const float *bn0_sc, *bn0_sh, *bn0_mu;   // BN_0 (8), all or none
  const float *bn1_sc, *bn1_sh, *bn1_mu;   // BN_1 (16), all or none
  float* y0;                  // [B][8][D][H][W]
  float* y1;                  // [B][on0][on1][on2][16]
  uint32_t* y1_bound;         // optional: y1's bound words (split.h), for the split-fp16 conv_1_1
  void* scv;                  // split cost volume on the box only: [B][8][r1 - r0 ...] x 16 B, or null
  const void* scv_in;         // PRE: the materialised split cost volume [B][8][D][H][W] x 16 B (split.h)
  int V, D, H, W;
  int w_exp0, w_exp1;
  int tiles_x, tiles_y, zchunks, total;
  int pad[3];                 // (z, y, x), odd
  int o0[3], on[3];           // conv_1_0 output region
  int r0[3], r1[3];           // SCV box [r0, r1)
#ifdef MVS_HEAD_STAMP
  unsigned long long* stamps;   // diagnostic build: [kStampWG][8 waves][kStampN] s_memtime stamps
#endif
};

#ifdef MVS_HEAD_STAMP
constexpr int kStampWG = 512, kStampN = 128;
#endif

__device__ inline float ror8(float v) {   // value of lane (l ^ 8) inside each 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
}

// PRE (mvs_split_head_fwd): the cost volume is already materialised as the split volume; the producer
// waves copy its planes into the ring (one 16-byte load and two 8-byte LDS stores per item) and, while
// the next planes' loads are in flight, run conv_1_0 (its three split products with their weight
// fragments in registers, and the window finish); the consumers run conv_0_0 -- both convolutions
// of the split path in ONE pass over the volume, bit-equal to conv3d_split.hip + conv3d_s2_split.hip.
template <int V, bool PRE = false>
__global__ __launch_bounds__(kThreads) void cv_head_kernel(HeadArgs a) {
  constexpr int NS = V - 1;
  __shared__ __attribute__((aligned(16))) char lds[lds_bytes<NS, PRE>()];
  char* const ring = lds;
  constexpr int RS = ring_slots<PRE>();
  char* const w1l = lds + RS * kSlotB;
  char* const coord = lds + RS * kSlotB + w1_lds_bytes<PRE>();
  char* const scr = coord + coord_bytes<NS, PRE>();

  const int wk = xcd_work_id((int)blockIdx.x, (int)gridDim.x);
  if (wk >= a.total) return;   // workgroup-uniform, before any barrier
  int t = wk;
  const int x0 = (t % a.tiles_x) * kTX;
  t /= a.tiles_x;
  const int y0 = (t % a.tiles_y) * kTY;
  t /= a.tiles_y;
  const int z0 = (t % a.zchunks) * kZC;
  const int b = t / a.zchunks;
  const int D = a.D, H = a.H, W = a.W;
  const int z1 = min(z0 + kZC, D);
  const int nsteps = (z1 - z0) >> 1;   // D even (checked by the C ABI)
  const int nbatch = nsteps + 1;       // batch j = planes z0 - 1 + 2j, z0 + 2j
  const int ex = cv_split_exponent(a.absmax);
  // the wave index through readfirstlane: role branches are scalar (s_cbranch_scc), not exec-masked
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wave < 4;
#ifdef MVS_HEAD_STAMP
  // diagnostic: lane 0 of every wave of the first kStampWG workgroups stamps s_memtime at segment ends
  unsigned long long* const stp = wk < kStampWG ? a.stamps + ((size_t)wk * 8 + wave) * kStampN : nullptr;
  int sti = 0;
  auto stamp = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (stp && lane == 0 && sti < kStampN) stp[sti] = t;
    ++sti;
  };
#else
  auto stamp = [&]() {};
#endif

  // conv_1_0 weight fragments -> LDS (every thread)
  if constexpr (!PRE) {
    const Rsrc rw = make_rsrc(a.w1, (uint32_t)kW1B);
#pragma unroll
    for (int j = 0; j < (kW1B / 16 + kThreads - 1) / kThreads; ++j) {
      const int e = tid + kThreads * j;
      if (e < kW1B / 16)
        *reinterpret_cast<f4v*>(w1l + e * 16) = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rw, e * 16, 0, 0));
    }
  }
  // ring slot of plane p (batch j = (p - z0 + 1) / 2 lives in slots 2j, 2j + 1 mod kRing)
  auto slot_of = [&](int p) { return (p - z0 + 1) % RS; };

  // ================================ producer state ================================
  const int ptid = tid - 256, pw = wave - 4;
  const size_t HW = (size_t)H * W;
  const PadGeom pg = pad_geom(H, W);
  const uint32_t pstride = (uint32_t)kC4 * 16u;   // bytes per padded pixel
  Rsrc rsv[NS];
  f4v ref[kItems];
  if (!consumer && !PRE) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      rsv[s] = make_rsrc(a.packed + (size_t)(b * V + 1 + s) * pg.plane * kC4, pg.plane * pstride);
#pragma unroll
    for (int u = 0; u < kItems; ++u) {   // the thread's (voxel, quad) items: the same every batch
      const int e = ptid + 256 * u;
      const int r = e >= kPlaneItems ? e - kPlaneItems : e;
      const int v = r >> 3, q = r & 7;
      const int yy = v / kHX, xx = v - yy * kHX;
      const int gx = x0 - 1 + xx, gy = y0 - 1 + yy;
      const bool in = e < kBatchItems && gx >= 0 && gx < W && gy >= 0 && gy < H;
      const float4 r4 = in ? a.refs[((size_t)(b * kC4 + q) * H + gy) * W + gx] : make_float4(0.f, 0.f, 0.f, 0.f);
      ref[u] = f4v{r4.x, r4.y, r4.z, r4.w};
    }
  }
  // plane-independent per-lane constants of the coordinate jobs: halo voxels lane and lane + 64, their
  // kornia-normalised reference coordinates (norm_coord: two IEEE divisions each, formed once) and
  // whether they lie in the image
  float cxn[2] = {0.f, 0.f}, cyn[2] = {0.f, 0.f};
  bool cin[2] = {false, false};
  if (kCoordsByConsumers == consumer && !PRE) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int v = lane + 64 * pass;
      const int yy = v / kHX, xx = v - yy * kHX;
      const int gx = x0 - 1 + xx, gy = y0 - 1 + yy;
      cin[pass] = v < kHV && gx >= 0 && gx < W && gy >= 0 && gy < H;
      cxn[pass] = norm_coord(cin[pass] ? gx : 0, W);
      cyn[pass] = norm_coord(cin[pass] ? gy : 0, H);
    }
  }
  // sampling state of batch j's planes for every (plane, view, halo voxel) -> coordinate buffer tb
  auto coords = [&](int j, int tb) {
    if constexpr (PRE) return;
    const int pbase = z0 - 1 + 2 * j;
    for (int c = wave & 3; c < 2 * NS; c += 4) {   // wave-uniform (plane, view) combos
      const int pl = c / NS, s = c - pl * NS;
      const int p = pbase + pl;
      const bool pok = p >= 0 && p < D;
      float G[9];
      load_matrix_uniform(a.sampling + ((size_t)(b * V + 1 + s) * D + (pok ? p : 0)) * 9, G);
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int v = lane + 64 * pass;
        if (v < kHV) {
          uint32_t pos;
          float wx, wy;
          src_coords(G, cxn[pass], cyn[pass], H, W, pok && cin[pass], pos, wx, wy);
          // an invalid sample's 4 taps read the zero padding at padded (w + 1, 0): (w + 1, 0), (0, 1)
          // [the next padded row], (w + 1, 1), (0, 2) -- in range: an out-of-range load returns at once,
          // which made the LDS-operand hazard of DESIGN.md §3.7 frequent; zero weights keep the sum 0
          if (pos == kInvalidTap) wx = wy = 0.0f;
          const uint32_t off = pos == kInvalidTap ? (uint32_t)(W + 1) * pstride
                                                  : ((uint32_t)(pos_y(pos) + 1) * (uint32_t)pg.pitch +
                                                     (uint32_t)(pos_x(pos) + 1)) * pstride;
          *reinterpret_cast<uint4*>(coord + (((tb * 2 + pl) * NS + s) * kHV + v) * 16) =
              make_uint4(off, __float_as_uint(wx), __float_as_uint(wy), 0u);
        }
      }
    }
  };
  const ViewDiv vd = view_div(V);
  // the box [r0, r1) of sample b's split volume: [8 quads][bz][by][bx] x 16 B
  const int bz = a.r1[0] - a.r0[0], by = a.r1[1] - a.r0[1], bxw = a.r1[2] - a.r0[2];
  const uint32_t bhw = (uint32_t)by * (uint32_t)bxw;
  const uint64_t box_bytes = (uint64_t)kC4 * (uint64_t)bz * bhw * 16ull;
  const Rsrc rscv = make_rsrc(a.scv ? static_cast<char*>(a.scv) + (size_t)b * box_bytes : nullptr,
                              a.scv ? (uint32_t)box_bytes : 0u);
  // variance of batch j's two planes -> ring slots.  Software-pipelined so the gathers of several
  // items are in flight together: item u + kAhead's sampling state (LDS) and 4 taps x NS views are
  // issued before item u is reduced (each wave keeps up to (kAhead + 1) x 4 x NS 16-byte gathers in
  // flight, waited by counted vmcnt).  The producers issue nothing but these gathers in the loop, all
  // in range (an out-of-range load returns at once and made hazard 1 of DESIGN.md §3.7 frequent).
  // (Measured and dropped: skipping the items of edge tiles whose 64 lanes lie outside the image --
  // 2.34 against 2.18 ms, the extra branches cost the interior tiles more than the edges save.)
#ifndef MVS_HEAD_AHEAD
#define MVS_HEAD_AHEAD 2
#endif
  constexpr int kAhead = MVS_HEAD_AHEAD;
  // per-item constants (the same every batch), packed: LDS offset inside a ring slot (bits 0-12), in
  // the image (13), plane of the batch (15), quad (16-18), halo voxel (19-25)
  uint32_t meta[kItems];
  if (!consumer) {
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      const int e = min(ptid + 256 * u, kBatchItems - 1);
      const int pl = e >= kPlaneItems ? 1 : 0;
      const int r = e - pl * kPlaneItems;
      // PRE (MVS_HEAD_VFAST): voxel fastest, so a wave's 64 loads are runs of one quad plane (rows of
      // 18 x 16 B) instead of 8 voxels x 8 quad planes 2^22 B apart
      const bool vfast = PRE && kPreVoxelFast;
      const int v = vfast ? r % kHV : r >> 3, q = vfast ? r / kHV : r & 7;
      const int yy = v / kHX, xx = v - yy * kHX;
      const int gx = x0 - 1 + xx, gy = y0 - 1 + yy;
      const bool vin = gx >= 0 && gx < W && gy >= 0 && gy < H;
      const uint32_t lo = (uint32_t)(yy * kRowB + xx * kVoxB + (((q >> 1) ^ ((xx >> 1) & 3)) << 4) + ((q & 1) << 3));
      meta[u] = lo | ((uint32_t)vin << 13) | ((uint32_t)pl << 15) | ((uint32_t)q << 16) | ((uint32_t)v << 19);
    }
  }
  const int zst0 = max(z0, a.r0[0]), zst1 = min(z1, a.r1[0]);   // planes stored to the SCV box
  // PRE: batch j's two planes copied from the split volume, software-pipelined across the step
  // barrier: pre_load(j + 1) is issued right after pre_store(j)'s LDS stores have completed, so its
  // HBM latency runs under a whole step of MFMAs (issued and stored in the same step, the loads were
  // the step's critical path); invalid items (outside the image or the volume) load the sample's first
  // element and store zeros -- no out-of-range load
  const Rsrc rin = make_rsrc(PRE ? static_cast<const char*>(a.scv_in) + (size_t)b * kC4 * D * HW * 16 : nullptr,
                             PRE ? (uint32_t)min((uint64_t)kC4 * D * HW * 16ull, 0xFFFFFFF0ull) : 0u);
  typedef __attribute__((ext_vector_type(4))) unsigned v4u;
  v4u pd[kPD][kItems];   // kPD batches in flight (buffer j % kPD)
  uint32_t pok[kPD];     // bit u: item u of the buffered batch is valid
  const int pnu = __builtin_amdgcn_readfirstlane(ptid + 256 * (kItems - 1) < kBatchItems ? kItems : kItems - 1);
  auto pre_load = [&](int j, int pb) {
#ifdef MVS_HEAD_NO_LOAD   // (timing ablation: the ring is never filled)
    return;
#endif
    const int pbase = z0 - 1 + 2 * j;
    pok[pb] = 0;
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      if (u == kItems - 1 && pnu != kItems) break;   // wave-uniform
      const uint32_t m = meta[u];
      const int pl = (m >> 15) & 1, q = (m >> 16) & 7, v = (int)(m >> 19);
      const int p = pbase + pl;
      const int yy = v / kHX, xx = v - yy * kHX;
      const bool ok = (m & (1u << 13)) && (unsigned)p < (unsigned)D;
      pok[pb] |= ok ? (1u << u) : 0u;
      const uint32_t off = ok ? ((((uint32_t)q * (uint32_t)D + (uint32_t)p) * (uint32_t)HW +
                                  (uint32_t)((y0 - 1 + yy) * W + (x0 - 1 + xx))) * 16u) : 0u;
      pd[pb][u] = __builtin_amdgcn_raw_buffer_load_b128(rin, (int)off, 0, 0);
    }
  };
  auto pre_store = [&](int j, int pb) {
#ifdef MVS_HEAD_NO_LOAD
    return;
#endif
    const int sl0 = slot_of(z0 - 1 + 2 * j);
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      if (u == kItems - 1 && pnu != kItems) break;
      const uint32_t m = meta[u];
      const int pl = (m >> 15) & 1;
      const bool ok = (pok[pb] >> u) & 1u;
      const uint2 hi = ok ? make_uint2(pd[pb][u].x, pd[pb][u].y) : make_uint2(0u, 0u);
      const uint2 lo = ok ? make_uint2(pd[pb][u].z, pd[pb][u].w) : make_uint2(0u, 0u);
      char* dst = ring + (sl0 + pl) * kSlotB + (m & 0x1FFFu);
      *reinterpret_cast<uint2*>(dst) = hi;
      *reinterpret_cast<uint2*>(dst + kPartB) = lo;
    }
    // the stores have read their data registers before the next batch's loads target them
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto items = [&](int j, int tb) {
    if constexpr (PRE) return;   // (pre_load / pre_store)
    const int pbase = z0 - 1 + 2 * j;
    const int sl0 = slot_of(pbase);   // even: the batch's second plane is the next slot
    const int nu = __builtin_amdgcn_readfirstlane(ptid + 256 * (kItems - 1) < kBatchItems ? kItems : kItems - 1);
    f4v tp[kAhead + 1][NS][4];
    float fx[kAhead + 1][NS], fy[kAhead + 1][NS];
    // item u's sampling state, read from LDS one item before its gathers are issued (the LDS round
    // trip off the gather issue path)
    uint32_t co[2][NS];
    float cx[2][NS], cy[2][NS];
    auto rdc = [&](int u) {
      const uint32_t m = meta[u];
      const int pl = (m >> 15) & 1, v = (int)(m >> 19);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint4 ce = *reinterpret_cast<const uint4*>(coord + (((tb * 2 + pl) * NS + s) * kHV + v) * 16);
#ifdef MVS_HEAD_RDC128   // experiment: all four words used (ce.w == 0), so the read is a ds_read_b128, not b96
        co[u & 1][s] = ce.x | ce.w;
#else
        co[u & 1][s] = ce.x;
#endif
        cx[u & 1][s] = __uint_as_float(ce.y);
        cy[u & 1][s] = __uint_as_float(ce.z);
      }
    };
    auto issue = [&](int u) {   // item u's 4 x NS tap gathers (its sampling state read by rdc(u))
      const int rr = u % (kAhead + 1);
      const uint32_t qo = ((meta[u] >> 16) & 7) * 16u;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t o = co[u & 1][s] + qo;
        fx[rr][s] = cx[u & 1][s];
        fy[rr][s] = cy[u & 1][s];
#ifdef MVS_HEAD_ABL_G
        {
          const float f = __uint_as_float(o);
          tp[rr][s][0] = f4v{f, f, f, f};
          tp[rr][s][1] = f4v{f, 1.f, f, f};
          tp[rr][s][2] = f4v{f, f, 2.f, f};
          tp[rr][s][3] = f4v{f, f, f, 3.f};
        }
#elif defined(MVS_HEAD_X2)   // experiment: each 16-byte tap as two 8-byte loads
        {
          typedef __attribute__((ext_vector_type(2))) unsigned v2u;
          const uint32_t offs[4] = {o, o + pstride, o + (uint32_t)pg.pitch * pstride, o + (uint32_t)pg.pitch * pstride + pstride};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const v2u a0 = __builtin_amdgcn_raw_buffer_load_b64(rsv[s], (int)offs[t], 0, 0);
            const v2u a1 = __builtin_amdgcn_raw_buffer_load_b64(rsv[s], (int)(offs[t] + 8u), 0, 0);
            tp[rr][s][t] = f4v{__uint_as_float(a0.x), __uint_as_float(a0.y), __uint_as_float(a1.x), __uint_as_float(a1.y)};
          }
        }
#elif defined(MVS_HEAD_GLOBAL)   // experiment: taps through global (flat-space) loads instead of buffer loads
        {
          const char* gb = reinterpret_cast<const char*>(a.packed) + (size_t)(b * V + 1 + s) * pg.plane * pstride;
          tp[rr][s][0] = *reinterpret_cast<const f4v*>(gb + o);
          tp[rr][s][1] = *reinterpret_cast<const f4v*>(gb + o + pstride);
          tp[rr][s][2] = *reinterpret_cast<const f4v*>(gb + o + (uint32_t)pg.pitch * pstride);
          tp[rr][s][3] = *reinterpret_cast<const f4v*>(gb + o + (uint32_t)pg.pitch * pstride + pstride);
        }
#else
        tp[rr][s][0] = ld4(rsv[s], o, 0);
        tp[rr][s][1] = ld4(rsv[s], o + pstride, 0);
        tp[rr][s][2] = ld4(rsv[s], o + (uint32_t)pg.pitch * pstride, 0);
        tp[rr][s][3] = ld4(rsv[s], o + (uint32_t)pg.pitch * pstride + pstride, 0);
#endif
      }
    };
    // items that exist for this wave: u < nu (wave-uniform)
    auto has = [&](int u) { return u < kItems - 1 || (u == kItems - 1 && nu == kItems); };
    // No gather is issued while an LDS instruction of this wave is outstanding (s_waitcnt lgkmcnt(0)
    // first): under the consumers' LDS load a ds_write / ds_read can still be reading its data or
    // address registers when a younger gather's data lands in them -- the register allocator reuses
    // a finished item's registers for the next gathers -- and the last lanes then write or address
    // the wrong values (sporadic, the first steps of a chunk).  So per item: its
    // gathers' wait, its variance, then the wait for the previous item's LDS operations (which had
    // the whole variance to finish), item u + kAhead's gathers, and only then this item's LDS work.
    auto lds_drain = [&]() {
      __builtin_amdgcn_sched_barrier(0);
#ifndef MVS_HEAD_NO_LDS_DRAIN   // (mutation build of tests/test_head_isa.py only: the rule's checker must fail)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
      __builtin_amdgcn_sched_barrier(0);
    };
    rdc(0);
    rdc(1);
    lds_drain();
#pragma unroll
    for (int u = 0; u < kAhead; ++u) issue(u);
#ifdef MVS_HEAD_RDC_FIRST
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    rdc(kAhead);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      if (!has(u)) break;   // wave-uniform (the last pass: waves 4-6 only)
      const uint32_t m = meta[u];
      const int pl = (m >> 15) & 1;
      const int p = pbase + pl;
      const bool valid = (m & (1u << 13)) && (unsigned)p < (unsigned)D;
      const int rr = u % (kAhead + 1);
#ifdef MVS_HEAD_VMWAIT   // experiment: item u's gathers explicitly waited for (item u + 1's may stay in flight), then nops
      __builtin_amdgcn_sched_barrier(0);
      if (kAhead > 1 && has(u + 1))
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_nop %1" ::"n"(4 * NS), "n"(MVS_HEAD_VMWAIT) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_nop %0" ::"n"(MVS_HEAD_VMWAIT) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#endif
      f4v xs[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) xs[s] = bilerp(tp[rr][s], fx[rr][s], fy[rr][s]);
      const f4v acc = variance_law4<NS>(ref[u], xs, vd);   // costvolume.py:12-14 (packed.h)
      uint2 hi, lo;
      split4(acc, ex, hi, lo);
      if (!valid) hi = lo = make_uint2(0u, 0u);
      lds_drain();
#ifdef MVS_HEAD_RDC_FIRST   // experiment: item u + kAhead + 1's sampling-state read before (not under) u + kAhead's gathers
      if (has(u + kAhead + 1)) rdc(u + kAhead + 1);
      lds_drain();
      if (has(u + kAhead)) issue(u + kAhead);
#else
      if (has(u + kAhead)) issue(u + kAhead);
      if (has(u + kAhead + 1)) rdc(u + kAhead + 1);
#endif
      char* dst = ring + (sl0 + pl) * kSlotB + (m & 0x1FFFu);
      // THE HAZARD: the item's two ds_write_b64 ring stores must not run while
      // any of this wave's tap gathers (buffer_load_dwordx4) is still in flight, and must complete before
      // the wave's next VALU work.  With gathers of later items outstanding across the stores, the last
      // 16-lane group of a ds_write_b64 (lanes 48-63, serviced last) stored wrong data in some launches
      // (bench geometry: 20 of 20 launches at V = 2 and V = 3); a wait for the stores alone cured V = 2,
      // not V = 3; both waits: 0 of 20 at every geometry (tools/dbg/stress_r6.sh, gpurun_out r6b / r6c).
      __builtin_amdgcn_sched_barrier(0);
#ifndef MVS_HEAD_NO_STORE_FENCE   // (mutation build of tests/test_head_isa.py only: the rule's checker must fail)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#ifdef MVS_HEAD_STORE_NOP   // experiment (DESIGN.md §3.7 residual): wait states between the item's VALU and its ring stores
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#endif
      __builtin_amdgcn_sched_barrier(0);
      *reinterpret_cast<uint2*>(dst) = hi;
      *reinterpret_cast<uint2*>(dst + kPartB) = lo;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // one item per scheduling region: without it the scheduler hoists every item's loads to the
      // top (all 7 items' gathers live at once: VGPR spills)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ================================ conv_1_0 state ================================
  // conv_1_0 (model.py:103) runs on the consumer waves, or in PRE on the producer waves, idle while
  // their loads are in flight; c1w = the wave's index in that role: 0-2 the three split products, 3
  // finishes each window from their partials (scratch, double buffered)
  const bool c1role = PRE ? !consumer : consumer;
  const int c1w = wave & 3;
  const int i16 = lane & 15, g4 = lane >> 4;
  float sc1 = 1.0f, sh1 = 0.0f, mu1 = 0.0f;
  auto load_bn1 = [&]() {
    if (a.bn1_sc) {
      sc1 = a.bn1_sc[i16];
      sh1 = a.bn1_sh[i16];
      mu1 = a.bn1_mu[i16];
    }
    asm volatile("" ::"v"(sc1), "v"(sh1), "v"(mu1));
  };
  const int oexp1 = -(ex + a.w_exp1);
  // PRE: the product wave's 27 (depth tap, tap) fragments of its weight part, in registers
  // (loaded inside the role's branch: live ranges of the two roles' fragments never overlap)
  h8v bw1[PRE ? 27 : 1];
  auto load_bw1 = [&]() {
    if (c1w < 3) {
      const Rsrc rw = make_rsrc(a.w1, (uint32_t)kW1B);
      const int bp = c1w == 1 ? 1 : 0;
#pragma unroll
      for (int j = 0; j < (PRE ? 27 : 1); ++j)
        bw1[j] = __builtin_bit_cast(h8v, __builtin_amdgcn_raw_buffer_load_b128(rw, ((j * 2 + bp) * 64 + lane) * 16, 0, 0));
    }
  };
  // conv_1_0: MFMA row i16 = window (jx, jy); product wave w < 3
  const int jx = i16 & 7, jy = i16 >> 3;
  const int apart = c1w == 2 ? kPartB : 0;    // x_lo for product 2
  const int bpart = c1w == 1 ? 1 : 0;         // w_lo for product 1
  int acol[3];
#pragma unroll
  for (int tx = 0; tx < 3; ++tx) {
    const int c = 2 * jx + tx;
    acol[tx] = apart + c * kVoxB + ((g4 ^ ((c >> 1) & 3)) << 4);
  }
  f4 cur = {0.f, 0.f, 0.f, 0.f}, nxt = cur;
  // acc += the 9 (ty, tx) taps of depth tap tz on plane slot sl (product wave's operands), in tap order;
  // conv3d_s2_split.hip's pipeline: operands read two taps ahead into a register ring, the schedule
  // pinned (sched_barrier) so no LDS read is re-targeted at registers an in-flight MFMA still reads
  auto mac1 = [&](f4& acc, int sl, int tz) {
    const char* base = ring + sl * kSlotB;
    auto ld = [&](int t, h8v& x, h8v& wv) {
      const int ty = t / 3, tx = t - 3 * (t / 3);
      x = *reinterpret_cast<const h8v*>(base + (2 * jy + ty) * kRowB + acol[tx]);
      if constexpr (PRE) wv = bw1[tz * 9 + t];
      else wv = *reinterpret_cast<const h8v*>(w1l + (((tz * 9 + t) * 2 + bpart) * 64 + lane) * 16);
    };
    h8v xr[3], wr[3];
    ld(0, xr[0], wr[0]);
    ld(1, xr[1], wr[1]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 2 < 9) ld(t + 2, xr[(t + 2) % 3], wr[(t + 2) % 3]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xr[t % 3], wr[t % 3], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // role wave 3: the completed window of depth start s from the partials in scratch buffer sb
  auto finish1 = [&](int s, int sb) {
    const f4 aa = *reinterpret_cast<const f4*>(scr + ((sb * 3 + 0) * 64 + lane) * 16);
    const f4 ab = *reinterpret_cast<const f4*>(scr + ((sb * 3 + 1) * 64 + lane) * 16);
    const f4 ac = *reinterpret_cast<const f4*>(scr + ((sb * 3 + 2) * 64 + lane) * 16);
    const int oz = (s + a.pad[0]) >> 1;
    if (oz < a.o0[0] || oz >= a.o0[0] + a.on[0]) return;   // wave-uniform
    float vmax = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g4 + r, wx_ = row & 7, wy_ = row >> 3;
      const int oy = (y0 - 1 + 2 * wy_ + a.pad[1]) >> 1, ox = (x0 - 1 + 2 * wx_ + a.pad[2]) >> 1;
      if (oy < a.o0[1] || oy >= a.o0[1] + a.on[1] || ox < a.o0[2] || ox >= a.o0[2] + a.on[2]) continue;
      float v = ldexpf(aa[r] + (ab[r] + ac[r]), oexp1);
      if (a.bn1_sc) v = fmaxf((v - mu1) * sc1 + sh1, 0.0f);
      vmax = fmaxf(vmax, fabsf(v));
      const size_t vx = (((size_t)(oz - a.o0[0]) * a.on[1] + (oy - a.o0[1])) * a.on[2] + (ox - a.o0[2]));
      a.y1[(((size_t)b * a.on[0] * a.on[1] * a.on[2]) + vx) * 16 + i16] = v;
    }
    if (a.y1_bound) bound_update<false>(a.y1_bound, vmax);   // mid-loop: no read-back
  };

  // conv_1_0 in step k: window zs - 1 completes (depth tap 2 on plane zs + 1), window zs + 1 starts
  auto conv1_step = [&](int k) {
    const int zs = z0 + 2 * k;
#if defined(MVS_HEAD_ABL_C) || defined(MVS_HEAD_NO_MAC1)
    if (false) {
#else
    if (c1w < 3) {
#endif
      if (k == 0) {
        mac1(cur, slot_of(z0 - 1), 0);
        mac1(cur, slot_of(z0), 1);
      }
      mac1(cur, slot_of(zs + 1), 2);   // completes window zs - 1
      mac1(nxt, slot_of(zs + 1), 0);   // window zs + 1: depth taps 0, 1
      mac1(nxt, slot_of(zs + 2), 1);
      *reinterpret_cast<f4*>(scr + (((k & 1) * 3 + c1w) * 64 + lane) * 16) = cur;
      cur = nxt;
      nxt = f4{0.f, 0.f, 0.f, 0.f};
    } else if (k > 0) {
      finish1(zs - 3, (k - 1) & 1);   // the window completed in step k - 1
    }
  };
  // the last step's window; the last chunk also owns the window starting at D - 1 (its taps on
  // planes D, D + 1 are zero: complete after the last step).  Contains the kernel's last barrier.
  auto conv1_tail = [&]() {
    const bool tail = z1 == D;
    if (c1w < 3 && tail) *reinterpret_cast<f4*>(scr + (((nsteps & 1) * 3 + c1w) * 64 + lane) * 16) = cur;
    if (c1w == 3) finish1(z1 - 3, (nsteps - 1) & 1);
    __syncthreads();
    if (c1w == 3 && tail) finish1(z1 - 1, nsteps & 1);
  };

  // ================================ schedule ================================
  // Both roles pass the same barriers (nsteps + 3): producers fill batches 0, 1 before step 0 and batch
  // k + 2 during step k; the sampling state of a batch is formed at least one barrier before its items.
  if (!consumer && PRE) {
    // batches 0 .. 1 + kPreAhead before the first step; batch k + 2 + kPreAhead stored during step k
    // (its slots were last read in step k - 1), its loads issued kPD steps earlier (buffer j % kPD:
    // the step loop unrolled by kPD keeps the index static)
    constexpr int A = kPreAhead;
    stamp();
    pre_load(0, 0);
    load_bw1();
    load_bn1();
    stamp();
    __syncthreads();
    stamp();
    pre_store(0, 0);
#pragma unroll
    for (int j = 1; j <= 1 + A; ++j) {
      if (j >= nbatch) break;   // uniform
      pre_load(j, 0);
      pre_store(j, 0);
    }
#pragma unroll
    for (int r = 0; r < kPD; ++r)
      if (2 + A + r < nbatch) pre_load(2 + A + r, (2 + A + r) % kPD);
    stamp();
    __syncthreads();
    stamp();
    stamp();
    __syncthreads();
    stamp();
    for (int k0 = 0; k0 < nsteps; k0 += kPD) {
#pragma unroll
      for (int r = 0; r < kPD; ++r) {
        const int k = k0 + r;
        if (k >= nsteps) break;   // uniform
        if (k + 2 + A < nbatch) pre_store(k + 2 + A, (r + 2 + A) % kPD);
        if (k + 2 + A + kPD < nbatch) pre_load(k + 2 + A + kPD, (r + 2 + A) % kPD);
        stamp();
        conv1_step(k);
        stamp();
        __syncthreads();
        stamp();
      }
    }
    conv1_tail();
    return;
  }
  if (!consumer) {
    stamp();
    if (!kCoordsByConsumers) {
      coords(0, 0);
      coords(1, 1);
    }
    stamp();
    __syncthreads();
    stamp();
    items(0, 0);
    items(1, 1);
    stamp();
    __syncthreads();
    stamp();
    if (!kCoordsByConsumers && 2 < nbatch) coords(2, 0);   // buffer 0 is free again (batch 0's items are done)
    stamp();
    __syncthreads();
    stamp();
    for (int k = 0; k < nsteps; ++k) {
      if (k + 2 < nbatch) items(k + 2, (k + 2) & 1);
      stamp();
      if (!kCoordsByConsumers && k + 3 < nbatch) coords(k + 3, (k + 3) & 1);
      stamp();
      __syncthreads();
      stamp();
    }
    __syncthreads();
    return;
  }
  // ================================ consumer state ================================
  h8v bw[27];
  float sc0 = 1.0f, sh0 = 0.0f, mu0 = 0.0f;
  {
    const Rsrc rwf = make_rsrc(a.w0, 27u * 64u * 16u);
#pragma unroll
    for (int tp = 0; tp < 27; ++tp)
      bw[tp] = __builtin_bit_cast(h8v, __builtin_amdgcn_raw_buffer_load_b128(rwf, lane * 16, tp * 1024, 0));
    if (a.bn0_sc) {
      sc0 = a.bn0_sc[lane & 7];
      sh0 = a.bn0_sh[lane & 7];
      mu0 = a.bn0_mu[lane & 7];
    }
    asm volatile("" ::"v"(sc0), "v"(sh0), "v"(mu0));
    if constexpr (!PRE) load_bn1();
  }
  const int gy_out = y0 + wave;   // consumer wave's conv_0_0 output row
  const bool row_on = consumer && gy_out < H && x0 < W;
  int aoff[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
    aoff[kx] = (wave & 3) * kRowB + (i16 + kx) * kVoxB + ((g4 ^ (((i16 + kx) >> 1) & 3)) << 4);
  const int oexp0 = -(ex + a.w_exp0);
  const int gx0 = x0 + 4 * g4;
  const bool store_lane = (lane & 15) < 8;
  const bool vec_store = (W & 3) == 0 && gx0 + 3 < W;
  const size_t DHW = (size_t)D * HW;
  // conv_2_0 / conv_3_0 read the SCV on their input box: the tile-interior voxels of this chunk's
  // planes (every in-volume voxel is interior to exactly one tile and one chunk), copied from plane p's
  // ring slot -- 512 (voxel, quad) items of 16 B, a wave's 64 lanes four 256-B rows of one quad
  auto box_store = [&](int p) {
    if (p < zst0 || p >= zst1) return;   // uniform
    const char* base = ring + slot_of(p) * kSlotB;
    typedef __attribute__((ext_vector_type(4))) unsigned v4u;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * (wave + 4 * r);
      const int xx = i & 15, yy = (i >> 4) & 3, q = i >> 6;
      const int gx = x0 + xx, gy = y0 + yy, hx = xx + 1;
      const int off = (yy + 1) * kRowB + hx * kVoxB + (((q >> 1) ^ ((hx >> 1) & 3)) << 4) + ((q & 1) << 3);
      const uint2 h = *reinterpret_cast<const uint2*>(base + off);
      const uint2 l = *reinterpret_cast<const uint2*>(base + kPartB + off);
      if (gx < W && gy < H && gx >= a.r0[2] && gx < a.r1[2] && gy >= a.r0[1] && gy < a.r1[1])
        __builtin_amdgcn_raw_buffer_store_b128(
            v4u{h.x, h.y, l.x, l.y}, rscv,
            (int)((((uint32_t)q * (uint32_t)bz + (uint32_t)(p - a.r0[0])) * bhw +
                   (uint32_t)((gy - a.r0[1]) * bxw + (gx - a.r0[2]))) * 16u),
            0, 0);
    }
  };
  stamp();
  if (kCoordsByConsumers) {
    coords(0, 0);
    coords(1, 1);
  }
  stamp();
  __syncthreads();
  stamp();
  stamp();
  __syncthreads();
  stamp();
  if (kCoordsByConsumers && 2 < nbatch) coords(2, 0);
  stamp();
  __syncthreads();
  stamp();
  for (int k = 0; k < nsteps; ++k) {
    const int zs = z0 + 2 * k;
    // ---- conv_0_0 on planes zs - 1 .. zs + 2 (conv3d_split.hip's item order) ----
#if defined(MVS_HEAD_ABL_C) || defined(MVS_HEAD_NO_C0)   // (timing ablations)
    if (false) {
#else
    if (row_on) {
#endif
      f4 ah[2], al[2];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        ah[d] = f4{0.f, 0.f, 0.f, 0.f};
        al[d] = f4{0.f, 0.f, 0.f, 0.f};
      }
      const char* base[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) base[p] = ring + ((2 * k + p) % RS) * kSlotB;
      constexpr int kIt = 9 * 4;
      auto lda = [&](int it, h8v& hi, h8v& lo) {
        const int grp = it / 4, p = it % 4, ky = grp / 3, kx = grp % 3;
        hi = *reinterpret_cast<const h8v*>(base[p] + ky * kRowB + aoff[kx]);
        lo = *reinterpret_cast<const h8v*>(base[p] + kPartB + ky * kRowB + aoff[kx]);
      };
      h8v rh[kPF + 1], rl[kPF + 1];
#pragma unroll
      for (int it = 0; it < kPF; ++it) lda(it, rh[it], rl[it]);
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int p = it % 4, grp = it / 4;
        if (it + kPF < kIt) lda(it + kPF, rh[(it + kPF) % (kPF + 1)], rl[(it + kPF) % (kPF + 1)]);
        const h8v ch = rh[it % (kPF + 1)], cl = rl[it % (kPF + 1)];
#pragma unroll
        for (int kz = 0; kz < 3; ++kz) {
          const int d = p - kz;
          if (d < 0 || d >= 2) continue;
          ah[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch, bw[kz * 9 + grp], ah[d], 0, 0, 0);
          al[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cl, bw[kz * 9 + grp], al[d], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float hh = ah[d][r], lh = al[d][r];
          const float hl = ror8(hh), ll = ror8(lh);
          float s = ldexpf(hh + ((lh + hl) + ll), oexp0);
          if (a.bn0_sc) s = fmaxf((s - mu0) * sc0 + sh0, 0.0f);
          v[r] = s;
        }
        const int z = zs + d;
        if (store_lane) {
          float* o = a.y0 + ((size_t)(b * 8 + (lane & 7)) * D + z) * HW + (size_t)gy_out * W + gx0;
          if (vec_store) {
            // non-temporal: the 0.5 GB output is read once, by deconv_1_0 much later in the step
            __builtin_nontemporal_store(f4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<f4v*>(o));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (gx0 + r < W) o[r] = v[r];
          }
        }
      }
    }
    stamp();
    if constexpr (!PRE) conv1_step(k);
    if (kCoordsByConsumers && k + 3 < nbatch) coords(k + 3, (k + 3) & 1);
    // batch k + 1's planes (and plane z0 of batch 0) to the box: resident in their slots this step
    if (k == 0) box_store(z0);
    box_store(zs + 1);
    box_store(zs + 2);
    stamp();
    __syncthreads();
    stamp();
  }
  if constexpr (PRE) __syncthreads();   // (the producers' conv1_tail barrier)
  else conv1_tail();
}

// Outputs of the conv_1_0 region whose depth / row / column window no tile owns: windows entirely in
// the zero padding (conv value 0), written as relu(BN_1(0)) exactly as conv3d_s2_split.hip's epilogue
// forms it.  Per sample three slabs: z faces (lz + hz planes, whole rows), then y faces of the other
// planes, then x faces of the rest; one thread per (voxel, channel).
__global__ __launch_bounds__(256) void head_faces_kernel(float* __restrict__ y1, int B, int on0, int on1, int on2,
                                                         int lz, int hz, int ly, int hy, int lx, int hx,
                                                         const float* __restrict__ sc, const float* __restrict__ sh,
                                                         const float* __restrict__ mu, uint32_t* __restrict__ y1_bound) {
  const long nzf = lz + hz, nyf = ly + hy, nxf = lx + hx;
  float vmax = 0.0f;   // the constants this thread wrote raise y1's bound words too
  const long mz = on0 - nzf, my = on1 - nyf;
  const long n0 = nzf * on1 * on2, n1 = mz * nyf * on2, n2 = mz * my * nxf;
  const long per = n0 + n1 + n2;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < (long)B * per * 16; e += (long)gridDim.x * blockDim.x) {
    const int co = (int)(e & 15);
    long i = e >> 4;
    const long bb = i / per;
    i -= bb * per;
    int oz, oy, ox;
    if (i < n0) {
      const int zi = (int)(i / ((long)on1 * on2));
      const long r = i - (long)zi * on1 * on2;
      oz = zi < lz ? zi : on0 - hz + (zi - lz);
      oy = (int)(r / on2);
      ox = (int)(r - (long)oy * on2);
    } else if (i < n0 + n1) {
      i -= n0;
      const int zi = (int)(i / (nyf * on2));
      const long r = i - (long)zi * nyf * on2;
      const int yi = (int)(r / on2);
      oz = lz + zi;
      oy = yi < ly ? yi : on1 - hy + (yi - ly);
      ox = (int)(r - (long)yi * on2);
    } else {
      i -= n0 + n1;
      const int zi = (int)(i / (my * nxf));
      const long r = i - (long)zi * my * nxf;
      const int yi = (int)(r / nxf);
      const int xi = (int)(r - (long)yi * nxf);
      oz = lz + zi;
      oy = ly + yi;
      ox = xi < lx ? xi : on2 - hx + (xi - lx);
    }
    float v = ldexpf(0.0f + (0.0f + 0.0f), 0);
    if (sc) v = fmaxf((v - mu[co]) * sc[co] + sh[co], 0.0f);
    y1[((((size_t)bb * on0 + oz) * on1 + oy) * on2 + ox) * 16 + co] = v;
    vmax = fmaxf(vmax, v);
  }
  if (y1_bound) bound_update<true>(y1_bound, vmax);   // every lane of every wave reaches it
}

// outputs of the conv_1_0 region whose window no tile owns (all-padding windows, head_faces_kernel)
void launch_head_faces(const Geometry& g, const HeadArgs& a, const float* const* bn1, float* y1, const int* pad,
                       const int* o0, const int* on, hipStream_t s, uint32_t* y1_bound = nullptr) {
  // per dim, per dim, region outputs whose window start 2 o - P lies below -1 (before tile 0) or at /
  // beyond the last owned start (n_tiles * tile - 1 in x / y, D - 1 + 2 in z)
  int lo[3], hi[3];
  const int own_hi[3] = {g.Dc - 1, a.tiles_y * kTY - 1, a.tiles_x * kTX - 1};   // first unowned start
  for (int d = 0; d < 3; ++d) {
    lo[d] = 0;
    while (lo[d] < on[d] && 2 * (o0[d] + lo[d]) - pad[d] < -1) ++lo[d];
    hi[d] = 0;
    while (hi[d] < on[d] - lo[d] && 2 * (o0[d] + on[d] - 1 - hi[d]) - pad[d] > own_hi[d] - (d == 0 ? 0 : 1)) ++hi[d];
  }
  if (lo[0] + hi[0] + lo[1] + hi[1] + lo[2] + hi[2] > 0) {
    const long n = (long)g.B * on[0] * on[1] * on[2] * 16;
    const int blocks = (int)std::min<long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(head_faces_kernel, dim3(blocks), dim3(256), 0, s, y1, g.B, on[0], on[1], on[2], lo[0], hi[0],
                       lo[1], hi[1], lo[2], hi[2], bn1[0], bn1[1], bn1[2], y1_bound);
  }
}

// grid and geometry fields shared by both launchers
int head_grid(const Geometry& g, HeadArgs& a, const int* pad, const int* o0, const int* on, const int* r0,
              const int* r1) {
  a.D = g.Dc;
  a.H = g.h;
  a.W = g.w;
  // tiles cover conv_0_0's outputs and every stride-2 window that touches the volume: a tile owns
  // window starts [x0 - 1, x0 + 15) / [y0 - 1, y0 + 3), the last start is n - 1 (P odd, n even)
  a.tiles_x = g.w / kTX + 1;
  a.tiles_y = g.h / kTY + 1;
  a.zchunks = (g.Dc + kZC - 1) / kZC;
  const long total = (long)a.tiles_x * a.tiles_y * a.zchunks * g.B;
  if (total >= (1L << 31) - 8) return MVS_ERR_TOO_LARGE;
  a.total = (int)total;
  for (int d = 0; d < 3; ++d) {
    a.pad[d] = pad[d];
    a.o0[d] = o0[d];
    a.on[d] = on[d];
    a.r0[d] = r0[d];
    a.r1[d] = r1[d];
  }
  return MVS_OK;
}

}  // namespace

size_t cv_head_lds_bytes(int V) { return V == 2 ? (size_t)lds_bytes<1>() : (size_t)lds_bytes<2>(); }

int launch_cv_head(const Geometry& g, const float* feat, const Cams& cm, float* ws, uint32_t* absmax,
                   const void* w0frag, int w_exp0, const void* w1frag, int w_exp1, const float* const* bn0,
                   const float* const* bn1, float* y0, float* y1, void* scv, const int* pad, const int* o0,
                   const int* on, const int* r0, const int* r1, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  float* smp = ws;
  float* packed = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) +
                                           align256((size_t)g.B * g.V * g.Dc * 9 * sizeof(float)));
  launch_cv_prologue_pm(g, feat, cm, smp, packed, absmax, s);
  HeadArgs a = {};
  a.packed = reinterpret_cast<const float4*>(packed);
  a.refs = a.packed + (size_t)g.B * g.V * kC4 * pad_geom(g.h, g.w).plane;
  a.sampling = smp;
  a.absmax = absmax;
  a.w0 = reinterpret_cast<const h8v*>(w0frag);
  a.w1 = reinterpret_cast<const h8v*>(w1frag);
  a.bn0_sc = bn0[0];
  a.bn0_sh = bn0[1];
  a.bn0_mu = bn0[2];
  a.bn1_sc = bn1[0];
  a.bn1_sh = bn1[1];
  a.bn1_mu = bn1[2];
  a.y0 = y0;
  a.y1 = y1;
  a.scv = scv;
  a.scv_in = nullptr;
  a.V = g.V;
  a.w_exp0 = w_exp0;
  a.w_exp1 = w_exp1;
  const int gst = head_grid(g, a, pad, o0, on, r0, r1);
  if (gst != MVS_OK) return gst;
#ifdef MVS_HEAD_STAMP
  static unsigned long long* stamps = nullptr;
  const size_t stamp_bytes = (size_t)kStampWG * 8 * kStampN * sizeof(unsigned long long);
  if (!stamps) (void)hipMalloc(&stamps, stamp_bytes);
  (void)hipMemsetAsync(stamps, 0, stamp_bytes, s);
  a.stamps = stamps;
#endif
  if (ev0) (void)hipEventRecord(ev0, s);
  if (g.V == 2)
    hipLaunchKernelGGL(cv_head_kernel<2>, xcd_grid(a.total), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(cv_head_kernel<3>, xcd_grid(a.total), dim3(kThreads), 0, s, a);
  if (ev1) (void)hipEventRecord(ev1, s);
#ifdef MVS_HEAD_STAMP
  if (const char* path = getenv("MVS_HEAD_STAMPS")) {   // diagnostic build only: synchronous dump
    std::vector<unsigned long long> h(stamp_bytes / sizeof(unsigned long long));
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), stamps, stamp_bytes, hipMemcpyDeviceToHost);
    if (FILE* f = fopen(path, "ab")) {
      fwrite(h.data(), 1, stamp_bytes, f);
      fclose(f);
    }
  }
#endif
  launch_head_faces(g, a, bn1, y1, pad, o0, on, s);
  return MVS_OK;
}

int launch_split_head(const Geometry& g, const void* scv_in, const uint32_t* absmax, const void* w0frag, int w_exp0,
                      const void* w1frag, int w_exp1, const float* const* bn0, const float* const* bn1, float* y0,
                      float* y1, const int* pad, const int* o0, const int* on, uint32_t* y1_bound, hipStream_t s,
                      hipEvent_t ev0, hipEvent_t ev1) {
  HeadArgs a = {};
  a.y1_bound = y1_bound;
  a.absmax = absmax;
  a.w0 = reinterpret_cast<const h8v*>(w0frag);
  a.w1 = reinterpret_cast<const h8v*>(w1frag);
  a.bn0_sc = bn0[0];
  a.bn0_sh = bn0[1];
  a.bn0_mu = bn0[2];
  a.bn1_sc = bn1[0];
  a.bn1_sh = bn1[1];
  a.bn1_mu = bn1[2];
  a.y0 = y0;
  a.y1 = y1;
  a.scv = nullptr;
  a.scv_in = scv_in;
  a.V = 2;
  a.w_exp0 = w_exp0;
  a.w_exp1 = w_exp1;
  const int zero[3] = {0, 0, 0};
  const int gst = head_grid(g, a, pad, o0, on, zero, zero);
  if (gst != MVS_OK) return gst;
#ifdef MVS_HEAD_STAMP
  static unsigned long long* stamps = nullptr;
  const size_t stamp_bytes = (size_t)kStampWG * 8 * kStampN * sizeof(unsigned long long);
  if (!stamps) (void)hipMalloc(&stamps, stamp_bytes);
  (void)hipMemsetAsync(stamps, 0, stamp_bytes, s);
  a.stamps = stamps;
#endif
  if (ev0) (void)hipEventRecord(ev0, s);
  hipLaunchKernelGGL((cv_head_kernel<2, true>), xcd_grid(a.total), dim3(kThreads), 0, s, a);
  if (ev1) (void)hipEventRecord(ev1, s);
#ifdef MVS_HEAD_STAMP
  if (const char* path = getenv("MVS_HEAD_STAMPS")) {   // diagnostic build only: synchronous dump
    std::vector<unsigned long long> h(stamp_bytes / sizeof(unsigned long long));
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), stamps, stamp_bytes, hipMemcpyDeviceToHost);
    if (FILE* f = fopen(path, "ab")) {
      fwrite(h.data(), 1, stamp_bytes, f);
      fclose(f);
    }
  }
#endif
  launch_head_faces(g, a, bn1, y1, pad, o0, on, s, y1_bound);
  return MVS_OK;
}

}  // namespace mvs
