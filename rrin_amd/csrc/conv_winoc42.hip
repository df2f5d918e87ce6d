// Exact-fp32 3x3 conv as Winograd F(4,3) x F(2,3) on fp32 records (R32): Winograd kind 14 of
// the record-layout conv table, the register-U structure of kind 6 (conv_winoc.hip) on patches
// 4 outputs wide and 2 tall.  24 transform points per patch instead of F(2x2,3x3)'s 16 per 4
// outputs: 3 MFMAs per output and input channel instead of 4 (0.75x), at the price of a 6-point
// column transform per lane and one co tile per transform (kind 6 feeds two).
//
// Replaces nn.Conv2d(3, pad=1) + LeakyReLU(0.1) (unet.py:29,59-63), the fused avg_pool2d output
// (unet.py:46), the cat by channel offset (unet.py:93) and the sub-pixel form of Upsample + up
// conv (unet.py:77-78), as every record-layout conv.
//
// Transforms (1D, in double by the packer for G; the input / output ones in fp32 here):
//   x (F(4,3)): B^T rows  v0 = 4 t0 - 5 t2 + t4        v1 = -4 (t1 + t2) + (t3 + t4)
//                         v2 = 4 (t1 - t2) + (t4 - t3)  v3 = -2 (t1 - t3) + (t4 - t2)
//                         v4 = 2 (t1 - t3) + (t4 - t2)  v5 = 4 t1 - 5 t3 + t5
//               A^T rows  Q0 = (M0 + (M1 + M2)) + (M3 + M4)        Q1 = (M1 - M2) + 2 (M3 - M4)
//                         Q2 = (M1 + M2) + 4 (M3 + M4)             Q3 = ((M1 - M2) + 8 (M3 - M4)) + M5
//   y (F(2,3)): kind 6's (wave yw owns B^T row yw; Y0 = (Q0 + Q1) + Q2, Y1 = (Q1 - Q2) - Q3).
// An output depends only on its 3x3 input footprint (the formulas omit the zero entries), so
// records past the image (the last tile's rows / columns) never reach a stored output.
//
// Tile: BM 32 output channels x 32 patches of 4 x 2: 32 px x 8 rows (8 columns x 4 rows of
// patches) or 16 px x 16 rows (4 x 8; W42<PCW>).  Wave yw (0-3) owns B^T_y row yw (points
// 6 yw .. 6 yw + 5); lane (j, hh): patch j (column pc = j % PCW, row pr = j / PCW) of the MFMA
// tile, record half hh (channels 4 hh .. + 3 of the 8-channel chunk; MFMA product e contracts
// channels e and 4 + e).  Per wave and chunk: 24 MFMAs, 6 U loads (one record per 4 MFMAs),
// 12 window reads, ~80 VALU, 3 (32 x 8) or 4 (16 x 16) LDS-DMA pieces.  Short K on a large grid (launch_winoc42): persistent workgroups that issue
// the next tile's raw(0), raw(1), U(0) before this tile's epilogue (W42P: the exchange in two
// halves, the stages past it).
// U: rrin_pack_conv3x3_wino_cfg for this kind, [cob][chunk][xi 24][hh][32 co][4 ch].
#include <type_traits>

#include "common.hpp"

#ifndef RRIN_WINO42_AGPR
#define RRIN_WINO42_AGPR 0
#endif
namespace rrin {

typedef float w42f16 __attribute__((ext_vector_type(16)));
typedef float w42f4 __attribute__((ext_vector_type(4)));

// Tile geometry PCW: 8 -> 32 px x 8 rows (8 x 4 patches), 4 -> 16 px x 16 rows (4 x 8 patches).
// Every output comes from the same patch, transforms and MFMA column arithmetic in both, so the
// geometry changes no bit of the result (tests/test_gpu_wino42.py); launch_winoc42 picks the one
// with fewer workgroup rounds (the 16 x 16 tile fits the level-4 grids, 80 x 45 at 1280 x 720).
template <int PCW_>
struct W42 {
  static constexpr int PCW = PCW_;                  // patch columns per tile
  static constexpr int PRW = 32 / PCW;              // patch rows per tile
  static constexpr int TW = 4 * PCW;                // output columns
  static constexpr int TH = 2 * PRW;                // output rows
  static constexpr int RC = TW + 2;                 // raw columns
  static constexpr int WM = (RC + 3) / 4;           // slots per column residue (w42_slot)
  // LDS slots per raw row: >= 4 WM, and 2 RW = 8 (PCW 8) or 4 / 12 (PCW 4) mod 16 records so a
  // ds_read_b128 group of 16 lanes (PCW columns x 16 / PCW rows) covers the 64 banks once
  static constexpr int RW = PCW == 8 ? 36 : 22;
  static_assert(RW >= 4 * WM, "raw row slots");
  static constexpr int RG = (TH + 2) * RW;          // per record group
  static constexpr int RAW = 2 * RG;                // per chunk (2 groups)
  static constexpr int PIECES = (RAW + 255) / 256;  // DMA pieces per thread
  static constexpr int STAGE = PIECES * 256;        // records per LDS stage (the tail is a dummy)
  static constexpr int NS = 3;                      // stages: chunk c + 2 lands while c computes
  static constexpr int XP = 65;                     // exchange pitch in records (64 lanes + 1)
  static constexpr int XREC = 4 * 16 * XP;          // output-transform exchange: 4 waves x 16 records
  static constexpr size_t LDS = (size_t)(NS * STAGE > XREC ? NS * STAGE : XREC) * 16;
};
static_assert(W42<8>::LDS == kWinoC42Lds && W42<4>::LDS == kWinoC42Lds, "LDS size (common.hpp)");
static_assert(2 * kWinoC42Lds <= 160 * 1024, "two blocks per CU");
// Persistent 32 x 8 tiles (short K): the next tile's first two raw chunks land
// during this tile's epilogue, so the stages may not overlay the exchange.  The exchange then
// runs in two halves of 8 records per lane (pitch 66: the gather's lane group reads slots
// 4 cx + patch, 16 distinct) and the stages sit past it.
struct W42P {
  static constexpr int XP = 66;
  static constexpr int XREC = 4 * 8 * XP;  // 2112 records
  static constexpr size_t LDS = (size_t)(XREC + W42<8>::NS * W42<8>::STAGE) * 16;
};
static_assert(2 * W42P::LDS <= 160 * 1024, "two blocks per CU (persistent)");

// LDS slot of raw column col (0 .. RC - 1) in its row: the PCW patch columns 4 pc + k of one k
// are consecutive slots, so a ds_read_b128 lane group (16 patches and their neighbours) covers
// the 64 banks once
template <int WM>
__device__ constexpr int w42_slot(int col) { return (col & 3) * WM + (col >> 2); }

// (the base through readfirstlane: a resource the compiler cannot prove uniform -- a base that
// changes per persistent tile -- turns every buffer load into a waterfall loop)
__device__ inline __amdgpu_buffer_rsrc_t w42_rsrc(const void* base) {
  const uint64_t p = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(p >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7fffffff, 0x00020000);
}

template <int EPI, int PCW, bool PERSIST>
__global__ __launch_bounds__(256, 2) void conv3x3_winoc42_kernel(ConvH8Args a) {
  using G = W42<PCW>;
  static_assert(!PERSIST || PCW == 8, "persistent tiles: the 32 x 8 geometry");
  constexpr int TH = G::TH, TW = G::TW, RG = G::RG, RW = G::RW, STAGE = G::STAGE, P = G::PIECES, WM = G::WM;
  constexpr int SB = PERSIST ? W42P::XREC : 0;  // first stage record
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int yw = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  const int pc = j % PCW, pr = j / PCW;
  int bid;
  {  // XCD-aware bijective remap (conv_mfma.hip): an XCD's workgroups are consecutive tiles
    const int nwg = (int)gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
  const int nch = a.nchunks;
  // tile -> (co block, x0, y0, image); co-block groups as kind 6 (launch_winoc42: U of a group
  // fits an XCD's L2).  PERSIST: workgroup b runs tiles b, b + grid, ...
  auto decode = [&](int tile, int& cob_, int& x0_, int& y0_, int& img_) {
    const int cpg = a.cob_group > 0 ? a.cob_group : a.co_blocks;
    const int gsz = cpg * (ntiles / a.co_blocks);
    const int g = tile / gsz;
    const int r = tile - g * gsz;
    const int cg = min(cpg, a.co_blocks - g * cpg);
    cob_ = g * cpg + r % cg;
    int t = r / cg;
    x0_ = (t % a.tiles_x) * TW;
    t /= a.tiles_x;
    y0_ = (t % a.tiles_y) * TH;
    img_ = t / a.tiles_y;
  };
  int tile = bid, cob, x0, y0, img;
  decode(tile, cob, x0, y0, img);

  // ---- raw tile: rows y0 - 1 .. y0 + TH, cols x0 - 1 .. x0 + TW of the chunk's two record
  // groups, buffer_load ... lds from a per-chunk base; slots past the tile re-read record 0
  auto tile_base = [&](int img_, int y0_, int x0_) {
    return a.src_hi + (int64_t)img_ * a.src_img + (int64_t)y0_ * a.src_wp + x0_ + (kH8PadLeft - 1);
  };
  const uint4* tbase = tile_base(img, y0, x0);
  // (a fixed bound: an array sized by the dependent P and captured by the lambda below drops the
  // kernel's host stub without a diagnostic -- hipcc 7.2)
  static_assert(P <= 4, "DMA pieces");
  uint32_t voff[4];
#pragma unroll
  for (int it = 0; it < P; ++it) {
    const int idx = tid + 256 * it;
    const int g = idx >= RG ? 1 : 0;
    const int rem = idx < G::RAW ? idx - g * RG : 0;
    const int r = rem / RW, pos = rem - r * RW;
    const int m = pos / WM, q = pos - m * WM;
    const int col = 4 * q + m;
    const bool ok = idx < G::RAW && m < 4 && col < G::RC;
    voff[it] = ok ? (uint32_t)((int64_t)g * a.src_gp + (int64_t)r * a.src_wp + col) * 16u : 0u;
  }
  const int64_t chunk_stride = 2 * a.src_gp;
  auto issue_raw_at = [&](const uint4* base, int s) {
    const auto rs = w42_rsrc(base);
#pragma unroll
    for (int it = 0; it < P; ++it)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(smem4 + SB + s * STAGE + 256 * it + 64 * yw), 16, voff[it], 0, 0,
          0);
  };
  const uint4* raw_next = tbase;  // raw(c + 2)'s base, set per tile

  // ---- U straight into registers: record (chunk c, xi = 6 yw + x, hh, co j) of the co block;
  // the chunk and the point's upper part in the scalar offset, the rest < 4 KB immediate
  // (the resource built at each load from the co block's base: w42_rsrc's readfirstlane keeps it
  // scalar also when the base is a loop-carried value of the persistent tile loop)
  auto u_base = [&](int cob_) { return a.w_hi + (int64_t)cob_ * nch * 1536; };
  const uint4* ub = u_base(cob);
  const uint32_t uvoff = (uint32_t)(hh * 32 + j) * 16u;
  auto load_u = [&](int c, int x) {
    const int soff = c * (1536 * 16) + (6 * yw + (x & 4)) * 1024;
    return __builtin_bit_cast(w42f4,
                              __builtin_amdgcn_raw_buffer_load_b128(w42_rsrc(ub), uvoff + (x & 3) * 1024, soff, 0));
  };

  // ---- B operands: B^T_y row yw combines raw rows ra, rb of the patch (kind 6's rows)
  const int ra = yw == 0 ? 0 : (yw == 2 ? 2 : 1);
  const int rb = yw == 0 ? 2 : (yw == 1 ? 2 : (yw == 2 ? 1 : 3));
  const float sg = yw == 1 ? 1.f : -1.f;
  const int lbase = hh * RG + 2 * pr * RW + pc;
  const int oa = lbase + ra * RW, ob = lbase + rb * RW;

  w42f16 acc[6];  // set by chunk 0's first MFMA of each point (C = 0: no 96 zeroing moves per tile)
  // U of the chunk being computed (point x reloaded for the next chunk after its MFMAs; a
  // prefetch distance of two chunks needs a second set: 256 VGPRs and spills)
  w42f4 ua[6];
  w42f4 v[6];   // B operands of the chunk being computed
  w42f4 d[12];  // window records of the next chunk: rows ra / rb, columns 0-5

  auto read_raw = [&](int s) {
    const uint4* rw = smem4 + SB + s * STAGE;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      d[2 * k] = __builtin_bit_cast(w42f4, rw[oa + w42_slot<WM>(k)]);
      d[2 * k + 1] = __builtin_bit_cast(w42f4, rw[ob + w42_slot<WM>(k)]);
    }
  };
  w42f4 t[6];
  auto rows = [&]() {
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[k][e] = fmaf(sg, d[2 * k + 1][e], d[2 * k][e]);
  };
  auto cols_a = [&]() {  // points 0-2
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[0][e] = fmaf(4.f, t[0][e], fmaf(-5.f, t[2][e], t[4][e]));
      v[1][e] = fmaf(-4.f, t[1][e] + t[2][e], t[3][e] + t[4][e]);
      v[2][e] = fmaf(4.f, t[1][e] - t[2][e], t[4][e] - t[3][e]);
    }
  };
  auto cols_b = [&]() {  // points 3-5
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float p = t[1][e] - t[3][e], s = t[4][e] - t[2][e];
      v[3][e] = fmaf(-2.f, p, s);
      v[4][e] = fmaf(2.f, p, s);
      v[5][e] = fmaf(4.f, t[1][e], fmaf(-5.f, t[3][e], t[5][e]));
    }
  };
  auto mfma_point = [&](const w42f4(&u)[6], int x, const bool first) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(u[x][e], v[x][e], first && e == 0 ? w42f16{} : acc[x], 0, 0, 0);
  };
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };

  // Chunk c (U(c) in u, its B operands in v), MORE: it has a successor.  Points 0-2, each
  // followed by the load of its U for chunk c + 1; the wait for raw(c + 1) (issued a chunk ago; the
  // previous chunk's U pts 3-5 and this chunk's U pts 0-2 stay in flight); the barrier; raw(c + 2)
  // -> the free stage; chunk c + 1's window reads under points 3-4, its row combination and points
  // 0-2 transform, point 5, its points 3-5 transform; U pts 3-5 after their MFMAs.  VMEM order
  // per chunk: U pts 0-2, raw(c + 2), U pts 3-5 -- the same every chunk.  The prologue issues
  // raw(0), raw(1), U(0) (also when it is the previous tile's prefetch), so chunk 0's wait for
  // raw(1) leaves 9 loads in flight: U(0) and U(1) pts 0-2.
  auto chunk = [&](int c, int s, const bool more, const bool first, w42f4(&u)[6]) {
    const int cu = c + 1;
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      mfma_point(u, x, first);
      if (more) u[x] = load_u(cu, x);
      fence();
    }
    if (more) {
      if (first)
        RRIN_VMWAIT(0, 9);
      else
        RRIN_VMWAIT(0, 6);
      bar();
      issue_raw_at(raw_next, s == 0 ? 2 : s - 1);
      if (c + 3 < nch) raw_next += chunk_stride;
      read_raw(s == 2 ? 0 : s + 1);
    }
    fence();
    mfma_point(u, 3, first);
    if (more) u[3] = load_u(cu, 3);
    fence();
    mfma_point(u, 4, first);
    if (more) u[4] = load_u(cu, 4);
    fence();
    if (more) {
      rows();
      cols_a();
    }
    fence();
    mfma_point(u, 5, first);
    if (more) u[5] = load_u(cu, 5);
    fence();
    if (more) cols_b();
  };
  auto next_stage = [](int s) { return s == 2 ? 0 : s + 1; };

  // prologue: raw(0), raw(1), U(0) -- the order the cross-tile prefetch issues them in too
  auto issue_prologue_raw = [&]() {
    issue_raw_at(tbase, 0);
    issue_raw_at(nch > 1 ? tbase + chunk_stride : tbase, 1);
    vm_fence();
  };
  auto issue_prologue_u = [&]() {
#pragma unroll
    for (int x = 0; x < 6; ++x) ua[x] = load_u(0, x);
    vm_fence();
  };
  issue_prologue_raw();
  issue_prologue_u();

  // ---- output transform: Q[c] = A^T_x row c of this wave's six points, record k (values
  // 4 k .. 4 k + 3 of c = k >> 2) per lane into X[wave][record][lane].  Wave yw then finishes
  // patch row prw = yw (PCW 8; PCW 4: rows 2 yw and 2 yw + 1 in lanes 0-15 and 16-31): lane
  // (xo, hh) takes pixel column x0 + xo (patch xo >> 2, column xo & 3) of output rows y0 + 2 prw
  // and + 1 from the four waves' Q with kind 6's A^T_y, so each store instruction writes runs of
  // TW consecutive pixels of a record group (the patch-per-lane layout wrote 16 B of every 64 B:
  // the stores were a quarter of a short-K tile's time).  One pass of 16 records
  // (pitch 65 over the stages) or, PERSIST, two of 8 (pitch 66, past them: W42P).
  constexpr int NPR = 32 / TW;  // patch rows a wave finishes
  const int xo = lane & (TW - 1), cx = xo & 3;
  const int prw = yw * NPR + (NPR == 1 ? 0 : (lane >> 4) & 1);
  const int src = (xo >> 2) + PCW * prw + 32 * hh;  // the lane of the MFMA layout holding this patch
  auto qrec = [&](int k) {
    w42f4 g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int vi = 4 * k + e, c = vi >> 4, i = vi & 15;
      const float m0 = acc[0][i], m1 = acc[1][i], m2 = acc[2][i], m3 = acc[3][i], m4 = acc[4][i], m5 = acc[5][i];
      g[e] = c == 0   ? (m0 + (m1 + m2)) + (m3 + m4)
             : c == 1 ? fmaf(2.f, m3 - m4, m1 - m2)
             : c == 2 ? fmaf(4.f, m3 + m4, m1 + m2)
                      : fmaf(8.f, m3 - m4, m1 - m2) + m5;
    }
    return g;
  };
  w42f4* X = reinterpret_cast<w42f4*>(smem4);
  float bsv[16];
  int ncob = 0;
  // the epilogue of the current tile; PF: the next tile's raw(0), raw(1) are in flight, its U(0)
  // loads follow the exchange (the accumulators are dead by then)
  auto epilogue = [&](auto pf) {
    float yv[2][16];  // rows 0 / 1 of the patch row, 16 channels
    if constexpr (!PERSIST) {
      constexpr int XP = G::XP;
#pragma unroll
      for (int k = 0; k < 16; ++k) X[(yw * 16 + k) * XP + lane] = qrec(k);
      __syncthreads();
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const int k = 4 * cx + k4;
        const w42f4 q0 = X[(0 * 16 + k) * XP + src];
        const w42f4 q1 = X[(1 * 16 + k) * XP + src];
        const w42f4 q2 = X[(2 * 16 + k) * XP + src];
        const w42f4 q3 = X[(3 * 16 + k) * XP + src];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          yv[0][4 * k4 + e] = (q0[e] + q1[e]) + q2[e];
          yv[1][4 * k4 + e] = (q1[e] - q2[e]) - q3[e];
        }
      }
    } else {
      constexpr int XP = W42P::XP;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // records k with k & 3 in {2 h, 2 h + 1}: kk = 2 (k >> 2) + (k & 1)
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) X[(yw * 8 + kk) * XP + lane] = qrec(4 * (kk >> 1) + 2 * h + (kk & 1));
        __syncthreads();
#pragma unroll
        for (int k4h = 0; k4h < 2; ++k4h) {
          const int kk = 2 * cx + k4h, k4 = 2 * h + k4h;
          const w42f4 q0 = X[(0 * 8 + kk) * XP + src];
          const w42f4 q1 = X[(1 * 8 + kk) * XP + src];
          const w42f4 q2 = X[(2 * 8 + kk) * XP + src];
          const w42f4 q3 = X[(3 * 8 + kk) * XP + src];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            yv[0][4 * k4 + e] = (q0[e] + q1[e]) + q2[e];
            yv[1][4 * k4 + e] = (q1[e] - q2[e]) - q3[e];
          }
        }
        if (h == 0) __syncthreads();  // every gather of half 0 done before half 1 overwrites X
      }
      if constexpr (decltype(pf)::value) {
        ub = u_base(ncob);
        issue_prologue_u();
      }
    }
    uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
    auto store4 = [&](int64_t rec, const float* vv) {
      dst[rec] = make_uint4(__float_as_uint(vv[0]), __float_as_uint(vv[1]), __float_as_uint(vv[2]), __float_as_uint(vv[3]));
    };
    const int x = x0 + xo, yb = y0 + 2 * prw;
    if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
      const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
  #pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int y = yb + r;
        if (cob * 32 < a.cout && y < a.h && x < a.w) {
  #pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int Y = 2 * y + (qq >> 1), XX = 2 * x + (qq & 1);
            const int64_t ri = ring_index(Y, XX, HH, WW);
            if (ri >= 0) {
  #pragma unroll
              for (int e = 0; e < 4; ++e)
                a.edge[((int64_t)img * creal + cob * 8 + 4 * hh + e) * a.ring + ri] = yv[r][4 * qq + e];
            } else {
              float vv[4];
  #pragma unroll
              for (int e = 0; e < 4; ++e) vv[e] = yv[r][4 * qq + e] + bsv[4 * qq + e];
              store4((int64_t)(2 * cob + hh) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + XX + kH8PadLeft, vv);
            }
          }
        }
      }
    } else {
      float vv[2][16];
  #pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int y = yb + r;
  #pragma unroll
        for (int i = 0; i < 16; ++i) {
          float tv = yv[r][i] + bsv[i];
          if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
          vv[r][i] = tv;
        }
  #pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (cob * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
            const int64_t rec = (int64_t)(cob * 8 + 2 * qq + hh) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
            store4(rec, &vv[r][4 * qq]);
            if constexpr (EPI == RRIN_EPI_LEAKY_REP) {  // edge replicate into the padding ring
              const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
              const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
              for (int dy = dy0; dy <= dy1; ++dy)
                for (int dx = dx0; dx <= dx1; ++dx)
                  if (dy | dx) store4(rec + (int64_t)dy * a.dst_wp + dx, &vv[r][4 * qq]);
            }
          }
        }
      }
      if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
        // a pool pair: rows yb, yb + 1 in this lane, columns x, x + 1 in lanes xo, xo ^ 1 (DPP
        // quad_perm [1, 0, 3, 2]); the even lane writes avg = 0.25 ((Y00 + Y10) + (Y01 + Y11))
        const int yp = yb;
        uint4* pdst = a.pool_hi + (int64_t)img * a.pool_img;
  #pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          float s4[4];
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float col = vv[0][4 * qq + e] + vv[1][4 * qq + e];
            const float nb = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(col), 0xB1, 0xF, 0xF, false));
            s4[e] = 0.25f * (col + nb);
          }
          if ((xo & 1) == 0 && cob * 32 + 8 * qq < a.cout && yp < a.h && x < a.w) {
            const int64_t rec =
                (int64_t)(cob * 8 + 2 * qq + hh) * a.pool_gp + (int64_t)(yp / 2 + 1) * a.pool_wp + x / 2 + kH8PadLeft;
            pdst[rec] = make_uint4(__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                                   __float_as_uint(s4[3]));
          }
        }
      }
    }
  };

  for (;;) {
    // wait for raw(0); chunk 0's B operands
    raw_next = tbase + (nch > 2 ? 2 : nch - 1) * chunk_stride;
    RRIN_VMWAIT(P, 6);
    bar();
    read_raw(0);
    rows();
    cols_a();
    cols_b();
    {
      int s = 0;
      if (nch > 1) {
        chunk(0, s, true, true, ua);
        s = next_stage(s);
        for (int c = 1; c + 1 < nch; ++c) {
          chunk(c, s, true, false, ua);
          s = next_stage(s);
        }
        chunk(nch - 1, s, false, false, ua);
      } else {
        chunk(0, s, false, true, ua);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA past the end has landed
#pragma unroll
    for (int i = 0; i < 16; ++i) bsv[i] = a.bias[cob * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
    vm_fence();  // the bias loads stay older than the next tile's prologue (make check-isa)
#if RRIN_WINO42_AGPR
    asm volatile("" ::"a"(acc[0][0]));
#endif
    __syncthreads();  // every read of the stages done before the exchange / the next tile's DMA
    if constexpr (!PERSIST) {
      epilogue(std::false_type{});
      break;
    } else {
      // the next tile's raw(0), raw(1), U(0) -- after the last tile a dummy re-issue of this
      // one's, so every path into the prologue wait carries the same loads (make check-isa)
      const int next = tile + (int)gridDim.x;
      const bool more = next < ntiles;
      int nx0, ny0, nimg;
      decode(more ? next : tile, ncob, nx0, ny0, nimg);
      tbase = tile_base(nimg, ny0, nx0);
      issue_prologue_raw();
      epilogue(std::true_type{});
      if (!more) break;
      tile = next;
      cob = ncob, x0 = nx0, y0 = ny0, img = nimg;
    }
  }
  if constexpr (PERSIST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy prologue has landed
}

template <int EPI, int PCW, bool PERSIST>
static int launch_winoc42_k(const ConvH8Args& a, int64_t grid, hipStream_t st) {
  auto k = conv3x3_winoc42_kernel<EPI, PCW, PERSIST>;
  constexpr size_t lds = PERSIST ? W42P::LDS : kWinoC42Lds;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)lds, st)) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  return hip_code(hipGetLastError());
}

// geometry policy (rrin_conv_h8_set_wino42_geom): 0 auto, 1 32 x 8 tiles, 2 16 x 16 tiles, 3 32 x 8
// tiles, one workgroup per tile
#ifndef RRIN_WINO42_GEOM_DEFAULT
#define RRIN_WINO42_GEOM_DEFAULT 0  // A/B builds (tools/build_wino_variant.sh): another start policy
#endif
static std::atomic<int> g_wino42_geom{RRIN_WINO42_GEOM_DEFAULT};

// persistent 32 x 8 tiles for short K: at most this many chunks (0: never), this many workgroups
#ifndef RRIN_WINO42_PERSIST_MAXCH
#define RRIN_WINO42_PERSIST_MAXCH 8
#endif
#ifndef RRIN_WINO42_PERSIST_WG
#define RRIN_WINO42_PERSIST_WG 512
#endif
#ifndef RRIN_WINO42_PERSIST_MINT  // fewest tiles (two per workgroup at least)
#define RRIN_WINO42_PERSIST_MINT 768
#endif

// co-block groups whose U fits kWinoCUGroupBytes of an XCD's L2 (as launch_winoc)
#ifndef RRIN_WINO42_UGROUP_KB
#define RRIN_WINO42_UGROUP_KB 2048
#endif
int launch_winoc42(const ConvH8Args& a, int epi, hipStream_t st) {
  ConvH8Args b = a;
  const int64_t per_cob = (int64_t)a.nchunks * 1536 * 16;
  b.cob_group = 0;
  if (RRIN_WINO42_UGROUP_KB > 0 && (int64_t)a.co_blocks * per_cob > (int64_t)RRIN_WINO42_UGROUP_KB * 1024) {
    int g = 1;
    while (2 * g < a.co_blocks && 2 * g * per_cob <= (int64_t)RRIN_WINO42_UGROUP_KB * 1024) g *= 2;
    b.cob_group = g;
  }
  // the 16 x 16 tile when it needs fewer rounds of the 512 resident workgroups (two per CU):
  // 1280 x 720's level 4 (80 x 45) is 576 tiles of 32 x 8 (1.1 rounds, 28 % of the area past
  // the image) but 480 of 16 x 16; elsewhere the 32 x 8 tile (10 raw rows per 8, not 18 per 16)
  const int64_t per_tile = (int64_t)a.co_blocks * a.n;
  const int64_t wide = per_tile * a.tiles_x * a.tiles_y;
  const int64_t tall = per_tile * ((a.w + 15) / 16) * ((a.h + 15) / 16);
  const int mode = g_wino42_geom.load(std::memory_order_relaxed);
  const bool use_tall = mode == 2 || (mode == 0 && (tall + 511) / 512 < (wide + 511) / 512);
  if (use_tall) {
    b.tiles_x = (a.w + 15) / 16;
    b.tiles_y = (a.h + 15) / 16;
  }
  // short K (level 0 at 1280 x 720: 4-8 chunks per tile, as long as its prologue and epilogue):
  // persistent workgroups that prefetch the next tile's first raw chunks under the epilogue
  const bool persist = !use_tall && mode != 3 && RRIN_WINO42_PERSIST_MAXCH > 0 &&
                       a.nchunks <= RRIN_WINO42_PERSIST_MAXCH && wide >= RRIN_WINO42_PERSIST_MINT;
  const int64_t grid = persist ? std::min<int64_t>(RRIN_WINO42_PERSIST_WG, wide / 2) : use_tall ? tall : wide;
#define RRIN_W42_CASE(E)                                                       \
  case E:                                                                      \
    return use_tall  ? launch_winoc42_k<E, 4, false>(b, grid, st)              \
           : persist ? launch_winoc42_k<E, 8, true>(b, grid, st)               \
                     : launch_winoc42_k<E, 8, false>(b, grid, st);
  switch (epi) {
    RRIN_W42_CASE(RRIN_EPI_LINEAR)
    RRIN_W42_CASE(RRIN_EPI_LEAKY)
    RRIN_W42_CASE(RRIN_EPI_LEAKY_POOL)
    RRIN_W42_CASE(RRIN_EPI_LEAKY_REP)
    RRIN_W42_CASE(RRIN_EPI_SUBPIXEL)
  }
#undef RRIN_W42_CASE
  return RRIN_E_ARG;
}

}  // namespace rrin

using namespace rrin;

// Kind-14 tile geometry policy (process-wide; results are the same bits either way): 0 auto
// (fewer workgroup rounds), 1 always 32 x 8, 2 always 16 x 16, 3 always 32 x 8 with one workgroup
// per tile (no persistent short-K launch).  Returns the previous policy.
extern "C" int rrin_conv_h8_set_wino42_geom(int32_t mode) {
  if (mode < 0 || mode > 3) return RRIN_E_ARG;
  return g_wino42_geom.exchange(mode);
}

// Kind-14 packing: [co block of 32][8-channel chunk][point xi = 6 eta + xi_x][record half][32 co][4 ch],
// U(eta, xi_x) = sum G2[eta][ky] G4[xi_x][kx] g[ky][kx] in double, rounded once to fp32
extern "C" int64_t rrin_pack_conv3x3_wino42_floats(int32_t cout, int32_t cin) {
  if (cout < 1 || cin < 1) return RRIN_E_ARG;
  return (int64_t)((cout + 31) / 32) * ((cin + 7) / 8) * 24 * 2 * 32 * 4;
}

extern "C" int rrin_pack_conv3x3_wino42(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                                        float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G2[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
  static const double G4[6][3] = {{0.25, 0.0, 0.0},
                                  {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                  {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                  {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                  {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                  {0.0, 0.0, 1.0}};
  const int cob_n = (cout + 31) / 32, nch = (cin + 7) / 8;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 24; ++xi)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < 32; ++col)
            for (int e = 0; e < 4; ++e) {
              const int co = cob * 32 + col, ch = c * 8 + hh * 4 + e;
              double u = 0.0;
              if (co < cout && ch < cin) {
                const float* g = w + ((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9;
                for (int ky = 0; ky < 3; ++ky)
                  for (int kx = 0; kx < 3; ++kx) u += G2[xi / 6][ky] * G4[xi % 6][kx] * (double)g[ky * 3 + kx];
              }
              wpack[o++] = (float)u;
            }
  for (int co = 0; co < cob_n * 32; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}
