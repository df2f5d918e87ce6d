// Exact-fp32 3x3 conv as Winograd F(2x2,3x3) on fp32 records (R32): the
// persistent register-U tile for the 32-output-channel convs, Winograd kind 8 of
// the record-layout conv table.  Same tile, wave roles and arithmetic order as
// kind 3 (conv3x3_winoq_kernel, conv_wino.hip): the outputs are bitwise those of
// configs 18-24.
//
// Replaces nn.Conv2d(3, pad=1) + LeakyReLU(0.1) (unet.py:29,59-63) and the fused
// avg_pool2d output (unet.py:46) of the level-0 convs (cout 32: UNetConvBlock of
// the first level, UNetUpBlock.conv_block of the last up level).
//
// Why (tools/clock_probe.py --kernel winoq): a level-0 conv has a K
// loop of 2-8 chunks, and a kind-3 workgroup spent only 36-69 % of its life in it
// -- 2-3.5 us waiting for chunk 0 to land and 2.5-4.4 us in the epilogue of an
// 8-21 us life.  Here a workgroup computes tiles bid, bid + G, ... (G = the grid,
// a few workgroups per CU) and stages the next tile's chunk 0 while its current
// tile's last chunk computes, so the chunk-0 latency hides behind that chunk and
// the epilogue:
//   * U straight from L2 into registers (buffer loads a chunk ahead; kind 6's
//     scheme), so LDS holds only 2 raw stages (2 x 680 records) and a separate
//     exchange area (2048 records): the next tile's DMA never meets the exchange;
//   * the epilogue's syncs are bare barriers (LDS only) and its stores buffer
//     stores with a fixed count per wave (an out-of-range offset drops a store),
//     so the next tile's chunk-0 wait is a counted vmcnt that skips them.
// cout <= 32 (one co block); epilogues LINEAR, LEAKY, LEAKY_POOL.
// Measured 20-33 % slower than kind 3 on every level-0 conv: built only
// into the lab library (`make lab`, RRIN_LAB).
#include "common.hpp"

#ifdef RRIN_LAB
#ifndef RRIN_WINOP_TILES
#define RRIN_WINOP_TILES 4  // tiles per workgroup (the grid is ntiles / this, rounded up)
#endif

namespace rrin {

typedef float pfloatx16 __attribute__((ext_vector_type(16)));
typedef float pfloatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int pu32x4 __attribute__((ext_vector_type(4)));

constexpr int kPCols = 34, kPRG = 10 * kPCols, kPRaw = 2 * kPRG;  // 680 raw records per stage
constexpr int kPU = 16 * 2 * 32;                                   // U records per chunk: [xi][half][co]
constexpr int kPX = 2048;                                          // exchange records
constexpr int kPBias = 2 * kPRaw + kPX;                            // record index of the 32 bias floats
static_assert((size_t)(kPBias * 16 + 128) == kWinoPLds, "LDS size");
static_assert(2 * kWinoPLds <= 160 * 1024, "two blocks per CU");

__device__ inline int wp_col(int col) { return (col & 1) * 17 + (col >> 1); }
__device__ inline void wp_dma16(__amdgpu_buffer_rsrc_t rs, uint4* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
}

template <int EPI>
__global__ __launch_bounds__(512, 4) void conv3x3_winop_kernel(ConvH8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int yw = wv & 3, pt = wv >> 2;
  const int G = gridDim.x;
  int bid;
  {  // XCD-aware bijective remap: an XCD's workgroups take consecutive first tiles
    const int q = G >> 3, r = G & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
  const int nch = a.nchunks;
  float* sbias = reinterpret_cast<float*>(smem4 + kPBias);
  if (tid < 32) sbias[tid] = a.bias[tid];  // visible after chunk 0's barrier

  // the lane id through an opaque move: values derived from it inside the loops are
  // recomputed where used instead of being hoisted into registers held across the
  // whole kernel (the 4-waves-per-SIMD budget is 128 VGPRs)
  auto lane_id = [&]() {
    int v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(tid));
    return v;
  };
  const bool tail_lane = tid < kPRaw - 512;  // second piece (waves 0-2)
  // a tile's origin: record (row y0 - 1, col x0 - 1) of group 0 of its image
  auto tile_src = [&](int t, int& y0) {
    const int x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    y0 = (t % a.tiles_y) * 8;
    const int img = t / a.tiles_y;
    return a.src_hi + (int64_t)img * a.src_img + (int64_t)y0 * a.src_wp + x0 + (kH8PadLeft - 1);
  };
  auto issue_raw = [&](const uint4* ts, int y0, int c, int stage) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(ts) - (int64_t)y0 * a.src_wp, 0, 0x7fffffff,
                                                      0x00020000);
    // rs starts at the tile column's top padding row: channel groups past cin read it (zeros)
    const unsigned rowoff = (unsigned)((int64_t)y0 * a.src_wp * 16);
    const int tl = lane_id();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      if (it == 0 || tail_lane) {
        // raw staging (kind 3's layout): record idx of the stage's 680, byte offsets from
        // the tile's origin (an image is < 2^32 bytes)
        const int idx = tl + 512 * it;
        const int g = idx >= kPRG ? 1 : 0;
        const int rem = idx - g * kPRG;
        const int r = rem / kPCols, pos = rem - r * kPCols;
        const int col = pos < 17 ? 2 * pos : 2 * (pos - 17) + 1;
        const int gg = 2 * c + g;
        const unsigned off = gg * 4 < a.cin
                                 ? rowoff + (unsigned)((((int64_t)(2 * c) + g) * a.src_gp + (int64_t)r * a.src_wp + col) * 16)
                                 : (unsigned)col * 16u;
        wp_dma16(rs, smem4 + stage * kPRaw + 512 * it + (tid & ~63), off);
      }
    }
  };
  // U record (xi = 4 yw + x, hh, co = j) of chunk c, straight into registers
  const auto urs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(a.w_hi), 0, 0x7fffffff, 0x00020000);
  auto load_u = [&](int c, int x) {
    const int tl = lane_id() & 63;  // (hh, j) = (tl >> 5, tl & 31)
    const unsigned uvoff = (unsigned)(((4 * yw) * 64 + tl) * 16);
    return __builtin_bit_cast(pfloatx4, __builtin_amdgcn_raw_buffer_load_b128(urs, uvoff + x * 1024, c * kPU * 16, 0));
  };

  const int ra = yw == 0 ? 0 : (yw == 2 ? 2 : 1);
  const int rb = yw == 0 ? 2 : (yw == 1 ? 2 : (yw == 2 ? 1 : 3));
  const float sg = yw == 1 ? 1.f : -1.f;
  const int oa = ra * kPCols, ob = rb * kPCols;

  pfloatx16 acc[4];
  pfloatx4 ur[4];  // U of the chunk being computed (point x reloaded after its MFMAs)
  // a chunk in raw stage s; U of chunk next_c loaded after each point when `more`
  auto chunk = [&](int s, bool more, int next_c) {
    const int tl = lane_id();
    const int lj = tl & 31, lhh = (tl >> 5) & 1, lpr = 2 * pt + (lj >> 4), ljx = (lj + 12 * (lj >> 4)) & 15;
    const uint4* rw = smem4 + s * kPRaw + lhh * kPRG + (2 * lpr) * kPCols;
    pfloatx4 t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pck = wp_col(2 * ljx + k);
      const pfloatx4 d0 = __builtin_bit_cast(pfloatx4, rw[oa + pck]);
      const pfloatx4 d1 = __builtin_bit_cast(pfloatx4, rw[ob + pck]);
#pragma unroll
      for (int e = 0; e < 4; ++e) t[k][e] = fmaf(sg, d1[e], d0[e]);
    }
    pfloatx4 v[4];
    v[0] = t[0] - t[2];
    v[1] = t[1] + t[2];
    v[2] = t[2] - t[1];
    v[3] = t[1] - t[3];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(ur[x][e], v[x][e], acc[x], 0, 0, 0);
      }
      if (more) ur[x] = load_u(next_c, x);
    }
  };
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  pfloatx4* X = reinterpret_cast<pfloatx4*>(smem4 + 2 * kPRaw);
  const int r = yw & 1, cc = yw >> 1;
  // fixed count of epilogue stores per wave (buffer stores, dropped when out of range)
  constexpr bool kPool = EPI == RRIN_EPI_LEAKY_POOL;

  int t = bid, y0;
  const uint4* ts = tile_src(t, y0);
  int g = 0;  // chunks computed by this workgroup: raw stage g & 1
  issue_raw(ts, y0, 0, 0);
#pragma unroll
  for (int x = 0; x < 4; ++x) ur[x] = load_u(0, x);
  bool first_tile = true;
  for (;;) {
    const int tn = t + G;
    const bool more_t = tn < ntiles;
    int ny0 = 0;
    const uint4* nts = more_t ? tile_src(tn, ny0) : ts;
    // zeroed per tile (0 + the first product: kind 3's first MFMA on a zero accumulator),
    // so the previous tile's accumulators are dead once its exchange has read them
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[x] = pfloatx16{};
    // chunk 0: its raw tile and U(0) were issued before the previous tile's epilogue
    // stores (4 per wave, 8 for the pooling waves): wait for all but those
    if (first_tile) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (kPool && yw == 0) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    first_tile = false;
    bar();  // chunk 0 landed everywhere; stage (g + 1) & 1 was last read in chunk g - 1
    if (nch > 1) {
      issue_raw(ts, y0, 1, (g + 1) & 1);
      chunk(g & 1, true, 1);
      ++g;
      for (int c = 1; c + 1 < nch; ++c, ++g) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
        issue_raw(ts, y0, c + 1, (g + 1) & 1);
        chunk(g & 1, true, c + 1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    // the last chunk: the next tile's chunk 0 goes to the free stage
    if (more_t) issue_raw(nts, ny0, 0, (g + 1) & 1);
    chunk(g & 1, false, 0);
    ++g;

    // ---- output transform (kind 3's order): exchange Q[c] of the four yw waves of a
    // patch-row pair through the exchange area, one column per pass
    int x0, yt0, img;
    {
      int tt = t;
      x0 = (tt % a.tiles_x) * 32;
      tt /= a.tiles_x;
      yt0 = (tt % a.tiles_y) * 8;
      img = tt / a.tiles_y;
    }
    const int el = lane_id() & 63, ej = el & 31;
    const int pr = 2 * pt + (ej >> 4), jx = (ej + 12 * (ej >> 4)) & 15;
    const int y = yt0 + 2 * pr + r, x = x0 + 2 * jx + cc;
    float yv[16];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        pfloatx4 q;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * k4 + e;
          const float m0 = acc[0][i], m1 = acc[1][i], m2 = acc[2][i], m3 = acc[3][i];
          q[e] = p == 0 ? (m0 + m1) + m2 : (m1 - m2) - m3;
        }
        X[((pt * 4 + yw) * 4 + k4) * 64 + lane] = q;
      }
      bar();
      if (cc == p) {
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const pfloatx4 q0 = X[((pt * 4 + 0) * 4 + k4) * 64 + lane];
          const pfloatx4 q1 = X[((pt * 4 + 1) * 4 + k4) * 64 + lane];
          const pfloatx4 q2 = X[((pt * 4 + 2) * 4 + k4) * 64 + lane];
          const pfloatx4 q3 = X[((pt * 4 + 3) * 4 + k4) * 64 + lane];
#pragma unroll
          for (int e = 0; e < 4; ++e) yv[4 * k4 + e] = r == 0 ? (q0[e] + q1[e]) + q2[e] : (q1[e] - q2[e]) - q3[e];
        }
      }
      bar();
    }
    // the next tile's U(0), issued after the raw DMA of its chunk 0 and before this tile's
    // stores (the counted wait above relies on that order); the accumulators are dead now
    if (more_t) {
#pragma unroll
      for (int xx = 0; xx < 4; ++xx) ur[xx] = load_u(0, xx);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep those loads ahead of the stores below
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(a.dst_hi + (int64_t)img * a.dst_img, 0, 0x7fffffff, 0x00020000);
    const bool in = y < a.h && x < a.w;
    // 32-bit byte offsets within the image (an image is < 2^32 bytes)
    const unsigned ehh = (unsigned)(el >> 5);
    const unsigned pix = (unsigned)(((y + 1) * a.dst_wp + x + kH8PadLeft) * 16);
    const unsigned gs = (unsigned)(a.dst_gp * 16);
    float vv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float tv = yv[i] + sbias[8 * (i >> 2) + 4 * (int)ehh + (i & 3)];
      if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
      vv[i] = tv;
    }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const bool ok = in && 8 * qq < a.cout;
      const pu32x4 v4 = {__float_as_uint(vv[4 * qq]), __float_as_uint(vv[4 * qq + 1]), __float_as_uint(vv[4 * qq + 2]),
                         __float_as_uint(vv[4 * qq + 3])};
      __builtin_amdgcn_raw_buffer_store_b128(v4, drs, ok ? (2 * qq + ehh) * gs + pix : 0x80000000u, 0, 0);
    }
    if constexpr (kPool) {
      // the patch's four outputs (yw = (r, c)) meet in the exchange area; wave yw 0 writes
      // avg = 0.25 ((Y00 + Y10) + (Y01 + Y11)), kind 3's order
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pfloatx4 q;
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = vv[4 * k + e];
        X[((pt * 4 + yw) * 4 + k) * 64 + lane] = q;
      }
      bar();
      if (yw == 0) {
        const int xp = x0 + 2 * jx, yp = yt0 + 2 * pr;
        const auto prs =
            __builtin_amdgcn_make_buffer_rsrc(a.pool_hi + (int64_t)img * a.pool_img, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const pfloatx4 y00 = X[((pt * 4 + 0) * 4 + qq) * 64 + lane];
          const pfloatx4 y10 = X[((pt * 4 + 1) * 4 + qq) * 64 + lane];
          const pfloatx4 y01 = X[((pt * 4 + 2) * 4 + qq) * 64 + lane];
          const pfloatx4 y11 = X[((pt * 4 + 3) * 4 + qq) * 64 + lane];
          const bool ok = 8 * qq < a.cout && yp < a.h && xp < a.w;
          float s4[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) s4[e] = 0.25f * ((y00[e] + y10[e]) + (y01[e] + y11[e]));
          const unsigned poff = (2 * qq + ehh) * (unsigned)(a.pool_gp * 16) +
                                (unsigned)(((yp / 2 + 1) * a.pool_wp + xp / 2 + kH8PadLeft) * 16);
          const pu32x4 v4 = {__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                             __float_as_uint(s4[3])};
          __builtin_amdgcn_raw_buffer_store_b128(v4, prs, ok ? poff : 0x80000000u, 0, 0);
        }
      }
      bar();  // the exchange area is rewritten by the next tile's epilogue
    }
    if (!more_t) break;
    t = tn;
    ts = nts;
    y0 = ny0;
  }
}

template <int EPI>
static int launch_winop_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_winop_kernel<EPI>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)kWinoPLds, st)) return e;
  const int64_t ntiles = (int64_t)a.tiles_x * a.tiles_y * a.n;
  const int64_t grid = (ntiles + RRIN_WINOP_TILES - 1) / RRIN_WINOP_TILES;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(512), kWinoPLds, st, a);
  return hip_code(hipGetLastError());
}

int launch_winop(const ConvH8Args& a, int epi, hipStream_t st) {
  if (a.co_blocks != 1) return RRIN_E_CONFIG;  // one co block (cout <= 32)
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_winop_k<RRIN_EPI_LINEAR>(a, st);
    case RRIN_EPI_LEAKY: return launch_winop_k<RRIN_EPI_LEAKY>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_winop_k<RRIN_EPI_LEAKY_POOL>(a, st);
  }
  return RRIN_E_CONFIG;
}

}  // namespace rrin
#endif  // RRIN_LAB
