// Exact-fp32 3x3 conv as Winograd F(2x2, 3x3) on fp32 records (R32) with the
// f32-input matrix cores (v_mfma_f32_32x32x2_f32).  Tile config kWinoCfg of
// the record-layout conv table (rrin_conv3x3_h8_fwd, precision F32R).
//
// Replaces the same reference ops as conv3x3_h8_kernel: nn.Conv2d(3, pad=1) +
// LeakyReLU(0.1) (unet.py:29,59-63), the fused avg_pool2d output (unet.py:46),
// the cat by channel offset (unet.py:93), and the sub-pixel form of Upsample +
// up conv (unet.py:77-78).
//
// Arithmetic: every operation is an IEEE fp32 operation -- no reduced-precision
// operand anywhere.  Per 2x2 output patch and input channel the 4x4 input window
// d becomes V = B^T d B (adds only), the weights U = G g G^T (host, in double,
// rounded once to fp32), and per transform point xi (16) the channel
// contraction M[xi] = sum_ci U[xi] V[xi] runs on the fp32 MFMA; the patch is
// Y = A^T M A (adds only).  16 multiplies per patch and channel pair instead of
// the direct form's 36: 2.25x fewer MFMA cycles for the same conv.
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   G   = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
//
// Block: 256 threads = 4 waves, tile = 32 output channels x 32 px x 8 rows =
// 64 patches (16 wide x 4 tall).  Wave (xh, ph) owns transform rows xi_y in
// {2xh, 2xh+1} (8 of the 16 points: 8 accumulators of 32 co x 32 patches, 128
// registers, so two blocks share a CU and cover each other's barriers) of the
// patch rows 2ph, 2ph+1.  K chunk = 8 channels (2 record groups): per point 4
// MFMAs (product e: lanes 0-31 channel e, lanes 32-63 channel 4+e).
// Each lane transforms exactly the B operands it feeds: the window rows of its
// patch (3 of 4: the two B^T rows of its xi_y pair), its 4 channels, straight
// from the LDS image of the raw input -- V never goes through LDS.
// Per chunk, double buffered in LDS (LDS-DMA, one chunk ahead):
//   raw input tile 2 groups x 10 rows x 34 cols (even columns, then odd, so
//                  the stride-2 window reads of 16 lanes are conflict-free)
//   U slab [xi][half][co] 16 x 2 x 32 records
// The output transform's two halves (xi_y 0-1, 2-3) meet through LDS: wave
// xh = 0 finishes output row 0 of each patch, xh = 1 row 1.
#include "common.hpp"

namespace rrin {

typedef float wfloatx16 __attribute__((ext_vector_type(16)));
typedef float wfloatx4 __attribute__((ext_vector_type(4)));
typedef float wfloatx2 __attribute__((ext_vector_type(2)));

constexpr int kWnRawCols = 34, kWnRawG = 10 * kWnRawCols, kWnRaw = 2 * kWnRawG, kWnRawStride = 704;
constexpr int kWnU = 16 * 2 * 32;  // records per U buffer: [xi][half][co]
static_assert(kWinoLds == (size_t)(2 * kWnRawStride + 2 * kWnU) * 16, "LDS size");
// LDS position of raw column col (0..33) within its row: even columns first
__device__ inline int wn_col(int col) { return (col & 1) * 17 + (col >> 1); }

// ABL: kernel-lab ablations only (built into librrin_lab.so under RRIN_LAB; the
// product library instantiates ABL = 0): 1 no weight DMA after chunk 0, 2 no raw
// DMA after chunk 0, 4 no MFMAs (operands kept live), 8 no transform arithmetic.
// PERS: persistent grid (2 blocks per CU); a block loops over the tiles bid,
// bid + grid, ... and stages chunk 0 of its next tile during the last chunk of the
// current one, so only its first tile waits for staging.  The output-transform
// exchange then uses the U buffer of the last chunk + its own 16 KB (kWinoPersLds).
template <int EPI, int ABL = 0, bool PERS = false>
__global__ __launch_bounds__(256, 2) void conv3x3_wino_kernel(ConvH8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  uint4* s_raw = smem4;                      // [2][kWnRawStride]: [group][row][wn_col]
  uint4* s_u = smem4 + 2 * kWnRawStride;     // [2][16][2][32]
  uint4* s_x = s_u + 2 * kWnU;               // PERS: [4 waves][4][64] exchange records

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int xh = wv & 1, ph = wv >> 1, j = lane & 31, hh = lane >> 5;
  int bid;
  {  // XCD-aware bijective remap (see conv_mfma.hip)
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
  const int nch = a.nchunks;

  // Tile t -> (channel block, column, row, image); staging bases of its raw input
  // rows y0-1..y0+8, cols x0-1..x0+32 and of its U slabs.
  struct Tile {
    int cob, x0, y0, img;
    const uint4* src;
    const uint4* wsrc;
  };
  auto tile_of = [&](int t) {
    Tile T;
    T.cob = t % a.co_blocks;
    t /= a.co_blocks;
    T.x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    T.y0 = (t % a.tiles_y) * 8;
    T.img = t / a.tiles_y;
    T.src = a.src_hi + (int64_t)T.img * a.src_img + (int64_t)T.y0 * a.src_wp + T.x0 + (kH8PadLeft - 1);
    T.wsrc = a.w_hi + (int64_t)T.cob * nch * kWnU + tid;
    return T;
  };

  // ---- staging.  Per thread and DMA piece (3): its group of the chunk, its offset
  // inside the group plane, and its column (groups past cin read the same column
  // of the zero top-padding row of group 0 instead: they meet zero weights).
  int p_g[3], p_off[3], p_col[3];
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const int idx = tid + 256 * it;
    const int g = idx >= kWnRawG ? 1 : 0;
    const int rem = idx - g * kWnRawG;
    const int r = rem / kWnRawCols, pos = rem - r * kWnRawCols;
    const int col = pos < 17 ? 2 * pos : 2 * (pos - 17) + 1;
    p_g[it] = g;
    p_off[it] = r * a.src_wp + col;
    p_col[it] = col;
  }
  auto issue_raw = [&](const Tile& T, int c, int buf) {
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      if (it < 2 || tid + 512 < kWnRaw) {
        const int gg = 2 * c + p_g[it];
        const int64_t off =
            gg * 4 < a.cin ? (int64_t)gg * a.src_gp + p_off[it] : (int64_t)p_col[it] - (int64_t)T.y0 * a.src_wp;
        dma16(T.src + off, s_raw + buf * kWnRawStride + 256 * it + (tid & ~63));
      }
    }
  };
  auto issue_u = [&](const Tile& T, int c, int buf) {
#pragma unroll
    for (int it = 0; it < 4; ++it)
      dma16(T.wsrc + (int64_t)c * kWnU + 256 * it, s_u + buf * kWnU + 256 * it + (tid & ~63));
  };

  // ---- per chunk: this lane's B operands V[xi][4hh + e][patch j] from its window:
  // B^T rows 2xh, 2xh+1 as t0 = d[ra] - d[rb], t1 = d[rc] + sgn d[rd] (no branch on xh),
  // then 8 points x 4 products
  wfloatx16 acc[8];
  // MFMA column j -> patch (row pr, column jx).  The second row's columns are
  // rotated by 12 so the window reads of the two rows (68 records apart) fall on
  // distinct banks in every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}).
  const int pr = 2 * ph + (j >> 4), jx = (j + 12 * (j >> 4)) & 15;
  const int ra = xh ? 2 : 0, rb = xh ? 1 : 2, rd = xh ? 3 : 2;  // rc = 1
  const float sgn = xh ? -1.f : 1.f;
  // One B^T row yl of this wave's pair (t = d[ra] - d[rb] or d[1] + sgn d[rd]) and
  // its 4 points' U operands, for chunk buffer b.
  auto transform = [&](int b, int yl, wfloatx4* u4, wfloatx4* v4) {
    const uint4* su = s_u + b * kWnU + (8 * xh + 4 * yl) * 64 + hh * 32 + j;
#pragma unroll
    for (int x = 0; x < 4; ++x) u4[x] = __builtin_bit_cast(wfloatx4, su[x * 64]);
    const uint4* rw = s_raw + b * kWnRawStride + hh * kWnRawG + (2 * pr) * kWnRawCols;
    wfloatx4 c4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pc = wn_col(2 * jx + k);
      const wfloatx4 d0 = __builtin_bit_cast(wfloatx4, rw[(yl ? 1 : ra) * kWnRawCols + pc]);
      const wfloatx4 d1 = __builtin_bit_cast(wfloatx4, rw[(yl ? rd : rb) * kWnRawCols + pc]);
      if constexpr ((ABL & 8) != 0) {
        c4[k] = d0;
      } else if (yl == 0) {
        c4[k] = d0 - d1;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) c4[k][e] = fmaf(sgn, d1[e], d0[e]);
      }
    }
    if constexpr ((ABL & 8) != 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) v4[x] = c4[x];
      return;
    }
    v4[0] = c4[0] - c4[2];
    v4[1] = c4[1] + c4[2];
    v4[2] = c4[2] - c4[1];
    v4[3] = c4[1] - c4[3];
  };
  auto mfmas = [&](int yl, const wfloatx4* u4, const wfloatx4* v4) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        if constexpr ((ABL & 4) != 0)
          asm volatile("" ::"v"(u4[x][e]), "v"(v4[x][e]));
        else
          acc[4 * yl + x] = __builtin_amdgcn_mfma_f32_32x32x2f32(u4[x][e], v4[x][e], acc[4 * yl + x], 0, 0, 0);
      }
  };
  auto compute = [&](int b) {
    wfloatx4 u0[4], v0[4], u1[4], v1[4];
    transform(b, 0, u0, v0);
    mfmas(0, u0, v0);
    transform(b, 1, u1, v1);
    mfmas(1, u1, v1);
  };

  Tile cur = tile_of(bid);
  int b0 = 0;  // buffer of the current tile's chunk 0
  issue_raw(cur, 0, 0);
  issue_u(cur, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int tile = bid;;) {
    const int next = PERS ? tile + (int)gridDim.x : ntiles;
    const bool has_next = next < ntiles;
    Tile nxt = cur;
    if (has_next) nxt = tile_of(next);
#pragma unroll
    for (int l = 0; l < 8; ++l)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[l][i] = 0.f;
    for (int c = 0; c < nch; ++c) {
      const int b = (b0 + c) & 1;
      // buffers b^1 were last read in the previous chunk, before the barrier that ended it
      if (c + 1 < nch) {
        if constexpr (!(ABL & 2)) issue_raw(cur, c + 1, b ^ 1);
        if constexpr (!(ABL & 1)) issue_u(cur, c + 1, b ^ 1);
      } else if (has_next) {  // PERS: the next tile's chunk 0
        issue_raw(nxt, 0, b ^ 1);
        issue_u(nxt, 0, b ^ 1);
      }
      compute(b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const int bl = (b0 + nch - 1) & 1;  // buffers of the last chunk: free now

    // ---- output transform: Q[yl][c] = sum_x M[xi_y][x] A[x][c] for this wave's xi rows,
    // then Y[0][c] = Q0 + Q1 + Q2 (wave xh 0), Y[1][c] = Q1 - Q2 - Q3 (wave xh 1)
    float q[2][2][16];
#pragma unroll
    for (int yl = 0; yl < 2; ++yl)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float m0 = acc[4 * yl][i], m1 = acc[4 * yl + 1][i], m2 = acc[4 * yl + 2][i], m3 = acc[4 * yl + 3][i];
        q[yl][0][i] = (m0 + m1) + m2;
        q[yl][1][i] = (m1 - m2) - m3;
      }
    // wave xh 0 hands its Q1 (yl 1) to its partner, wave xh 1 its Q2 (yl 0): records
    // k 0-3 / 4-7 in the two U buffers, or (PERS: the other buffers hold the next
    // tile's chunk 0) in the last chunk's U buffer and the exchange area
    wfloatx4* xlo = reinterpret_cast<wfloatx4*>(PERS ? s_u + bl * kWnU : s_u);
    wfloatx4* xhi = reinterpret_cast<wfloatx4*>(PERS ? s_x : s_u + kWnU);
    auto xslot = [&](int w, int k) { return (k < 4 ? xlo : xhi) + (w * 4 + (k & 3)) * 64 + lane; };
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      wfloatx4 g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int v = 4 * k + e, c = v >> 4, i = v & 15;
        g[e] = xh ? q[0][c][i] : q[1][c][i];
      }
      *xslot(wv, k) = g;
    }
    __syncthreads();
    float yv[2][16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const wfloatx4 pv = *xslot(wv ^ 1, k);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int v = 4 * k + e, c = v >> 4, i = v & 15;
        yv[c][i] = xh ? (pv[e] - q[0][c][i]) - q[1][c][i] : (q[0][c][i] + q[1][c][i]) + pv[e];
      }
    }

    // ---- epilogue: this lane's pixels (y, x0 + 2 jx + c), 16 channels 8 qq + 4 hh + e
    const int cob = cur.cob, x0 = cur.x0, img = cur.img;
    const int y = cur.y0 + 2 * pr + xh;
    uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
    auto store4 = [&](int64_t rec, const float* v) {
      dst[rec] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    };
    if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
      // rows co' = cob*32 + 8 qq + 4 hh + e: group cob of 8 real channels, phase qq = (py, px)
      const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
      if (cob * 32 < a.cout && y < a.h) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int x = x0 + 2 * jx + c;
          if (x >= a.w) continue;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int Y = 2 * y + (qq >> 1), X = 2 * x + (qq & 1);
            const int64_t ri = ring_index(Y, X, HH, WW);
            if (ri >= 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                a.edge[((int64_t)img * creal + cob * 8 + 4 * hh + e) * a.ring + ri] = yv[c][4 * qq + e];
            } else {
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = yv[c][4 * qq + e] + a.bias[cob * 32 + 8 * qq + 4 * hh + e];
              store4((int64_t)(2 * cob + hh) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + X + kH8PadLeft, v);
            }
          }
        }
      }
    } else {
      float v[2][16];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float tv = yv[c][i] + a.bias[cob * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
          if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
          v[c][i] = tv;
        }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int x = x0 + 2 * jx + c;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (cob * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
            const int64_t rec = (int64_t)(cob * 8 + 2 * qq + hh) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
            store4(rec, &v[c][4 * qq]);
            if constexpr (EPI == RRIN_EPI_LEAKY_REP) {
              // edge replicate into the padding ring (read only by a sub-pixel up conv)
              const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
              const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
              for (int dy = dy0; dy <= dy1; ++dy)
                for (int dx = dx0; dx <= dx1; ++dx)
                  if (dy | dx) store4(rec + (int64_t)dy * a.dst_wp + dx, &v[c][4 * qq]);
            }
          }
        }
      }
      if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
        // row 1 of each patch (wave xh 1) meets row 0 (wave xh 0) in LDS: one-tile grids
        // use the raw buffers (idle now), PERS the exchange records (the next tile's chunk
        // 0 is in the other raw buffer) once every wave has read them (barrier);
        // avg = 0.25 ((v00 + v10) + (v01 + v11))
        wfloatx4* xp = reinterpret_cast<wfloatx4*>(s_raw);
        auto pslot = [&](int k) { return PERS ? xslot(ph, k) : xp + (ph * 8 + k) * 64 + lane; };
        if constexpr (PERS) __syncthreads();
        if (xh) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            wfloatx4 g;
#pragma unroll
            for (int e = 0; e < 4; ++e) g[e] = v[(4 * k + e) >> 4][(4 * k + e) & 15];
            *pslot(k) = g;
          }
        }
        __syncthreads();
        if (!xh) {
          float v1[2][16];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const wfloatx4 g = *pslot(k);
#pragma unroll
            for (int e = 0; e < 4; ++e) v1[(4 * k + e) >> 4][(4 * k + e) & 15] = g[e];
          }
          const int x = x0 + 2 * jx;
          uint4* pdst = a.pool_hi + (int64_t)img * a.pool_img;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (cob * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
              float s4[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int i = 4 * qq + e;
                s4[e] = 0.25f * ((v[0][i] + v1[0][i]) + (v[1][i] + v1[1][i]));
              }
              const int64_t rec =
                  (int64_t)(cob * 8 + 2 * qq + hh) * a.pool_gp + (int64_t)(y / 2 + 1) * a.pool_wp + x / 2 + kH8PadLeft;
              pdst[rec] = make_uint4(__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                                     __float_as_uint(s4[3]));
            }
          }
        }
      }
    }
    if (!has_next) break;
    // the next tile's chunk 1 is staged into buffers bl (exchange records) at its start
    __syncthreads();
    tile = next;
    cur = nxt;
    b0 = bl ^ 1;
  }
}

constexpr size_t kWinoPersLds = kWinoLds + (size_t)4 * 4 * 64 * 16;  // + exchange records

static int wino_num_cus() {
  static std::atomic<int> n[kMaxDevices] = {};
  const int dev = current_device();
  int v = n[dev].load(std::memory_order_relaxed);
  if (!v) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1) v = 256;
    n[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int EPI, int ABL = 0, bool PERS = false>
static int launch_wino_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_wino_kernel<EPI, ABL, PERS>;
  constexpr size_t lds = PERS ? kWinoPersLds : kWinoLds;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)lds)) return e;
  int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
#ifndef RRIN_WINO_PERS_BPC  // persistent blocks per CU (A/B builds)
#define RRIN_WINO_PERS_BPC 2
#endif
  const int64_t slots = (int64_t)RRIN_WINO_PERS_BPC * wino_num_cus();
  if (PERS && grid > slots) grid = slots;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  return hip_code(hipGetLastError());
}

#ifdef RRIN_LAB
// kernel lab (librrin_lab.so only): the LEAKY conv with ablation bits; bit 256 = PERS
int launch_wino_lab(const ConvH8Args& a, int abl, hipStream_t st) {
  switch (abl) {
    case 0: return launch_wino_k<RRIN_EPI_LEAKY, 0>(a, st);
    case 1: return launch_wino_k<RRIN_EPI_LEAKY, 1>(a, st);
    case 2: return launch_wino_k<RRIN_EPI_LEAKY, 2>(a, st);
    case 3: return launch_wino_k<RRIN_EPI_LEAKY, 3>(a, st);
    case 4: return launch_wino_k<RRIN_EPI_LEAKY, 4>(a, st);
    case 8: return launch_wino_k<RRIN_EPI_LEAKY, 8>(a, st);
    case 11: return launch_wino_k<RRIN_EPI_LEAKY, 11>(a, st);
    case 15: return launch_wino_k<RRIN_EPI_LEAKY, 15>(a, st);
    case 256: return launch_wino_k<RRIN_EPI_LEAKY, 0, true>(a, st);
    case 256 + 3: return launch_wino_k<RRIN_EPI_LEAKY, 3, true>(a, st);
    case 256 + 4: return launch_wino_k<RRIN_EPI_LEAKY, 4, true>(a, st);
  }
  return RRIN_E_CONFIG;
}
#endif

// Persistent grid (PERS) only in A/B builds (-DRRIN_WINO_PERS_MIN=k: from k tiles per
// block slot).  Alone it is faster (kernel lab, profiles/r02/wino_pers: full-resolution
// convs 2-10 %, level 1 2-3 %; 720p x 1 bench +1.2 %), but the default 2-stream
// forward loses 4 % (125.1 -> 120.3 pairs/s): a persistent grid holds every block
// slot for the whole launch, so the other stream's kernels no longer fill the
// slots one-tile blocks free as they finish.
#ifndef RRIN_WINO_PERS_MIN
#define RRIN_WINO_PERS_MIN 0
#endif
template <int EPI>
static int launch_wino_e(const ConvH8Args& a, hipStream_t st) {
  if constexpr (RRIN_WINO_PERS_MIN > 0) {
    const int64_t ntiles = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
    if (ntiles >= (int64_t)RRIN_WINO_PERS_MIN * RRIN_WINO_PERS_BPC * wino_num_cus())
      return launch_wino_k<EPI, 0, true>(a, st);
  }
  return launch_wino_k<EPI>(a, st);
}

int launch_wino(const ConvH8Args& a, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_wino_e<RRIN_EPI_LINEAR>(a, st);
    case RRIN_EPI_LEAKY: return launch_wino_e<RRIN_EPI_LEAKY>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_wino_e<RRIN_EPI_LEAKY_POOL>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_wino_e<RRIN_EPI_LEAKY_REP>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_wino_e<RRIN_EPI_SUBPIXEL>(a, st);
  }
  return RRIN_E_ARG;
}

}  // namespace rrin

using namespace rrin;

extern "C" int64_t rrin_pack_conv3x3_wino_floats(int32_t cout, int32_t cin) {
  if (cout < 1 || cin < 1) return RRIN_E_ARG;
  const int64_t cob = (cout + 31) / 32, nch = (cin + 7) / 8;
  return cob * nch * kWnU * 4;
}

extern "C" int rrin_pack_conv3x3_wino(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                                      float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
  const int cob_n = (cout + 31) / 32, nch = (cin + 7) / 8;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 16; ++xi)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < 32; ++col)
            for (int e = 0; e < 4; ++e) {
              const int co = cob * 32 + col, ch = c * 8 + hh * 4 + e;
              double u = 0.0;
              if (co < cout && ch < cin) {
                const float* g = w + ((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9;
                for (int ky = 0; ky < 3; ++ky)
                  for (int kx = 0; kx < 3; ++kx) u += G[xi >> 2][ky] * G[xi & 3][kx] * (double)g[ky * 3 + kx];
              }
              wpack[o++] = (float)u;
            }
  for (int co = 0; co < cob_n * 32; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}
