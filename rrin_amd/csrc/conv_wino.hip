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
// product library instantiates ABL = 0): 1 no weight DMA after chunk 1, 2 no raw
// DMA after chunk 1, 4 no MFMAs (operands kept live), 8 no transform arithmetic.
//
// Main loop: a register pipeline over half-chunks (half = one B^T row yl of the
// wave's pair = 16 MFMAs, point-major: the 4 products of point x back to back on
// accumulator 4 yl + x).  While the MFMAs of half H issue, the window reads of half
// H + 1 are in flight, and once point x's 4 MFMAs have issued its U / B registers
// take point x of half H + 1 (U read from LDS, B transformed in the MFMA shadows):
// no MFMA waits on an LDS round trip, and one operand set is live.  The chunk's
// barrier sits at the start of its second half: every read of the chunk's buffers
// has been consumed by then, so right after it those buffers take chunk c + 2's
// LDS-DMA and the reads of chunk c + 1 start.
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(256, 2) void conv3x3_wino_kernel(ConvH8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  uint4* s_raw = smem4;                      // [2][kWnRawStride]: [group][row][wn_col]
  uint4* s_u = smem4 + 2 * kWnRawStride;     // [2][16][2][32]

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

  // tile -> (channel block, column, row, image); staging bases of its raw input
  // rows y0-1..y0+8, cols x0-1..x0+32 and of its U slabs
  struct Tile {
    int cob, x0, y0, img;
  } cur;
  {
    int t = bid;
    cur.cob = t % a.co_blocks;
    t /= a.co_blocks;
    cur.x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    cur.y0 = (t % a.tiles_y) * 8;
    cur.img = t / a.tiles_y;
  }
  const uint4* tsrc = a.src_hi + (int64_t)cur.img * a.src_img + (int64_t)cur.y0 * a.src_wp + cur.x0 + (kH8PadLeft - 1);
  const uint4* wsrc = a.w_hi + (int64_t)cur.cob * nch * kWnU + tid;

  // ---- staging.  Per thread and DMA piece (3): its group of the chunk, its offset
  // inside the group plane (groups past cin read the same column of the zero
  // top-padding row of group 0 instead: they meet zero weights).
  int64_t p_off[3];
  int p_g[3], p_zero[3];
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const int idx = tid + 256 * it;
    const int g = idx >= kWnRawG ? 1 : 0;
    const int rem = idx - g * kWnRawG;
    const int r = rem / kWnRawCols, pos = rem - r * kWnRawCols;
    const int col = pos < 17 ? 2 * pos : 2 * (pos - 17) + 1;
    p_g[it] = g;
    p_off[it] = (int64_t)g * a.src_gp + r * a.src_wp + col;
    p_zero[it] = col - cur.y0 * a.src_wp;
  }
  auto issue_raw = [&](int c, int buf) {
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      if (it < 2 || tid + 512 < kWnRaw) {
        const int gg = 2 * c + p_g[it];
        const int64_t off = gg * 4 < a.cin ? (int64_t)(2 * c) * a.src_gp + p_off[it] : (int64_t)p_zero[it];
        dma16(tsrc + off, s_raw + buf * kWnRawStride + 256 * it + (tid & ~63));
      }
    }
  };
  auto issue_u = [&](int c, int buf) {
#pragma unroll
    for (int it = 0; it < 4; ++it) dma16(wsrc + (int64_t)c * kWnU + 256 * it, s_u + buf * kWnU + 256 * it + (tid & ~63));
  };
  auto issue = [&](int c, int buf) {
    if (!(ABL & 2) || c < 2) issue_raw(c, buf);
    if (!(ABL & 1) || c < 2) issue_u(c, buf);
  };

  // MFMA column j -> patch (row pr, column jx).  The second row's columns are
  // rotated by 12 so the window reads of the two rows (68 records apart) fall on
  // distinct banks in every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}).
  const int pr = 2 * ph + (j >> 4), jx = (j + 12 * (j >> 4)) & 15;
  const int ra = xh ? 2 : 0, rb = xh ? 1 : 2, rd = xh ? 3 : 2;  // rc = 1
  const float sgn = xh ? -1.f : 1.f;
  // LDS addresses (records) of this lane's operands in buffer 0: U of point
  // (8 xh + 4 yl + x) at su0 + yl * 256 + x * 64; window records at rw0 + row * 34 + pc[k]
  const int su0 = 2 * kWnRawStride + (8 * xh) * 64 + hh * 32 + j;
  const int rw0 = hh * kWnRawG + (2 * pr) * kWnRawCols;
  int pc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pc[k] = wn_col(2 * jx + k);
  const int r0a = (ra)*kWnRawCols, r0b = (rb)*kWnRawCols, r1a = kWnRawCols, r1b = (rd)*kWnRawCols;

  wfloatx16 acc[8];
  wfloatx4 u[4], v[4];  // operands of the half being issued; point x recycled after its MFMAs
  // U record of point (8 xh + 4 yl + x) of the chunk in buffer b
  auto read_u = [&](int b, int yl, int x) {
    return __builtin_bit_cast(wfloatx4, smem4[su0 + b * kWnU + yl * 256 + x * 64]);
  };
  // the 8 window records of B^T row yl (rows o0 / o1, 4 columns)
  auto read_raw = [&](int b, int yl, wfloatx4* d) {
    const uint4* rw = s_raw + b * kWnRawStride + rw0;
    const int o0 = yl ? r1a : r0a, o1 = yl ? r1b : r0b;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[2 * k] = __builtin_bit_cast(wfloatx4, rw[o0 + pc[k]]);
      d[2 * k + 1] = __builtin_bit_cast(wfloatx4, rw[o1 + pc[k]]);
    }
  };
  // column k of B^T row yl: t = d[ra] - d[rb] (yl 0) or d[1] + sgn d[rd] (yl 1)
  auto row_t = [&](int yl, const wfloatx4* d, int k) {
    if constexpr ((ABL & 8) != 0) return d[2 * k];
    wfloatx4 t;
    if (yl == 0) {
      t = d[2 * k] - d[2 * k + 1];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = fmaf(sgn, d[2 * k + 1][e], d[2 * k][e]);
    }
    return t;
  };
  // the 4 MFMAs of point x of half yl (FIRST: chunk 0 starts from zero)
  auto mfma_point = [&](int yl, int x, bool first) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr ((ABL & 4) != 0) {
        asm volatile("" ::"v"(u[x][e]), "v"(v[x][e]));
      } else {
        const wfloatx16 c = (first && e == 0) ? wfloatx16{} : acc[4 * yl + x];
        acc[4 * yl + x] = __builtin_amdgcn_mfma_f32_32x32x2f32(u[x][e], v[x][e], c, 0, 0, 0);
      }
    }
  };
  // one half: MFMAs of half yl (operands in u / v) while half (bn, yn) -- the next
  // one -- is read from buffer bn and transformed into u / v point by point
  // hard scheduling fence (RRIN_WINO_FENCE, default on): keeps each stage's
  // instructions between its fences, so the reads stay ahead of the MFMAs
#ifndef RRIN_WINO_FENCE
#define RRIN_WINO_FENCE 1
#endif
#ifndef RRIN_WINO_SGB
#define RRIN_WINO_SGB 0
#endif
  auto fence = [&]() {
    if constexpr (RRIN_WINO_FENCE) __builtin_amdgcn_sched_barrier(0);
  };
  auto half = [&](int yl, int bn, int yn, bool first) {
    wfloatx4 d[8], t[4];
    read_raw(bn, yn, d);
    fence();
    mfma_point(yl, 0, first);
    u[0] = read_u(bn, yn, 0);
    fence();
    t[0] = row_t(yn, d, 0);
    t[2] = row_t(yn, d, 2);
    mfma_point(yl, 1, first);
    v[0] = (ABL & 8) ? t[0] : t[0] - t[2];
    u[1] = read_u(bn, yn, 1);
    fence();
    t[1] = row_t(yn, d, 1);
    mfma_point(yl, 2, first);
    v[1] = (ABL & 8) ? t[1] : t[1] + t[2];
    u[2] = read_u(bn, yn, 2);
    fence();
    t[3] = row_t(yn, d, 3);
    mfma_point(yl, 3, first);
    v[2] = (ABL & 8) ? t[2] : t[2] - t[1];
    v[3] = (ABL & 8) ? t[3] : t[1] - t[3];
    u[3] = read_u(bn, yn, 3);
    fence();
#if RRIN_WINO_SGB
    // pin the order: window reads, point 0, then one MFMA per 2-3 VALU
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#endif
  };

  // ---- prologue: chunk 0 staged, its first half's operands in u / v; chunk 1 in flight
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nch > 1) issue(1, 1);
  {
    wfloatx4 d[8], t[4];
    read_raw(0, 0, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = row_t(0, d, k);
    v[0] = (ABL & 8) ? t[0] : t[0] - t[2];
    v[1] = (ABL & 8) ? t[1] : t[1] + t[2];
    v[2] = (ABL & 8) ? t[2] : t[2] - t[1];
    v[3] = (ABL & 8) ? t[3] : t[1] - t[3];
#pragma unroll
    for (int x = 0; x < 4; ++x) u[x] = read_u(0, 0, x);
  }
  half(0, 0, 1, true);  // half (0, 0); reads of half (0, 1)
  // step c: half (c, 1) and half (c + 1, 0), the barrier at its top: chunk c + 1
  // landed everywhere and every read of chunk c's buffers (b) was consumed before
  // it, so b takes chunk c + 2's DMA.  No LDS read is pending across the barrier.
  auto step = [&](int c, bool first) {
    const int b = c & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 2 < nch) issue(c + 2, b);
    half(1, b ^ 1, 0, first);   // half (c, 1); reads of half (c + 1, 0)
    half(0, b ^ 1, 1, false);   // half (c + 1, 0); reads of half (c + 1, 1)
  };
  if (nch > 1) step(0, true);
  for (int c = 1; c + 1 < nch; ++c) step(c, false);
  // the last chunk's second half (its "next half" reads fetch stale records)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  half(1, ((nch - 1) & 1) ^ 1, 0, nch == 1);
  // those reads complete before the epilogue reuses the LDS
  __syncthreads();

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
    // k 0-3 / 4-7 in the two U buffers (no DMA in flight and every read of them
    // consumed since the last chunk's barrier)
    wfloatx4* xlo = reinterpret_cast<wfloatx4*>(s_u);
    wfloatx4* xhi = reinterpret_cast<wfloatx4*>(s_u + kWnU);
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
        // row 1 of each patch (wave xh 1) meets row 0 (wave xh 0) in LDS, in the raw
        // buffers (idle now); avg = 0.25 ((v00 + v10) + (v01 + v11))
        wfloatx4* xp = reinterpret_cast<wfloatx4*>(s_raw);
        auto pslot = [&](int k) { return xp + (ph * 8 + k) * 64 + lane; };
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
}

template <int EPI, int ABL = 0>
static int launch_wino_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_wino_kernel<EPI, ABL>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)kWinoLds, st)) return e;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), kWinoLds, st, a);
  return hip_code(hipGetLastError());
}


int launch_wino(const ConvH8Args& a, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_wino_k<RRIN_EPI_LINEAR>(a, st);
    case RRIN_EPI_LEAKY: return launch_wino_k<RRIN_EPI_LEAKY>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_wino_k<RRIN_EPI_LEAKY_POOL>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_wino_k<RRIN_EPI_LEAKY_REP>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_wino_k<RRIN_EPI_SUBPIXEL>(a, st);
  }
  return RRIN_E_ARG;
}




// ============================================================================
// 4-waves-per-SIMD tile (config kWinoQCfg): the 32-channel tile of cfg 18 (same
// packing, staging and arithmetic order: bitwise equal outputs) run by 8 waves
// of 4 accumulators each -- wave (yw, pt) owns B^T row yw (points 4 yw .. +3)
// of patch rows 2 pt, 2 pt + 1 -- at <= 128 VGPRs, so two blocks give every
// SIMD four waves: more independent waves to keep the matrix pipe fed while
// others wait on LDS, barriers or their transform, instead of a deeper
// per-wave pipeline.  The output transform meets through LDS as in cfg 19.
// ============================================================================
// RRIN_WINOQ_EPIWAIT 1: a compiler-visible vmcnt(0) after the main loop, before the
// epilogue's bias loads (0: the A/B build without it; profiles/r04/winoq_epiwait/)
#ifndef RRIN_WINOQ_EPIWAIT
#define RRIN_WINOQ_EPIWAIT 1
#endif
// RRIN_WINOQ_RU (A/B): the U operands straight from L2 into registers (buffer loads a
// chunk ahead, as conv_winoc.hip) instead of LDS-DMA + LDS reads (2-stage loop only)
#ifndef RRIN_WINOQ_RU
#define RRIN_WINOQ_RU 0
#endif
// Diagnostic build only (tools/clock_probe.py --kernel winoq): per-workgroup s_memtime
// stamps after chunk 0 landed, at the end of the main loop and at the end, and the
// s_memrealtime span and start
#ifndef RRIN_WINOQ_CLOCK
#define RRIN_WINOQ_CLOCK 0
#endif
#ifndef RRIN_WINOQ_STAGES
#define RRIN_WINOQ_STAGES 2
#endif
#ifndef RRIN_WINOQ_ORDER
#define RRIN_WINOQ_ORDER 0  // A/B builds only: tile order of the workgroup index
#endif
#ifndef RRIN_WINOQ_AGPR
#define RRIN_WINOQ_AGPR 0
#endif
#ifndef RRIN_WINOQ_PRIO
#define RRIN_WINOQ_PRIO 0  // A/B builds only: 1 s_setprio around each MFMA cluster, 2 static for waves 4-7
#endif
constexpr int kWqStages = RRIN_WINOQ_STAGES;
#if RRIN_WINOQ_CLOCK
constexpr int kQClkSlots = 1 << 16;
__device__ unsigned long long g_winoq_clk[kQClkSlots * 6];
#endif
constexpr int kWqStage = kWnRaw + kWnU;  // records per stage of the 8-wave tile (raw 680 + U 1024)
static_assert(kWinoQLds >= (size_t)kWqStages * kWqStage * 16, "LDS size");
static_assert(2 * kWinoQLds <= 160 * 1024, "two blocks per CU");

// ABL (lab builds only, librrin_lab.so): 1 no U DMA after chunk 0, 2 no raw DMA
// after chunk 0, 4 no MFMAs, 8 no transform arithmetic, 16 no window reads after
// chunk 0 (registers reused), 32 no U reads after chunk 0, 64 no epilogue stores
// PT: patch-row pairs per tile -- 2: 8 waves, TH 8 (cfg 20); 1: 4 waves, TH 4
// (cfg 21, twice the tiles for the few-tile deep levels of small workloads).
// ---- sub-pixel ring fold (RF) ---------------------------------------------------
// A sub-pixel up conv computes conv3x3(upsample_x2(x)) from phase weights over the
// edge-replicated low-res x; on the 1-pixel ring of the 2h x 2w output the true conv
// reads zero padding where the phase form read the clamped upsample, so the ring
// pixels take  y = (phase value - corr) + bias  with corr = sum over ci of the
// out-of-image taps w[c][ci][ky][kx] * up(ci, clamp(Y + ky - 1), clamp(X + kx - 1))
// (the arithmetic of edge_fix_h8_kernel, conv_f16.hip, which runs as a separate
// launch for the other configs).  Ring segment seg of (image, co block): top / bottom
// row under tile column tx (seg tx / tiles_x + tx: X in [64 tx, 64 tx + 64)), left /
// right column beside tile row ty (2 tiles_x + ty / 2 tiles_x + tiles_y + ty:
// Y in [16 ty, 16 ty + 16) within [1, H - 2]); 8 real channels (the co block).
struct RingSeg {
  int line, idx, np;  // line 0 top 1 bottom 2 left 3 right; tile column / row; pixels (64 / 16)
  int Y0, X0;         // first pixel
  int lo, hi;         // valid pixel positions [lo, hi) along the line
};
__device__ inline RingSeg ring_seg(const ConvH8Args& a, int seg) {
  RingSeg r;
  const int H = 2 * a.h, W = 2 * a.w;
  if (seg < 2 * a.tiles_x) {
    r.line = seg < a.tiles_x ? 0 : 1;
    r.idx = seg - r.line * a.tiles_x;
    r.np = 64;
    r.X0 = 64 * r.idx;
    r.Y0 = r.line == 0 ? 0 : H - 1;
    r.lo = 0;
    r.hi = min(64, W - r.X0);
  } else {
    const int t = seg - 2 * a.tiles_x;
    r.line = t < a.tiles_y ? 2 : 3;
    r.idx = t - (r.line - 2) * a.tiles_y;
    r.np = 16;
    r.Y0 = 16 * r.idx;
    r.X0 = r.line == 2 ? 0 : W - 1;
    r.lo = max(0, 1 - r.Y0);
    r.hi = max(r.lo, min(16, H - 1 - r.Y0));
  }
  return r;
}
// bilinear x2 upsample (align_corners = False, edge clamp) of channel ci of image img
// at output pixel (Y, X), in upsample_bilinear2d's order (edge_fix_h8_kernel's Up8)
__device__ inline float ring_up(const ConvH8Args& a, int img, int ci, int Y, int X) {
  int ra, rb, ca, cb;
  float wa, wc;
  if (Y & 1) { ra = Y >> 1; rb = min(ra + 1, a.h - 1); wa = 0.75f; }
  else { rb = Y >> 1; ra = max(rb - 1, 0); wa = 0.25f; }
  if (X & 1) { ca = X >> 1; cb = min(ca + 1, a.w - 1); wc = 0.75f; }
  else { cb = X >> 1; ca = max(cb - 1, 0); wc = 0.25f; }
  const float* src = reinterpret_cast<const float*>(a.src_hi + (int64_t)img * a.src_img + (int64_t)(ci >> 2) * a.src_gp +
                                                    kH8PadLeft) + (ci & 3);
  const float v0 = src[((int64_t)(ra + 1) * a.src_wp + ca) * 4], v1 = src[((int64_t)(ra + 1) * a.src_wp + cb) * 4];
  const float v2 = src[((int64_t)(rb + 1) * a.src_wp + ca) * 4], v3 = src[((int64_t)(rb + 1) * a.src_wp + cb) * 4];
  const float wb = 1.0f - wa, wd = 1.0f - wc;
  const float top = wc * v0 + wd * v1;
  const float bot = wc * v2 + wd * v3;
  return wa * top + wb * bot;
}
// segment (img, cob, seg) done by both of its writers: the later one writes its ring
// pixels, (phase value - corr) + bias, from the edge and corr scratch (after the
// caller's agent-scope acquire)
__device__ inline void ring_combine(const ConvH8Args& a, int img, int cob, int seg, int tid) {
  const RingSeg r = ring_seg(a, seg);
  const int p = tid & (r.np - 1), c = tid / r.np;
  if (c >= 8 || p < r.lo || p >= r.hi) return;
  const int H = 2 * a.h, W = 2 * a.w, creal = a.cout >> 2;
  const int Y = r.line < 2 ? r.Y0 : r.Y0 + p, X = r.line < 2 ? r.X0 + p : r.X0;
  const int ch = cob * 8 + c;
  // sc1 loads (write-through stores of other workgroups, possibly on other XCDs)
  const auto er = __builtin_amdgcn_make_buffer_rsrc(a.edge, 0, 0x7fffffff, 0x00020000);
  const float e = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
      er, (int)((((int64_t)img * creal + ch) * a.ring + ring_index(Y, X, H, W)) * 4), 0, 16));
  float* slab = a.corr + ((int64_t)(img * a.co_blocks + cob) * a.nseg + seg) * 512;
  const auto cr = __builtin_amdgcn_make_buffer_rsrc(slab, 0, 512 * 4, 0x00020000);
  const float corr = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(cr, (c * r.np + p) * 4, 0, 16));
  float* dst = reinterpret_cast<float*>(a.dst_hi);
  dst[(((int64_t)img * a.dst_img + (int64_t)(ch >> 2) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + X + kH8PadLeft) << 2) +
      (ch & 3)] = (e - corr) + a.bias_raw[ch];
}
// one ticket of segment (img, cob, seg) by lane 0 (after every wave drained its
// write-through stores and the barrier); returns on every thread whether this
// workgroup was the segment's second writer (then after an agent-scope acquire)
__device__ inline bool ring_ticket(const ConvH8Args& a, int img, int cob, int seg, int tid, int* s_flag) {
  if (tid == 0) {
    int* cnt = a.rcnt + (img * a.co_blocks + cob) * a.nseg + seg;
    const int last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    *s_flag = last;
  }
  __syncthreads();
  const bool last = *s_flag != 0;
  __syncthreads();  // s_flag reusable
  // every load of the handed-off values is an sc1 load (ring_combine): no agent-scope
  // acquire (it would drop this CU's cached lines), only the compiler-ordering fence
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return last;
}
// correction workgroup rb (< n * co_blocks * nseg; 512 threads): corr of its segment,
// 64 input channels per LDS stage (the segment's upsampled line +-1 and the two corner
// values, the 9 taps x 8 channels of weights: 36 KB), so a stage is one round of loads
__device__ inline void ring_block(const ConvH8Args& a, int rb, float* sm) {
  const int tid = threadIdx.x;
  const int seg = rb % a.nseg, t = rb / a.nseg, cob = t % a.co_blocks, img = t / a.co_blocks;
  const RingSeg r = ring_seg(a, seg);
  if (r.lo >= r.hi) return;  // an empty column segment (its conv tile does not count it either)
  const int H = 2 * a.h, W = 2 * a.w, creal = a.cout >> 2;
  const bool row = r.line < 2;
  const int nl = r.np + 2;           // staged line: positions -1 .. np
  constexpr int RC = 64;             // input channels per LDS stage (one load round per stage)
  float* s_l = sm;                   // [RC][nl]
  float* s_e = sm + RC * 66;         // [RC][2] corner extras (row lines)
  float* s_w = s_e + RC * 2;         // [RC ci][9 taps][8 c]
  const int p = tid & (r.np - 1), c = tid / r.np;
  const bool act = c < 8 && p >= r.lo && p < r.hi;
  const int X = row ? r.X0 + p : r.X0;
  // extras: the second row in (top: 1, bottom: H - 2) at the corner columns
  const int Ye = r.line == 0 ? min(1, H - 1) : max(H - 2, 0);
  float acc = 0.f;
  for (int c0 = 0; c0 < a.cin; c0 += RC) {
    const int nc = min(RC, a.cin - c0);
    for (int i = tid; i < nc * nl; i += 512) {
      const int ci = i / nl, j = i - ci * nl;
      const int Yv = row ? r.Y0 : min(max(r.Y0 - 1 + j, 0), H - 1);
      const int Xv = row ? min(max(r.X0 - 1 + j, 0), W - 1) : r.X0;
      s_l[ci * nl + j] = ring_up(a, img, c0 + ci, Yv, Xv);
    }
    if (row && tid < 2 * nc) s_e[tid] = ring_up(a, img, c0 + (tid >> 1), Ye, (tid & 1) ? W - 1 : 0);
    for (int i = tid; i < nc * 72; i += 512) {
      const int ci = i / 72, tap = (i / 8) % 9, cc = i & 7;
      s_w[i] = cob * 8 + cc < creal ? a.wedge[((int64_t)(c0 + ci) * 9 + tap) * creal + cob * 8 + cc] : 0.f;
    }
    __syncthreads();
    if (act) {
      for (int ci = 0; ci < nc; ++ci) {
        const float* l = s_l + ci * nl;
        const float* w = s_w + ci * 72 + c;
        if (r.line == 0 || r.line == 1) {  // the outside kernel row ky (0 top, 2 bottom), then the corners
          const int ky = r.line == 0 ? 0 : 2;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) acc = fmaf(w[(ky * 3 + kx) * 8], l[p + kx], acc);
          if (X == 0) {
            acc = fmaf(w[((r.line == 0 ? 1 : 0) * 3) * 8], r.line == 0 ? l[p] : s_e[ci * 2], acc);
            acc = fmaf(w[((r.line == 0 ? 2 : 1) * 3) * 8], r.line == 0 ? s_e[ci * 2] : l[p], acc);
          }
          if (X == W - 1) {
            acc = fmaf(w[((r.line == 0 ? 1 : 0) * 3 + 2) * 8], r.line == 0 ? l[p + 2] : s_e[ci * 2 + 1], acc);
            acc = fmaf(w[((r.line == 0 ? 2 : 1) * 3 + 2) * 8], r.line == 0 ? s_e[ci * 2 + 1] : l[p + 2], acc);
          }
        } else {  // the outside kernel column kx (0 left, 2 right)
          const int kx = r.line == 2 ? 0 : 2;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) acc = fmaf(w[(ky * 3 + kx) * 8], l[p + ky], acc);
        }
      }
    }
    __syncthreads();
  }
  if (act) {
    float* slab = a.corr + ((int64_t)(img * a.co_blocks + cob) * a.nseg + seg) * 512;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, 512 * 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc), rsrc, (c * r.np + p) * 4, 0, 16 /* sc1 */);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring_ticket(a, img, cob, seg, tid, reinterpret_cast<int*>(sm + 9216))) ring_combine(a, img, cob, seg, tid);
}

//
// SK (split-K, a.ksplit > 1): the grid has a.ksplit blocks per tile, slice ks running
// chunks [ks * a.kper, ..).  After its output transform a slice stores its pre-bias
// outputs (16 floats per lane) to a.part and counts itself in a.cnt[tile]
// (agent-scope release / acquire: the slices may run on different XCDs); the slice that
// counts last reads the tile's slices back, sums them in slice order (so the result
// does not depend on which slice finished last), resets the counter and runs the
// epilogue.  A different association of the K sum than one slice (not bitwise equal to
// cfg 20), fixed per conv: batch and per-sample outputs stay bitwise equal.
//
// RF (EPI_SUBPIXEL, PT 2, no split): the ring fold -- the first a.nring workgroups of the
// grid are ring correction blocks (ring_block), the rest the conv tiles; a tile on the
// image border stores its ring values write-through and counts itself in the ticket of
// each ring segment it covers (ring_combine by the later writer).
template <int EPI, int ABL = 0, int PT = 2, int SK = 0, int RF = 0>
__global__ __launch_bounds__(256 * PT, 2) void conv3x3_winoq_kernel(ConvH8Args a) {
  static_assert(!RF || (EPI == RRIN_EPI_SUBPIXEL && PT == 2 && !SK), "ring fold: 8-wave sub-pixel conv");
  constexpr int NT = 256 * PT, TH = 4 * PT;
  constexpr int RG = (TH + 2) * kWnRawCols, RAW = 2 * RG, STAGE = RAW + kWnU;
  static_assert(RAW > NT && RAW <= 2 * NT && kWnU % NT == 0, "two raw pieces, whole U pieces");
  constexpr int NS = PT == 2 ? kWqStages : 2;  // the 3-stage A/B ring is built for the 8-wave tile
  constexpr int UP = kWnU / NT;  // U pieces per thread
  constexpr bool RU = RRIN_WINOQ_RU != 0 && NS == 2;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  // kWqStages stages of [raw RAW | U 1024] records
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int yw = wv & 3, pt = wv >> 2, j = lane & 31, hh = lane >> 5;
  // RF: groups of 8 ring blocks (one per XCD) at the head of every a.rstride workgroups,
  // so the dispatcher interleaves them with the tiles; the tiles' index space skips them
  int cidx = blockIdx.x;
  if constexpr (RF) {
    const int g = blockIdx.x / a.rstride, off = blockIdx.x - g * a.rstride, ng = a.nring >> 3;
    if (g < ng && off < 8) {
      const int rb = 8 * g + off;
      if (rb < a.n * a.co_blocks * a.nseg) ring_block(a, rb, reinterpret_cast<float*>(smem4));
      return;
    }
    cidx -= 8 * min(g + 1, ng);
  }
  int bid;
  {
    const int nwg = gridDim.x - (RF ? a.nring : 0), q = nwg >> 3, r = nwg & 7;
    const int xcd = cidx & 7, slot = cidx >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  const int ksn = SK ? a.ksplit : 1;  // K slices per tile
  if (bid >= ntiles * ksn) return;
  const int tile = SK ? bid / ksn : bid, ks = SK ? bid - tile * ksn : 0;
#if RRIN_WINOQ_CLOCK
  const unsigned long long qc_t0 = __builtin_amdgcn_s_memtime(), qc_r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long qc_t1 = 0;
#endif
  // this slice's chunks [c0, c0 + nch) of the conv's a.nchunks; staging below counts chunks
  // from c0 (source and weight bases moved by c0 chunks, cin_loc channels from there)
  const int c0 = SK ? ks * a.kper : 0;
  const int nch = SK ? min(a.nchunks - c0, a.kper) : a.nchunks;
  const int cin_loc = a.cin - 8 * c0;
  int cob, x0, y0, img;
  {
    int t = tile;
#if RRIN_WINOQ_ORDER == 1  // A/B: tile column fastest, then the co block
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    cob = t % a.co_blocks;
    t /= a.co_blocks;
#elif RRIN_WINOQ_ORDER == 2  // A/B: the co block outermost within an image
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    const int ty_ = t % a.tiles_y;
    t /= a.tiles_y;
    cob = t % a.co_blocks;
    t /= a.co_blocks;
    t = t * a.tiles_y + ty_;
#else  // groups of a.cob_group co blocks (0: one group of all), tile positions within a group,
       // the group's co blocks of a tile position on consecutive workgroups (they share its raw
       // tile); an XCD runs consecutive workgroups, so with groups it streams one group's U
    {
      const int cpg = a.cob_group > 0 ? a.cob_group : a.co_blocks;
      const int gsz = cpg * (ntiles / a.co_blocks);
      const int g = t / gsz;
      const int r = t - g * gsz;
      const int cg = min(cpg, a.co_blocks - g * cpg);
      cob = g * cpg + r % cg;
      t = r / cg;
    }
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
#endif
    y0 = (t % a.tiles_y) * TH;
    img = t / a.tiles_y;
  }
  const uint4* tsrc =
      a.src_hi + (int64_t)img * a.src_img + (int64_t)(2 * c0) * a.src_gp + (int64_t)y0 * a.src_wp + x0 + (kH8PadLeft - 1);
  const uint4* wsrc = a.w_hi + ((int64_t)cob * a.nchunks + c0) * kWnU + tid;
  // staging: raw RAW records = NT + the rest, U 1024 = UP x NT
  int64_t p_off[2];
  int p_g[2], p_zero[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + NT * it;
    const int g = idx >= RG ? 1 : 0;
    const int rem = idx - g * RG;
    const int r = rem / kWnRawCols, pos = rem - r * kWnRawCols;
    const int col = pos < 17 ? 2 * pos : 2 * (pos - 17) + 1;
    p_g[it] = g;
    p_off[it] = (int64_t)g * a.src_gp + r * a.src_wp + col;
    p_zero[it] = col - y0 * a.src_wp;
  }
  // LDS: NS == 2: stages [raw | U] x 2; NS == 3 (A/B): a raw ring of 3 stages (chunk c + 2
  // staged while c computes) and a U ring of 2 (U is L2-resident: one chunk ahead)
  auto raw_stage = [&](int c) { return NS == 3 ? smem4 + (c % 3) * RAW : smem4 + (c & 1) * STAGE; };
  auto u_stage = [&](int c) { return NS == 3 ? smem4 + 3 * RAW + (c & 1) * kWnU : smem4 + (c & 1) * STAGE + RAW; };
  auto issue_raw = [&](int c) {
    uint4* base = raw_stage(c);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      if ((it == 0 || tid < RAW - NT) && !((ABL & 2) && c > 0)) {
        const int gg = 2 * c + p_g[it];
        const int64_t off = gg * 4 < cin_loc ? (int64_t)(2 * c) * a.src_gp + p_off[it] : (int64_t)p_zero[it];
        dma16(tsrc + off, base + NT * it + (tid & ~63));
      }
    }
  };
  auto issue_u = [&](int c) {
    if constexpr (!RU) {
      uint4* base = u_stage(c);
#pragma unroll
      for (int it = 0; it < UP; ++it)
        if (!((ABL & 1) && c > 0)) dma16(wsrc + (int64_t)c * kWnU + NT * it, base + NT * it + (tid & ~63));
    }
  };
  auto issue = [&](int c) {
    issue_raw(c);
    issue_u(c);
  };
  // RU: U record (xi = 4 yw + x, hh, co = j) of chunk c straight into registers
  const auto urs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(a.w_hi + ((int64_t)cob * a.nchunks + c0) * kWnU),
                                                     0, 0x7fffffff, 0x00020000);
  auto load_u = [&](int c, int x) {
    const unsigned voff = (unsigned)(((4 * yw + x) * 64 + hh * 32 + j) * 16);
    return __builtin_bit_cast(wfloatx4, __builtin_amdgcn_raw_buffer_load_b128(urs, voff, c * kWnU * 16, 0));
  };
  wfloatx4 ur[4];  // RU: U of the chunk being computed (point x reloaded after its MFMAs)
  const int pr = 2 * pt + (j >> 4), jx = (j + 12 * (j >> 4)) & 15;
  const int ra = yw == 0 ? 0 : (yw == 2 ? 2 : 1);
  const int rb = yw == 0 ? 2 : (yw == 1 ? 2 : (yw == 2 ? 1 : 3));
  const float sg = yw == 1 ? 1.f : -1.f;
  const int rw0 = hh * RG + (2 * pr) * kWnRawCols;
  const int oa = ra * kWnRawCols, ob = rb * kWnRawCols;
  int pc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pc[k] = wn_col(2 * jx + k);
  const int su0 = (4 * yw) * 64 + hh * 32 + j;  // U of point 4 yw + x: + x * 64 (layout [xi][half][32 co])

  wfloatx16 acc[4];
  wfloatx4 dk[8], uk[4];  // ABL 16 / 32: chunk 0's reads kept
  // one chunk in buffer b: window reads -> B^T row -> 4 points, then per point
  // its U record and 4 MFMAs (point-major, the cfg 18 accumulation order)
  auto chunk = [&](bool first, int c) {
    const uint4* rw = raw_stage(c) + rw0;
    wfloatx4 t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      wfloatx4 d0, d1;
      if (!(ABL & 16) || first) {
        d0 = __builtin_bit_cast(wfloatx4, rw[oa + pc[k]]);
        d1 = __builtin_bit_cast(wfloatx4, rw[ob + pc[k]]);
        if constexpr ((ABL & 16) != 0) dk[2 * k] = d0, dk[2 * k + 1] = d1;
      } else {
        d0 = dk[2 * k];
        d1 = dk[2 * k + 1];
      }
      if constexpr ((ABL & 8) != 0) {
        t[k] = d0;
        asm volatile("" ::"v"(d1));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) t[k][e] = fmaf(sg, d1[e], d0[e]);
      }
    }
    wfloatx4 v[4];
    if constexpr ((ABL & 8) != 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = t[x];
    } else {
      v[0] = t[0] - t[2];
      v[1] = t[1] + t[2];
      v[2] = t[2] - t[1];
      v[3] = t[1] - t[3];
    }
    const uint4* su = u_stage(c) + su0;
#if RRIN_WINOQ_PRIO == 1
    __builtin_amdgcn_s_setprio(1);  // A/B: priority around the MFMA cluster (guide T5)
#endif
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      wfloatx4 u;
      if constexpr (RU) {
        u = ur[x];
      } else if (!(ABL & 32) || first) {
        u = __builtin_bit_cast(wfloatx4, su[x * 64]);
        if constexpr ((ABL & 32) != 0) uk[x] = u;
      } else {
        u = uk[x];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr ((ABL & 4) != 0) {
          asm volatile("" ::"v"(u[e]), "v"(v[x][e]));
        } else {
          const wfloatx16 cin_acc = (first && e == 0) ? wfloatx16{} : acc[x];
          acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(u[e], v[x][e], cin_acc, 0, 0, 0);
        }
      }
      if constexpr (RU) {
        if (c + 1 < nch) ur[x] = load_u(c + 1, x);
      }
    }
#if RRIN_WINOQ_PRIO == 1
    __builtin_amdgcn_s_setprio(0);
#endif
  };
#if RRIN_WINOQ_PRIO == 2
  // A/B: static priority for the younger half of the workgroup (guide T5, static form)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
  // kWqStages = 3 (A/B builds): the raw tile of chunk c + 2 and the U slab of chunk c + 1
  // are issued at the top of chunk c, U first; at the top of chunk c a wave waits until
  // only its raw pieces of chunk c + 1 are in flight (2 for waves 0-2, which also stage
  // the raw tile's 168-record tail, 1 for the rest), then the bare barrier makes every
  // wave's pieces visible and ends every read of chunk c - 1, whose raw stage takes
  // chunk c + 2 and whose U stage takes chunk c + 1.  (Round 3's 3-stage ring kept U in
  // the same 3 stages: 82 KB per block.)
  const bool tail_wave = __builtin_amdgcn_readfirstlane(wv) < 3;
  auto wait_chunk = [&](bool next_in_flight) {
    if (!next_in_flight) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (tail_wave) {
      RRIN_VMWAIT(2, 0);
    } else {
      RRIN_VMWAIT(1, 0);
    }
  };
  if constexpr ((ABL & 4) != 0) {
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[x] = wfloatx16{};
  }
  {
  if constexpr (NS == 3) {
    issue_u(0);
    issue_raw(0);
    if (nch > 1) issue_raw(1);
  } else {
    issue(0);
  }
  if constexpr (RU) {
#pragma unroll
    for (int x = 0; x < 4; ++x) ur[x] = load_u(0, x);
  }
  for (int c = 0; c < nch; ++c) {
    if constexpr (NS == 3) {
      wait_chunk(c + 1 < nch);
      // bare barrier: __syncthreads() would drain vmcnt to 0 and wait for chunk c + 1 too
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (c + 1 < nch) issue_u(c + 1);
      if (c + 2 < nch) issue_raw(c + 2);
      chunk(c == 0, c);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // chunk c landed everywhere; stage (c + 1) & 1 was last read in chunk c - 1
#if RRIN_WINOQ_CLOCK
      if (c == 0) qc_t1 = __builtin_amdgcn_s_memtime();
#endif
      if (c + 1 < nch) issue(c + 1);
      chunk(c == 0, c);
    }
  }
  }
#if RRIN_WINOQ_CLOCK
  const unsigned long long qc_t2 = __builtin_amdgcn_s_memtime();
#endif
  // every stage DMA has landed (the last chunk waited for it): said with a wait the
  // compiler sees, so that it does not drain vmcnt at the exchange barrier below for the
  // LDS-DMA it cannot see completed -- which would wait out the bias loads too
#if RRIN_WINOQ_EPIWAIT
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
  // the epilogue's bias values, loaded now: their latency hides behind the exchange
  // instead of stalling the stores (the bias blob is padded to whole 32-row blocks)
  float bsv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bsv[i] = a.bias[cob * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
  __syncthreads();  // every read done before the exchange reuses the LDS
#if RRIN_WINOQ_AGPR
  asm volatile("" ::"a"(acc[0][0]));  // A/B: MFMA accumulators in AGPRs
#endif

  // ---- output transform (cfg 19 scheme, one co tile): the four yw waves of a
  // patch-row pair exchange their Q[c] = sum_x M[x] A[x][c] through LDS, one
  // column c per pass; wave (yw, pt) finishes output row r = yw & 1 of column
  // cc = yw >> 1, Y[0] = (Q0 + Q1) + Q2, Y[1] = (Q1 - Q2) - Q3 (cfg 18's order)
  wfloatx4* X = reinterpret_cast<wfloatx4*>(smem4);
  const int r = yw & 1, cc = yw >> 1;
  const int y = y0 + 2 * pr + r, x = x0 + 2 * jx + cc;
  uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
  auto store4 = [&](int64_t rec, const float* vv) {
    if constexpr ((ABL & 64) != 0) {
      asm volatile("" ::"v"(vv[0]), "v"(vv[1]), "v"(vv[2]), "v"(vv[3]));
      if (vv[0] != 12345.f) return;  // keeps the values live; never stores in practice
    }
    dst[rec] = make_uint4(__float_as_uint(vv[0]), __float_as_uint(vv[1]), __float_as_uint(vv[2]), __float_as_uint(vv[3]));
  };
  // two passes (column c = 0, 1): the Q records of one column are 32 KB
  float yv[16];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      wfloatx4 g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * k4 + e;
        const float m0 = acc[0][i], m1 = acc[1][i], m2 = acc[2][i], m3 = acc[3][i];
        g[e] = p == 0 ? (m0 + m1) + m2 : (m1 - m2) - m3;
      }
      X[((pt * 4 + yw) * 4 + k4) * 64 + lane] = g;
    }
    __syncthreads();
    if (cc == p) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const wfloatx4 q0 = X[((pt * 4 + 0) * 4 + k4) * 64 + lane];
        const wfloatx4 q1 = X[((pt * 4 + 1) * 4 + k4) * 64 + lane];
        const wfloatx4 q2 = X[((pt * 4 + 2) * 4 + k4) * 64 + lane];
        const wfloatx4 q3 = X[((pt * 4 + 3) * 4 + k4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) yv[4 * k4 + e] = r == 0 ? (q0[e] + q1[e]) + q2[e] : (q1[e] - q2[e]) - q3[e];
      }
    }
    __syncthreads();
  }
  if constexpr (SK) {
    // slice partial: plane q of the slice = NT lanes x 4 floats (coalesced per wave).
    // Split-K seam (cdna_hip_programming.md, split-K reduction recipe, sc1 form): the slice
    // drawing ksn - 1 reduces, reading every slab with sc1 loads.  Correct for any
    // placement of a tile's slices over CUs / XCDs.
    // The slab stores are write-through (sc1), so no release fence: every wave drains, the
    // barrier, then lane 0's relaxed ticket.
    {
      float* slab = a.part + (int64_t)(tile * ksn) * 4 * NT * 4;  // block-uniform base
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, ksn * 4 * NT * 16, 0x00020000);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = {__float_as_uint(yv[4 * q]), __float_as_uint(yv[4 * q + 1]), __float_as_uint(yv[4 * q + 2]),
                         __float_as_uint(yv[4 * q + 3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, ((ks * 4 + q) * NT + tid) * 16, 0, 16 /* sc1 */);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // "last slice" flag in the dynamic LDS array (right past the exchange records: 2048 of TH 8, 1024 of TH 4)
    int* s_last = reinterpret_cast<int*>(smem4 + 2048);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == ksn - 1;
      if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      *s_last = last;
    }
    __syncthreads();
    if (!*s_last) return;
    // the slabs are read with sc1 loads (no agent-scope acquire, which would drop this
    // CU's cached lines); the wavefront fence only keeps the loads below the ticket
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(a.part + (int64_t)(tile * ksn) * 4 * NT * 4, 0,
                                                       ksn * 4 * NT * 16, 0x00020000);
    auto ld = [&](int k, int q) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(srs, ((k * 4 + q) * NT + tid) * 16, 0, 16);
      return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 sum = ld(0, q);
      for (int k = 1; k < ksn; ++k) {
        const float4 v = ld(k, q);
        sum.x += v.x;
        sum.y += v.y;
        sum.z += v.z;
        sum.w += v.w;
      }
      yv[4 * q] = sum.x;
      yv[4 * q + 1] = sum.y;
      yv[4 * q + 2] = sum.z;
      yv[4 * q + 3] = sum.w;
    }
  }
  if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
    const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
    if (cob * 32 < a.cout && y < a.h && x < a.w) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int Y = 2 * y + (qq >> 1), XX = 2 * x + (qq & 1);
        const int64_t ri = ring_index(Y, XX, HH, WW);
        if (ri >= 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t k = ((int64_t)img * creal + cob * 8 + 4 * hh + e) * a.ring + ri;
            if constexpr (RF) {  // write-through: the segment's other writer may combine it
              const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(a.edge, 0, 0x7fffffff, 0x00020000);
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(yv[4 * qq + e]), rsrc, (int)(k * 4), 0, 16);
            } else {
              a.edge[k] = yv[4 * qq + e];
            }
          }
        } else {
          float vv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) vv[e] = yv[4 * qq + e] + bsv[4 * qq + e];
          store4((int64_t)(2 * cob + hh) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + XX + kH8PadLeft, vv);
        }
      }
    }
    if constexpr (RF) {
      // the ring segments this tile writes (its tile column's top / bottom row, its tile
      // row's left / right column): one ticket each, the later writer combines
      const int tx = x0 >> 5, ty = y0 / TH;
      const bool on[4] = {ty == 0, ty == a.tiles_y - 1, tx == 0, tx == a.tiles_x - 1};
      if (on[0] || on[1] || on[2] || on[3]) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* s_flag = reinterpret_cast<int*>(smem4 + 2048);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!on[k]) continue;
          const int seg = k == 0 ? tx : k == 1 ? a.tiles_x + tx : k == 2 ? 2 * a.tiles_x + ty : 2 * a.tiles_x + a.tiles_y + ty;
          const RingSeg rs = ring_seg(a, seg);
          if (rs.lo >= rs.hi) continue;  // empty column segment: no ring block counts it either
          if (ring_ticket(a, img, cob, seg, tid, s_flag)) ring_combine(a, img, cob, seg, tid);
        }
      }
    }
  } else {
    float vv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float tv = yv[i] + bsv[i];
      if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
      vv[i] = tv;
    }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      if (cob * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
        const int64_t rec = (int64_t)(cob * 8 + 2 * qq + hh) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
        store4(rec, &vv[4 * qq]);
        if constexpr (EPI == RRIN_EPI_LEAKY_REP) {
          const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
          const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
          for (int dy = dy0; dy <= dy1; ++dy)
            for (int dx = dx0; dx <= dx1; ++dx)
              if (dy | dx) store4(rec + (int64_t)dy * a.dst_wp + dx, &vv[4 * qq]);
        }
      }
    }
    if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        wfloatx4 g;
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = vv[4 * k + e];
        X[((pt * 4 + yw) * 4 + k) * 64 + lane] = g;
      }
      __syncthreads();
      if (yw == 0) {
        const int xp = x0 + 2 * jx, yp = y0 + 2 * pr;
        uint4* pdst = a.pool_hi + (int64_t)img * a.pool_img;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const wfloatx4 y00 = X[((pt * 4 + 0) * 4 + qq) * 64 + lane];
          const wfloatx4 y10 = X[((pt * 4 + 1) * 4 + qq) * 64 + lane];
          const wfloatx4 y01 = X[((pt * 4 + 2) * 4 + qq) * 64 + lane];
          const wfloatx4 y11 = X[((pt * 4 + 3) * 4 + qq) * 64 + lane];
          if (cob * 32 + 8 * qq < a.cout && yp < a.h && xp < a.w) {
            float s4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) s4[e] = 0.25f * ((y00[e] + y10[e]) + (y01[e] + y11[e]));
            const int64_t rec =
                (int64_t)(cob * 8 + 2 * qq + hh) * a.pool_gp + (int64_t)(yp / 2 + 1) * a.pool_wp + xp / 2 + kH8PadLeft;
            pdst[rec] = make_uint4(__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                                   __float_as_uint(s4[3]));
          }
        }
      }
    }
  }
#if RRIN_WINOQ_CLOCK
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores done
  const unsigned long long qc_t3 = __builtin_amdgcn_s_memtime(), qc_r3 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    unsigned long long* g = g_winoq_clk + (size_t)(bid % kQClkSlots) * 6;
    g[0] = qc_t1 - qc_t0;  // core clocks until chunk 0 landed
    g[1] = qc_t2 - qc_t0;  // ... until the end of the main loop
    g[2] = qc_t3 - qc_t0;  // ... until the stores completed
    g[3] = qc_r3 - qc_r0;  // 100 MHz ticks, whole workgroup
    g[4] = qc_r0;          // start (100 MHz ticks)
    g[5] = qc_r3;          // end
  }
#endif
}

template <int EPI, int ABL = 0, int PT = 2, int SK = 0, int RF = 0>
static int launch_winoq_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_winoq_kernel<EPI, ABL, PT, SK, RF>;
  static LdsAttr attr;
  constexpr size_t raw = (size_t)2 * (4 * PT + 2) * kWnRawCols;
  constexpr size_t lds = (PT == 2 && kWqStages == 3) ? (3 * raw + 2 * kWnU) * 16 : 2 * (raw + kWnU) * 16;
  if (int e = attr.ensure((const void*)k, (int)lds, st)) return e;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n * (SK ? a.ksplit : 1) + (RF ? a.nring : 0);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256 * PT), lds, st, a);
  return hip_code(hipGetLastError());
}

template <int PT>
static int launch_winoq_sk(const ConvH8Args& a, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_winoq_k<RRIN_EPI_LINEAR, 0, PT, 1>(a, st);
    case RRIN_EPI_LEAKY: return launch_winoq_k<RRIN_EPI_LEAKY, 0, PT, 1>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_winoq_k<RRIN_EPI_LEAKY_POOL, 0, PT, 1>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_winoq_k<RRIN_EPI_LEAKY_REP, 0, PT, 1>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_winoq_k<RRIN_EPI_SUBPIXEL, 0, PT, 1>(a, st);
  }
  return RRIN_E_ARG;
}

// Workgroup order of kinds 3 / 4 (as kind 6's, conv_winoc.hip::winoc_cob_group): when the co
// blocks' U (nchunks x 16 KB each) exceeds RRIN_WINOQ_UGROUP_KB, groups of co blocks whose U fits
// it, each group's workgroups consecutive -- an XCD then streams one group's U instead of every
// co block's (the deep split-K convs of small images read each U once per XCD otherwise).  The
// order changes no result.  Ring-folding launches keep their own index space.
#ifndef RRIN_WINOQ_UGROUP_KB
#define RRIN_WINOQ_UGROUP_KB 2048
#endif
static int winoq_cob_group(const ConvH8Args& a) {
  const int64_t per_cob = (int64_t)a.nchunks * kWnU * 16;
  const int64_t cap = (int64_t)RRIN_WINOQ_UGROUP_KB * 1024;
  if (RRIN_WINOQ_UGROUP_KB <= 0 || a.nring > 0 || (int64_t)a.co_blocks * per_cob <= cap) return 0;
  int g = 1;
  while (2 * g < a.co_blocks && 2 * g * per_cob <= cap) g *= 2;
  return g;
}

int launch_winoq(const ConvH8Args& a0, int epi, int th, hipStream_t st) {
  ConvH8Args a = a0;
  a.cob_group = winoq_cob_group(a0);
  if (a.ksplit > 1) return th == 4 ? launch_winoq_sk<1>(a, epi, st) : launch_winoq_sk<2>(a, epi, st);
  if (a.nring > 0) {
    if (th != 8 || epi != RRIN_EPI_SUBPIXEL) return RRIN_E_CONFIG;
    return launch_winoq_k<RRIN_EPI_SUBPIXEL, 0, 2, 0, 1>(a, st);
  }
  if (th == 4) {
    switch (epi) {
      case RRIN_EPI_LINEAR: return launch_winoq_k<RRIN_EPI_LINEAR, 0, 1>(a, st);
      case RRIN_EPI_LEAKY: return launch_winoq_k<RRIN_EPI_LEAKY, 0, 1>(a, st);
      case RRIN_EPI_LEAKY_POOL: return launch_winoq_k<RRIN_EPI_LEAKY_POOL, 0, 1>(a, st);
      case RRIN_EPI_LEAKY_REP: return launch_winoq_k<RRIN_EPI_LEAKY_REP, 0, 1>(a, st);
      case RRIN_EPI_SUBPIXEL: return launch_winoq_k<RRIN_EPI_SUBPIXEL, 0, 1>(a, st);
    }
    return RRIN_E_ARG;
  }
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_winoq_k<RRIN_EPI_LINEAR>(a, st);
    case RRIN_EPI_LEAKY: return launch_winoq_k<RRIN_EPI_LEAKY>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_winoq_k<RRIN_EPI_LEAKY_POOL>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_winoq_k<RRIN_EPI_LEAKY_REP>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_winoq_k<RRIN_EPI_SUBPIXEL>(a, st);
  }
  return RRIN_E_ARG;
}

#ifdef RRIN_LAB
// kernel lab (librrin_lab.so only): the LEAKY conv with ablation bits
int launch_wino_lab(const ConvH8Args& a, int abl, hipStream_t st) {
  switch (abl) {  // 1024 + bits: the 4-waves-per-SIMD tile (cfg 20)
    case 1024 + 0: return launch_winoq_k<RRIN_EPI_LEAKY, 0>(a, st);
    case 1024 + 3: return launch_winoq_k<RRIN_EPI_LEAKY, 3>(a, st);
    case 1024 + 4: return launch_winoq_k<RRIN_EPI_LEAKY, 4>(a, st);
    case 1024 + 8: return launch_winoq_k<RRIN_EPI_LEAKY, 8>(a, st);
    case 1024 + 16: return launch_winoq_k<RRIN_EPI_LEAKY, 16>(a, st);
    case 1024 + 32: return launch_winoq_k<RRIN_EPI_LEAKY, 32>(a, st);
    case 1024 + 48: return launch_winoq_k<RRIN_EPI_LEAKY, 48>(a, st);
    case 1024 + 56: return launch_winoq_k<RRIN_EPI_LEAKY, 56>(a, st);
    case 1024 + 59: return launch_winoq_k<RRIN_EPI_LEAKY, 59>(a, st);
    case 1024 + 64: return launch_winoq_k<RRIN_EPI_LEAKY, 64>(a, st);
    case 1024 + 123: return launch_winoq_k<RRIN_EPI_LEAKY, 123>(a, st);
    case 0: return launch_wino_k<RRIN_EPI_LEAKY, 0>(a, st);
    case 1: return launch_wino_k<RRIN_EPI_LEAKY, 1>(a, st);
    case 2: return launch_wino_k<RRIN_EPI_LEAKY, 2>(a, st);
    case 3: return launch_wino_k<RRIN_EPI_LEAKY, 3>(a, st);
    case 4: return launch_wino_k<RRIN_EPI_LEAKY, 4>(a, st);
    case 8: return launch_wino_k<RRIN_EPI_LEAKY, 8>(a, st);
    case 11: return launch_wino_k<RRIN_EPI_LEAKY, 11>(a, st);
    case 15: return launch_wino_k<RRIN_EPI_LEAKY, 15>(a, st);
  }
  return RRIN_E_CONFIG;
}
#endif

}  // namespace rrin

using namespace rrin;

#if RRIN_WINOQ_CLOCK
// diagnostic builds only: copy n workgroup stamps (6 x u64 each) to host memory
extern "C" int rrin_winoq_clock_read(unsigned long long* host, int n) {
  if (!host || n < 1 || n > rrin::kQClkSlots) return RRIN_E_ARG;
  return rrin::hip_code(hipMemcpyFromSymbol(host, HIP_SYMBOL(rrin::g_winoq_clk), (size_t)n * 6 * 8, 0,
                                            hipMemcpyDeviceToHost));
}
#endif

extern "C" int64_t rrin_pack_conv3x3_wino_floats(int32_t cout, int32_t cin) {
  return rrin_pack_conv3x3_wino_bm_floats(cout, cin, 32);
}

extern "C" int64_t rrin_pack_conv3x3_wino_bm_floats(int32_t cout, int32_t cin, int32_t bm) {
  if (cout < 1 || cin < 1 || (bm != 32 && bm != 64)) return RRIN_E_ARG;
  const int64_t cob = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  return cob * nch * 16 * 2 * bm * 4;
}

extern "C" int rrin_pack_conv3x3_wino(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                                      float* wpack, float* bpack) {
  return rrin_pack_conv3x3_wino_bm(w, b, cout, cin, 32, perm, wpack, bpack);
}

// [co block of bm][8-channel chunk][transform point xi][record half][bm co][4 channels]
extern "C" int rrin_pack_conv3x3_wino_bm(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                                         const int32_t* perm, float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1 || (bm != 32 && bm != 64)) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
  const int cob_n = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 16; ++xi)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < bm; ++col)
            for (int e = 0; e < 4; ++e) {
              const int co = cob * bm + col, ch = c * 8 + hh * 4 + e;
              double u = 0.0;
              if (co < cout && ch < cin) {
                const float* g = w + ((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9;
                for (int ky = 0; ky < 3; ++ky)
                  for (int kx = 0; kx < 3; ++kx) u += G[xi >> 2][ky] * G[xi & 3][kx] * (double)g[ky * 3 + kx];
              }
              wpack[o++] = (float)u;
            }
  for (int co = 0; co < cob_n * bm; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}
