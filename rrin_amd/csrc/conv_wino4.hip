// Exact-fp32 3x3 conv as Winograd F(4x4, 3x3) on fp32 records (R32) with the
// f32-input matrix cores (v_mfma_f32_32x32x2_f32).  Tile config kWino4Cfg of the
// record-layout conv table (rrin_conv3x3_h8_fwd, precision F32R); the same
// reference ops as conv_wino.hip (nn.Conv2d(3, pad=1) + LeakyReLU(0.1),
// unet.py:29,59-63; fused avg_pool2d, unet.py:46; sub-pixel Upsample + up conv,
// unet.py:77-78).
//
// Per 4x4 output patch and input channel the 6x6 input window d becomes
// V = B^T d B, the weights U = G g G^T (host, in double, rounded once to fp32),
// per transform point xi (36) M[xi] = sum_ci U[xi] V[xi] on the fp32 MFMA, and
// the patch Y = A^T M A: 36 multiplies per 16 outputs and channel pair, against
// F(2x2)'s 16 per 4 (1.78x fewer MFMA cycles) and the direct form's 144 per 16.
// Interpolation points 0, 1, -1, 1/2, -2, inf -- the most accurate F(4,3) set in
// fp32 (about 6x F(2x2)'s rounding error, max-abs 1e-5 on a 256-channel conv
// of unit inputs; every operation stays an IEEE fp32 operation) -- with the
// rows of B^T scaled to small integers (the inverse scale folded into G):
//   B^T = [ 2 -3 -4  3  2  0]    G = [ 1/2    0     0  ]   A^T = [1 1  1   1    1 0]
//         [ 0 -2  1  5  2  0]        [ 1/6   1/6   1/6 ]         [0 1 -1  1/2  -2 0]
//         [ 0 -2  5 -1 -2  0]        [ 1/6  -1/6   1/6 ]         [0 1  1  1/4   4 0]
//         [ 0  2  1 -2 -1  0]        [16/15  8/15  4/15]         [0 1 -1  1/8  -8 1]
//         [ 0  1 -2 -1  2  0]        [ 1/30 -1/15  2/15]
//         [ 0  2 -3 -4  3  2]        [ 0     0     1/2 ]
//
// Block: 384 threads = 6 waves; tile = 32 output channels x 32 px x 16 rows =
// 32 patches (8 wide x 4 tall, the MFMA's N).  Wave i owns B^T row i: it
// combines the window rows of its patch into t_k = sum_r B^T[i][r] d[r][k]
// (k = 0..5), then the 6 points (i, j) are v_j = sum_k B^T[j][k] t_k, each
// contracted on its own accumulator (6 x 16 registers).  K chunk = 4 channels
// (one record group): lanes 0-31 carry channels 0-1 of the record, lanes 32-63
// channels 2-3 (8-byte LDS reads), 2 MFMAs per point.  Per chunk, double
// buffered in LDS (LDS-DMA, one chunk ahead): the raw tile (18 rows x 34 cols,
// columns by phase col % 4) and U [xi][half][co][2]; 55 KB per block, so two blocks
// share a CU (12 waves, 3 per SIMD).  The output transform meets through LDS
// in two column passes.
#include <type_traits>

#include "common.hpp"

namespace rrin {

// The F(4x4) tile (kind 5) lost to F(2x2) on every Net shape: its
// kernel is built only into the lab library (`make lab`, RRIN_LAB); the product
// library keeps the host packing below and reports config kind 5 as not built.
#ifdef RRIN_LAB
typedef float w4x16 __attribute__((ext_vector_type(16)));
typedef float w4x4 __attribute__((ext_vector_type(4)));
typedef float w4x2 __attribute__((ext_vector_type(2)));

constexpr int kW4Cols = 34, kW4Rows = 18, kW4Raw = kW4Rows * kW4Cols;  // 612 records
constexpr int kW4U = 36 * 2 * 32 * 2 / 4;                               // 1152 records: [xi][half][co][2]
constexpr int kW4Stage = kW4Raw + kW4U;                                 // 1764 records
constexpr int kW4NT = 384;
static_assert(kWino4Lds == (size_t)2 * kW4Stage * 16, "LDS size");
static_assert(2 * kWino4Lds <= 160 * 1024, "two blocks per CU");
static_assert(kW4Raw > kW4NT && kW4Raw <= 2 * kW4NT && kW4U % kW4NT == 0, "staging pieces");

#ifndef W4_KGROUP
#define W4_KGROUP 6
#endif

// B^T with integer rows (the scale lives in G, rrin_pack_conv3x3_wino4)
constexpr float kBT4[6][6] = {{2, -3, -4, 3, 2, 0},  {0, -2, 1, 5, 2, 0},  {0, -2, 5, -1, -2, 0},
                              {0, 2, 1, -2, -1, 0}, {0, 1, -2, -1, 2, 0}, {0, 2, -3, -4, 3, 2}};

// LDS position of raw column col (0..33) within its row: four phases by col % 4
// (9, 9, 8, 8 columns), so the 8 patches of a row (columns 4 pc + k) read
// consecutive records and, with the 34-record row stride, the tile's 32 patches
// cover every LDS bank once per read
__device__ inline int w4_col(int col) { return (col & 3) * 9 - ((col & 3) == 3 ? 1 : 0) + (col >> 2); }

// A^T rows applied to six values (Q = M A or Y = A^T Q), fixed order
__device__ inline w4x4 w4_at(int r, const w4x4* m) {
  switch (r) {
    case 0: return (((m[0] + m[1]) + m[2]) + m[3]) + m[4];
    case 1: return ((m[1] - m[2]) + 0.5f * m[3]) - 2.0f * m[4];
    case 2: return ((m[1] + m[2]) + 0.25f * m[3]) + 4.0f * m[4];
    default: return (((m[1] - m[2]) + 0.125f * m[3]) - 8.0f * m[4]) + m[5];
  }
}

// ABL (lab builds only, librrin_lab.so): 1 no DMA after chunk 0, 2 (with 1) no
// wait / barrier per chunk, 4 no MFMAs, 8 no transform arithmetic, 32 no U reads
// after chunk 0
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(kW4NT) __attribute__((amdgpu_waves_per_eu(3))) void conv3x3_wino4_kernel(ConvH8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  int bid;
  {  // consecutive tiles on one XCD (blocks are dealt to the 8 XCDs round robin)
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
  const int nch = a.nchunks;
  int cob, x0, y0, img;
  {
    int t = bid;
    cob = t % a.co_blocks;
    t /= a.co_blocks;
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    y0 = (t % a.tiles_y) * 16;
    img = t / a.tiles_y;
  }
  // raw tile: padded rows y0 .. y0 + 17 (image rows y0 - 1 .. y0 + 16), cols x0 - 1 .. x0 + 32
  const uint4* tsrc = a.src_hi + (int64_t)img * a.src_img + (int64_t)y0 * a.src_wp + x0 + (kH8PadLeft - 1);
  const uint4* wsrc = a.w_hi + (int64_t)cob * nch * kW4U + tid;
  int64_t p_off[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + kW4NT * it;
    const int r = idx / kW4Cols, pos = idx - r * kW4Cols;
    const int col = pos < 9 ? 4 * pos : pos < 18 ? 4 * (pos - 9) + 1 : pos < 26 ? 4 * (pos - 18) + 2 : 4 * (pos - 26) + 3;
    p_off[it] = (int64_t)r * a.src_wp + col;
  }
  auto issue = [&](int c, int b) {
    if ((ABL & 1) && c > 0) return;
    uint4* base = smem4 + b * kW4Stage;
    const int64_t g = (int64_t)c * a.src_gp;  // chunk c = record group c (4 channels)
    dma16(tsrc + g + p_off[0], base + (tid & ~63));
    if (tid < kW4Raw - kW4NT) dma16(tsrc + g + p_off[1], base + kW4NT + (tid & ~63));
#pragma unroll
    for (int it = 0; it < kW4U / kW4NT; ++it)
      dma16(wsrc + (int64_t)c * kW4U + kW4NT * it, base + kW4Raw + kW4NT * it + (tid & ~63));
  };
  const int pr = j >> 3, pc = j & 7;  // patch of this lane
  int pcol[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) pcol[k] = w4_col(4 * pc + k);
  const int rw0 = (4 * pr) * kW4Cols;  // window row 0 of the patch

  w4x16 acc[6];
  w4x2 uk[6];  // ABL 32: chunk 0's U kept
  if constexpr ((ABL & 4) != 0) {
#pragma unroll
    for (int x = 0; x < 6; ++x) acc[x] = w4x16{};
  }
  // one chunk in stage b for B^T row I
  auto chunk = [&](auto I_, int b, bool first) {
    constexpr int I = decltype(I_)::value;
    const w4x2* rw = reinterpret_cast<const w4x2*>(smem4 + b * kW4Stage) + 2 * rw0 + hh;
    w4x2 t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      bool any = false;
#pragma unroll
      for (int rr = 0; rr < 6; ++rr) {
        const float cf = kBT4[I][rr];
        if (cf != 0.f) {
          const w4x2 d = rw[2 * (rr * kW4Cols + pcol[k])];
          if constexpr ((ABL & 8) != 0) {
            if (!any) t[k] = d;
            else asm volatile("" ::"v"(d));
            any = true;
          } else if (!any) {
            t[k] = cf * d;
            any = true;
          } else {
            t[k][0] = fmaf(cf, d[0], t[k][0]);
            t[k][1] = fmaf(cf, d[1], t[k][1]);
          }
        }
      }
      // window reads of at most W4_KGROUP columns in flight (register pressure: M takes 96)
      if ((k + 1) % W4_KGROUP == 0) asm volatile("" ::: "memory");
    }
    const w4x2* su = reinterpret_cast<const w4x2*>(smem4 + b * kW4Stage + kW4Raw) + (6 * I * 2 + hh) * 32 + j;
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      w4x2 v;
      bool any = false;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float cf = kBT4[jj][k];
        if ((ABL & 8) != 0 && cf != 0.f) {
          if (!any) v = t[k];
          any = true;
        } else if (cf != 0.f) {
          if (!any) {
            v = cf * t[k];
            any = true;
          } else {
            v[0] = fmaf(cf, t[k][0], v[0]);
            v[1] = fmaf(cf, t[k][1], v[1]);
          }
        }
      }
      w4x2 u;
      if (!(ABL & 32) || first) {
        u = su[jj * 64];
        if constexpr ((ABL & 32) != 0) uk[jj] = u;
      } else {
        u = uk[jj];
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if constexpr ((ABL & 4) != 0) {
          asm volatile("" ::"v"(u[e]), "v"(v[e]));
        } else {
          const w4x16 c = (first && e == 0) ? w4x16{} : acc[jj];
          acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(u[e], v[e], c, 0, 0, 0);
        }
      }
    }
  };
  auto main_loop = [&](auto I_) {
    issue(0, 0);
    for (int c = 0; c < nch; ++c) {
      if (!((ABL & 2) && c > 1)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk c landed everywhere; stage (c + 1) & 1 was last read in chunk c - 1
      }
      if (c + 1 < nch) issue(c + 1, (c + 1) & 1);
      chunk(I_, c & 1, c == 0);
    }
  };
  switch (wv) {
    case 0: main_loop(std::integral_constant<int, 0>{}); break;
    case 1: main_loop(std::integral_constant<int, 1>{}); break;
    case 2: main_loop(std::integral_constant<int, 2>{}); break;
    case 3: main_loop(std::integral_constant<int, 3>{}); break;
    case 4: main_loop(std::integral_constant<int, 4>{}); break;
    default: main_loop(std::integral_constant<int, 5>{}); break;
  }
  __syncthreads();  // every read done before the exchange reuses the LDS

  // ---- output transform: Q[i][c] = sum_j M[i][j] A[j][c] in the wave, then
  // Y[r][c] = sum_i A^T[r][i] Q[i][c] across the waves, two columns per pass
  w4x4* X = reinterpret_cast<w4x4*>(smem4);
  uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
  auto store4 = [&](int64_t rec, const float* vv) {
    dst[rec] = make_uint4(__float_as_uint(vv[0]), __float_as_uint(vv[1]), __float_as_uint(vv[2]), __float_as_uint(vv[3]));
  };
  // the 16 channel values of output (r, c) of this lane's patch: co = 8 (k4) + 4 hh + e
  auto output = [&](int r, int c, float* yv) {
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      w4x4 q[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) q[i] = X[((i * 2 + (c & 1)) * 4 + k4) * 64 + lane];
      const w4x4 y = w4_at(r, q);
#pragma unroll
      for (int e = 0; e < 4; ++e) yv[4 * k4 + e] = y[e];
      asm volatile("" ::: "memory");  // one k4 group of Q reads in flight
    }
  };
  // bias (+ leaky) and the stores of output pixel (y, x); POOL: the values kept in vv
  auto emit = [&](int y, int x, const float* yv, float* vv) {
    if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
      const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
      if (cob * 32 < a.cout && y < a.h && x < a.w) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int Y = 2 * y + (qq >> 1), XX = 2 * x + (qq & 1);
          const int64_t ri = ring_index(Y, XX, HH, WW);
          if (ri >= 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) a.edge[((int64_t)img * creal + cob * 8 + 4 * hh + e) * a.ring + ri] = yv[4 * qq + e];
          } else {
            float ov[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = yv[4 * qq + e] + a.bias[cob * 32 + 8 * qq + 4 * hh + e];
            store4((int64_t)(2 * cob + hh) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + XX + kH8PadLeft, ov);
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float tv = yv[i] + a.bias[cob * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
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
    }
  };
  const int py = y0 + 4 * pr, px = x0 + 4 * pc;  // output pixel (0, 0) of the patch
  // Q[i][c] for the four columns up front (64 registers instead of the 96 of M)
  w4x4 qc[4][4];
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) {
    w4x4 m[6];
#pragma unroll
    for (int jj = 0; jj < 6; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[jj][e] = acc[jj][4 * k4 + e];
#pragma unroll
    for (int c = 0; c < 4; ++c) qc[c][k4] = w4_at(c, m);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int cl = 0; cl < 2; ++cl)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) X[((wv * 2 + cl) * 4 + k4) * 64 + lane] = qc[2 * p + cl][k4];
    __syncthreads();
    if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
      // wave w < 2 finishes rows 2w, 2w + 1 of columns 2p, 2p + 1: one pool window,
      // avg = 0.25 ((Y00 + Y10) + (Y01 + Y11)) of the leaky outputs
      if (wv < 2) {
        float yv[16], vv[16], va[16], s0[16];
        output(2 * wv, 2 * p, yv);
        emit(py + 2 * wv, px + 2 * p, yv, va);
        output(2 * wv + 1, 2 * p, yv);
        emit(py + 2 * wv + 1, px + 2 * p, yv, vv);
#pragma unroll
        for (int i = 0; i < 16; ++i) s0[i] = va[i] + vv[i];
        output(2 * wv, 2 * p + 1, yv);
        emit(py + 2 * wv, px + 2 * p + 1, yv, va);
        output(2 * wv + 1, 2 * p + 1, yv);
        emit(py + 2 * wv + 1, px + 2 * p + 1, yv, vv);
        const int yp = py + 2 * wv, xp = px + 2 * p;
        uint4* pdst = a.pool_hi + (int64_t)img * a.pool_img;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (cob * 32 + 8 * qq < a.cout && yp < a.h && xp < a.w) {
            float s4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * qq + e;
              s4[e] = 0.25f * (s0[i] + (va[i] + vv[i]));
            }
            const int64_t rec =
                (int64_t)(cob * 8 + 2 * qq + hh) * a.pool_gp + (int64_t)(yp / 2 + 1) * a.pool_wp + xp / 2 + kH8PadLeft;
            pdst[rec] = make_uint4(__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                                   __float_as_uint(s4[3]));
          }
        }
      }
    } else {
      // wave w < 4 finishes row w of columns 2p, 2p + 1
      if (wv < 4) {
#pragma unroll
        for (int cl = 0; cl < 2; ++cl) {
          float yv[16], vv[16];
          output(wv, 2 * p + cl, yv);
          emit(py + wv, px + 2 * p + cl, yv, vv);
        }
      }
    }
    __syncthreads();
  }
}

template <int EPI, int ABL = 0>
static int launch_wino4_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_wino4_kernel<EPI, ABL>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)kWino4Lds, st)) return e;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kW4NT), kWino4Lds, st, a);
  return hip_code(hipGetLastError());
}

int launch_wino4(const ConvH8Args& a, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_wino4_k<RRIN_EPI_LINEAR>(a, st);
    case RRIN_EPI_LEAKY: return launch_wino4_k<RRIN_EPI_LEAKY>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_wino4_k<RRIN_EPI_LEAKY_POOL>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_wino4_k<RRIN_EPI_LEAKY_REP>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_wino4_k<RRIN_EPI_SUBPIXEL>(a, st);
  }
  return RRIN_E_ARG;
}

int launch_wino4_lab(const ConvH8Args& a, int abl, hipStream_t st) {
  switch (abl) {
    case 0: return launch_wino4_k<RRIN_EPI_LEAKY, 0>(a, st);
    case 1: return launch_wino4_k<RRIN_EPI_LEAKY, 1>(a, st);
    case 3: return launch_wino4_k<RRIN_EPI_LEAKY, 3>(a, st);
    case 4: return launch_wino4_k<RRIN_EPI_LEAKY, 4>(a, st);
    case 8: return launch_wino4_k<RRIN_EPI_LEAKY, 8>(a, st);
    case 12: return launch_wino4_k<RRIN_EPI_LEAKY, 12>(a, st);
    case 32: return launch_wino4_k<RRIN_EPI_LEAKY, 32>(a, st);
    case 35: return launch_wino4_k<RRIN_EPI_LEAKY, 35>(a, st);
    case 43: return launch_wino4_k<RRIN_EPI_LEAKY, 43>(a, st);
  }
  return RRIN_E_CONFIG;
}
#endif  // RRIN_LAB

}  // namespace rrin

using namespace rrin;

extern "C" int64_t rrin_pack_conv3x3_wino4_floats(int32_t cout, int32_t cin) {
  if (cout < 1 || cin < 1) return RRIN_E_ARG;
  const int64_t cob = (cout + 31) / 32, nch = (cin + 3) / 4;
  return cob * nch * 36 * 2 * 32 * 2;
}

// [co block of 32][4-channel chunk][transform point xi = 6 a + b][half][32 co][2 channels]:
// U[xi] = G4[a] g G4[b]^T in double, rounded once; channel = 4 chunk + 2 half + e
extern "C" int rrin_pack_conv3x3_wino4(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                                       float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G[6][3] = {{1.0 / 2, 0.0, 0.0},          {1.0 / 6, 1.0 / 6, 1.0 / 6},
                                 {1.0 / 6, -1.0 / 6, 1.0 / 6}, {16.0 / 15, 8.0 / 15, 4.0 / 15},
                                 {1.0 / 30, -1.0 / 15, 2.0 / 15}, {0.0, 0.0, 1.0 / 2}};
  const int cob_n = (cout + 31) / 32, nch = (cin + 3) / 4;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 36; ++xi)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < 32; ++col)
            for (int e = 0; e < 2; ++e) {
              const int co = cob * 32 + col, ch = c * 4 + hh * 2 + e;
              double u = 0.0;
              if (co < cout && ch < cin) {
                const float* g = w + ((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9;
                for (int ky = 0; ky < 3; ++ky)
                  for (int kx = 0; kx < 3; ++kx) u += G[xi / 6][ky] * G[xi % 6][kx] * (double)g[ky * 3 + kx];
              }
              wpack[o++] = (float)u;
            }
  for (int co = 0; co < cob_n * 32; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}
