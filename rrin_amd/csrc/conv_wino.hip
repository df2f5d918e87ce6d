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
// 64 patches (16 wide x 4 tall).  Wave (xh, ph): transform rows xi_y in
// {2xh, 2xh+1} (8 of the 16 points: 8 accumulators of 32 co x 32 patches, 128
// registers, so two blocks share a CU and cover each other's barriers) of the
// patch rows 2ph, 2ph+1.  K chunk = one record group (4 channels): per point 2
// MFMAs (product e: lanes 0-31 channel e, lanes 32-63 channel 2+e).
// Per chunk, all stages in LDS and double buffered:
//   raw input tile 10 x 34 records  (LDS-DMA, two chunks ahead)
//   U slab [xi][co] 16 x 32 records (LDS-DMA, one chunk ahead)
//   V      [xi][patch] 16 x 64      (input transform by the block, one chunk ahead)
// The output transform's two halves (xi_y 0-1, 2-3) meet through LDS: wave
// xh = 0 finishes output row 0 of each patch, xh = 1 row 1.
#include "common.hpp"

namespace rrin {

typedef float wfloatx16 __attribute__((ext_vector_type(16)));
typedef float wfloatx4 __attribute__((ext_vector_type(4)));
typedef float wfloatx2 __attribute__((ext_vector_type(2)));

constexpr int kWnRawCols = 34, kWnRaw = 10 * kWnRawCols, kWnRawStride = 352;
constexpr int kWnV = 16 * 64;  // records per V buffer
constexpr int kWnU = 16 * 32;  // records per U buffer
static_assert(kWinoLds == (size_t)(2 * kWnRawStride + 2 * kWnV + 2 * kWnU) * 16, "LDS size");

template <int EPI>
__global__ __launch_bounds__(256, 2) void conv3x3_wino_kernel(ConvH8Args a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  uint4* s_raw = smem4;                      // [2][kWnRawStride]
  uint4* s_v = smem4 + 2 * kWnRawStride;     // [2][16][64]
  uint4* s_u = s_v + 2 * kWnV;               // [2][16][32]

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
  int t = bid;
  const int cob = t % a.co_blocks;
  t /= a.co_blocks;
  const int x0 = (t % a.tiles_x) * 32;
  t /= a.tiles_x;
  const int y0 = (t % a.tiles_y) * 8;
  const int img = t / a.tiles_y;
  const int nch = a.nchunks;

  // ---- staging: raw input rows y0-1..y0+8, cols x0-1..x0+32 of record group c
  const uint4* src = a.src_hi + (int64_t)img * a.src_img + (int64_t)y0 * a.src_wp + x0 + (kH8PadLeft - 1);
  auto issue_raw = [&](int c, int buf) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kWnRaw) {
        const int r = idx / kWnRawCols, col = idx - r * kWnRawCols;
        dma16(src + (int64_t)c * a.src_gp + (int64_t)r * a.src_wp + col,
              s_raw + buf * kWnRawStride + 256 * it + (tid & ~63));
      }
    }
  };
  const uint4* wsrc = a.w_hi + (int64_t)cob * nch * kWnU;
  auto issue_u = [&](int c, int buf) {
#pragma unroll
    for (int it = 0; it < 2; ++it)
      dma16(wsrc + (int64_t)c * kWnU + tid + 256 * it, s_u + buf * kWnU + 256 * it + (tid & ~63));
  };

  // ---- input transform: thread (patch tp, xi row txy) -> V[txy*4 + xi_x][tp], 4 channels
  const int tp = tid & 63, txy = tid >> 6;
  const int tpr = 2 * (tp >> 5) + ((tp & 31) >> 4), tjx = tp & 15;
  const int tra = txy == 0 ? 0 : 1, trb = txy == 3 ? 3 : 2;  // the two window rows of B^T row txy
  auto transform = [&](int rb, int vb) {
    const uint4* base = s_raw + rb * kWnRawStride + (2 * tpr) * kWnRawCols + 2 * tjx;
    wfloatx4 tt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const wfloatx4 da = __builtin_bit_cast(wfloatx4, base[tra * kWnRawCols + k]);
      const wfloatx4 db = __builtin_bit_cast(wfloatx4, base[trb * kWnRawCols + k]);
      tt[k] = txy == 1 ? da + db : (txy == 2 ? db - da : da - db);
    }
    uint4* vd = s_v + vb * kWnV + txy * 4 * 64 + tp;
    vd[0] = __builtin_bit_cast(uint4, tt[0] - tt[2]);
    vd[64] = __builtin_bit_cast(uint4, tt[1] + tt[2]);
    vd[128] = __builtin_bit_cast(uint4, tt[2] - tt[1]);
    vd[192] = __builtin_bit_cast(uint4, tt[1] - tt[3]);
  };

  // ---- channel contraction: 8 points (xi = 8 xh + l) x 2 products per chunk
  wfloatx16 acc[8];
#pragma unroll
  for (int l = 0; l < 8; ++l)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[l][i] = 0.f;
  auto compute = [&](int b) {
    const wfloatx2* su = reinterpret_cast<const wfloatx2*>(s_u + b * kWnU + 8 * xh * 32 + j) + hh;
    const wfloatx2* sv = reinterpret_cast<const wfloatx2*>(s_v + b * kWnV + 8 * xh * 64 + ph * 32 + j) + hh;
    wfloatx2 av[8], bv[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      av[l] = su[l * 32 * 2];
      bv[l] = sv[l * 64 * 2];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int l = 0; l < 8; ++l) acc[l] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[l][e], bv[l][e], acc[l], 0, 0, 0);
  };

  issue_raw(0, 0);
  if (nch > 1) issue_raw(1, 1);
  issue_u(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  transform(0, 0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int b = c & 1;
    // raw buffer b held chunk c (transformed last iteration); U / V buffer b^1 were read last iteration
    if (c + 2 < nch) issue_raw(c + 2, b);
    if (c + 1 < nch) {
      issue_u(c + 1, b ^ 1);
      transform(b ^ 1, b ^ 1);
    }
    compute(b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

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
  // wave xh 0 hands its Q1 (yl 1) to its partner, wave xh 1 its Q2 (yl 0)
  wfloatx4* xch = reinterpret_cast<wfloatx4*>(s_v);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wfloatx4 g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v = 4 * k + e, c = v >> 4, i = v & 15;
      g[e] = xh ? q[0][c][i] : q[1][c][i];
    }
    xch[(wv * 8 + k) * 64 + lane] = g;
  }
  __syncthreads();
  float yv[2][16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const wfloatx4 pv = xch[((wv ^ 1) * 8 + k) * 64 + lane];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v = 4 * k + e, c = v >> 4, i = v & 15;
      yv[c][i] = xh ? (pv[e] - q[0][c][i]) - q[1][c][i] : (q[0][c][i] + q[1][c][i]) + pv[e];
    }
  }

  // ---- epilogue: this lane's pixels (y, x0 + 2 jx + c), 16 channels 8 qq + 4 hh + e
  const int pr = 2 * ph + (j >> 4), jx = j & 15;
  const int y = y0 + 2 * pr + xh;
  uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
  auto store4 = [&](int64_t rec, const float* v) {
    dst[rec] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  };
  if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
    // rows co' = cob*32 + 8 qq + 4 hh + e: group cob of 8 real channels, phase qq = (py, px)
    const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
    if (cob * 32 >= a.cout || y >= a.h) return;
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
      // row 1 of each patch (wave xh 1) meets row 0 (wave xh 0) in LDS; avg = 0.25 ((v00 + v10) + (v01 + v11))
      wfloatx4* xp = reinterpret_cast<wfloatx4*>(s_u);
      if (xh) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          wfloatx4 g;
#pragma unroll
          for (int e = 0; e < 4; ++e) g[e] = v[(4 * k + e) >> 4][(4 * k + e) & 15];
          xp[(ph * 8 + k) * 64 + lane] = g;
        }
      }
      __syncthreads();
      if (!xh) {
        float v1[2][16];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const wfloatx4 g = xp[(ph * 8 + k) * 64 + lane];
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

template <int EPI>
static int launch_wino_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_wino_kernel<EPI>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)kWinoLds)) return e;
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

}  // namespace rrin

using namespace rrin;

extern "C" int64_t rrin_pack_conv3x3_wino_floats(int32_t cout, int32_t cin) {
  if (cout < 1 || cin < 1) return RRIN_E_ARG;
  const int64_t cob = (cout + 31) / 32, nch = (cin + 3) / 4;
  return cob * nch * kWnU * 4;
}

extern "C" int rrin_pack_conv3x3_wino(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                                      float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
  const int cob_n = (cout + 31) / 32, nch = (cin + 3) / 4;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 16; ++xi)
        for (int col = 0; col < 32; ++col)
          for (int e = 0; e < 4; ++e) {
            const int co = cob * 32 + col, ch = c * 4 + e;
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
