// Training path (autograd on): NCHW fp32 HIP kernels for the forward operators
// of the reference's differentiable Net.forward and their backward.
//
// The reference trains with Net.forward under autograd (train.py:98) and
// loss.backward() (train.py:144); its operators are nn.Conv2d(3, pad=1) + bias
// (unet.py:29,38,59,62,78), LeakyReLU(0.1) (unet.py:47,60,63), F.avg_pool2d(2)
// (unet.py:46), nn.Upsample(x2, bilinear) (unet.py:77) and F.grid_sample in warp
// (model.py:8-21).  rrin_amd.train (Python) wraps each kernel pair below in a
// torch.autograd.Function; the model.py glue (cat, t-blend, sigmoid, blend,
// clamp) stays PyTorch elementwise autograd.
//
// conv3x3 is one implicit-GEMM kernel on the fp32 matrix cores
// (v_mfma_f32_32x32x2_f32, exact fp32 products, fp32 accumulation), block tile
// 64 x 64, K step 16 staged in LDS, three index maps:
//   FWD   C[co][p]            = sum_{ci,tap} W[co][ci][tap] x[ci][p + tap]       (+ bias, leaky)
//   DGRAD C[ci][p]            = sum_{co,tap} W[co][ci][8 - tap] g'[co][p + tap]   (flipped, transposed W)
//   WGRAD C[co][(ci,tap) | 1] = sum_{img,p} g'[co][p] x[ci][p + tap]            (last column: the bias grad)
// with g' = g * leaky'(y) applied on the fly (y = the forward's output: with a
// positive slope its sign is the pre-activation's), so leaky backward is fused
// into both gradient convs.  WGRAD splits its K (images x pixels) into fixed
// slices whose partial tiles are summed in slice order: deterministic.
//
// grid_sample backward (warp): the flow gradient is local per output pixel;
// the image gradient is a scatter (bilinear taps at data-dependent positions),
// accumulated in 64-bit fixed point (2^-scale units, scale from the gradient's
// max) so the sum is exact and order-independent, hence deterministic.
#include <string.h>

#include "common.hpp"

namespace rrin {

typedef float tfloatx16 __attribute__((ext_vector_type(16)));

enum { TC_FWD = 0, TC_DGRAD = 1, TC_WGRAD = 2 };

struct TConvArgs {
  int n, cin, cout, h, w;
  int leaky;
  float slope;
  const float* x;    // FWD / WGRAD: input [n][cin][h][w]
  const float* g;    // DGRAD / WGRAD: incoming gradient [n][cout][h][w]
  const float* y;    // leaky backward: forward output [n][cout][h][w]
  const float* wt;   // OIHW [cout][cin][3][3]
  const float* bias; // FWD (nullable)
  float* out;        // FWD y, DGRAD gx, WGRAD partials [slices][cout][cin*9+1]
  int M, N;          // GEMM dims
  int64_t K;         // GEMM reduction length
  int64_t kslice;    // WGRAD: K per slice (multiple of 16)
};

constexpr int TBM = 64, TBN = 64, TBK = 16;

// A(m, k) and B(k, n) of the three maps; tap = ky * 3 + kx
template <int MODE>
__device__ inline float tc_a(const TConvArgs& a, int m, int64_t k, int img) {
  if constexpr (MODE == TC_FWD) {
    return (m < a.M && k < a.K) ? a.wt[(int64_t)m * a.K + k] : 0.f;
  } else if constexpr (MODE == TC_DGRAD) {
    if (m >= a.M || k >= a.K) return 0.f;
    const int co = (int)(k / 9), tap = (int)(k - (int64_t)co * 9);
    return a.wt[((int64_t)co * a.cin + m) * 9 + (8 - tap)];
  } else {  // WGRAD: g'[img][co = m][p]
    if (m >= a.M || k >= a.K) return 0.f;
    const int64_t hw = (int64_t)a.h * a.w;
    const int im = (int)(k / hw);
    const int64_t p = k - (int64_t)im * hw;
    const int64_t o = ((int64_t)im * a.cout + m) * hw + p;
    float gv = a.g[o];
    if (a.leaky) gv *= a.y[o] > 0.f ? 1.f : a.slope;
    return gv;
  }
}

template <int MODE>
__device__ inline float tc_b(const TConvArgs& a, int64_t k, int n, int img) {
  const int64_t hw = (int64_t)a.h * a.w;
  if constexpr (MODE == TC_FWD || MODE == TC_DGRAD) {
    if (k >= a.K || n >= a.N) return 0.f;
    const int c = (int)(k / 9), tap = (int)(k - (int64_t)c * 9);
    const int py = n / a.w, px = n - py * a.w;
    const int yy = py + tap / 3 - 1, xx = px + tap % 3 - 1;
    if (yy < 0 || yy >= a.h || xx < 0 || xx >= a.w) return 0.f;
    if constexpr (MODE == TC_FWD) {
      return a.x[((int64_t)img * a.cin + c) * hw + (int64_t)yy * a.w + xx];
    } else {
      const int64_t o = ((int64_t)img * a.cout + c) * hw + (int64_t)yy * a.w + xx;
      float gv = a.g[o];
      if (a.leaky) gv *= a.y[o] > 0.f ? 1.f : a.slope;
      return gv;
    }
  } else {  // WGRAD: B(k = (img, p), n = (ci, tap) | bias column)
    if (k >= a.K || n >= a.N) return 0.f;
    if (n == a.N - 1) return 1.f;
    const int im = (int)(k / hw);
    const int64_t p = k - (int64_t)im * hw;
    const int py = (int)(p / a.w), px = (int)(p - (int64_t)py * a.w);
    const int ci = n / 9, tap = n - ci * 9;
    const int yy = py + tap / 3 - 1, xx = px + tap % 3 - 1;
    if (yy < 0 || yy >= a.h || xx < 0 || xx >= a.w) return 0.f;
    return a.x[((int64_t)im * a.cin + ci) * hw + (int64_t)yy * a.w + xx];
  }
}

// grid: x = N tiles, y = M tiles, z = images (FWD / DGRAD) or K slices (WGRAD)
template <int MODE>
__global__ __launch_bounds__(256) void tconv3x3_kernel(TConvArgs a) {
  __shared__ float sa[TBK][TBM];
  __shared__ float sb[TBK][TBN];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;  // wave's 32 x 32 sub-tile
  const int m0 = blockIdx.y * TBM, n0 = blockIdx.x * TBN;
  const int img = MODE == TC_WGRAD ? 0 : (int)blockIdx.z;
  int64_t k0 = 0, k1 = a.K;
  if constexpr (MODE == TC_WGRAD) {
    k0 = (int64_t)blockIdx.z * a.kslice;
    k1 = k0 + a.kslice < a.K ? k0 + a.kslice : a.K;
  }
  tfloatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // staging: thread -> (k row, 4 consecutive m / n)
  const int sk = tid >> 4, sc = (tid & 15) * 4;
  for (int64_t kb = k0; kb < k1; kb += TBK) {
    const int64_t k = kb + sk;
    const bool kin = k < k1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sa[sk][sc + j] = kin ? tc_a<MODE>(a, m0 + sc + j, k, img) : 0.f;
      sb[sk][sc + j] = kin ? tc_b<MODE>(a, k, n0 + sc + j, img) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TBK; kk += 2) {
      const float av = sa[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float bv = sb[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C[m][n] of register r: m = 8 (r / 4) + 4 (lane / 32) + r % 4, n = lane % 32
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= a.N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
    if (m >= a.M) continue;
    float v = acc[r];
    if constexpr (MODE == TC_FWD) {
      if (a.bias) v += a.bias[m];
      if (a.leaky) v = v > 0.f ? v : v * a.slope;
      a.out[((int64_t)img * a.cout + m) * ((int64_t)a.h * a.w) + n] = v;
    } else if constexpr (MODE == TC_DGRAD) {
      a.out[((int64_t)img * a.cin + m) * ((int64_t)a.h * a.w) + n] = v;
    } else {
      a.out[((int64_t)blockIdx.z * a.M + m) * a.N + n] = v;
    }
  }
}

// WGRAD: sum the slices' partials in slice order -> gw [cout][cin*9], gb [cout]
__global__ void twgrad_reduce_kernel(const float* __restrict__ part, int slices, int M, int N, float* gw,
                                     float* gb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  float s = 0.f;
  for (int k = 0; k < slices; ++k) s += part[(int64_t)k * M * N + i];
  const int m = i / N, c = i - m * N;
  if (c == N - 1) {
    if (gb) gb[m] = s;
  } else {
    gw[(int64_t)m * (N - 1) + c] = s;
  }
}

// ---- avg_pool2d(2): y[i][j] = 0.25 ((x00 + x01) + (x10 + x11)) (CPU kernel's order)
__global__ void tpool2_fwd_kernel(const float* __restrict__ x, float* y, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ho = h / 2, wo = w / 2;
  const int xo = (int)(i % wo);
  const int64_t t = i / wo;
  const int yo = (int)(t % ho);
  const int64_t c = t / ho;
  const float* p = x + c * h * w + (int64_t)(2 * yo) * w + 2 * xo;
  y[i] = (((p[0] + p[1]) + p[w]) + p[w + 1]) * 0.25f;
}

__global__ void tpool2_bwd_kernel(const float* __restrict__ gy, float* gx, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int xx = (int)(i % w);
  const int64_t t = i / w;
  const int yy = (int)(t % h);
  const int64_t c = t / h;
  gx[i] = gy[c * (h / 2) * (w / 2) + (int64_t)(yy / 2) * (w / 2) + xx / 2] * 0.25f;
}

// ---- Upsample(x2, bilinear, align_corners=False), separable: output o of a line
// of n inputs reads i0 = floor(s), i1 = min(i0 + 1, n - 1) with s = max((o + .5) / 2 - .5, 0),
// weights 1 - l, l (l = s - i0).  Forward = the reference formula (unet.py:77).
__device__ inline void up_taps(int o, int n, int& i0, int& i1, float& l) {
  float s = ((float)o + 0.5f) * 0.5f - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + 1 < n ? i0 + 1 : n - 1;
  l = s - (float)i0;
}

__global__ void tup2_fwd_kernel(const float* __restrict__ x, float* y, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int W2 = 2 * w, H2 = 2 * h;
  const int ox = (int)(i % W2);
  const int64_t t = i / W2;
  const int oy = (int)(t % H2);
  const int64_t c = t / H2;
  int y0, y1, x0, x1;
  float ly, lx;
  up_taps(oy, h, y0, y1, ly);
  up_taps(ox, w, x0, x1, lx);
  const float* p = x + c * h * w;
  const float a = p[(int64_t)y0 * w + x0], b = p[(int64_t)y0 * w + x1];
  const float cc = p[(int64_t)y1 * w + x0], d = p[(int64_t)y1 * w + x1];
  y[i] = (1.f - ly) * ((1.f - lx) * a + lx * b) + ly * ((1.f - lx) * cc + lx * d);
}

// backward as a gather: input i of a line receives from outputs 2i-2 .. 2i+3 the
// weight each of them gave it (both taps may be i at the clamped edge)
__device__ inline float up_w(int o, int n, int i) {
  int i0, i1;
  float l;
  up_taps(o, n, i0, i1, l);
  return (i0 == i ? 1.f - l : 0.f) + (i1 == i ? l : 0.f);
}

__global__ void tup2_bwd_kernel(const float* __restrict__ gy, float* gx, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ix = (int)(i % w);
  const int64_t t = i / w;
  const int iy = (int)(t % h);
  const int64_t c = t / h;
  const int W2 = 2 * w, H2 = 2 * h;
  const float* g = gy + c * H2 * W2;
  float s = 0.f;
  for (int oy = 2 * iy - 2; oy <= 2 * iy + 3; ++oy) {
    if (oy < 0 || oy >= H2) continue;
    const float wy = up_w(oy, h, iy);
    if (wy == 0.f) continue;
    float r = 0.f;
    for (int ox = 2 * ix - 2; ox <= 2 * ix + 3; ++ox) {
      if (ox < 0 || ox >= W2) continue;
      const float wx = up_w(ox, w, ix);
      if (wx != 0.f) r += wx * g[(int64_t)oy * W2 + ox];
    }
    s += wy * r;
  }
  gx[i] = s;
}

// ---- grid_sample backward of warp (model.py:8-21)
// max |g| per call (order-free) -> fixed-point scale for the image gradient
__global__ void tabsmax_kernel(const float* __restrict__ g, int64_t total, unsigned* mx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float v = i < total ? fabsf(g[i]) : 0.f;
  if (!(v <= 3.0e38f)) v = 3.0e38f;  // NaN / inf: saturate (the fixed-point sum then saturates too)
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) atomicMax(mx, __float_as_uint(v));
}

// 2^s with max|g| * 2^s < 2^(62 - hb), hb = ceil(log2(h w)): a source pixel receives at
// most one tap from each of the image's h w output pixels (weight <= 1), so its signed
// 64-bit sum cannot overflow at any size; the ulp stays 2^-(62 - hb) of max|g| (2^-39 at
// 4K).  s is capped at 126 so the scale stays finite for tiny gradients (those that fall
// below the ulp then count as zero, as they would in fp32 against max|g|).
__device__ inline float fx_scale(const unsigned* mx, int64_t hw) {
  const float m = __uint_as_float(*mx);
  if (!(m > 0.f)) return 1.f;
  int e;
  frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
  int hb = 0;
  while (((int64_t)1 << hb) < hw) ++hb;
  return ldexpf(1.f, min(62 - hb - e, 126));
}

__global__ void twarp_bwd_kernel(const float* __restrict__ img, const float* __restrict__ flow,
                                 const float* __restrict__ gout, unsigned long long* acc, float* gflow,
                                 const unsigned* mx, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int n = (int)(t / h);
  const int64_t hw = (int64_t)h * w;
  const float u = flow[(int64_t)n * 2 * hw + (int64_t)y * w + x];
  const float v = flow[(int64_t)n * 2 * hw + hw + (int64_t)y * w + x];
  const WarpTaps tp = warp_taps(x, y, u, v, h, w);
  const float sc = fx_scale(mx, hw);
  float gix = 0.f, giy = 0.f;
  // tap weights nw = s e, ne = s we, sw = n e, se = n we (common.hpp warp_taps)
  const float we_ = tp.wx, e_ = 1.0f - tp.wx, n_ = tp.wy, s_ = 1.0f - tp.wy;
  for (int ch = 0; ch < c; ++ch) {
    const float go = gout[((int64_t)n * c + ch) * hw + (int64_t)y * w + x];
    const float* plane = img + ((int64_t)n * c + ch) * hw;
    const float* p = plane + (int64_t)tp.y0 * w + tp.x0;
    const float a = (tp.vy0 && tp.vx0) ? p[0] : 0.f;
    const float b = (tp.vy0 && tp.vx1) ? p[1] : 0.f;
    const float cc = (tp.vy1 && tp.vx0) ? p[w] : 0.f;
    const float d = (tp.vy1 && tp.vx1) ? p[w + 1] : 0.f;
    // d out / d ix, d out / d iy (PyTorch grid_sampler_2d_backward)
    gix += go * ((b - a) * s_ + (d - cc) * n_);
    giy += go * ((cc - a) * e_ + (d - b) * we_);
    unsigned long long* q = acc + ((int64_t)n * c + ch) * hw + (int64_t)tp.y0 * w + tp.x0;
    auto add = [&](bool ok, int64_t off, float wgt) {
      if (ok && wgt != 0.f) atomicAdd(q + off, (unsigned long long)(long long)llrintf(go * wgt * sc));
    };
    add(tp.vy0 && tp.vx0, 0, tp.nw);
    add(tp.vy0 && tp.vx1, 1, tp.ne);
    add(tp.vy1 && tp.vx0, w, tp.sw);
    add(tp.vy1 && tp.vx1, w + 1, tp.se);
  }
  // ix = (gx + 1) W / 2 - 0.5 with gx = 2 (x / W - 0.5): d ix / d u = (W / 2) (2 / W)
  gflow[(int64_t)n * 2 * hw + (int64_t)y * w + x] = gix * ((float)w / 2.0f) * (2.0f / (float)w);
  gflow[(int64_t)n * 2 * hw + hw + (int64_t)y * w + x] = giy * ((float)h / 2.0f) * (2.0f / (float)h);
}

__global__ void tfix_to_float_kernel(const unsigned long long* __restrict__ acc, const unsigned* mx, float* out,
                                     int64_t total, int64_t hw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  out[i] = (float)((double)(long long)acc[i] / (double)fx_scale(mx, hw));
}

inline int grid_of(int64_t total) { return (int)((total + 255) / 256); }

}  // namespace rrin

using namespace rrin;

static int tconv_check(const rrin_tconv_desc* d) {
  if (!d || !d->wt || !d->out || !d->x) return RRIN_E_ARG;
  if (d->n < 1 || d->cin < 1 || d->cout < 1 || d->h < 1 || d->w < 1) return RRIN_E_ARG;
  if (d->leaky && !(d->slope > 0.f && d->slope <= 1.f)) return RRIN_E_ARG;
  if (d->mode == RRIN_TCONV_DGRAD && d->leaky && !d->y) return RRIN_E_ARG;
  if ((int64_t)d->h * d->w > 0x7fffffff) return RRIN_E_SHAPE;
  return 0;
}

extern "C" int rrin_tconv3x3(const rrin_tconv_desc* d, void* stream) {
  if (int e = tconv_check(d)) return e;
  if (d->mode != RRIN_TCONV_FWD && d->mode != RRIN_TCONV_DGRAD) return RRIN_E_ARG;
  TConvArgs a;
  memset(&a, 0, sizeof(a));
  a.n = d->n, a.cin = d->cin, a.cout = d->cout, a.h = d->h, a.w = d->w;
  a.leaky = d->leaky, a.slope = d->slope, a.wt = d->wt, a.bias = d->bias, a.out = d->out;
  a.N = d->h * d->w;
  const hipStream_t st = (hipStream_t)stream;
  if (d->mode == RRIN_TCONV_FWD) {
    a.x = d->x;
    a.M = d->cout;
    a.K = (int64_t)d->cin * 9;
    dim3 grid((a.N + TBN - 1) / TBN, (a.M + TBM - 1) / TBM, d->n);
    hipLaunchKernelGGL(tconv3x3_kernel<TC_FWD>, grid, dim3(256), 0, st, a);
  } else {
    a.g = d->x;  // the incoming gradient [n][cout][h][w]
    a.y = d->y;
    a.M = d->cin;
    a.K = (int64_t)d->cout * 9;
    dim3 grid((a.N + TBN - 1) / TBN, (a.M + TBM - 1) / TBM, d->n);
    hipLaunchKernelGGL(tconv3x3_kernel<TC_DGRAD>, grid, dim3(256), 0, st, a);
  }
  return hip_code(hipGetLastError());
}

// ---- weight gradient, row-tiled (round 4): C[co][ci * 9 + tap] = sum over the pixels of a
// slice of whole image rows of g'[co][p] x[ci][p + tap] on v_mfma_f32_32x32x2_f32.  A K chunk
// is a 64-pixel segment of one row: g' for the block's co tiles and the 3 x 66-pixel input
// rows (halo, zero padding) of 32 ci are staged in LDS, the pixels split by parity (pixel
// 2 s + kh is K step s of MFMA lane half kh), the input rows also one-shifted, so every
// operand of 4 K steps is one aligned ds_read_b128 and the 9 taps reuse the staged rows.
// Wave (co tile ct, tap group tg) owns taps 3 tg .. 3 tg + 2: 3 accumulators.  Slices are
// fixed per shape and summed in slice order (twgrad_reduce_kernel): deterministic.
struct TWArgs {
  int n, cin, cout, h, w, leaky;
  float slope;
  const float* x;
  const float* g;
  const float* y;
  float* part;   // [slices][cout][cin * 9 + 1]
  int rows_per_slice;
};
constexpr int kWgPx = 64, kWgSj = 36;  // pixels per K chunk; parity-row stride (33 + pad, 16-B aligned)

template <int CT>
constexpr size_t twgrad_lds() {
  return (size_t)(CT * 32 * 2 * 32 + 2 * 32 * 3 * 2 * kWgSj) * 4;
}

template <int CT>
__global__ __launch_bounds__(192 * CT, 2) void twgrad_tile_kernel(TWArgs a) {
  extern __shared__ __attribute__((aligned(16))) float tw_smem[];
  float* sA = tw_smem;                      // [CT * 32 co][2 kh][32 s]
  float* sB = tw_smem + CT * 32 * 2 * 32;   // [2 copies][32 ci][3 ky][2 p][kWgSj]
  constexpr int NT = 192 * CT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = wv % CT, tg = wv / CT;
  const int ci0 = blockIdx.x * 32, co0 = blockIdx.y * (32 * CT), slice = blockIdx.z;
  const int64_t hw = (int64_t)a.h * a.w;
  const int rows = a.n * a.h;
  const int r0 = slice * a.rows_per_slice, r1 = min(rows, r0 + a.rows_per_slice);
  tfloatx16 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = tfloatx16{};
  const int j = lane & 31, kh = lane >> 5;
  // per tap: the LDS float offset of this lane's B operand run (copy, ky, parity) at s = 0
  int boff[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tap = 3 * tg + t, ky = tap / 3, kx = tap % 3, c = kh + kx;
    boff[t] = ((((c >> 1) * 32 + j) * 3 + ky) * 2 + (c & 1)) * kWgSj;
  }
  const int aoff = ((ct * 32 + j) * 2 + kh) * 32;
  for (int R = r0; R < r1; ++R) {
    const int img = R / a.h, yrow = R - img * a.h;
    for (int x0 = 0; x0 < a.w; x0 += kWgPx) {
      __syncthreads();  // every read of the previous chunk done
      // A: g'[co][x0 .. x0 + 63], 4 pixels per item (one float4 load when w % 4 == 0),
      // zero past w / cout
      for (int i = tid; i < CT * 32 * 16; i += NT) {
        const int col = i >> 4, q = i & 15, co = co0 + col, px = x0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (co < a.cout && px < a.w) {
          const int64_t o = ((int64_t)img * a.cout + co) * hw + (int64_t)yrow * a.w + px;
          float4 yv = make_float4(1.f, 1.f, 1.f, 1.f);
          if ((a.w & 3) == 0) {
            v = *reinterpret_cast<const float4*>(a.g + o);
            if (a.leaky) yv = *reinterpret_cast<const float4*>(a.y + o);
          } else {
            float gv[4] = {0.f, 0.f, 0.f, 0.f}, yy4[4] = {1.f, 1.f, 1.f, 1.f};
            for (int e = 0; e < 4 && px + e < a.w; ++e) {
              gv[e] = a.g[o + e];
              if (a.leaky) yy4[e] = a.y[o + e];
            }
            v = make_float4(gv[0], gv[1], gv[2], gv[3]);
            yv = make_float4(yy4[0], yy4[1], yy4[2], yy4[3]);
          }
          if (a.leaky) {
            v.x *= yv.x > 0.f ? 1.f : a.slope;
            v.y *= yv.y > 0.f ? 1.f : a.slope;
            v.z *= yv.z > 0.f ? 1.f : a.slope;
            v.w *= yv.w > 0.f ? 1.f : a.slope;
          }
        }
        *reinterpret_cast<float2*>(sA + (col * 2 + 0) * 32 + 2 * q) = make_float2(v.x, v.z);
        *reinterpret_cast<float2*>(sA + (col * 2 + 1) * 32 + 2 * q) = make_float2(v.y, v.w);
      }
      // B: x[ci][yrow - 1 .. yrow + 1][x0 - 1 .. x0 + 64], zero outside; k = 2 jj + p
      for (int i = tid; i < 32 * 3 * 66; i += NT) {
        const int cl = i / 198, rem = i - cl * 198, ky = rem / 66, k = rem - ky * 66;
        const int ci = ci0 + cl, yy = yrow + ky - 1, px = x0 - 1 + k;
        float v = 0.f;
        if (ci < a.cin && yy >= 0 && yy < a.h && px >= 0 && px < a.w)
          v = a.x[((int64_t)img * a.cin + ci) * hw + (int64_t)yy * a.w + px];
        const int p = k & 1, jj = k >> 1;
        sB[((0 * 32 + cl) * 3 + ky) * 2 * kWgSj + p * kWgSj + jj] = v;
        if (jj >= 1) sB[((1 * 32 + cl) * 3 + ky) * 2 * kWgSj + p * kWgSj + jj - 1] = v;
      }
      __syncthreads();
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) {
        const float4 av = *reinterpret_cast<const float4*>(sA + aoff + 4 * s4);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const float4 bv = *reinterpret_cast<const float4*>(sB + boff[t] + 4 * s4);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc[t], 0, 0, 0);
        }
      }
    }
  }
  // C[co][ci] of register r: co = 8 (r / 4) + 4 (lane / 32) + r % 4, ci = lane % 32
  const int N = a.cin * 9 + 1, ci = ci0 + j;
  if (ci >= a.cin) return;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tap = 3 * tg + t;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + ct * 32 + 8 * (r >> 2) + 4 * kh + (r & 3);
      if (co < a.cout) a.part[((int64_t)slice * a.cout + co) * N + ci * 9 + tap] = acc[t][r];
    }
  }
}

// the bias column of a slice's partials: sum of g' over its rows, fixed order (per thread a
// strided run, then a fixed tree): deterministic
__global__ __launch_bounds__(256) void twgrad_bias_kernel(TWArgs a) {
  __shared__ float red[256];
  const int co = blockIdx.x, slice = blockIdx.y, tid = threadIdx.x;
  const int64_t hw = (int64_t)a.h * a.w;
  const int rows = a.n * a.h;
  const int r0 = slice * a.rows_per_slice, r1 = min(rows, r0 + a.rows_per_slice);
  float s = 0.f;
  for (int R = r0; R < r1; ++R) {
    const int img = R / a.h, yrow = R - img * a.h;
    const int64_t base = ((int64_t)img * a.cout + co) * hw + (int64_t)yrow * a.w;
    for (int px = tid; px < a.w; px += 256) {
      float v = a.g[base + px];
      if (a.leaky) v *= a.y[base + px] > 0.f ? 1.f : a.slope;
      s += v;
    }
  }
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) a.part[((int64_t)slice * a.cout + co) * (a.cin * 9 + 1) + a.cin * 9] = red[0];
}

// slices of whole rows: ~1024 tile workgroups per weight gradient
static void twgrad_slices(int n, int cin, int cout, int h, int* rows_per_slice, int* slices) {
  const int ct = cout % 64 == 0 ? 2 : 1;
  const int64_t per = (int64_t)((cin + 31) / 32) * ((cout + 32 * ct - 1) / (32 * ct));
  const int rows = n * h;
  int64_t sl = (1024 + per - 1) / per;
  if (sl > rows) sl = rows;
  if (sl < 1) sl = 1;
  *rows_per_slice = (int)((rows + sl - 1) / sl);
  *slices = (rows + *rows_per_slice - 1) / *rows_per_slice;
}

extern "C" int64_t rrin_tconv3x3_wgrad_work_floats(int32_t n, int32_t cin, int32_t cout, int32_t h, int32_t w) {
  if (n < 1 || cin < 1 || cout < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  int rps, sl;
  twgrad_slices(n, cin, cout, h, &rps, &sl);
  return (int64_t)sl * cout * ((int64_t)cin * 9 + 1);
}

template <int CT>
static int launch_twgrad(const TWArgs& a, int slices, hipStream_t st) {
  auto k = twgrad_tile_kernel<CT>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)twgrad_lds<CT>(), st)) return e;
  dim3 grid((unsigned)((a.cin + 31) / 32), (unsigned)((a.cout + 32 * CT - 1) / (32 * CT)), (unsigned)slices);
  hipLaunchKernelGGL(k, grid, dim3(192 * CT), twgrad_lds<CT>(), st, a);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_tconv3x3_wgrad(const rrin_twgrad_desc* d, void* stream) {
  if (!d || !d->x || !d->g || !d->gw || !d->work || (d->leaky && !d->y)) return RRIN_E_ARG;
  if (d->n < 1 || d->cin < 1 || d->cout < 1 || d->h < 1 || d->w < 1) return RRIN_E_ARG;
  if (d->leaky && !(d->slope > 0.f && d->slope <= 1.f)) return RRIN_E_ARG;
  TWArgs a;
  memset(&a, 0, sizeof(a));
  a.n = d->n, a.cin = d->cin, a.cout = d->cout, a.h = d->h, a.w = d->w;
  a.leaky = d->leaky, a.slope = d->slope, a.x = d->x, a.g = d->g, a.y = d->y, a.part = d->work;
  int slices;
  twgrad_slices(a.n, a.cin, a.cout, a.h, &a.rows_per_slice, &slices);
  const hipStream_t st = (hipStream_t)stream;
  const int rc = a.cout % 64 == 0 ? launch_twgrad<2>(a, slices, st) : launch_twgrad<1>(a, slices, st);
  if (rc) return rc;
  hipLaunchKernelGGL(twgrad_bias_kernel, dim3((unsigned)a.cout, (unsigned)slices), dim3(256), 0, st, a);
  const int M = a.cout, N = a.cin * 9 + 1;
  hipLaunchKernelGGL(twgrad_reduce_kernel, dim3(grid_of((int64_t)M * N)), dim3(256), 0, st, (const float*)d->work,
                     slices, M, N, d->gw, d->gb);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_tpool2_fwd(const float* x, float* y, int32_t nc, int32_t h, int32_t w, void* stream) {
  if (!x || !y || nc < 1 || h < 2 || w < 2 || (h & 1) || (w & 1)) return RRIN_E_ARG;
  const int64_t total = (int64_t)nc * (h / 2) * (w / 2);
  hipLaunchKernelGGL(tpool2_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, x, y, h, w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_tpool2_bwd(const float* gy, float* gx, int32_t nc, int32_t h, int32_t w, void* stream) {
  if (!gy || !gx || nc < 1 || h < 2 || w < 2 || (h & 1) || (w & 1)) return RRIN_E_ARG;
  const int64_t total = (int64_t)nc * h * w;
  hipLaunchKernelGGL(tpool2_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, gy, gx, h, w,
                     total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_tup2_fwd(const float* x, float* y, int32_t nc, int32_t h, int32_t w, void* stream) {
  if (!x || !y || nc < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  const int64_t total = (int64_t)nc * 4 * h * w;
  hipLaunchKernelGGL(tup2_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, x, y, h, w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_tup2_bwd(const float* gy, float* gx, int32_t nc, int32_t h, int32_t w, void* stream) {
  if (!gy || !gx || nc < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  const int64_t total = (int64_t)nc * h * w;
  hipLaunchKernelGGL(tup2_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, gy, gx, h, w, total);
  return hip_code(hipGetLastError());
}

extern "C" int64_t rrin_twarp_bwd_work_bytes(int32_t n, int32_t c, int32_t h, int32_t w) {
  if (n < 1 || c < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  return (int64_t)n * c * h * w * 8 + 256;
}

extern "C" int rrin_twarp_bwd(const float* img, const float* flow, const float* gout, float* gimg, float* gflow,
                              void* work, int64_t work_bytes, int32_t n, int32_t c, int32_t h, int32_t w,
                              void* stream) {
  if (!img || !flow || !gout || !gimg || !gflow || !work || n < 1 || c < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  const int64_t total = (int64_t)n * c * h * w;
  if (work_bytes < rrin_twarp_bwd_work_bytes(n, c, h, w)) return RRIN_E_WORKSPACE;
  const hipStream_t st = (hipStream_t)stream;
  unsigned long long* acc = static_cast<unsigned long long*>(work);
  unsigned* mx = reinterpret_cast<unsigned*>(acc + total);
  if (hipError_t e = hipMemsetAsync(work, 0, (size_t)total * 8 + 256, st)) return (int)e;
  hipLaunchKernelGGL(tabsmax_kernel, dim3(grid_of(total)), dim3(256), 0, st, gout, total, mx);
  const int64_t px = (int64_t)n * h * w;
  hipLaunchKernelGGL(twarp_bwd_kernel, dim3(grid_of(px)), dim3(256), 0, st, img, flow, gout, acc, gflow,
                     (const unsigned*)mx, c, h, w, px);
  hipLaunchKernelGGL(tfix_to_float_kernel, dim3(grid_of(total)), dim3(256), 0, st, (const unsigned long long*)acc,
                     (const unsigned*)mx, gimg, total, (int64_t)h * w);
  return hip_code(hipGetLastError());
}

// ---- Winograd weight pack on the device (training: the weights change every optimizer
// step).  The layout and arithmetic of rrin_pack_conv3x3_wino_bm (conv_wino.hip): per
// output row o, input channel i and point xi, u = sum_ky sum_kx G[xi/4][ky] G[xi%4][kx] g,
// in double, that order, no contraction, rounded once -- the host packing's bits.
// mode 0: g = W[o][i] (the forward conv); mode 1: g = W[i][o] flipped in y and x (the
// data-gradient conv: out rows = cin, in channels = cout).
#pragma clang fp contract(off)
__global__ void tpack_wino_kernel(const float* __restrict__ w, int cout, int cin, int rows, int cols, int bm,
                                  int mode, float* __restrict__ wpack, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  // i = (((cob * nch + c) * 16 + xi) * 2 + hh) * bm * 4 + col * 4 + e
  const int e = (int)(i & 3);
  int64_t t = i >> 2;
  const int col = (int)(t % bm);
  t /= bm;
  const int hh = (int)(t & 1);
  t >>= 1;
  const int xi = (int)(t & 15);
  t >>= 4;
  const int nch = (cols + 7) / 8;
  const int c = (int)(t % nch);
  const int cob = (int)(t / nch);
  const int o = cob * bm + col, ch = c * 8 + hh * 4 + e;
  double u = 0.0;
  if (o < rows && ch < cols) {
    const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
    const float* g = mode ? w + ((int64_t)ch * cin + o) * 9 : w + ((int64_t)o * cin + ch) * 9;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        const double gv = (double)(mode ? g[(2 - ky) * 3 + (2 - kx)] : g[ky * 3 + kx]);
        const double p = G[xi >> 2][ky] * G[xi & 3][kx];
        u = u + p * gv;
      }
  }
  wpack[i] = (float)u;
}
#pragma clang fp contract(on)

extern "C" int rrin_tpack_wino(const float* w, int32_t cout, int32_t cin, int32_t bm, int32_t mode, float* wpack,
                               void* stream) {
  if (!w || !wpack || cout < 1 || cin < 1 || (bm != 32 && bm != 64) || (mode != 0 && mode != 1)) return RRIN_E_ARG;
  const int rows = mode ? cin : cout, cols = mode ? cout : cin;
  const int64_t total = rrin_pack_conv3x3_wino_bm_floats(rows, cols, bm);
  if (total < 0) return (int)total;
  hipLaunchKernelGGL(tpack_wino_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, w, cout, cin, rows,
                     cols, bm, mode, wpack, total);
  return hip_code(hipGetLastError());
}
