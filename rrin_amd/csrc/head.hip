// Head convs (Cout <= 4) fused with the Net glue they feed, plus the layout
// and standalone backwarp kernels.
//
//   FLOW   Flow.last        -> t-blend            model.py:37-39
//   REFINE refine_flow.last -> residual + 2 warps  model.py:44-48 (warp: model.py:8-21)
//   MASK   Mask.last        -> sigmoid + blend     model.py:52-55
//   FINAL  final.last       -> + out, clamp(0,1)   model.py:62-63
//
// A 3x3 conv with 2-4 outputs cannot fill a 32-wide MFMA tile (>= 87 % waste)
// and is HBM-bound anyway (32 ch in, <= 4 out per pixel), so it runs on the
// VALU: one thread per pixel, 8-channel chunks of the 32-channel input staged
// through LDS exactly like the MFMA conv, weights read as wave-uniform scalars.
//
// The 16-channel Net buffer g16 holds [x0 0-2 | x1 3-5 | Ft0 6-7 | Ft1 8-9 |
// xt1 10-12 | xt2 13-15].  Every fused update is pointwise (reads and writes of
// g16 at the thread's own pixel only), so in-place writes are race-free.
#include "common.hpp"

namespace rrin {

// ---- head conv ----------------------------------------------------------------
struct HeadArgs {
  const float* src;  // cin-channel PP, channel 0 of image 0
  int64_t src_img, src_plane;
  int src_wp;
  float* g;          // g16 channel 0 of image 0 (or PLAIN dst view)
  int64_t g_img, g_plane;
  int g_wp;
  const float* w;    // OIHW
  const float* bias;
  const float* coef; // [n][8]
  float* out;        // FINAL: NCHW
  float* flow_raw;   // FLOW: raw output (4 PP planes), nullable
  int64_t fr_img, fr_plane;
  int fr_wp;
  int h, w_, tiles_x, tiles_y;
  float* raw;        // optional: conv output before the glue, NCHW
};

constexpr int HC = 8;        // channels per staged chunk
constexpr int HROWS = 10;    // 8 output rows + halo
constexpr int HLC = 40;
constexpr int HIN_V4 = HC * HROWS * HLC / 4;  // 800

template <int COUT, int MODE>
__global__ void __launch_bounds__(256) head_kernel(HeadArgs a) {
  constexpr int CIN = 32;
  __shared__ __attribute__((aligned(16))) float s_in[HC * HROWS * HLC];
  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int img = bid / a.tiles_y;
  const int x0 = tx * 32, y0 = ty * 8;
  const int r = tid >> 5, xl = tid & 31;

  float acc[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc[co] = a.bias[co];

  const float* src_img = a.src + img * a.src_img;
  for (int c = 0; c < CIN / HC; ++c) {
    float4* s4 = reinterpret_cast<float4*>(s_in);
#pragma unroll
    for (int it = 0; it < (HIN_V4 + 255) / 256; ++it) {
      const int idx = tid + 256 * it;
      if (idx < HIN_V4) {
        const int ci = idx / (HROWS * 10);
        const int rem = idx - ci * (HROWS * 10);
        const int rr = rem / 10;
        const int q = rem - rr * 10;
        s4[idx] = *reinterpret_cast<const float4*>(src_img + (int64_t)(c * HC + ci) * a.src_plane +
                                                   (int64_t)(y0 + rr) * a.src_wp + x0 + (kPadLeft - 4) + 4 * q);
      }
    }
    __syncthreads();
#pragma unroll
    for (int ci = 0; ci < HC; ++ci) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float v = s_in[(ci * HROWS + r + ky) * HLC + xl + 3 + kx];
#pragma unroll
          for (int co = 0; co < COUT; ++co)
            acc[co] = fmaf(a.w[((co * CIN) + c * HC + ci) * 9 + ky * 3 + kx], v, acc[co]);
        }
      }
    }
    __syncthreads();
  }

  const int y = y0 + r, x = x0 + xl;
  if (y >= a.h || x >= a.w_) return;
  float* gi = a.g + img * a.g_img;
  const int64_t pix = (int64_t)(y + 1) * a.g_wp + x + kPadLeft;
  auto G = [&](int ch) -> float& { return gi[(int64_t)ch * a.g_plane + pix]; };
  const float* cf = a.coef + img * 8;
  if (a.raw)
#pragma unroll
    for (int co = 0; co < COUT; ++co) a.raw[(((int64_t)img * COUT + co) * a.h + y) * a.w_ + x] = acc[co];

  if constexpr (MODE == RRIN_HEAD_PLAIN) {
#pragma unroll
    for (int co = 0; co < COUT; ++co) G(co) = acc[co];
  } else if constexpr (MODE == RRIN_HEAD_FLOW) {
    // Ft0 = (-(1-t)t)*F01 + (t*t)*F10 ; Ft1 = ((1-t)^2)*F01 - (t(1-t))*F10
#pragma clang fp contract(off)
    if (a.flow_raw) {
      float* fr = a.flow_raw + img * a.fr_img + (int64_t)(y + 1) * a.fr_wp + x + kPadLeft;
      for (int k = 0; k < 4; ++k) fr[k * a.fr_plane] = acc[k];
    }
    for (int k = 0; k < 2; ++k) {
      G(6 + k) = cf[0] * acc[k] + cf[1] * acc[2 + k];
      G(8 + k) = cf[2] * acc[k] - cf[3] * acc[2 + k];
    }
  } else if constexpr (MODE == RRIN_HEAD_REFINE) {
#pragma clang fp contract(off)
    const float f0u = G(6) + acc[0], f0v = G(7) + acc[1];
    const float f1u = G(8) + acc[2], f1v = G(9) + acc[3];
    G(6) = f0u;
    G(7) = f0v;
    G(8) = f1u;
    G(9) = f1v;
    const int64_t off = (int64_t)a.g_wp + kPadLeft;  // pixel (0,0) inside a plane
    const WarpTaps t0 = warp_taps(x, y, f0u, f0v, a.h, a.w_);
    const WarpTaps t1 = warp_taps(x, y, f1u, f1v, a.h, a.w_);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      G(10 + ch) = warp_apply(t0, gi + (int64_t)ch * a.g_plane, a.g_wp, off);
      G(13 + ch) = warp_apply(t1, gi + (int64_t)(3 + ch) * a.g_plane, a.g_wp, off);
    }
  } else if constexpr (MODE == RRIN_HEAD_MASK) {
#pragma clang fp contract(off)
    const float m0 = 1.0f / (1.0f + expf(-acc[0]));
    const float m1 = 1.0f / (1.0f + expf(-acc[1]));
    const float w1 = cf[4] * m0, w2 = cf[5] * m1;
    const float den = w1 + w2 + 1e-8f;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) G(6 + ch) = (w1 * G(10 + ch) + w2 * G(13 + ch)) / den;
  } else {  // FINAL
#pragma clang fp contract(off)
    float* o = a.out + ((int64_t)img * 3) * a.h * a.w_ + (int64_t)y * a.w_ + x;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float v = acc[ch] + G(6 + ch);
      o[(int64_t)ch * a.h * a.w_] = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);  // NaN passes
    }
  }
}

template <int COUT, int MODE>
static int head_launch(const HeadArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((head_kernel<COUT, MODE>), dim3(grid), dim3(256), 0, st, a);
  return hip_code(hipGetLastError());
}

// ---- layout kernels -----------------------------------------------------------
__global__ void nchw_to_pp_kernel(const float* __restrict__ src, float* dst, int64_t dst_img,
                                  int64_t plane, int wp, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  dst[n * dst_img + ch * plane + (int64_t)(y + 1) * wp + x + kPadLeft] = src[i];
}

__global__ void pp_to_nchw_kernel(const float* __restrict__ src, int64_t src_img, int64_t plane,
                                  int wp, float* dst, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  dst[i] = src[n * src_img + ch * plane + (int64_t)(y + 1) * wp + x + kPadLeft];
}

__global__ void warp_nchw_kernel(const float* __restrict__ img, const float* __restrict__ flow,
                                 float* out, int c, int h, int w, int64_t total) {
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
  for (int ch = 0; ch < c; ++ch) {
    const float* plane = img + ((int64_t)n * c + ch) * hw;
    out[((int64_t)n * c + ch) * hw + (int64_t)y * w + x] = warp_apply(tp, plane, w, 0);
  }
}

__global__ void flow_tblend_kernel(const float* __restrict__ fr, int64_t fr_img, int64_t fr_plane, int fr_wp,
                                   float* g, int64_t g_img, int64_t g_plane, int g_wp, const float* coef, int h,
                                   int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int img = (int)(t / h);
  const float* f = fr + img * fr_img + (int64_t)(y + 1) * fr_wp + x + kPadLeft;
  float* gp = g + img * g_img + (int64_t)(y + 1) * g_wp + x + kPadLeft;
  const float* cf = coef + img * 8;
  for (int k = 0; k < 2; ++k) {
#pragma clang fp contract(off)
    const float f01 = f[k * fr_plane], f10 = f[(2 + k) * fr_plane];
    gp[(6 + k) * g_plane] = cf[0] * f01 + cf[1] * f10;
    gp[(8 + k) * g_plane] = cf[2] * f01 - cf[3] * f10;
  }
}

}  // namespace rrin

using namespace rrin;

extern "C" int rrin_flow_tblend_fwd(const rrin_pp* fr, const rrin_pp* g16, const float* coef, int32_t n,
                                    void* stream) {
  if (!fr || !g16 || !fr->base || !g16->base || !coef || n < 1) return RRIN_E_ARG;
  if (fr->channels < 4 || g16->channels < 16 || g16->ch_off != 0) return RRIN_E_ARG;
  if (fr->g.h != g16->g.h || fr->g.w != g16->g.w) return RRIN_E_SHAPE;
  const int64_t total = (int64_t)n * g16->g.h * g16->g.w;
  hipLaunchKernelGGL(flow_tblend_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, fr->base + (int64_t)fr->ch_off * fr->g.plane, fr->img_stride,
                     fr->g.plane, fr->g.wp, g16->base, g16->img_stride, g16->g.plane, g16->g.wp, coef,
                     g16->g.h, g16->g.w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_head_fwd(const rrin_head_desc* d, void* stream) {
  if (!d || !d->src.base || !d->g16.base || !d->w || !d->bias) return RRIN_E_ARG;
  if (d->cin != 32 || d->n < 1) return RRIN_E_ARG;
  const int h = d->src.g.h, w = d->src.g.w;
  if (d->g16.g.h != h || d->g16.g.w != w) return RRIN_E_SHAPE;
  const rrin_geom gg = make_geom(h, w);
  if (gg.wp != d->src.g.wp || gg.hp != d->src.g.hp || gg.wp != d->g16.g.wp || gg.hp != d->g16.g.hp)
    return RRIN_E_SHAPE;
  if (d->src.channels < 32) return RRIN_E_ARG;
  if (d->mode != RRIN_HEAD_PLAIN) {
    if (d->g16.channels < 16 || d->g16.ch_off != 0 || !d->coef) return RRIN_E_ARG;
  } else if (d->g16.channels < d->cout) {
    return RRIN_E_ARG;
  }
  if (d->mode == RRIN_HEAD_FINAL && !d->out) return RRIN_E_ARG;
  HeadArgs a;
  a.src = d->src.base + (int64_t)d->src.ch_off * d->src.g.plane;
  a.src_img = d->src.img_stride;
  a.src_plane = d->src.g.plane;
  a.src_wp = d->src.g.wp;
  a.g = d->g16.base + (int64_t)d->g16.ch_off * d->g16.g.plane;
  a.g_img = d->g16.img_stride;
  a.g_plane = d->g16.g.plane;
  a.g_wp = d->g16.g.wp;
  a.w = d->w;
  a.bias = d->bias;
  a.coef = d->coef;
  a.out = d->out;
  a.raw = d->raw_out;
  a.flow_raw = nullptr;
  if (d->mode == RRIN_HEAD_FLOW && d->flow_raw.base) {
    if (d->flow_raw.channels < 4 || d->flow_raw.g.h != h || d->flow_raw.g.w != w || d->flow_raw.g.wp != gg.wp)
      return RRIN_E_SHAPE;
    a.flow_raw = d->flow_raw.base + (int64_t)d->flow_raw.ch_off * d->flow_raw.g.plane;
    a.fr_img = d->flow_raw.img_stride;
    a.fr_plane = d->flow_raw.g.plane;
    a.fr_wp = d->flow_raw.g.wp;
  }
  a.h = h;
  a.w_ = w;
  a.tiles_x = (w + 31) / 32;
  a.tiles_y = (h + 7) / 8;
  const int grid = a.tiles_x * a.tiles_y * d->n;
  hipStream_t st = (hipStream_t)stream;
  switch (d->mode) {
    case RRIN_HEAD_PLAIN:
      if (d->cout == 1) return head_launch<1, RRIN_HEAD_PLAIN>(a, grid, st);
      if (d->cout == 2) return head_launch<2, RRIN_HEAD_PLAIN>(a, grid, st);
      if (d->cout == 3) return head_launch<3, RRIN_HEAD_PLAIN>(a, grid, st);
      if (d->cout == 4) return head_launch<4, RRIN_HEAD_PLAIN>(a, grid, st);
      return RRIN_E_ARG;
    case RRIN_HEAD_FLOW:
      return d->cout == 4 ? head_launch<4, RRIN_HEAD_FLOW>(a, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_REFINE:
      return d->cout == 4 ? head_launch<4, RRIN_HEAD_REFINE>(a, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_MASK:
      return d->cout == 2 ? head_launch<2, RRIN_HEAD_MASK>(a, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_FINAL:
      return d->cout == 3 ? head_launch<3, RRIN_HEAD_FINAL>(a, grid, st) : RRIN_E_ARG;
  }
  return RRIN_E_ARG;
}

static inline bool pp_ok(const rrin_pp* v) {
  if (!v || !v->base) return false;
  const rrin_geom g = make_geom(v->g.h, v->g.w);
  return g.wp == v->g.wp && g.hp == v->g.hp && g.plane == v->g.plane;
}

extern "C" int rrin_nchw_to_pp(const float* src, int32_t n, int32_t c, const rrin_pp* dst, void* stream) {
  if (!src || !pp_ok(dst) || n < 1 || c < 1 || c > dst->channels) return RRIN_E_ARG;
  const int64_t total = (int64_t)n * c * dst->g.h * dst->g.w;
  const int grid = (int)((total + 255) / 256);
  hipLaunchKernelGGL(nchw_to_pp_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src,
                     dst->base + (int64_t)dst->ch_off * dst->g.plane, dst->img_stride, dst->g.plane,
                     dst->g.wp, c, dst->g.h, dst->g.w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_pp_to_nchw(const rrin_pp* src, int32_t n, int32_t c, float* dst, void* stream) {
  if (!dst || !pp_ok(src) || n < 1 || c < 1 || c > src->channels) return RRIN_E_ARG;
  const int64_t total = (int64_t)n * c * src->g.h * src->g.w;
  const int grid = (int)((total + 255) / 256);
  hipLaunchKernelGGL(pp_to_nchw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     src->base + (int64_t)src->ch_off * src->g.plane, src->img_stride, src->g.plane,
                     src->g.wp, dst, c, src->g.h, src->g.w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_warp_fwd(const float* img, const float* flow, float* out, int32_t n, int32_t c,
                             int32_t h, int32_t w, void* stream) {
  if (!img || !flow || !out || n < 1 || c < 1 || h < 1 || w < 1) return RRIN_E_ARG;
  const int64_t total = (int64_t)n * h * w;
  const int grid = (int)((total + 255) / 256);
  hipLaunchKernelGGL(warp_nchw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, img, flow, out, c,
                     h, w, total);
  return hip_code(hipGetLastError());
}
