// conv3x3 (pad 1) + bias [+ LeakyReLU] [+ fused 2x2 avg-pool output]
// [+ fused bilinear x2 upsample of the input] as an implicit GEMM on the gfx950
// f32-input matrix cores (v_mfma_f32_32x32x2_f32: exact fp32, fmaf chain).
//
// Replaces, per SURVEY.md §8(a) rows a6-a9:
//   nn.Conv2d(k=3,pad=1)       /root/reference/unet.py:29,59,62,78
//   LeakyReLU(0.1)             unet.py:47,60,63  (epilogue)
//   F.avg_pool2d(x,2)          unet.py:46        (second output of the epilogue)
//   nn.Upsample(bilinear,x2)   unet.py:77        (input staging)
//   torch.cat((up,bridge),1)   unet.py:93        (channel-offset addressing)
//
// GEMM view: D[co][p] = sum_k W[co][k] * X[k][p], k = (ci, ky, kx).
// A block owns BM output channels x (TH rows x 32 cols) output pixels and walks
// K in chunks of 8 input channels x 9 taps.  Per chunk it stages into LDS
//   input  [8 ch][TH+2 rows][40 cols]  (cols x0-4 .. x0+35, 16-B vector loads)
//   weight [8 ch][9 taps][BM]          (pre-packed, one contiguous slab)
// double-buffered: chunk c+1 is staged by LDS-DMA (global_load_lds_dwordx4)
// while the MFMAs run on chunk c (UPSAMPLE2X: register prefetch of the low-res
// tile + expansion in LDS).
// One 32x32x2 MFMA covers a channel PAIR at one tap: lanes 0-31 carry channel
// 2p, lanes 32-63 channel 2p+1, so every operand read is one conflict-free
// ds_read_b32 with a compile-time immediate offset.
#include "common.hpp"

namespace rrin {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct ConvArgs {
  const float* src;
  int64_t src_img, src_plane;
  int src_wp, src_h, src_w;     // src logical size (h/2,w/2 when upsampling)
  int cin, nchunks;
  float* dst;
  int64_t dst_img, dst_plane;
  int dst_wp, cout;
  float* pool;
  int64_t pool_img, pool_plane;
  int pool_wp;
  const float* wpack;
  const float* bias;
  int h, w;                     // output size
  int co_blocks, tiles_x, tiles_y, n;
  float slope;
};

constexpr int CK = 8;     // input channels per K chunk
constexpr int LC = 40;    // LDS row length (floats): cols x0-4 .. x0+35

template <int WAVES_M, int WAVES_N, int WM, int WN>
struct Tile {
  static constexpr int BM = 32 * WM * WAVES_M;
  static constexpr int TH = WN * WAVES_N;
  static constexpr int ROWS = TH + 2;
  static constexpr int IN_F = CK * ROWS * LC;
  static constexpr int W_F = CK * 9 * BM;
  static constexpr int IN_V4 = IN_F / 4;
  static constexpr int W_V4 = W_F / 4;
  static constexpr int IN_IT = (IN_V4 + 255) / 256;
  static constexpr int W_IT = (W_V4 + 255) / 256;
  static constexpr int LR_ROWS = TH / 2 + 2;
  static constexpr int LR_COLS = 20;
  static constexpr int LR_F = CK * LR_ROWS * LR_COLS;
  static constexpr int LR_IT = (LR_F + 255) / 256;
  static constexpr size_t LDS_BYTES = 2 * (size_t)(IN_F + W_F) * sizeof(float);
  static constexpr size_t LDS_BYTES_UP = LDS_BYTES + (size_t)LR_F * sizeof(float);
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
  static_assert(16 % TH == 0, "TH must divide the 16-row plane padding");
};

// Lab-only ablations (template SCHED, librrin_lab32.so; wrong outputs, they
// time what is left): NO_DMA skips staging later chunks (keeps computing on
// chunk 0), NO_MFMA keeps the LDS operand reads but drops the MFMAs, NO_EPI
// drops the epilogue stores, NO_SYNC drops the per-chunk wait + barrier.
enum : int { S32_NO_DMA = 1, S32_NO_MFMA = 2, S32_NO_EPI = 4, S32_NO_SYNC = 8 };

template <int WAVES_M, int WAVES_N, int WM, int WN, int SRC, int EPI, int SCHED = 0>
__global__ void __launch_bounds__(256) conv3x3_mfma_kernel(ConvArgs a) {
  using T = Tile<WAVES_M, WAVES_N, WM, WN>;
  constexpr bool kNoDma = (SCHED & S32_NO_DMA) != 0, kNoMfma = (SCHED & S32_NO_MFMA) != 0;
  constexpr bool kNoEpi = (SCHED & S32_NO_EPI) != 0, kNoSync = (SCHED & S32_NO_SYNC) != 0;
  constexpr int BM = T::BM, TH = T::TH, ROWS = T::ROWS;
  constexpr int IN_F = T::IN_F, W_F = T::W_F;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_in = smem;            // [2][IN_F]
  float* s_w = smem + 2 * IN_F;  // [2][W_F]
  float* s_lr = s_w + 2 * W_F;   // [LR_F] low-res tile (UPSAMPLE2X)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;
  const int j = lane & 31;
  const int hh = lane >> 5;

  // XCD-aware remap (bijective): hardware deals blocks round-robin over the 8
  // XCDs, so give each XCD one contiguous run of logical blocks.  Logical order
  // has the co-blocks of a tile adjacent, then neighbouring tiles: blocks that
  // stage the same input rows share one L2.  Placement affects speed only.
  int bid;
  {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int cob = bid % a.co_blocks;
  bid /= a.co_blocks;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int img = bid / a.tiles_y;
  const int x0 = tx * 32;
  const int y0 = ty * TH;

  const float* src_img = a.src + img * a.src_img;
  const float* wsrc = a.wpack + (int64_t)cob * a.nchunks * W_F;

  float4 rw[SRC == RRIN_SRC_DIRECT ? 1 : T::W_IT];

  // DIRECT: LDS-DMA staging (global_load_lds_dwordx4, lane-linear LDS image,
  // no staging VGPRs, no LDS store pass).  Channels past cin source the zero
  // top-padding row.
  auto dma16 = [&](const float* g, float* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
  };
  auto issue = [&](int c, int buf) {
#pragma unroll
    for (int it = 0; it < T::IN_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::IN_V4) {
        const int ci = idx / (ROWS * 10);
        const int rem = idx - ci * (ROWS * 10);
        const int r = rem / 10;
        const int q = rem - r * 10;
        const int ch = c * CK + ci;
        const int64_t off = ch < a.cin ? (int64_t)ch * a.src_plane + (int64_t)(y0 + r) * a.src_wp + x0 +
                                             (kPadLeft - 4) + 4 * q
                                       : (int64_t)(x0 + (kPadLeft - 4) + 4 * q);
        dma16(src_img + off, s_in + buf * IN_F + 4 * (256 * it + wave * 64));
      }
    }
    const float* g = wsrc + (int64_t)c * W_F;
#pragma unroll
    for (int it = 0; it < T::W_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::W_V4) dma16(g + 4 * idx, s_w + buf * W_F + 4 * (256 * it + wave * 64));
    }
  };

  auto load_w = [&](int c) {
    const float4* g = reinterpret_cast<const float4*>(wsrc + (int64_t)c * W_F);
#pragma unroll
    for (int it = 0; it < T::W_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::W_V4) rw[it] = g[idx];
    }
  };
  auto store_w = [&](int buf) {
    float4* s = reinterpret_cast<float4*>(s_w + buf * W_F);
#pragma unroll
    for (int it = 0; it < T::W_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::W_V4) s[idx] = rw[it];
    }
  };
  // UPSAMPLE2X (unet.py:77, bilinear x2, align_corners=False).  The low-res
  // tile this block needs (TH/2+2 rows x 20 cols per channel, edge-clamped
  // coordinates) is prefetched into registers during the MFMAs, stored to LDS,
  // and expanded there into the hi-res input tile, two output columns per item:
  //   X = 2i   : .25 L[i-1] + .75 L[i]      X = 2i+1 : .75 L[i] + .25 L[i+1]
  // (rows likewise; clamping is carried by the clamped loads).  Positions
  // outside the hi-res frame are the conv's zero padding.
  const int ly0 = y0 / 2 - 1, lx0 = x0 / 2 - 2;
  float rlr[T::LR_IT];
  auto load_lr = [&](int c) {
#pragma unroll
    for (int it = 0; it < T::LR_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::LR_F) {
        const int ci = idx / (T::LR_ROWS * T::LR_COLS);
        const int rem = idx - ci * (T::LR_ROWS * T::LR_COLS);
        const int r = rem / T::LR_COLS;
        const int q = rem - r * T::LR_COLS;
        const int ch = c * CK + ci;
        const int yy = min(max(ly0 + r, 0), a.src_h - 1);
        const int xx = min(max(lx0 + q, 0), a.src_w - 1);
        rlr[it] = ch < a.cin ? src_img[(int64_t)ch * a.src_plane + (int64_t)(yy + 1) * a.src_wp + xx + kPadLeft] : 0.f;
      }
    }
  };
  auto expand_up = [&](int buf) {
#pragma unroll
    for (int it = 0; it < T::LR_IT; ++it) {
      const int idx = tid + 256 * it;
      if (idx < T::LR_F) s_lr[idx] = rlr[it];
    }
    __syncthreads();
    float* so = s_in + buf * IN_F;
    constexpr int PAIRS = 18;  // i = x0/2-1 .. x0/2+16 -> X = x0-2 .. x0+33 (LDS cols 2..37)
    constexpr int ITEMS = CK * ROWS * PAIRS;
#pragma unroll
    for (int it = 0; it < (ITEMS + 255) / 256; ++it) {
      const int idx = tid + 256 * it;
      if (idx < ITEMS) {
        const int ci = idx / (ROWS * PAIRS);
        const int rem = idx - ci * (ROWS * PAIRS);
        const int r = rem / PAIRS;
        const int pi = rem - r * PAIRS;
        const int Y = y0 - 1 + r;
        const int Xe = x0 - 2 + 2 * pi;  // even output column of the pair
        float2 o = make_float2(0.f, 0.f);
        if (Y >= 0 && Y < a.h) {
          const int iy = Y >> 1;
          const int ra = (Y & 1) ? iy : iy - 1;         // upper source row
          const float wa = (Y & 1) ? 0.75f : 0.25f;      // its weight
          const float* la = s_lr + (ci * T::LR_ROWS + (ra - ly0)) * T::LR_COLS + (x0 / 2 - 1 + pi - lx0);
          const float* lb = la + T::LR_COLS;
          const float wb = 1.0f - wa;
          // horizontal first, then vertical (the order of upsample_bilinear2d)
          const float ae = 0.25f * la[-1] + 0.75f * la[0], ao = 0.75f * la[0] + 0.25f * la[1];
          const float be = 0.25f * lb[-1] + 0.75f * lb[0], bo = 0.75f * lb[0] + 0.25f * lb[1];
          if (Xe >= 0 && Xe < a.w) o.x = wa * ae + wb * be;
          if (Xe + 1 >= 0 && Xe + 1 < a.w) o.y = wa * ao + wb * bo;
        }
        *reinterpret_cast<float2*>(so + (ci * ROWS + r) * LC + 2 + 2 * pi) = o;
      }
    }
  };

  floatx16 acc[WM][WN];
#pragma unroll
  for (int mt = 0; mt < WM; ++mt)
#pragma unroll
    for (int nt = 0; nt < WN; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.f;

  // 36 k-steps (4 channel pairs x 9 taps) per chunk; operands of step s+1 are
  // read from LDS before the MFMAs of step s issue, so the ds_read latency
  // hides under 64-cycle MFMAs instead of stalling in front of them.
  auto compute = [&](int buf) {
    const float* si = s_in + buf * IN_F + hh * ROWS * LC + (wn * WN) * LC + j + 3;
    const float* sw = s_w + buf * W_F + hh * 9 * BM + (wm * WM) * 32 + j;
    float av[2][WM], bv[2][WN];
    auto ld = [&](int st, int slot) {
      const int cp = st / 9, tap = st % 9, ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) av[slot][mt] = sw[(2 * cp * 9 + tap) * BM + mt * 32];
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) bv[slot][nt] = si[(2 * cp * ROWS + nt + ky) * LC + kx];
    };
    ld(0, 0);
#pragma unroll
    for (int st = 0; st < (CK / 2) * 9; ++st) {
      if (st + 1 < (CK / 2) * 9) ld(st + 1, (st + 1) & 1);
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt) {
          if constexpr (kNoMfma)
            asm volatile("" ::"v"(av[st & 1][mt]), "v"(bv[st & 1][nt]));
          else
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[st & 1][mt], bv[st & 1][nt], acc[mt][nt], 0, 0, 0);
        }
    }
  };

  if constexpr (SRC == RRIN_SRC_DIRECT) {
    // ---- DMA pipeline: chunk c+1 lands in buf^1 while the MFMAs run on c
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c < a.nchunks; ++c) {
      const int buf = kNoDma ? 0 : c & 1;
      if (!kNoDma && (c + 1) < a.nchunks) issue(c + 1, buf ^ 1);  // buf^1 last read before the previous barrier
      compute(buf);
      if constexpr (!kNoSync) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    // ---- UPSAMPLE2X: register prefetch of weights + low-res tile, LDS expansion
    load_w(0);
    load_lr(0);
    expand_up(0);
    store_w(0);
    __syncthreads();
    for (int c = 0; c < a.nchunks; ++c) {
      const int buf = c & 1;
      const bool more = (c + 1) < a.nchunks;
      if (more) {
        load_w(c + 1);
        load_lr(c + 1);
      }
      compute(buf);
      if (more) {
        expand_up(buf ^ 1);  // contains one extra barrier (s_lr hand-off)
        store_w(buf ^ 1);
      }
      __syncthreads();
    }
  }

  // ---- epilogue: bias, leaky, store (+ 2x2 average pool)
  if constexpr (kNoEpi) {
#pragma unroll
    for (int mt = 0; mt < WM; ++mt)
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(acc[mt][nt][i]));
    return;
  }
  const int yb = y0 + wn * WN;
  const int x = x0 + j;
#pragma unroll
  for (int mt = 0; mt < WM; ++mt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = cob * BM + (wm * WM + mt) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      const float bias = a.bias[co];
      float v[WN];
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        float t = acc[mt][nt][i] + bias;
        if constexpr (EPI != RRIN_EPI_LINEAR) t = t > 0.f ? t : t * a.slope;
        v[nt] = t;
        const int y = yb + nt;
        if (co < a.cout && y < a.h && x < a.w)
          a.dst[img * a.dst_img + (int64_t)co * a.dst_plane + (int64_t)(y + 1) * a.dst_wp + x + kPadLeft] = t;
      }
      if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
#pragma unroll
        for (int p = 0; p < WN / 2; ++p) {
          float s = v[2 * p] + v[2 * p + 1];
          s += __shfl_xor(s, 1);
          const int y = yb + 2 * p;
          if (!(j & 1) && co < a.cout && y < a.h && x < a.w)
            a.pool[img * a.pool_img + (int64_t)co * a.pool_plane + (int64_t)(y / 2 + 1) * a.pool_wp +
                   x / 2 + kPadLeft] = 0.25f * s;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------
// Config table.  cfg -> (WAVES_M, WAVES_N, WM, WN)
//   0: BM 32,  TH 8   (1x4 waves, 32co x 2 rows each)
//   1: BM 64,  TH 8   (1x4 waves, 64co x 2 rows each)
//   2: BM 128, TH 4   (2x2 waves, 64co x 2 rows each)
//   3: BM 32,  TH 16  (1x4 waves, 32co x 4 rows each)
//   4: BM 64,  TH 4   (2x2 waves, 32co x 2 rows each)
//   5: BM 128, TH 8   (1x4 waves, 128co x 2 rows each)
#define RRIN_CONV_CFGS(X) \
  X(0, 1, 4, 1, 2)        \
  X(1, 1, 4, 2, 2)        \
  X(2, 2, 2, 2, 2)        \
  X(3, 1, 4, 1, 4)        \
  X(4, 2, 2, 1, 2)        \
  X(5, 1, 4, 4, 2)

struct CfgInfo {
  int bm, th;
  size_t lds;
};

static const CfgInfo kCfg[] = {
#define X(id, a, b, c, d) {Tile<a, b, c, d>::BM, Tile<a, b, c, d>::TH, Tile<a, b, c, d>::LDS_BYTES},
    RRIN_CONV_CFGS(X)
#undef X
};
static constexpr int kNumCfg = sizeof(kCfg) / sizeof(kCfg[0]);

template <int A, int B, int C, int D, int SRC, int EPI, int SCHED = 0>
static int launch_t(const ConvArgs& args, int grid, hipStream_t st) {
  using T = Tile<A, B, C, D>;
  constexpr size_t lds = SRC == RRIN_SRC_UPSAMPLE2X ? T::LDS_BYTES_UP : T::LDS_BYTES;
  auto k = conv3x3_mfma_kernel<A, B, C, D, SRC, EPI, SCHED>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)lds, st)) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, args);
  return hip_code(hipGetLastError());
}

template <int A, int B, int C, int D>
static int launch_cfg(const ConvArgs& args, int src, int epi, int grid, hipStream_t st) {
  if (src == RRIN_SRC_DIRECT) {
    if (epi == RRIN_EPI_LINEAR) return launch_t<A, B, C, D, RRIN_SRC_DIRECT, RRIN_EPI_LINEAR>(args, grid, st);
    if (epi == RRIN_EPI_LEAKY) return launch_t<A, B, C, D, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY>(args, grid, st);
    return launch_t<A, B, C, D, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY_POOL>(args, grid, st);
  }
  if (epi == RRIN_EPI_LINEAR) return launch_t<A, B, C, D, RRIN_SRC_UPSAMPLE2X, RRIN_EPI_LINEAR>(args, grid, st);
  if (epi == RRIN_EPI_LEAKY) return launch_t<A, B, C, D, RRIN_SRC_UPSAMPLE2X, RRIN_EPI_LEAKY>(args, grid, st);
  return launch_t<A, B, C, D, RRIN_SRC_UPSAMPLE2X, RRIN_EPI_LEAKY_POOL>(args, grid, st);
}

}  // namespace rrin

using namespace rrin;

extern "C" int rrin_conv_cfg_count(void) { return kNumCfg; }
extern "C" int rrin_conv_cfg_bm(int32_t cfg) { return (cfg >= 0 && cfg < kNumCfg) ? kCfg[cfg].bm : RRIN_E_CONFIG; }
extern "C" int rrin_conv_cfg_th(int32_t cfg) { return (cfg >= 0 && cfg < kNumCfg) ? kCfg[cfg].th : RRIN_E_CONFIG; }

// Validate a descriptor and fill the kernel arguments; grid = one block per tile.
static int conv_prepare(const rrin_conv_desc* d, ConvArgs& a, int& grid_out) {
  if (!d || !d->src.base || !d->dst.base || !d->wpack || !d->bias) return RRIN_E_ARG;
  if (d->cfg < 0 || d->cfg >= kNumCfg) return RRIN_E_CONFIG;
  if (d->n < 1 || d->cin < 1 || d->cout < 1) return RRIN_E_ARG;
  if (d->src_mode != RRIN_SRC_DIRECT && d->src_mode != RRIN_SRC_UPSAMPLE2X) return RRIN_E_ARG;
  if (d->epi_mode < RRIN_EPI_LINEAR || d->epi_mode > RRIN_EPI_LEAKY_POOL) return RRIN_E_ARG;
  const CfgInfo& ci = kCfg[d->cfg];
  const int h = d->dst.g.h, w = d->dst.g.w;
  if (d->cin > d->src.channels || d->cout > d->dst.channels) return RRIN_E_ARG;
  if (d->src_mode == RRIN_SRC_DIRECT) {
    if (d->src.g.h != h || d->src.g.w != w) return RRIN_E_SHAPE;
  } else {
    if (d->src.g.h * 2 != h || d->src.g.w * 2 != w) return RRIN_E_SHAPE;
  }
  if (d->epi_mode == RRIN_EPI_LEAKY_POOL) {
    if (!d->pool.base || (h & 1) || (w & 1) || d->pool.g.h * 2 != h || d->pool.g.w * 2 != w ||
        d->cout > d->pool.channels)
      return RRIN_E_SHAPE;
  }
  // plane geometry must be the library's (reads past w/h rely on the padding)
  const rrin_geom gs = make_geom(d->src.g.h, d->src.g.w);
  const rrin_geom gd = make_geom(h, w);
  if (gs.wp != d->src.g.wp || gs.hp != d->src.g.hp || gd.wp != d->dst.g.wp || gd.hp != d->dst.g.hp)
    return RRIN_E_SHAPE;

  a = ConvArgs{};
  a.src = d->src.base + (int64_t)d->src.ch_off * d->src.g.plane;
  a.src_img = d->src.img_stride;
  a.src_plane = d->src.g.plane;
  a.src_wp = d->src.g.wp;
  a.src_h = d->src.g.h;
  a.src_w = d->src.g.w;
  a.cin = d->cin;
  a.nchunks = (d->cin + CK - 1) / CK;
  a.dst = d->dst.base + (int64_t)d->dst.ch_off * d->dst.g.plane;
  a.dst_img = d->dst.img_stride;
  a.dst_plane = d->dst.g.plane;
  a.dst_wp = d->dst.g.wp;
  a.cout = d->cout;
  a.pool = nullptr;
  a.pool_img = a.pool_plane = 0;
  a.pool_wp = 0;
  if (d->epi_mode == RRIN_EPI_LEAKY_POOL) {
    a.pool = d->pool.base + (int64_t)d->pool.ch_off * d->pool.g.plane;
    a.pool_img = d->pool.img_stride;
    a.pool_plane = d->pool.g.plane;
    a.pool_wp = d->pool.g.wp;
  }
  a.wpack = d->wpack;
  a.bias = d->bias;
  a.h = h;
  a.w = w;
  a.co_blocks = (d->cout + ci.bm - 1) / ci.bm;
  a.tiles_x = (w + 31) / 32;
  a.tiles_y = (h + ci.th - 1) / ci.th;
  a.n = d->n;
  a.slope = d->slope;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (grid > 0x7fffffff) return RRIN_E_SHAPE;
  grid_out = (int)grid;
  return 0;
}

extern "C" int rrin_conv3x3_fwd(const rrin_conv_desc* d, void* stream) {
  ConvArgs a;
  int grid = 0;
  const int rc = conv_prepare(d, a, grid);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  switch (d->cfg) {
#define X(id, A, B, C, D) \
  case id:                \
    return launch_cfg<A, B, C, D>(a, d->src_mode, d->epi_mode, grid, st);
    RRIN_CONV_CFGS(X)
#undef X
  }
  return RRIN_E_CONFIG;
}

#ifdef RRIN_LAB
// Kernel lab (tools/conv_lab.py ablate32; librrin_lab32.so, `make lab`): one
// direct LEAKY conv of any config with the ablation bits S32_* in `sched`.
template <int A, int B, int C, int D>
static int lab32_cfg(const ConvArgs& a, int sched, int grid, hipStream_t st) {
  switch (sched) {
#define L(v) \
  case v:    \
    return launch_t<A, B, C, D, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, v>(a, grid, st);
    L(0) L(1) L(2) L(3) L(4) L(8) L(9) L(12) L(13)
#undef L
  }
  return RRIN_E_CONFIG;
}

extern "C" int rrin_conv3x3_lab32(const rrin_conv_desc* d, int32_t sched, void* stream) {
  if (!d || d->src_mode != RRIN_SRC_DIRECT || d->epi_mode != RRIN_EPI_LEAKY) return RRIN_E_ARG;
  ConvArgs a;
  int grid = 0;
  const int rc = conv_prepare(d, a, grid);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  switch (d->cfg) {
#define X(id, A, B, C, D) \
  case id:                \
    return lab32_cfg<A, B, C, D>(a, sched, grid, st);
    RRIN_CONV_CFGS(X)
#undef X
  }
  return RRIN_E_CONFIG;
}
#endif
