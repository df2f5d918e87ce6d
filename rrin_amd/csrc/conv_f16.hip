// Split-fp16 ("F16X3") and fp16 ("F16") path of the RRIN hot path on the
// gfx950 f16 matrix cores (v_mfma_f32_32x32x16_f16, fp32 accumulate).
//
// Numerics (F16X3): every fp32 value v lives as hi = f16(v) and a pre-scaled
// lo' = f16((v - hi) * 2^11), so v = hi + lo' 2^-11 to ~2^-22 |v| and lo' stays
// a normal fp16 down to |v| ~ 1e-4.  A product a*w is computed as
// a_hi*w_hi (accumulator acc) + (a_hi*w_lo' + a_lo'*w_hi) (accumulator accx,
// scaled back by 2^-11 in the epilogue) — every term exact in fp32 — with fp32
// accumulation in the MFMA; the dropped lo*lo term is <= 2^-22 |a w|.
// Weights are pre-scaled by 2^s (exact), max |w| 2^s in [2^12, 2^13); the
// epilogue multiplies by 2^-s.  F16 keeps hi only (fp16 configs).
//
// Replaces (as conv_mfma.hip): nn.Conv2d(3,pad=1) + LeakyReLU(0.1)
// (/root/reference/unet.py:29,59-63,78), F.avg_pool2d (unet.py:46, fused second
// output), torch.cat (unet.py:93, channel-offset views); nn.Upsample(bilinear,x2)
// (unet.py:77) runs as its own pass (rrin_upsample2x_h8); the head convs +
// model.py glue as head_h8_kernel.
//
// H8 activation layout: per image and 8-channel group an hp x wp plane of
// 16-B records (8 halves).  A pixel's 8 channels are one record, so the MFMA
// operands (8 consecutive k per lane) are single ds_read_b128s of the staged
// tile, and epilogue stores of 32 pixels x 8 B per half-wave are contiguous.
#include <math.h>
#include <string.h>

#include <type_traits>

#include "common.hpp"
#include "edge_fix.hpp"

namespace rrin {

constexpr int H8_LC = 34;  // staged input row: records of pixels x0-1 .. x0+32

typedef _Float16 half2v __attribute__((ext_vector_type(2)));
// hi/lo split of 4 consecutive channels into two 8-B record halves: hi = RNE fp16
// of v (v_cvt_pk_f16_f32, two values per op), lo = fp16 of (v - hi) * 2^11 as one
// v_fma_mix_f32 (hi read as f16) on v * 2^11 -- the exact difference, so the same
// bits as lo_of (the kernels are built without packed FP32 ops).
__device__ inline void split4(const float* v, uint2& hv, uint2& lv) {
  const half2v h0 = __builtin_convertvector((float2v){v[0], v[1]}, half2v);
  const half2v h1 = __builtin_convertvector((float2v){v[2], v[3]}, half2v);
  const float l0 = fmaf((float)h0[0], -kLoScale, v[0] * kLoScale), l1 = fmaf((float)h0[1], -kLoScale, v[1] * kLoScale);
  const float l2 = fmaf((float)h1[0], -kLoScale, v[2] * kLoScale), l3 = fmaf((float)h1[1], -kLoScale, v[3] * kLoScale);
  hv = make_uint2(__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1));
  lv = make_uint2(__builtin_bit_cast(unsigned, __builtin_convertvector((float2v){l0, l1}, half2v)),
                  __builtin_bit_cast(unsigned, __builtin_convertvector((float2v){l2, l3}, half2v)));
}



template <int NW, int WM, int WN, int PLANES>
struct TileH8 {
  static constexpr int NT = 64 * NW;
  static constexpr int BM = 32 * WM;
  static constexpr int TH = WN * NW;
  static constexpr int ROWS = TH + 2;
  static constexpr int IN_REC = 2 * ROWS * H8_LC;  // per plane: 2 groups x rows x cols
  static constexpr int W_REC = 9 * 2 * BM;          // per plane: taps x halves x co
  static constexpr int IN_IT = (IN_REC + NT - 1) / NT;
  static constexpr int W_IT = (W_REC + NT - 1) / NT;
  static constexpr size_t LDS = 2 * (size_t)PLANES * (IN_REC + W_REC) * 16;
  static_assert(16 % TH == 0, "TH must divide the 16-row plane padding");
};

// keep floats [0, nvalid) of an fp32 record (nvalid in 1..3)
__device__ inline uint4 mask_floats(uint4 v, int nvalid) {
  if (nvalid < 2) v.y = 0u;
  if (nvalid < 3) v.z = 0u;
  v.w = 0u;
  return v;
}

__device__ inline uint4 mask_halves(uint4 v, int nvalid) {
  // keep halves [0, nvalid) of a record (nvalid in 1..7)
  unsigned* d = reinterpret_cast<unsigned*>(&v);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (2 * k >= nvalid)
      d[k] = 0u;
    else if (2 * k + 1 >= nvalid)
      d[k] &= 0xFFFFu;
  }
  return v;
}


// Schedule knobs of the kernel (template SCHED; the cfg table picks them per
// layer, tools/conv_lab.py ablate times them).  SPREAD issues the next chunk's
// DMA pieces between the first kSpreadTaps taps of the current chunk instead
// of in one burst before it; STAGGER lets waves NW/2.. issue theirs after tap
// kStaggerTap instead (the two wave halves of a SIMD then load at different
// times); WRES keeps every weight chunk of the block's channel block resident
// in LDS, staged once per block.  Lab-only ablations (wrong outputs, they time
// what is left): NO_WDMA / NO_IDMA keep reading the chunk-0 weight slab /
// input tile instead of staging later chunks, NO_MFMA keeps the LDS operand
// reads but drops the MFMAs, NO_EPI drops the epilogue; MFMA16 issues every
// 32x32x16 product as two v_mfma_f32_16x16x32_f16 of the same FLOPs on the
// same operands (a clock/throughput probe of the other MFMA shape).
// Epilogue bias of the record kernel: 0 = each epilogue piece loads its 4 bias floats
// just before its stores (then waits out every earlier store of the tile: vmcnt counts
// stores too); 1 = every piece's bias loaded at the start of the epilogue (one wait);
// 2 = loaded at the start of the tile, landed during the chunk loop (no wait, but 16 WM
// more VGPRs live across it).  -1 (default): per tile shape, as measured at C3 fp16
// (profiles/r04/h8_bias/): 2 where the accumulators are small (WM WN <= 2: the level-0
// and level-4 tiles, 6-14 % faster per conv), 1 on the other unspread tiles (cfg 0 -8 %,
// cfg 5 -3 %), 0 on the SPREAD tiles (cfg 10 / 11, which lose 1-7 % with either).
#ifndef RRIN_H8_WIDE
#define RRIN_H8_WIDE 1
#endif
#ifndef RRIN_H8_BIAS
#define RRIN_H8_BIAS -1
#endif

enum : int {
  SCHED_NO_WDMA = 1, SCHED_NO_IDMA = 2, SCHED_NO_MFMA = 4, SCHED_NO_EPI = 8,
  SCHED_SPREAD = 16, SCHED_WRES = 32, SCHED_STAGGER = 64, SCHED_MFMA16 = 128
};
constexpr int kSpreadTaps = 6, kStaggerTap = 3;

// DMA = true: stage with LDS-DMA (requires cin % 8 == 0: no partial channel
// group to mask); false: register staging with masking (first convs, cin 6/9/10).
//
// A block computes the output tiles (BM channels x TH rows x 32 columns of one
// image, channel block fastest) bid, bid + gridDim.x, ...  With a grid of every
// tile that is one tile per block; with a persistent grid (a few blocks per
// CU) chunk 0 of a block's next tile is staged while the last chunk of the
// current one computes, so only its first tile waits for staging.  WRES needs
// every tile of a block in one channel block (gridDim.x % co_blocks == 0).
//
// F32 (exact fp32, "R32" records): a record holds 4 fp32 channels, a chunk is
// 2 groups = 8 input channels, and each tap's K8 block is 4
// v_mfma_f32_32x32x2_f32 (product e: lanes 0-31 channel e, lanes 32-63 channel
// 4+e of the chunk; one ds_read_b128 per operand feeds all 4).  Same tiles,
// LDS images and DMA as the fp16 kernel; weights unscaled; whole-record stores.
template <int NW, int WM, int WN, int PLANES, int EPI, bool DMA, int SCHED = 0, bool F32 = false>
__global__ void RRIN_PK_CONV_ATTR __launch_bounds__(64 * NW) conv3x3_h8_kernel(ConvH8Args a) {
  using T = TileH8<NW, WM, WN, PLANES>;
  // EPI_SUBPIXEL with the ring from scratch in this launch: workgroups [0, nfix) run the FULL
  // fix-up -- one ring tile per 256-thread slice, one K group each (the summation order of every
  // ring_full conv whatever its tile, so the outputs do not depend on the config) -- and leave;
  // the conv tiles follow
  if constexpr (EPI == RRIN_EPI_SUBPIXEL && NW >= 4) {
    if ((int)blockIdx.x < a.nfix) {
      const int vg = threadIdx.x >> 8;
      const int r = (int)blockIdx.x * (NW / 4) + vg;
      const bool act = r < a.fix_real;
      const int rr = act ? r : 0;
      edge_fix_body<PLANES, 1, F32, true>(a.fix, rr % a.fix_gx, (rr / a.fix_gx) % a.fix_gy, rr / (a.fix_gx * a.fix_gy),
                                          vg, act);
      return;
    }
  }
  const int cgrid = (int)gridDim.x - a.nfix, cblk = (int)blockIdx.x - a.nfix;  // the conv's part of the grid
  static_assert(!F32 || PLANES == 1, "fp32 records: one plane");
  constexpr int CPR = F32 ? 4 : 8;  // channels per record
  constexpr int NT = T::NT, BM = T::BM, TH = T::TH, ROWS = T::ROWS;
  constexpr int IN_REC = T::IN_REC, W_REC = T::W_REC;
  constexpr bool kNoW = (SCHED & SCHED_NO_WDMA) != 0, kNoIn = (SCHED & SCHED_NO_IDMA) != 0;
  constexpr bool kNoMfma = (SCHED & SCHED_NO_MFMA) != 0, kNoEpi = (SCHED & SCHED_NO_EPI) != 0;
  constexpr bool kSpread = DMA && (SCHED & SCHED_SPREAD) != 0;
  constexpr bool kStagger = DMA && !kSpread && (SCHED & SCHED_STAGGER) != 0 && NW >= 2;
  constexpr bool kWRes = DMA && (SCHED & SCHED_WRES) != 0;
  constexpr bool kMfma16 = (SCHED & SCHED_MFMA16) != 0;
  constexpr int kBias = RRIN_H8_BIAS >= 0 ? RRIN_H8_BIAS : (WM * WN <= 2 ? 2 : (SCHED & SCHED_SPREAD) ? 0 : 1);
  // whole-record epilogue stores on H8 records (epi_pair; RRIN_H8_WIDE=0: per-piece half-records)
  constexpr bool kWide = RRIN_H8_WIDE && !F32 && EPI != RRIN_EPI_SUBPIXEL;
  // DMA pieces (one 16-B record per thread and plane) of one chunk: input tile, then weight slab
  constexpr int NPIECE = T::IN_IT + (kWRes ? 0 : T::W_IT);

  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  uint4* s_in = smem4;                          // [buf][plane][IN_REC]
  uint4* s_w = smem4 + 2 * PLANES * IN_REC;     // [buf][plane][W_REC]; WRES: [chunk][plane][W_REC]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wn = tid >> 6;  // waves stacked along output rows
  const int j = lane & 31;
  const int hh = lane >> 5;

  int bid;
  {  // XCD-aware bijective remap (see conv_mfma.hip); nfix is a multiple of 8
    const int nwg = cgrid, q = nwg >> 3, r = nwg & 7;
    const int xcd = cblk & 7, slot = cblk >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  struct TileId {
    int cob, x0, y0, img;
  };
  auto tile_id = [&](int t) {
    TileId o;
    o.cob = t % a.co_blocks;
    t /= a.co_blocks;
    o.x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    o.y0 = (t % a.tiles_y) * TH;
    o.img = t / a.tiles_y;
    return o;
  };

  uint4 rin[PLANES][DMA ? 1 : T::IN_IT];
  uint4 rw[PLANES][DMA ? 1 : T::W_IT];

  // LDS-DMA staging of chunk c of tile tl: input piece `it` into buffer buf,
  // weight piece `it` into weight slot `slot` (both planes).  buffer_load ... lds from a
  // per-chunk base (scalar arithmetic) at a per-lane byte offset computed once per kernel:
  // no vector address arithmetic in the chunk loop (it cost ~80 VALU per chunk beside 36
  // MFMAs on the SPREAD tiles, each VALU stalling the MFMA pipe -- DESIGN.md §5e)
  uint32_t in_off[DMA ? T::IN_IT : 1], in_zoff[DMA ? T::IN_IT : 1];
  if constexpr (DMA) {
#pragma unroll
    for (int it = 0; it < T::IN_IT; ++it) {
      const int idx = min(tid + NT * it, IN_REC - 1);
      const int g = idx / (ROWS * H8_LC);
      const int rem = idx - g * (ROWS * H8_LC);
      const int r = rem / H8_LC;
      const int col = rem - r * H8_LC;
      in_off[it] = (uint32_t)(g * a.src_gp + r * a.src_wp + col) * 16u;
      in_zoff[it] = (uint32_t)col * 16u;  // the zero top-padding row of group 0 (groups past cin)
    }
  }
  auto dma_rs = [&](const void* base, uint32_t voff, int soff, uint4* d) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000),
        (__attribute__((address_space(3))) void*)d, 16, voff, soff, 0, 0);
  };
  auto issue_in = [&](const TileId& tl, int c, int buf, int it) {
    // (a full piece needs no lane test: the condition folds for every piece but the last)
    if (NT * (it + 1) <= IN_REC || tid + NT * it < IN_REC) {
      uint4* d = s_in + buf * PLANES * IN_REC + NT * it + (tid & ~63);
      // one base per tile (scalar); the chunk's group pair and the tile row in the lane offset
      const int64_t tb = (int64_t)tl.img * a.src_img + tl.x0 + (kH8PadLeft - 1);
      const uint32_t c0 = (uint32_t)(2 * c) * (uint32_t)a.src_gp * 16u;
      uint32_t vo = in_off[it] + c0 + (uint32_t)tl.y0 * (uint32_t)a.src_wp * 16u;
      // the chunk's second group past cin: its lanes read the zero top-padding row of the
      // chunk's first group instead (uniform test; a select only in that chunk)
      if ((2 * c + 1) * CPR >= a.cin && tid + NT * it >= ROWS * H8_LC) vo = c0 + in_zoff[it];
      dma_rs(a.src_hi + tb, vo, 0, d);
      if constexpr (PLANES == 2) dma_rs(a.src_lo + tb, vo, 0, d + IN_REC);
    }
  };
  auto issue_w = [&](const TileId& tl, int c, int slot, int it) {
    if (NT * (it + 1) <= W_REC || tid + NT * it < W_REC) {
      const int64_t off = ((int64_t)tl.cob * a.nchunks + c) * W_REC;
      uint4* d = s_w + slot * PLANES * W_REC + NT * it + (tid & ~63);
      dma_rs(a.w_hi + off, (uint32_t)tid * 16u, NT * it * 16, d);
      if constexpr (PLANES == 2) dma_rs(a.w_lo + off, (uint32_t)tid * 16u, NT * it * 16, d + W_REC);
    }
  };
  auto issue_piece = [&](const TileId& tl, int c, int buf, int k) {
    if (k < T::IN_IT) {
      if constexpr (!kNoIn) issue_in(tl, c, buf, k);
    } else {
      if constexpr (!kNoW) issue_w(tl, c, buf, k - T::IN_IT);
    }
  };

  auto load_in = [&](const TileId& tl, int c) {
    const uint4* src[2] = {a.src_hi, a.src_lo};
#pragma unroll
    for (int it = 0; it < T::IN_IT; ++it) {
      const int idx = tid + NT * it;
      if (idx < IN_REC) {
        const int g = idx / (ROWS * H8_LC);
        const int rem = idx - g * (ROWS * H8_LC);
        const int r = rem / H8_LC;
        const int col = rem - r * H8_LC;
        const int gg = c * 2 + g;
        const int nval = a.cin - gg * CPR;
        const int64_t off = (int64_t)tl.img * a.src_img + (int64_t)gg * a.src_gp + (int64_t)(tl.y0 + r) * a.src_wp +
                            tl.x0 + (kH8PadLeft - 1) + col;
#pragma unroll
        for (int p = 0; p < PLANES; ++p) {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (nval > 0) {
            v = src[p][off];
            if (nval < CPR) v = F32 ? mask_floats(v, nval) : mask_halves(v, nval);
          }
          rin[p][it] = v;
        }
      }
    }
  };
  auto store_in = [&](int buf) {
#pragma unroll
    for (int p = 0; p < PLANES; ++p)
#pragma unroll
      for (int it = 0; it < T::IN_IT; ++it) {
        const int idx = tid + NT * it;
        if (idx < IN_REC) s_in[(buf * PLANES + p) * IN_REC + idx] = rin[p][it];
      }
  };
  auto load_w = [&](const TileId& tl, int c) {
    const uint4* wsrc[2] = {a.w_hi, a.w_lo};
#pragma unroll
    for (int p = 0; p < PLANES; ++p)
#pragma unroll
      for (int it = 0; it < T::W_IT; ++it) {
        const int idx = tid + NT * it;
        if (idx < W_REC) rw[p][it] = wsrc[p][((int64_t)tl.cob * a.nchunks + c) * W_REC + idx];
      }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int p = 0; p < PLANES; ++p)
#pragma unroll
      for (int it = 0; it < T::W_IT; ++it) {
        const int idx = tid + NT * it;
        if (idx < W_REC) s_w[(buf * PLANES + p) * W_REC + idx] = rw[p][it];
      }
  };

  // acc: hi*hi products; accx (F16X3): hi*lo' + lo'*hi, 2^11 too large
  floatx16 acc[WM][WN], accx[WM][WN];
  floatx4 p16[kMfma16 ? WM : 1][kMfma16 ? WN : 1][2][PLANES];  // MFMA16 probe accumulators

  // 9 taps per chunk; one K16 block = 16 input channels at one tap (lanes
  // 0-31 carry channels 0-7 of the chunk, lanes 32-63 channels 8-15).
  // Operands of tap t+1 are read before the MFMAs of tap t issue; after_tap(t)
  // runs behind tap t's MFMAs (SPREAD / STAGGER: DMA pieces of the next chunk).
  // zc (std::true_type for the tile's first chunk): the first MFMA of each accumulator takes C = 0,
  // so a tile starts without zeroing its accumulator registers
  auto compute_f32 = [&](int buf, int wslot, auto&& after_tap, auto zc) {
    const uint4* si = s_in + (kNoIn ? 0 : buf) * IN_REC + (hh * ROWS + wn * WN) * H8_LC + j;
    const uint4* sw = s_w + (kNoW ? 0 : wslot) * W_REC + hh * BM + j;
    floatx4 av[2][WM], bv[2][WN];
    auto ld = [&](int t, int slot) {
      const int ky = t / 3, kx = t % 3;
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) av[slot][mt] = __builtin_bit_cast(floatx4, sw[t * 2 * BM + mt * 32]);
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) bv[slot][nt] = __builtin_bit_cast(floatx4, si[(nt + ky) * H8_LC + kx]);
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
      const int s = t & 1;
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int mt = 0; mt < WM; ++mt)
#pragma unroll
          for (int nt = 0; nt < WN; ++nt) {
            if constexpr (kNoMfma)
              asm volatile("" ::"v"(av[s][mt][e]), "v"(bv[s][nt][e]));
            else
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                  av[s][mt][e], bv[s][nt][e], decltype(zc)::value && t == 0 && e == 0 ? floatx16{} : acc[mt][nt], 0, 0, 0);
          }
      after_tap(t);
    }
  };
  auto compute = [&](int buf, int wslot, auto&& after_tap, auto zc) {
    if constexpr (F32) {
      compute_f32(buf, wslot, after_tap, zc);
      return;
    }
    constexpr bool kZc = decltype(zc)::value;
    const uint4* si[PLANES];
    const uint4* sw[PLANES];
#pragma unroll
    for (int p = 0; p < PLANES; ++p) {
      si[p] = s_in + ((kNoIn ? 0 : buf) * PLANES + p) * IN_REC + (hh * ROWS + wn * WN) * H8_LC + j;
      sw[p] = s_w + ((kNoW ? 0 : wslot) * PLANES + p) * W_REC + hh * BM + j;
    }
    half8 av[2][PLANES][WM], bv[2][PLANES][WN];
    auto ld = [&](int t, int slot) {
      const int ky = t / 3, kx = t % 3;
#pragma unroll
      for (int p = 0; p < PLANES; ++p) {
#pragma unroll
        for (int mt = 0; mt < WM; ++mt) av[slot][p][mt] = __builtin_bit_cast(half8, sw[p][t * 2 * BM + mt * 32]);
#pragma unroll
        for (int nt = 0; nt < WN; ++nt) bv[slot][p][nt] = __builtin_bit_cast(half8, si[p][(nt + ky) * H8_LC + kx]);
      }
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
      const int s = t & 1;
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt) {
          if constexpr (kNoMfma) {
            asm volatile("" ::"v"(av[s][0][mt]), "v"(bv[s][0][nt]));
            if constexpr (PLANES == 2) asm volatile("" ::"v"(av[s][1][mt]), "v"(bv[s][1][nt]));
          } else if constexpr (kMfma16) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              if constexpr (PLANES == 2) {
                p16[mt][nt][u][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[s][1][mt], bv[s][0][nt],
                                                                           p16[mt][nt][u][1], 0, 0, 0);
                p16[mt][nt][u][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[s][0][mt], bv[s][1][nt],
                                                                           p16[mt][nt][u][1], 0, 0, 0);
              }
              p16[mt][nt][u][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[s][0][mt], bv[s][0][nt],
                                                                         p16[mt][nt][u][0], 0, 0, 0);
            }
          } else {
            if constexpr (PLANES == 2) {
              accx[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s][1][mt], bv[s][0][nt],
                                                                   kZc && t == 0 ? floatx16{} : accx[mt][nt], 0, 0, 0);
              accx[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s][0][mt], bv[s][1][nt], accx[mt][nt], 0, 0, 0);
            }
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s][0][mt], bv[s][0][nt],
                                                                kZc && t == 0 ? floatx16{} : acc[mt][nt], 0, 0, 0);
          }
        }
      after_tap(t);
    }
  };

  // fp16 range guard of the stored values, accumulated per lane over the workgroup's tiles and
  // written once at its end (one conditional store instead of one per epilogue piece)
  bool bad = false;
  // ---- epilogue piece (mt, q) of tile tl: V = the combined accumulators
  // (acc + accx 2^-11, weight scale still applied): scale, bias, leaky, split,
  // 8-B half-record stores (+ pool / edge-replicate / sub-pixel ring scratch).
  // 4 consecutive channels of one pixel (lane hh's share of record co0/8, or
  // the whole fp32 record co0/4 + hh) -> record `rec` of the group plane set `d`
  auto store4 = [&](uint4* const* d, int64_t rec, const float* v) {
    if constexpr (F32) {
      d[0][rec] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                             __float_as_uint(v[3]));
    } else {
      // fp16 range guard: a value fp16 cannot hold would become inf / NaN and
      // could end as a finite but wrong pixel (e.g. a warp of an inf flow
      // samples zeros); flag it (the FINAL head then poisons the output)
      bad |= !(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))) <= kF16Max);
      uint2 hv, lv;
      split4(v, hv, lv);
      reinterpret_cast<uint2*>(d[0] + rec)[hh] = hv;
      if constexpr (PLANES == 2) reinterpret_cast<uint2*>(d[1] + rec)[hh] = lv;
    }
  };
  auto epi_piece = [&](const TileId& tl, const auto& V, int mt, int q, const float* bs) {
    const int cob = tl.cob, x0 = tl.x0, img = tl.img;
    const int yb = tl.y0 + wn * WN;
    const int x = x0 + j;
    uint4* dst[2] = {a.dst_hi + img * a.dst_img, PLANES == 2 ? a.dst_lo + img * a.dst_img : nullptr};
    if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
      // rows co' = (co/8)*32 + phase*8 + co%8: an MFMA row block (mt) is one
      // 8-channel group, q its phase (py, px); LR pixel (y, x) -> HR (2y+py, 2x+px)
      const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
      const int grp = (cob * BM + mt * 32) >> 5;
      if (grp * 32 >= a.cout) return;
      const int py = q >> 1, px = q & 1;
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        const int y = yb + nt;
        if (y >= a.h || x >= a.w) continue;
        const int Y = 2 * y + py, X = 2 * x + px;
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = F32 ? V[mt][nt][4 * q + e] : V[mt][nt][4 * q + e] * a.inv_wscale;
        const int64_t ri = ring_index(Y, X, HH, WW);
        if (ri >= 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) a.edge[((int64_t)img * creal + grp * 8 + 4 * hh + e) * a.ring + ri] = t[e];
        } else {
          const int rg = F32 ? 2 * grp + hh : grp;  // record group of channels grp*8 + 4hh ..
          const int64_t rec = (int64_t)rg * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + X + kH8PadLeft;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = t[e] + bs[e];
          store4(dst, rec, v);
        }
      }
    } else {
      uint4* pdst[2] = {nullptr, nullptr};
      if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
        pdst[0] = a.pool_hi + img * a.pool_img;
        if (PLANES == 2) pdst[1] = a.pool_lo + img * a.pool_img;
      }
      const int co0 = cob * BM + mt * 32 + 8 * q;  // first channel of the 8-channel block
      const int grp = F32 ? (co0 >> 2) + hh : co0 >> 3;  // record group this lane writes
      float v[WN][4];
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        const int y = yb + nt;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = V[mt][nt][4 * q + e];
          t = F32 ? t + bs[e] : t * a.inv_wscale + bs[e];
          if constexpr (EPI != RRIN_EPI_LINEAR) t = leaky(t, a.slope);
          v[nt][e] = t;
        }
        if (co0 < a.cout && y < a.h && x < a.w) {
          const int64_t rec = (int64_t)grp * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
          store4(dst, rec, v[nt]);
          if constexpr (EPI == RRIN_EPI_LEAKY_REP) {
            // edge replicate into the padding ring (read only by a sub-pixel up conv)
            const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
            const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
            for (int dy = dy0; dy <= dy1; ++dy)
              for (int dx = dx0; dx <= dx1; ++dx)
                if (dy | dx) store4(dst, rec + (int64_t)dy * a.dst_wp + dx, v[nt]);
          }
        }
      }
      if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
#pragma unroll
        for (int p2 = 0; p2 < WN / 2; ++p2) {
          float s4[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float s = v[2 * p2][e] + v[2 * p2 + 1][e];
            s4[e] = 0.25f * (s + __shfl_xor(s, 1));
          }
          const int y = yb + 2 * p2;
          if (!(j & 1) && co0 < a.cout && y < a.h && x < a.w) {
            const int64_t rec = (int64_t)grp * a.pool_gp + (int64_t)(y / 2 + 1) * a.pool_wp + x / 2 + kH8PadLeft;
            store4(pdst, rec, s4);
          }
        }
      }
    }
  };
  // ---- epilogue pieces (mt, 2 qp) and (mt, 2 qp + 1) together, H8 records (kWide): each lane
  // forms its two 8-B half-records, halves_to_record (v_permlane32_swap) turns them into one whole
  // 16-B record -- lane (j, hh) stores 8-channel block 2 qp + hh of its pixel -- and the wave
  // stores whole records: half the store instructions of epi_piece, the same bytes and bits.
  // (Not the sub-pixel epilogue: its ring pixels go to the fp32 edge scratch per channel.)
  auto epi_pair = [&](const TileId& tl, const auto& V, int mt, int qp, const float* bs0, const float* bs1) {
    const int cob = tl.cob, x0 = tl.x0, img = tl.img;
    const int yb = tl.y0 + wn * WN;
    const int x = x0 + j;
    uint4* dst[2] = {a.dst_hi + img * a.dst_img, PLANES == 2 ? a.dst_lo + img * a.dst_img : nullptr};
    const int cq0 = cob * BM + mt * 32 + 16 * qp;  // first channel of block 2 qp
    const int col = cq0 + 8 * hh;                  // first channel of the block this lane stores
    float v[2][WN][4];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = V[mt][nt][4 * (2 * qp + k) + e];
          t = t * a.inv_wscale + (k ? bs1 : bs0)[e];
          if constexpr (EPI != RRIN_EPI_LINEAR) t = leaky(t, a.slope);
          v[k][nt][e] = t;
        }
    // range guard on each lane's own values (as store4: only where that block is stored)
    auto guard = [&](const float* u) {
      bad |= !(fmaxf(fmaxf(fabsf(u[0]), fabsf(u[1])), fmaxf(fabsf(u[2]), fabsf(u[3]))) <= kF16Max);
    };
    auto store_rec = [&](uint4* const* d, int64_t rec, const uint4* r) {
      d[0][rec] = r[0];
      if constexpr (PLANES == 2) d[1][rec] = r[1];
    };
    // both blocks' halves -> this lane's whole record (hi, and lo for two planes)
    auto records = [&](const float* u0, const float* u1, uint4* r) {
      uint2 h0, l0, h1, l1;
      split4(u0, h0, l0);
      split4(u1, h1, l1);
      r[0] = halves_to_record(h0, h1);
      if constexpr (PLANES == 2) r[1] = halves_to_record(l0, l1);
    };
#pragma unroll
    for (int nt = 0; nt < WN; ++nt) {
      const int y = yb + nt;
      const bool pix = y < a.h && x < a.w;
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (pix && cq0 + 8 * k < a.cout) guard(v[k][nt]);
      uint4 r[2];
      records(v[0][nt], v[1][nt], r);  // every lane: the swap reads the partner lane
      if (pix && col < a.cout) {
        const int64_t rec = (int64_t)(col >> 3) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
        store_rec(dst, rec, r);
        if constexpr (EPI == RRIN_EPI_LEAKY_REP) {
          // edge replicate into the padding ring (read only by a sub-pixel up conv)
          const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
          const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
          for (int dy = dy0; dy <= dy1; ++dy)
            for (int dx = dx0; dx <= dx1; ++dx)
              if (dy | dx) store_rec(dst, rec + (int64_t)dy * a.dst_wp + dx, r);
        }
      }
    }
    if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
      uint4* pdst[2] = {a.pool_hi + img * a.pool_img, PLANES == 2 ? a.pool_lo + img * a.pool_img : nullptr};
#pragma unroll
      for (int p2 = 0; p2 < WN / 2; ++p2) {
        float s4[2][4];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float s = v[k][2 * p2][e] + v[k][2 * p2 + 1][e];
            s4[k][e] = 0.25f * (s + __shfl_xor(s, 1));
          }
        const int y = yb + 2 * p2;
        const bool pix = !(j & 1) && y < a.h && x < a.w;
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (pix && cq0 + 8 * k < a.cout) guard(s4[k]);
        uint4 r[2];
        records(s4[0], s4[1], r);
        if (pix && col < a.cout)
          store_rec(pdst, (int64_t)(col >> 3) * a.pool_gp + (int64_t)(y / 2 + 1) * a.pool_wp + x / 2 + kH8PadLeft, r);
      }
    }
  };
  // combined accumulators: V = acc + accx 2^-11 (F16X3), V = acc (F16)
  auto combine = [&](floatx16 (&V)[WM][WN]) {
#pragma unroll
    for (int mt = 0; mt < WM; ++mt)
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          V[mt][nt][i] = PLANES == 2 ? fmaf(accx[mt][nt][i], kLoUnscale, acc[mt][nt][i]) : acc[mt][nt][i];
  };
  constexpr int NPIECE_EPI = WM * 4;
  // bias of epilogue piece (mt, q): channels co0 + 4hh .. co0 + 4hh + 3 of lane half hh,
  // co0 = cob BM + 32 mt + 8 q (pieces past cout store nothing: their bias stays 0)
  auto load_bias_piece = [&](int cob, int mt, int q, float* bq) {
    const int co0 = cob * BM + mt * 32 + 8 * q;
#pragma unroll
    for (int e = 0; e < 4; ++e) bq[e] = co0 < a.cout ? a.bias[co0 + 4 * hh + e] : 0.f;
  };
  float bsv[kBias ? WM : 1][4][4];
  auto load_bias = [&](int cob) {
#pragma unroll
    for (int p = 0; p < NPIECE_EPI; ++p) load_bias_piece(cob, p / 4, p % 4, bsv[kBias ? p / 4 : 0][p % 4]);
  };

  int tile = bid;
  if (tile >= ntiles) return;
  TileId cur = tile_id(tile);
  // prologue: chunk 0 of the block's first tile (WRES: and every weight chunk)
  if constexpr (DMA) {
#pragma unroll
    for (int it = 0; it < T::IN_IT; ++it) issue_in(cur, 0, 0, it);
    for (int c = 0; c < (kWRes ? a.nchunks : 1); ++c)
#pragma unroll
      for (int it = 0; it < T::W_IT; ++it) issue_w(cur, c, c, it);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load_w(cur, 0);
    load_in(cur, 0);
    store_in(0);
    store_w(0);
  }
  __syncthreads();
  int buf = 0;
  for (;;) {
    const int ntile = tile + cgrid;
    const bool more = ntile < ntiles;
    const TileId nxt = tile_id(more ? ntile : tile);
    if constexpr (kNoMfma || kMfma16) {  // probes: the accumulators are not written by the chunk loop's MFMAs
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            acc[mt][nt][i] = 0.f;
            accx[mt][nt][i] = 0.f;
            if constexpr (kMfma16) p16[mt][nt][i >> 3][(i >> 2) & (PLANES - 1)][i & 3] = 0.f;
          }
    }
    if constexpr (kBias == 2) load_bias(cur.cob);
    // chunk 0 peeled (its MFMAs start the accumulators from C = 0), then chunks 1 .. nchunks - 1
    auto chunk_iter = [&](const int c, auto zc) {
      // staged during this chunk: chunk c+1 of this tile, or chunk 0 of the next tile
      const bool last = c + 1 == a.nchunks;
      const bool pre = !last || more;
      const TileId& pt = last ? nxt : cur;
      const int pc = last ? 0 : c + 1;
      const int wslot = kWRes ? c : buf;
      if constexpr (DMA) {
        // buf^1 was last read in the previous chunk, before the barrier that ended it
        if constexpr (kSpread) {
          compute(buf, wslot, [&](int t) {
            if (t < kSpreadTaps && pre) {
              // pieces [t NPIECE / kSpreadTaps, (t + 1) NPIECE / kSpreadTaps) with tap t; the piece
              // index a compile-time constant (a runtime index put the per-piece offsets in scratch)
#pragma unroll
              for (int k = 0; k < NPIECE; ++k)
                if (t * NPIECE / kSpreadTaps <= k && k < (t + 1) * NPIECE / kSpreadTaps) issue_piece(pt, pc, buf ^ 1, k);
            }
          }, zc);
        } else if constexpr (kStagger) {
          const bool late = __builtin_amdgcn_readfirstlane(tid) >= NT / 2;
          if (pre && !late) {
#pragma unroll
            for (int k = 0; k < NPIECE; ++k) issue_piece(pt, pc, buf ^ 1, k);
          }
          compute(buf, wslot, [&](int t) {
            if (t == kStaggerTap && pre && late) {
#pragma unroll
              for (int k = 0; k < NPIECE; ++k) issue_piece(pt, pc, buf ^ 1, k);
            }
          }, zc);
        } else {
          if (pre) {
#pragma unroll
            for (int k = 0; k < NPIECE; ++k) issue_piece(pt, pc, buf ^ 1, k);
          }
          compute(buf, wslot, [](int) {}, zc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      } else {
        if (pre) {
          load_w(pt, pc);
          load_in(pt, pc);
        }
        compute(buf, buf, [](int) {}, zc);
        if (pre) {
          store_in(buf ^ 1);
          store_w(buf ^ 1);
        }
        __syncthreads();
      }
      buf ^= 1;
    };
    chunk_iter(0, std::true_type{});
    for (int c = 1; c < a.nchunks; ++c) chunk_iter(c, std::false_type{});

    if constexpr (kMfma16) {  // probe: keep the results live (values are not the conv)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc[mt][nt][i] = p16[mt][nt][i >> 2][0][i & 3];
            accx[mt][nt][i] = p16[mt][nt][i >> 2][PLANES - 1][i & 3];
          }
    }

    if constexpr (kNoEpi) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(acc[mt][nt][i]), "v"(accx[mt][nt][i]));
    } else {
      floatx16 V[WM][WN];
      combine(V);
      if constexpr (kBias == 1) load_bias(cur.cob);
      // the bias has landed (mode 2: long ago, the chunk loop drained vmcnt): a wait the
      // compiler sees, so that it does not wait out each piece's stores before the next
      // piece's bias (vmcnt(0), as s_waitcnt's 16-bit immediate)
      if constexpr (kBias != 0) __builtin_amdgcn_s_waitcnt(0x0F70);
      if constexpr (kWide) {
#pragma unroll
        for (int pp = 0; pp < NPIECE_EPI / 2; ++pp) {
          const int mt = pp / 2, qp = pp % 2;
          if constexpr (kBias == 0) {
            float b0[4], b1[4];
            load_bias_piece(cur.cob, mt, 2 * qp, b0);
            load_bias_piece(cur.cob, mt, 2 * qp + 1, b1);
            epi_pair(cur, V, mt, qp, b0, b1);
          } else {
            epi_pair(cur, V, mt, qp, bsv[mt][2 * qp], bsv[mt][2 * qp + 1]);
          }
        }
      } else {
#pragma unroll
        for (int p = 0; p < NPIECE_EPI; ++p) {
          if constexpr (kBias == 0) {
            float bq[4];
            load_bias_piece(cur.cob, p / 4, p % 4, bq);
            epi_piece(cur, V, p / 4, p % 4, bq);
          } else {
            epi_piece(cur, V, p / 4, p % 4, bsv[p / 4][p % 4]);
          }
        }
      }
    }
    if (!more) break;
    tile = ntile;
    cur = nxt;
  }
  if (bad && a.status) *a.status = 1;
}

// ---- bilinear x2 upsample pass (unet.py:77, align_corners=False) -------------
template <int PLANES>
__global__ void up2x_h8_kernel(const uint4* __restrict__ s_hi, const uint4* __restrict__ s_lo, int64_t s_img,
                               int64_t s_gp, int s_wp, int sh, int sw, uint4* d_hi, uint4* d_lo, int64_t d_img,
                               int64_t d_gp, int d_wp, int groups, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int w = 2 * sw, h = 2 * sh;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int g = (int)(t % groups);
  const int img = (int)(t / groups);
  // Y even (2i): 0.25 row(i-1) + 0.75 row(i); odd: 0.75 row(i) + 0.25 row(i+1); edges clamp
  int ra, rb, ca, cb;
  float wa, wc;
  if (y & 1) { ra = y >> 1; rb = min(ra + 1, sh - 1); wa = 0.75f; }
  else { rb = y >> 1; ra = max(rb - 1, 0); wa = 0.25f; }
  if (x & 1) { ca = x >> 1; cb = min(ca + 1, sw - 1); wc = 0.75f; }
  else { cb = x >> 1; ca = max(cb - 1, 0); wc = 0.25f; }
  const float wb = 1.0f - wa, wd = 1.0f - wc;
  const int64_t base = img * s_img + g * s_gp;
  const int64_t r00 = base + (int64_t)(ra + 1) * s_wp + ca + kH8PadLeft;
  const int64_t r01 = base + (int64_t)(ra + 1) * s_wp + cb + kH8PadLeft;
  const int64_t r10 = base + (int64_t)(rb + 1) * s_wp + ca + kH8PadLeft;
  const int64_t r11 = base + (int64_t)(rb + 1) * s_wp + cb + kH8PadLeft;
  half8 q[4][PLANES];
  const int64_t rr[4] = {r00, r01, r10, r11};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[k][0] = __builtin_bit_cast(half8, s_hi[rr[k]]);
    if constexpr (PLANES == 2) q[k][1] = __builtin_bit_cast(half8, s_lo[rr[k]]);
  }
  half8 ohi, olo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = PLANES == 2 ? join(q[k][0][e], q[k][PLANES - 1][e]) : (float)q[k][0][e];
    // horizontal first, then vertical (upsample_bilinear2d order)
    const float top = wc * v[0] + wd * v[1];
    const float bot = wc * v[2] + wd * v[3];
    const float o = wa * top + wb * bot;
    ohi[e] = (_Float16)o;
    olo[e] = lo_of(o, ohi[e]);
  }
  const int64_t drec = img * d_img + g * d_gp + (int64_t)(y + 1) * d_wp + x + kH8PadLeft;
  d_hi[drec] = __builtin_bit_cast(uint4, ohi);
  if constexpr (PLANES == 2) d_lo[drec] = __builtin_bit_cast(uint4, olo);
}

template <int PLANES, int KS, bool F32 = false, bool FULL = false>
__global__ void RRIN_PK_EDGE_ATTR __launch_bounds__(256 * KS) edge_fix_h8_kernel(EdgeFixArgs a) {
  edge_fix_body<PLANES, KS, F32, FULL>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---- layout kernels ------------------------------------------------------------
__device__ inline int64_t h8_half_index(int64_t img_stride, int64_t gp, int wp, int img, int ch, int y, int x) {
  return ((int64_t)img * img_stride + (int64_t)(ch >> 3) * gp + (int64_t)(y + 1) * wp + x + kH8PadLeft) * 8 +
         (ch & 7);
}

__global__ void nchw_to_h8_kernel(const float* __restrict__ src, _Float16* hi, _Float16* lo, int64_t img_stride,
                                  int64_t gp, int wp, int ch_off, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  const float v = src[i];
  const int64_t k = h8_half_index(img_stride, gp, wp, n, ch_off + ch, y, x);
  const _Float16 vh = (_Float16)v;
  hi[k] = vh;
  if (lo) lo[k] = lo_of(v, vh);
}

template <int PLANES>
__global__ void pack_g16_h8_kernel(const float* __restrict__ i0, const float* __restrict__ i1, uint4* ghi,
                                   uint4* glo, int64_t img_stride, int64_t gp, int wp, int h, int w,
                                   int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int img = (int)(t / h);
  const int64_t hw = (int64_t)h * w;
  const int64_t px = (int64_t)img * 3 * hw + (int64_t)y * w + x;
  half8 hi = {}, lo = {};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float a = i0[px + c * hw], b = i1[px + c * hw];
    hi[c] = (_Float16)a;
    hi[3 + c] = (_Float16)b;
    lo[c] = lo_of(a, hi[c]);
    lo[3 + c] = lo_of(b, hi[3 + c]);
  }
  const int64_t rec = (int64_t)img * img_stride + (int64_t)(y + 1) * wp + x + kH8PadLeft;
  ghi[rec] = __builtin_bit_cast(uint4, hi);
  ghi[rec + gp] = make_uint4(0u, 0u, 0u, 0u);
  if constexpr (PLANES == 2) {
    glo[rec] = __builtin_bit_cast(uint4, lo);
    glo[rec + gp] = make_uint4(0u, 0u, 0u, 0u);
  }
}

__global__ void h8_to_nchw_kernel(const _Float16* __restrict__ hi, const _Float16* __restrict__ lo, int64_t img_stride,
                                  int64_t gp, int wp, int ch_off, float* dst, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  const int64_t k = h8_half_index(img_stride, gp, wp, n, ch_off + ch, y, x);
  dst[i] = lo ? join(hi[k], lo[k]) : (float)hi[k];
}

// ---- head conv (Cout <= 4) + Net glue on the H8 Net buffer --------------------
struct HeadH8Args {
  const uint4* src_hi;
  const uint4* src_lo;
  int64_t src_img, src_gp;
  int src_wp;
  _Float16* g_hi;  // g16: 2 groups
  _Float16* g_lo;
  int64_t g_img, g_gp;
  int g_wp;
  const float* w;
  const float* bias;
  const float* coef;
  float* out;
  _Float16* fr_hi;  // FLOW: raw output (1 group), nullable
  _Float16* fr_lo;
  int64_t fr_img, fr_gp;
  int fr_wp;
  int h, w_, tiles_x, tiles_y;
  uint4* g32;       // F32R: g16 as 4 records of 4 fp32 channels (g_img / g_gp / g_wp in records)
  uint4* fr32;      // F32R: raw Flow output, 1 record (nullable)
  float* raw;       // optional: head conv output before the glue, NCHW [n][COUT][h][w]
  int* status;      // optional fp16 range flag: glue stores set it, FINAL poisons on it
};

template <int COUT, int MODE, int PLANES>
__global__ void __launch_bounds__(256) head_h8_kernel(HeadH8Args a) {
  // tile 16 rows x 32 cols; thread = 2 vertically adjacent pixels (packed fp32 FMA)
  constexpr int CIN = 32, HROWS = 18, HLC = 40;
  __shared__ __attribute__((aligned(16))) float s_in[8 * HROWS * HLC];
  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int img = bid / a.tiles_y;
  const int x0 = tx * 32, y0 = ty * 16;
  const int r2 = 2 * (tid >> 5), xl = tid & 31;

  // weights are wave-uniform: scalar loads, no LDS traffic
  float2v acc2[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc2[co] = float2v{a.bias[co], a.bias[co]};
  // records of rows y0-1..y0+16, cols x0-1..x0+32 of one channel group, fetched
  // one group ahead into registers, then converted to fp32 planar LDS
  constexpr int kRec = HROWS * H8_LC, kIt = (kRec + 255) / 256;
  uint4 pre[kIt][PLANES];
  auto fetch = [&](int g) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kRec) {
        const int rr = idx / H8_LC, col = idx - rr * H8_LC;
        const int64_t rec = img * a.src_img + (int64_t)g * a.src_gp + (int64_t)(y0 + rr) * a.src_wp + x0 +
                            (kH8PadLeft - 1) + col;
        pre[it][0] = a.src_hi[rec];
        if constexpr (PLANES == 2) pre[it][1] = a.src_lo[rec];
      }
    }
  };
  fetch(0);
  for (int g = 0; g < CIN / 8; ++g) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kRec) {
        const int rr = idx / H8_LC, col = idx - rr * H8_LC;
        const half8 vh = __builtin_bit_cast(half8, pre[it][0]);
        half8 vl = {};
        if constexpr (PLANES == 2) vl = __builtin_bit_cast(half8, pre[it][PLANES - 1]);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          s_in[(e * HROWS + rr) * HLC + col + 3] = PLANES == 2 ? join(vh[e], vl[e]) : (float)vh[e];
      }
    }
    __syncthreads();
    if (g + 1 < CIN / 8) fetch(g + 1);
#pragma unroll
    for (int ci = 0; ci < 8; ++ci) {
      float rows[4][3];  // input rows r2-1 .. r2+2 (staged rows r2 .. r2+3), cols xl-1 .. xl+1
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) rows[k][kx] = s_in[(ci * HROWS + r2 + k) * HLC + xl + 3 + kx];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float2v v = {rows[ky][kx], rows[ky + 1][kx]};
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float w = a.w[((co * CIN) + g * 8 + ci) * 9 + ky * 3 + kx];
            acc2[co] = __builtin_elementwise_fma(float2v{w, w}, v, acc2[co]);
          }
        }
    }
    __syncthreads();
  }

  for (int p = 0; p < 2; ++p) {
  float acc[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc[co] = acc2[co][p];
  const int y = y0 + r2 + p, x = x0 + xl;
  if (y >= a.h || x >= a.w_) continue;
  // Net buffer records of this pixel: group 0 = ch 0-7, group 1 = ch 8-15
  const int64_t rec0 = img * a.g_img + (int64_t)(y + 1) * a.g_wp + x + kH8PadLeft, rec1 = rec0 + a.g_gp;
  uint4* ghi = reinterpret_cast<uint4*>(a.g_hi);
  uint4* glo = reinterpret_cast<uint4*>(a.g_lo);
  auto load8 = [&](int64_t rec, float* v) {
    const half8 h = __builtin_bit_cast(half8, ghi[rec]);
    half8 l = {};
    if constexpr (PLANES == 2) l = __builtin_bit_cast(half8, glo[rec]);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = PLANES == 2 ? join(h[e], l[e]) : (float)h[e];
  };
  // n consecutive channels starting at half `e0` of record `rec` (one 2/4/8/16-B store per plane)
  auto store = [&](int64_t rec, int e0, const float* v, int n) {
    _Float16 hv[8], lv[8];
    for (int e = 0; e < n; ++e)
      if (a.status && !(fabsf(v[e]) <= kF16Max)) *a.status = 1;
    for (int e = 0; e < n; ++e) {
      hv[e] = (_Float16)v[e];
      lv[e] = lo_of(v[e], hv[e]);
    }
    _Float16* ph = reinterpret_cast<_Float16*>(ghi + rec) + e0;
    _Float16* pl = reinterpret_cast<_Float16*>(glo + rec) + e0;
    if (n == 8) {
      *reinterpret_cast<uint4*>(ph) = __builtin_bit_cast(uint4, hv);
      if constexpr (PLANES == 2) *reinterpret_cast<uint4*>(pl) = __builtin_bit_cast(uint4, lv);
    } else if (n == 2) {
      *reinterpret_cast<uint32_t*>(ph) = (uint32_t)__builtin_bit_cast(uint16_t, hv[0]) |
                                         ((uint32_t)__builtin_bit_cast(uint16_t, hv[1]) << 16);
      if constexpr (PLANES == 2)
        *reinterpret_cast<uint32_t*>(pl) = (uint32_t)__builtin_bit_cast(uint16_t, lv[0]) |
                                           ((uint32_t)__builtin_bit_cast(uint16_t, lv[1]) << 16);
    } else {
      for (int e = 0; e < n; ++e) {
        ph[e] = hv[e];
        if constexpr (PLANES == 2) pl[e] = lv[e];
      }
    }
  };
  const float* cf = a.coef + img * 8;
  if (a.raw)
#pragma unroll
    for (int co = 0; co < COUT; ++co) a.raw[(((int64_t)img * COUT + co) * a.h + y) * a.w_ + x] = acc[co];

  if constexpr (MODE == RRIN_HEAD_PLAIN) {
    for (int co = 0; co < COUT; ++co) {
      const int64_t k = h8_half_index(a.g_img, a.g_gp, a.g_wp, img, co, y, x);
      const _Float16 vh = (_Float16)acc[co];
      a.g_hi[k] = vh;
      if constexpr (PLANES == 2) a.g_lo[k] = lo_of(acc[co], vh);
    }
  } else if constexpr (MODE == RRIN_HEAD_FLOW) {
#pragma clang fp contract(off)
    // round the raw flow to its stored form first, so that a later t-blend of the
    // kept raw flow (skip_flow) reproduces these Ft bit for bit
    _Float16 rh[4], rl[4];
    for (int k = 0; k < 4; ++k)
      if (a.status && !(fabsf(acc[k]) <= kF16Max)) *a.status = 1;
    for (int k = 0; k < 4; ++k) {
      rh[k] = (_Float16)acc[k];
      rl[k] = lo_of(acc[k], rh[k]);
      acc[k] = PLANES == 2 ? join(rh[k], rl[k]) : (float)rh[k];
    }
    if (a.fr_hi) {
      const int64_t kk = h8_half_index(a.fr_img, a.fr_gp, a.fr_wp, img, 0, y, x);
      *reinterpret_cast<uint2*>(a.fr_hi + kk) = __builtin_bit_cast(uint2, rh);
      if constexpr (PLANES == 2) *reinterpret_cast<uint2*>(a.fr_lo + kk) = __builtin_bit_cast(uint2, rl);
    }
    float f0[2], f1[2];
    for (int k = 0; k < 2; ++k) {
      f0[k] = cf[0] * acc[k] + cf[1] * acc[2 + k];
      f1[k] = cf[2] * acc[k] - cf[3] * acc[2 + k];
    }
    store(rec0, 6, f0, 2);
    store(rec1, 0, f1, 2);
  } else if constexpr (MODE == RRIN_HEAD_REFINE) {
#pragma clang fp contract(off)
    float g0[8], g1[8];
    load8(rec0, g0);
    load8(rec1, g1);
    const float f0[2] = {g0[6] + acc[0], g0[7] + acc[1]};
    float o1[8];
    o1[0] = g1[0] + acc[2];
    o1[1] = g1[1] + acc[3];
    const WarpTaps t0 = warp_taps(x, y, f0[0], f0[1], a.h, a.w_);
    const WarpTaps t1 = warp_taps(x, y, o1[0], o1[1], a.h, a.w_);
    // backwarp x0 (ch 0-2) with Ft0 and x1 (ch 3-5) with Ft1: one record load per tap and plane
    auto warp3 = [&](const WarpTaps& t, int c0, float* o) {
      float q[4][8];
      const bool ok[4] = {t.vy0 && t.vx0, t.vy0 && t.vx1, t.vy1 && t.vx0, t.vy1 && t.vx1};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (ok[k]) {
          load8(img * a.g_img + (int64_t)(t.y0 + (k >> 1) + 1) * a.g_wp + t.x0 + (k & 1) + kH8PadLeft, q[k]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) q[k][e] = 0.0f;
        }
      }
#pragma unroll
      for (int c = 0; c < 3; ++c)
        o[c] = q[0][c0 + c] * t.nw + q[1][c0 + c] * t.ne + q[2][c0 + c] * t.sw + q[3][c0 + c] * t.se;
    };
    warp3(t0, 0, o1 + 2);
    warp3(t1, 3, o1 + 5);
    store(rec0, 6, f0, 2);
    store(rec1, 0, o1, 8);
  } else if constexpr (MODE == RRIN_HEAD_MASK) {
#pragma clang fp contract(off)
    float g1[8];
    load8(rec1, g1);
    const float m0 = 1.0f / (1.0f + expf(-acc[0]));
    const float m1 = 1.0f / (1.0f + expf(-acc[1]));
    const float w1 = cf[4] * m0, w2 = cf[5] * m1;
    const float den = w1 + w2 + 1e-8f;
    float o[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) o[ch] = (w1 * g1[2 + ch] + w2 * g1[5 + ch]) / den;
    store(rec0, 6, o, 2);
    store(rec1, 0, o + 2, 1);
  } else {  // FINAL
#pragma clang fp contract(off)
    float g0[8], g1[8];
    load8(rec0, g0);
    load8(rec1, g1);
    const float base[3] = {g0[6], g0[7], g1[0]};
    float* o = a.out + ((int64_t)img * 3) * a.h * a.w_ + (int64_t)y * a.w_ + x;
    const bool poison = a.status && *a.status != 0;  // an fp16 overflow upstream (range guard)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float v = acc[ch] + base[ch];
      o[(int64_t)ch * a.h * a.w_] = poison ? __builtin_nanf("") : (v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v));
    }
  }
  }
}

template <int PLANES>
__global__ void flow_tblend_h8_kernel(const _Float16* __restrict__ fhi, const _Float16* __restrict__ flo,
                                      int64_t f_img, int64_t f_gp, int f_wp, _Float16* ghi, _Float16* glo,
                                      int64_t g_img, int64_t g_gp, int g_wp, const float* coef, int h, int w,
                                      int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int img = (int)(t / h);
  const float* cf = coef + img * 8;
  float f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t kk = h8_half_index(f_img, f_gp, f_wp, img, k, y, x);
    f[k] = PLANES == 2 ? join(fhi[kk], flo[kk]) : (float)fhi[kk];
  }
  float o[4];
  for (int k = 0; k < 2; ++k) {
#pragma clang fp contract(off)
    o[k] = cf[0] * f[k] + cf[1] * f[2 + k];
    o[2 + k] = cf[2] * f[k] - cf[3] * f[2 + k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t kk = h8_half_index(g_img, g_gp, g_wp, img, 6 + k, y, x);
    const _Float16 vh = (_Float16)o[k];
    ghi[kk] = vh;
    if constexpr (PLANES == 2) glo[kk] = lo_of(o[k], vh);
  }
}

// ---- F32R (exact fp32, 4 channels per record) layout / glue kernels -----------------
__device__ inline int64_t r32_elem_index(int64_t img_stride, int64_t gp, int wp, int img, int ch, int y, int x) {
  return ((int64_t)img * img_stride + (int64_t)(ch >> 2) * gp + (int64_t)(y + 1) * wp + x + kH8PadLeft) * 4 +
         (ch & 3);
}
__device__ inline uint4 f4rec(float a, float b, float c, float d) {
  return make_uint4(__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d));
}

__global__ void nchw_to_r32_kernel(const float* __restrict__ src, float* dst, int64_t img_stride, int64_t gp, int wp,
                                   int ch_off, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  dst[r32_elem_index(img_stride, gp, wp, n, ch_off + ch, y, x)] = src[i];
}

__global__ void r32_to_nchw_kernel(const float* __restrict__ src, int64_t img_stride, int64_t gp, int wp, int ch_off,
                                   float* dst, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = (int)(t % c);
  const int n = (int)(t / c);
  dst[i] = src[r32_elem_index(img_stride, gp, wp, n, ch_off + ch, y, x)];
}

// x = cat(x0, x1) (model.py:33) into g16: record 0 = x0 0-2, x1 0; record 1 =
// x1 1-2, 0, 0; records 2-3 zero (whole-record stores).
__global__ void pack_g16_r32_kernel(const float* __restrict__ i0, const float* __restrict__ i1, uint4* g,
                                    int64_t img_stride, int64_t gp, int wp, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int img = (int)(t / h);
  const int64_t hw = (int64_t)h * w;
  const int64_t px = (int64_t)img * 3 * hw + (int64_t)y * w + x;
  const float a0 = i0[px], a1 = i0[px + hw], a2 = i0[px + 2 * hw];
  const float b0 = i1[px], b1 = i1[px + hw], b2 = i1[px + 2 * hw];
  const int64_t rec = (int64_t)img * img_stride + (int64_t)(y + 1) * wp + x + kH8PadLeft;
  g[rec] = f4rec(a0, a1, a2, b0);
  g[rec + gp] = f4rec(b1, b2, 0.f, 0.f);
  g[rec + 2 * gp] = make_uint4(0u, 0u, 0u, 0u);
  g[rec + 3 * gp] = make_uint4(0u, 0u, 0u, 0u);
}

// Ft0 / Ft1 (model.py:38-39) from a kept raw Flow record -> g16 channels 6-9
__global__ void flow_tblend_r32_kernel(const uint4* __restrict__ fr, int64_t f_img, int f_wp, uint4* g, int64_t g_img,
                                       int64_t g_gp, int g_wp, const float* coef, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int64_t t = i / w;
  const int y = (int)(t % h);
  const int img = (int)(t / h);
  const float* cf = coef + img * 8;
  const floatx4 f = __builtin_bit_cast(floatx4, fr[(int64_t)img * f_img + (int64_t)(y + 1) * f_wp + x + kH8PadLeft]);
  float o[4];
  for (int k = 0; k < 2; ++k) {
#pragma clang fp contract(off)
    o[k] = cf[0] * f[k] + cf[1] * f[2 + k];
    o[2 + k] = cf[2] * f[k] - cf[3] * f[2 + k];
  }
  const int64_t rec = (int64_t)img * g_img + (int64_t)(y + 1) * g_wp + x + kH8PadLeft;
  const floatx4 r1 = __builtin_bit_cast(floatx4, g[rec + g_gp]);
  const floatx4 r2 = __builtin_bit_cast(floatx4, g[rec + 2 * g_gp]);
  g[rec + g_gp] = f4rec(r1[0], r1[1], o[0], o[1]);
  g[rec + 2 * g_gp] = f4rec(o[2], o[3], r2[2], r2[3]);
}

// bilinear x2 (unet.py:77, align_corners=False, edge clamp) of fp32 records
__global__ void up2x_r32_kernel(const uint4* __restrict__ s, int64_t s_img, int64_t s_gp, int s_wp, int sh, int sw,
                                uint4* d, int64_t d_img, int64_t d_gp, int d_wp, int groups, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int w = 2 * sw, h = 2 * sh;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int g = (int)(t % groups);
  const int img = (int)(t / groups);
  int ra, rb, ca, cb;
  float wa, wc;
  if (y & 1) { ra = y >> 1; rb = min(ra + 1, sh - 1); wa = 0.75f; }
  else { rb = y >> 1; ra = max(rb - 1, 0); wa = 0.25f; }
  if (x & 1) { ca = x >> 1; cb = min(ca + 1, sw - 1); wc = 0.75f; }
  else { cb = x >> 1; ca = max(cb - 1, 0); wc = 0.25f; }
  const float wb = 1.0f - wa, wd = 1.0f - wc;
  const int64_t base = img * s_img + g * s_gp + kH8PadLeft;
  const floatx4 q0 = __builtin_bit_cast(floatx4, s[base + (int64_t)(ra + 1) * s_wp + ca]);
  const floatx4 q1 = __builtin_bit_cast(floatx4, s[base + (int64_t)(ra + 1) * s_wp + cb]);
  const floatx4 q2 = __builtin_bit_cast(floatx4, s[base + (int64_t)(rb + 1) * s_wp + ca]);
  const floatx4 q3 = __builtin_bit_cast(floatx4, s[base + (int64_t)(rb + 1) * s_wp + cb]);
  float o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float top = wc * q0[e] + wd * q1[e];  // horizontal first (upsample_bilinear2d order)
    const float bot = wc * q2[e] + wd * q3[e];
    o[e] = wa * top + wb * bot;
  }
  d[img * d_img + g * d_gp + (int64_t)(y + 1) * d_wp + x + kH8PadLeft] = f4rec(o[0], o[1], o[2], o[3]);
}

// Head conv (Cout <= 4) + Net glue on fp32 records: as head_h8_kernel, with the
// 32-channel input as 8 records of 4 channels and g16 as 4 records; every g16
// update is a whole 16-B record (records the glue only partly changes are read
// first), no partial-record writes.
template <int COUT, int MODE>
__global__ void __launch_bounds__(256) head_r32_kernel(HeadH8Args a) {
  constexpr int CIN = 32, HROWS = 18, HLC = 40;
  __shared__ __attribute__((aligned(16))) float s_in[8 * HROWS * HLC];
  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int img = bid / a.tiles_y;
  const int x0 = tx * 32, y0 = ty * 16;
  const int r2 = 2 * (tid >> 5), xl = tid & 31;

  float acc2[2][COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc2[0][co] = acc2[1][co] = a.bias[co];
  // records of rows y0-1..y0+16, cols x0-1..x0+32 of 8 channels (2 record groups),
  // fetched one channel octet ahead into registers, then stored to planar LDS
  constexpr int kRec = HROWS * H8_LC, kIt = (kRec + 255) / 256;
  uint4 pre[kIt][2];
  auto fetch = [&](int g8) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kRec) {
        const int rr = idx / H8_LC, col = idx - rr * H8_LC;
        const int64_t rec = img * a.src_img + (int64_t)(2 * g8) * a.src_gp + (int64_t)(y0 + rr) * a.src_wp + x0 +
                            (kH8PadLeft - 1) + col;
        pre[it][0] = a.src_hi[rec];
        pre[it][1] = a.src_hi[rec + a.src_gp];
      }
    }
  };
  fetch(0);
  for (int g8 = 0; g8 < CIN / 8; ++g8) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kRec) {
        const int rr = idx / H8_LC, col = idx - rr * H8_LC;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          s_in[(e * HROWS + rr) * HLC + col + 3] = __builtin_bit_cast(floatx4, pre[it][e >> 2])[e & 3];
      }
    }
    __syncthreads();
    if (g8 + 1 < CIN / 8) fetch(g8 + 1);
#pragma unroll
    for (int ci = 0; ci < 8; ++ci) {
      float rows[4][3];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) rows[k][kx] = s_in[(ci * HROWS + r2 + k) * HLC + xl + 3 + kx];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float w = a.w[((co * CIN) + g8 * 8 + ci) * 9 + ky * 3 + kx];
            acc2[0][co] = fmaf(w, rows[ky][kx], acc2[0][co]);
            acc2[1][co] = fmaf(w, rows[ky + 1][kx], acc2[1][co]);
          }
    }
    __syncthreads();
  }

  for (int p = 0; p < 2; ++p) {
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = acc2[p][co];
    const int y = y0 + r2 + p, x = x0 + xl;
    if (y >= a.h || x >= a.w_) continue;
    const int64_t rec0 = img * a.g_img + (int64_t)(y + 1) * a.g_wp + x + kH8PadLeft;
    auto ld = [&](int k) { return __builtin_bit_cast(floatx4, a.g32[rec0 + k * a.g_gp]); };
    auto st = [&](int k, float v0, float v1, float v2, float v3) { a.g32[rec0 + k * a.g_gp] = f4rec(v0, v1, v2, v3); };
    const float* cf = a.coef + img * 8;
    if (a.raw)
#pragma unroll
      for (int co = 0; co < COUT; ++co) a.raw[(((int64_t)img * COUT + co) * a.h + y) * a.w_ + x] = acc[co];
    if constexpr (MODE == RRIN_HEAD_PLAIN) {
      float* gf = reinterpret_cast<float*>(a.g32);
      for (int co = 0; co < COUT; ++co) gf[r32_elem_index(a.g_img, a.g_gp, a.g_wp, img, co, y, x)] = acc[co];
    } else if constexpr (MODE == RRIN_HEAD_FLOW) {
#pragma clang fp contract(off)
      if (a.fr32) a.fr32[img * a.fr_img + (int64_t)(y + 1) * a.fr_wp + x + kH8PadLeft] = f4rec(acc[0], acc[1], acc[2], acc[3]);
      float f0[2], f1[2];
      for (int k = 0; k < 2; ++k) {
        f0[k] = cf[0] * acc[k] + cf[1] * acc[2 + k];
        f1[k] = cf[2] * acc[k] - cf[3] * acc[2 + k];
      }
      const floatx4 r1 = ld(1), r2v = ld(2);
      st(1, r1[0], r1[1], f0[0], f0[1]);
      st(2, f1[0], f1[1], r2v[2], r2v[3]);
    } else if constexpr (MODE == RRIN_HEAD_REFINE) {
#pragma clang fp contract(off)
      const floatx4 q0 = ld(0), q1 = ld(1), q2 = ld(2);
      const float f0[2] = {q1[2] + acc[0], q1[3] + acc[1]};
      float o1[8];
      o1[0] = q2[0] + acc[2];
      o1[1] = q2[1] + acc[3];
      const WarpTaps t0 = warp_taps(x, y, f0[0], f0[1], a.h, a.w_);
      const WarpTaps t1 = warp_taps(x, y, o1[0], o1[1], a.h, a.w_);
      // backwarp x0 (ch 0-2) with Ft0 and x1 (ch 3-5) with Ft1: records 0-1 per tap
      auto warp3 = [&](const WarpTaps& t, int c0, float* o) {
        float q[4][8];
        const bool ok[4] = {t.vy0 && t.vx0, t.vy0 && t.vx1, t.vy1 && t.vx0, t.vy1 && t.vx1};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (ok[k]) {
            const int64_t r = img * a.g_img + (int64_t)(t.y0 + (k >> 1) + 1) * a.g_wp + t.x0 + (k & 1) + kH8PadLeft;
            const floatx4 lo = __builtin_bit_cast(floatx4, a.g32[r]);
            const floatx4 hi = __builtin_bit_cast(floatx4, a.g32[r + a.g_gp]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              q[k][e] = lo[e];
              q[k][4 + e] = hi[e];
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) q[k][e] = 0.0f;
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c)
          o[c] = q[0][c0 + c] * t.nw + q[1][c0 + c] * t.ne + q[2][c0 + c] * t.sw + q[3][c0 + c] * t.se;
      };
      warp3(t0, 0, o1 + 2);
      warp3(t1, 3, o1 + 5);
      (void)q0;
      st(1, q1[0], q1[1], f0[0], f0[1]);
      st(2, o1[0], o1[1], o1[2], o1[3]);
      st(3, o1[4], o1[5], o1[6], o1[7]);
    } else if constexpr (MODE == RRIN_HEAD_MASK) {
#pragma clang fp contract(off)
      const floatx4 r1 = ld(1), r2v = ld(2), r3 = ld(3);
      const float g1[8] = {r2v[0], r2v[1], r2v[2], r2v[3], r3[0], r3[1], r3[2], r3[3]};  // ch 8-15
      const float m0 = 1.0f / (1.0f + expf(-acc[0]));
      const float m1 = 1.0f / (1.0f + expf(-acc[1]));
      const float w1 = cf[4] * m0, w2 = cf[5] * m1;
      const float den = w1 + w2 + 1e-8f;
      float o[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) o[ch] = (w1 * g1[2 + ch] + w2 * g1[5 + ch]) / den;
      st(1, r1[0], r1[1], o[0], o[1]);
      st(2, o[2], r2v[1], r2v[2], r2v[3]);
    } else {  // FINAL
#pragma clang fp contract(off)
      const floatx4 r1 = ld(1), r2v = ld(2);
      const float base[3] = {r1[2], r1[3], r2v[0]};
      float* o = a.out + ((int64_t)img * 3) * a.h * a.w_ + (int64_t)y * a.w_ + x;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float v = acc[ch] + base[ch];
        o[(int64_t)ch * a.h * a.w_] = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
      }
    }
  }
}

// ---- host helpers ------------------------------------------------------------------
// fp32 -> fp16 bits, round to nearest even (host packing).
static uint16_t f2h_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const uint32_t au = u & 0x7FFFFFFFu;
  if (au >= 0x7F800000u) return (uint16_t)(sign | (au > 0x7F800000u ? 0x7E00u : 0x7C00u));
  if (au >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);  // rounds to >= 65520 -> inf
  if (au < 0x38800000u) {                                     // subnormal / zero in fp16
    const float af = fabsf(f);
    const uint32_t m = (uint32_t)lrintf(af * 16777216.0f);     // units of 2^-24, RNE
    return (uint16_t)(sign | m);
  }
  const uint32_t e = ((au >> 23) - 112u) << 10;  // rebias 127 -> 15
  uint32_t m = (au >> 13) & 0x3FFu;
  const uint32_t rest = au & 0x1FFFu;
  uint32_t h = e | m;
  if (rest > 0x1000u || (rest == 0x1000u && (m & 1u))) h += 1u;
  return (uint16_t)(sign | h);
}

static float h2f(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
  float f;
  if (e == 0) {
    f = ldexpf((float)m, -24);
  } else if (e == 31) {
    uint32_t u = sign | 0x7F800000u | (m << 13);
    memcpy(&f, &u, 4);
    return f;
  } else {
    uint32_t u = ((e + 112u) << 23) | (m << 13);
    memcpy(&f, &u, 4);
  }
  return sign ? -f : f;
}

// Config table: cfg -> (NW waves along rows, WM co-tiles, WN rows per wave,
// SC schedule knobs SCHED_*, PE grid: 0 = one tile per block, k = k x the
// blocks a CU holds at once, persistent).  16-17 (BM 32 x TH 4) are for the
// few-tile deep levels of small workloads (engine size classes).
#define RRIN_H8_CFGS(X)  \
  X(0, 8, 2, 2, 0, 0)    \
  X(1, 8, 1, 2, 0, 0)    \
  X(2, 4, 2, 2, 0, 0)    \
  X(3, 4, 1, 4, 0, 0)    \
  X(4, 4, 2, 1, 0, 0)    \
  X(5, 8, 4, 2, 0, 0)    \
  X(6, 4, 1, 2, 0, 0)    \
  X(7, 2, 1, 4, 0, 0)    \
  X(8, 4, 1, 2, 32, 1)   \
  X(9, 8, 1, 2, 32, 1)   \
  X(10, 8, 2, 2, 16, 1)  \
  X(11, 8, 2, 2, 16, 0)  \
  X(12, 4, 1, 2, 16, 1)  \
  X(13, 8, 1, 2, 16, 1)  \
  X(14, 4, 1, 2, 48, 1)  \
  X(15, 8, 1, 2, 48, 1)  \
  X(16, 4, 1, 1, 16, 1)  \
  X(17, 2, 1, 2, 16, 1)

// Shared memory of one block: double-buffered input tile and weight slab, or
// with WRES every chunk's weight slab resident.
template <int NW, int WM, int WN, int PLANES>
constexpr size_t h8_lds_bytes(bool wres, int nchunks) {
  using T = TileH8<NW, WM, WN, PLANES>;
  return ((size_t)2 * T::IN_REC + (size_t)(wres && nchunks > 2 ? nchunks : 2) * T::W_REC) * PLANES * 16;
}

struct CfgH8 {
  int bm, th;
  size_t lds1, lds2;  // at two weight slabs (WRES: at <= 2 chunks)
  size_t wslab;       // bytes of one weight slab per plane (WRES: one more per chunk past 2)
  bool pool_ok;
  int sched, persist;
  int nt;  // threads per workgroup (the direct-form tiles; 0: Winograd configs)
};
static constexpr size_t kRetiredLds = (size_t)1 << 30;  // > kMaxLds: never usable
static const CfgH8 kCfgH8[] = {
#define X(id, nw, wm, wn, sc, pe)                                                                               \
  {TileH8<nw, wm, wn, 1>::BM, TileH8<nw, wm, wn, 1>::TH, h8_lds_bytes<nw, wm, wn, 1>((sc & SCHED_WRES) != 0, 2), \
   h8_lds_bytes<nw, wm, wn, 2>((sc & SCHED_WRES) != 0, 2), (size_t)TileH8<nw, wm, wn, 1>::W_REC * 16,     \
   (wn % 2) == 0, sc, pe, 64 * nw},
    RRIN_H8_CFGS(X)
#undef X
    // kWinoCfg: Winograd F(2x2,3x3) on fp32 records (conv_wino.hip), BM 32 x TH 8
    {32, 8, kWinoLds, (size_t)1 << 30, 0, true, 0, 0},
    // config 19, retired in round 6: the kind-2 Winograd tile (BM 64, 8 waves, one block per CU)
    // lost to kinds 3 and 6 and was removed; the id stays reserved so ids 20-24 keep their meaning
    {64, 8, kRetiredLds, kRetiredLds, 0, true, 0, 0},
    // kWinoQCfg: cfg 18's tile and packing, 8 waves of 4 accumulators (conv3x3_winoq_kernel)
    {32, 8, (size_t)2 * (680 + 1024) * 16, (size_t)1 << 30, 0, true, 0, 0},
    // kWinoQ4Cfg: the same on half-height tiles (TH 4, 4 waves): twice the tiles
    {32, 4, (size_t)2 * (408 + 1024) * 16, (size_t)1 << 30, 0, true, 0, 0},
    // config 22, retired in round 6: Winograd F(4x4,3x3) (kind 5), 1.28-1.58x kind 3's time
    {32, 16, kRetiredLds, kRetiredLds, 0, true, 0, 0},
    // kWinoC2Cfg: register-U tile, BM 64 x TH 4, 4 waves of 2 co tiles (conv_winoc.hip); at fp16
    // the same tile with f16 MFMAs (conv_winoh.hip)
    {64, 4, kWinoCLds1, (size_t)1 << 30, 0, true, 0, 0},
    // kWinoC1Cfg: register-U tile, BM 32 x TH 8, 4 waves of 2 patch tiles
    {32, 8, kWinoCLds2, (size_t)1 << 30, 0, true, 0, 0},
    // kWinoC42Cfg (round 6): register-U tile in F(4,3) x F(2,3), BM 32 x TH 8 (conv_winoc42.hip)
    {32, 8, kWinoC42Lds, (size_t)1 << 30, 0, true, 0, 0},
};
static constexpr int kNumCfgH8 = sizeof(kCfgH8) / sizeof(kCfgH8[0]);
static constexpr int kWinoCfg = 18;
static constexpr int kRetired19Cfg = 19;
static constexpr int kWinoQCfg = 20;
static constexpr int kWinoQ4Cfg = 21;
static constexpr int kRetired22Cfg = 22;
static constexpr int kWinoC2Cfg = 23;
static constexpr int kWinoC1Cfg = 24;
static constexpr int kWinoC42Cfg = 25;
static_assert(kNumCfgH8 == 26, "config ids (engine tables, rrin_hip.h)");
static inline bool is_winoc(int cfg) { return cfg == kWinoC2Cfg || cfg == kWinoC1Cfg; }
// Round 6 removed the rejected Winograd tiles (kinds 2, 5, 8-13; DESIGN.md §5b-§5e keep their
// measurements): ids 19 and 22 stay reserved (rrin_conv_h8_cfg_ok 0, RRIN_E_CONFIG), 25-30 are gone.
static inline bool retired(int cfg) { return cfg == kRetired19Cfg || cfg == kRetired22Cfg; }
static inline bool is_wino(int cfg) {
  return cfg == kWinoCfg || cfg == kWinoQCfg || cfg == kWinoQ4Cfg || is_winoc(cfg) || cfg == kWinoC42Cfg;
}
// the fp16 Winograd tile (conv_winoh.hip): kind 6
static inline bool is_winoh(int cfg) { return cfg == kWinoC2Cfg; }
static constexpr size_t kMaxLds = 160 * 1024;
static constexpr int kMaxKSplit = 16;

static int num_cus(int dev) {
  static std::atomic<int> n[kMaxDevices] = {};
  int v = n[dev].load(std::memory_order_relaxed);
  if (!v) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1) v = 256;
    n[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int NW, int WM, int WN, int PLANES, int EPI, bool DMA, int SCHED, bool F32 = false>
static int launch_h8_k(const ConvH8Args& args, int persist, hipStream_t st) {
  using T = TileH8<NW, WM, WN, PLANES>;
  auto k = conv3x3_h8_kernel<NW, WM, WN, PLANES, EPI, DMA, SCHED, F32>;
  constexpr bool wres = DMA && (SCHED & SCHED_WRES) != 0;
  const size_t lds = h8_lds_bytes<NW, WM, WN, PLANES>(wres, args.nchunks);
  if (lds > kMaxLds) return RRIN_E_CONFIG;
  static LdsAttr attr;
  // resident blocks per CU, per device and LDS footprint (WRES: chunk count)
  static std::atomic<int> per_cu[kMaxDevices][40] = {};
  if (int e = attr.ensure((const void*)k, (int)kMaxLds, st)) return e;
  const int64_t ntiles = (int64_t)args.co_blocks * args.tiles_x * args.tiles_y * args.n;
  int64_t grid = ntiles;
  if (persist > 0) {
    const int dev = stream_device(st);
    std::atomic<int>& slot = per_cu[dev][wres ? (args.nchunks < 40 ? args.nchunks : 39) : 0];
    int pc = slot.load(std::memory_order_relaxed);
    if (!pc) {
      hipError_t e = on_device(dev, [&] {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, (const void*)k, T::NT, lds);
      });
      if (e != hipSuccess) return (int)e;
      if (pc < 1) pc = 1;
      slot.store(pc, std::memory_order_relaxed);
    }
    int64_t g = (int64_t)persist * pc * num_cus(dev);
    g -= g % args.co_blocks;  // WRES: every tile of a block in the block's channel block
    if (g < args.co_blocks) g = args.co_blocks;
    if (g < grid) grid = g;
  }
  if constexpr (EPI == RRIN_EPI_SUBPIXEL && T::NT >= 256) {
    if (args.fix_real > 0) {  // the FULL ring fix-up in workgroups [0, nfix) of this launch
      constexpr int VG = T::NT / 256;  // ring tiles per workgroup, one per 256-thread slice
      ConvH8Args b = args;
      b.nfix = ((args.fix_real + VG - 1) / VG + 7) & ~7;
      b.fix.nslices = F32 ? b.fix.cin / kFixCi : 1;  // fp32: runs of one chunk, added in run order
      b.fix.cross = 0;
      const size_t flds = (size_t)VG * kFixSubFloats * sizeof(float);
      hipLaunchKernelGGL(k, dim3((unsigned)(grid + b.nfix)), dim3(T::NT), lds > flds ? lds : flds, st, b);
      return hip_code(hipGetLastError());
    }
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(T::NT), lds, st, args);
  return hip_code(hipGetLastError());
}

template <int NW, int WM, int WN, int PLANES, int EPI, int SCHED, bool F32 = false>
static int launch_h8_t(const ConvH8Args& args, int persist, hipStream_t st) {
  using T = TileH8<NW, WM, WN, PLANES>;
  if constexpr (T::LDS > kMaxLds) {
    return RRIN_E_CONFIG;
  } else {
    if (args.cin % 8 == 0 || args.tail_finite)
      return launch_h8_k<NW, WM, WN, PLANES, EPI, true, SCHED, F32>(args, persist, st);
    if constexpr (EPI == RRIN_EPI_LEAKY_REP || EPI == RRIN_EPI_SUBPIXEL) {
      return RRIN_E_CONFIG;  // decoder-side modes: always whole channel groups
    } else {
      return launch_h8_k<NW, WM, WN, PLANES, EPI, false, 0, F32>(args, persist, st);  // knobs need DMA
    }
  }
}

template <int NW, int WM, int WN, int SCHED>
static int launch_h8_cfg(const ConvH8Args& args, int prec, int epi, int persist, hipStream_t st) {
  const int planes = prec == RRIN_PREC_F16X3 ? 2 : 1;
  if (prec == RRIN_PREC_F32R) {
    switch (epi) {
      case RRIN_EPI_LINEAR: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LINEAR, SCHED, true>(args, persist, st);
      case RRIN_EPI_LEAKY: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY, SCHED, true>(args, persist, st);
      case RRIN_EPI_LEAKY_POOL: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY_POOL, SCHED, true>(args, persist, st);
      case RRIN_EPI_LEAKY_REP: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY_REP, SCHED, true>(args, persist, st);
      default: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_SUBPIXEL, SCHED, true>(args, persist, st);
    }
  }
  if (planes == 2) {
    switch (epi) {
      case RRIN_EPI_LINEAR: return launch_h8_t<NW, WM, WN, 2, RRIN_EPI_LINEAR, SCHED>(args, persist, st);
      case RRIN_EPI_LEAKY: return launch_h8_t<NW, WM, WN, 2, RRIN_EPI_LEAKY, SCHED>(args, persist, st);
      case RRIN_EPI_LEAKY_POOL: return launch_h8_t<NW, WM, WN, 2, RRIN_EPI_LEAKY_POOL, SCHED>(args, persist, st);
      case RRIN_EPI_LEAKY_REP: return launch_h8_t<NW, WM, WN, 2, RRIN_EPI_LEAKY_REP, SCHED>(args, persist, st);
      default: return launch_h8_t<NW, WM, WN, 2, RRIN_EPI_SUBPIXEL, SCHED>(args, persist, st);
    }
  }
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LINEAR, SCHED>(args, persist, st);
    case RRIN_EPI_LEAKY: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY, SCHED>(args, persist, st);
    case RRIN_EPI_LEAKY_POOL: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY_POOL, SCHED>(args, persist, st);
    case RRIN_EPI_LEAKY_REP: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_LEAKY_REP, SCHED>(args, persist, st);
    default: return launch_h8_t<NW, WM, WN, 1, RRIN_EPI_SUBPIXEL, SCHED>(args, persist, st);
  }
}

static bool h8_ok(const rrin_h8& v, int prec) {
  if (!v.hi || (prec == RRIN_PREC_F16X3 && !v.lo)) return false;
  if (prec == RRIN_PREC_F32R && v.lo) return false;  // one plane
  const rrin_geom g = make_geom_h8(v.g.h, v.g.w);
  return g.hp == v.g.hp && g.wp == v.g.wp && g.plane == v.g.plane;
}

static inline int64_t ring_pixels(int h, int w) {
  return h < 2 ? (int64_t)w : 2 * (int64_t)w + 2 * (int64_t)(h - 2);
}

static inline int planes_of(int prec) { return prec == RRIN_PREC_F16X3 ? 2 : 1; }
// record-layout precisions: F16X3 / F16 (8 halves per record), F32R (4 floats)
static inline bool rec_prec(int prec) {
  return prec == RRIN_PREC_F16X3 || prec == RRIN_PREC_F16 || prec == RRIN_PREC_F32R;
}
static inline int chans_per_rec(int prec) { return prec == RRIN_PREC_F32R ? 4 : 8; }

// Validate a conv descriptor and turn it into kernel arguments.
}  // namespace rrin
// the ring fix-up's host side (defined with its kernels below, at file scope)
static int edge_fix_prepare(const rrin_edge_fix_desc* d, rrin::EdgeFixArgs& a, dim3& grid);
static int edge_fix_run(rrin::EdgeFixArgs a, dim3 grid, int prec, bool full, const rrin_edge_fix_desc* d,
                        hipStream_t st, bool one_group = false);
namespace rrin {

static int h8_prepare(const rrin_conv_h8_desc* d, ConvH8Args& a, bool need_scratch = true) {
  if (!d || !d->whi || !d->bias) return RRIN_E_ARG;
  if (!rec_prec(d->prec)) return RRIN_E_ARG;
  if (d->prec == RRIN_PREC_F16X3 && !d->wlo) return RRIN_E_ARG;
  if (d->cfg < 0 || d->cfg >= kNumCfgH8 || retired(d->cfg) ||
      (planes_of(d->prec) == 2 ? kCfgH8[d->cfg].lds2 : kCfgH8[d->cfg].lds1) > kMaxLds)
    return RRIN_E_CONFIG;
  if (d->n < 1 || d->cin < 1 || d->cout < 8 || (d->cout & 7)) return RRIN_E_ARG;
  if (d->epi_mode < RRIN_EPI_LINEAR || d->epi_mode > RRIN_EPI_SUBPIXEL) return RRIN_E_ARG;
  if (!h8_ok(d->src, d->prec) || !h8_ok(d->dst, d->prec)) return RRIN_E_SHAPE;
  const bool sub = d->epi_mode == RRIN_EPI_SUBPIXEL;
  const int h = d->src.g.h, w = d->src.g.w;  // the grid the conv runs on
  if (d->dst.g.h != (sub ? 2 * h : h) || d->dst.g.w != (sub ? 2 * w : w)) return RRIN_E_SHAPE;
  const int cpr = chans_per_rec(d->prec);
  if (d->cin > cpr * d->src.groups || (sub ? d->cout / 4 : d->cout) > cpr * d->dst.groups) return RRIN_E_ARG;
  if (sub && ((d->cout & 31) || !d->edge)) return RRIN_E_ARG;
  if (!(d->slope >= 0.f && d->slope <= 1.f)) return RRIN_E_ARG;  // leaky() as max(t, slope t)
  if (d->epi_mode == RRIN_EPI_LEAKY_POOL) {
    if (!kCfgH8[d->cfg].pool_ok) return RRIN_E_CONFIG;  // a wave must own both rows of a pool pair
    if (!h8_ok(d->pool, d->prec) || (h & 1) || (w & 1) || d->pool.g.h * 2 != h || d->pool.g.w * 2 != w ||
        d->cout > cpr * d->pool.groups)
      return RRIN_E_SHAPE;
  }
  const int planes = planes_of(d->prec);
  const CfgH8& ci = kCfgH8[d->cfg];
  memset(&a, 0, sizeof(a));
  const int64_t sg = (int64_t)d->src.g_off * d->src.g.plane;
  a.src_hi = static_cast<const uint4*>(d->src.hi) + sg;
  a.src_lo = planes == 2 ? static_cast<const uint4*>(d->src.lo) + sg : nullptr;
  a.src_img = d->src.img_stride;
  a.src_gp = d->src.g.plane;
  a.src_wp = d->src.g.wp;
  a.cin = d->cin;
  a.nchunks = (d->cin + 2 * cpr - 1) / (2 * cpr);  // 2 record groups per chunk
  const int64_t dg = (int64_t)d->dst.g_off * d->dst.g.plane;
  a.dst_hi = static_cast<uint4*>(d->dst.hi) + dg;
  a.dst_lo = planes == 2 ? static_cast<uint4*>(d->dst.lo) + dg : nullptr;
  a.dst_img = d->dst.img_stride;
  a.dst_gp = d->dst.g.plane;
  a.dst_wp = d->dst.g.wp;
  a.cout = d->cout;
  if (d->epi_mode == RRIN_EPI_LEAKY_POOL) {
    const int64_t pg = (int64_t)d->pool.g_off * d->pool.g.plane;
    a.pool_hi = static_cast<uint4*>(d->pool.hi) + pg;
    a.pool_lo = planes == 2 ? static_cast<uint4*>(d->pool.lo) + pg : nullptr;
    a.pool_img = d->pool.img_stride;
    a.pool_gp = d->pool.g.plane;
    a.pool_wp = d->pool.g.wp;
  }
  a.w_hi = static_cast<const uint4*>(d->whi);
  a.w_lo = planes == 2 ? static_cast<const uint4*>(d->wlo) : nullptr;
  a.bias = d->bias;
  a.inv_wscale = d->prec == RRIN_PREC_F32R ? 1.0f : d->inv_wscale;
  a.slope = d->slope;
  a.tail_finite = d->tail_finite;
  a.status = d->status;
  a.h = h;
  a.w = w;
  if (sub) {
    a.edge = d->edge;
    a.ring = ring_pixels(2 * h, 2 * w);
  }
  a.co_blocks = (d->cout + ci.bm - 1) / ci.bm;
  a.tiles_x = (w + 31) / 32;
  a.tiles_y = (h + ci.th - 1) / ci.th;
  if (is_wino(d->cfg) && d->prec == RRIN_PREC_F16) {
    // fp16 Winograd (kind 6 only): 16-channel chunks of both record groups, no split / fold
    if (!is_winoh(d->cfg) || d->ksplit > 1 || d->ring_w) return RRIN_E_CONFIG;
    if ((d->cin & 15) && !d->tail_finite) return RRIN_E_CONFIG;
  } else if (is_wino(d->cfg)) {
    if (d->prec != RRIN_PREC_F32R) return RRIN_E_CONFIG;
    if ((d->cin & 3) && !d->tail_finite) return RRIN_E_CONFIG;  // stages whole records only
    // the register-U tiles stage both record groups of every chunk: they must exist
    if ((is_winoc(d->cfg) || d->cfg == kWinoC42Cfg) && (d->cin & 7) && !d->tail_finite) return RRIN_E_CONFIG;
    a.nchunks = (d->cin + 7) / 8;  // two record groups per K chunk
  }
  // the Winograd tiles stage every record group of every chunk (past cin against zero
  // weights): the source view must hold them, or the staging reads past the tensor
  if (is_wino(d->cfg) && 2 * a.nchunks > d->src.groups) return RRIN_E_SHAPE;
  {
    // LDS-DMA staging addresses the source through buffer resources (num_records 2^31 - 1) with
    // 32-bit byte offsets: the direct-form tiles from one base per image (every staged record
    // group of the image), the Winograd tiles from one base per tile and chunk (two groups).  A
    // larger span would stage zeros past the range -- a wrong result with no error -- so it is
    // rejected (a 64-channel fp16 view passes 2 GB near 6144x3456).
    const bool dma = is_wino(d->cfg) || d->cin % 8 == 0 || d->tail_finite;
    const int64_t span_groups = is_wino(d->cfg) ? 3 : 2 * (int64_t)a.nchunks;
    if (dma && span_groups * d->src.g.plane * 16 >= ((int64_t)1 << 31)) return RRIN_E_SHAPE;
  }
  a.n = d->n;
  if ((int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n > 0x7fffffff) return RRIN_E_SHAPE;
  a.ksplit = 1;
  if (d->ksplit > 1) {  // Winograd split-K: kinds 3 and 4 only
    if (d->cfg != kWinoQCfg && d->cfg != kWinoQ4Cfg) return RRIN_E_CONFIG;
    if (d->ksplit > kMaxKSplit || (need_scratch && (!d->part || !d->cnt))) return RRIN_E_ARG;
    a.kper = (a.nchunks + d->ksplit - 1) / d->ksplit;
    a.ksplit = (a.nchunks + a.kper - 1) / a.kper;  // every slice non-empty
    if ((int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n * a.ksplit > 0x7fffffff) return RRIN_E_SHAPE;
    a.part = d->part;
    a.cnt = d->cnt;
  }
  if (d->ring_w) {  // sub-pixel ring fold (kind 3, unsplit): no separate edge fix-up launch
    if (!sub || d->cfg != kWinoQCfg || a.ksplit > 1) return RRIN_E_CONFIG;
    if ((d->cin & 7) || !d->ring_bias || (need_scratch && (!d->ring_corr || !d->ring_cnt))) return RRIN_E_ARG;
    a.nseg = 2 * a.tiles_x + 2 * a.tiles_y;
    const int64_t rb = (int64_t)a.n * a.co_blocks * a.nseg;
    if (rb + (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n > 0x7fffffff) return RRIN_E_SHAPE;
    a.nring = (int)((rb + 7) & ~(int64_t)7);  // keeps the tiles' XCD remap aligned
    const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n + a.nring;
    a.rstride = 8 * (int)(grid / a.nring);    // ring groups spread over the whole grid
    a.wedge = d->ring_w;
    a.bias_raw = d->ring_bias;
    a.corr = d->ring_corr;
    a.rcnt = d->ring_cnt;
  }
  if (d->ring_full) {  // the ring from scratch with this conv (ABI 17)
    const rrin_edge_fix_desc* e = d->ring_full;
    if (!sub || d->ring_w || e->full != 1 || e->prec != d->prec || e->n != d->n || e->cout * 4 != d->cout)
      return RRIN_E_ARG;
    dim3 g;
    if (int rc = edge_fix_prepare(e, a.fix, g)) return rc;
    if (a.fix.s_hi != a.src_hi || a.fix.sh != h || a.fix.sw != w) return RRIN_E_ARG;  // this conv's input
    a.fix_gx = (int)g.x;
    a.fix_gy = (int)g.y;
    const int64_t nf = (int64_t)g.x * g.y * g.z;
    if (nf + (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n + 8 > 0x7fffffff) return RRIN_E_SHAPE;
    a.fix_real = (int)nf;
  }
  return 0;
}

// floats of rrin_conv_h8_desc.ring_corr and ints of .ring_cnt a ring-folding sub-pixel conv
// needs (0 and 0 when d->ring_w is NULL)
extern "C" int64_t rrin_conv_h8_ring_floats(const rrin_conv_h8_desc* d, int64_t* cnt_ints) {
  ConvH8Args a;
  const int rc = h8_prepare(d, a, false);
  if (rc) return rc;
  const int64_t segs = a.nring > 0 ? (int64_t)a.n * a.co_blocks * a.nseg : 0;
  if (cnt_ints) *cnt_ints = segs;
  return segs * 512;
}

// floats of rrin_conv_h8_desc.part and ints of .cnt a split-K conv needs (0 without a split)
extern "C" int64_t rrin_conv_h8_split_floats(const rrin_conv_h8_desc* d, int64_t* cnt_ints) {
  ConvH8Args a;
  const int rc = h8_prepare(d, a, false);
  if (rc) return rc;
  const int64_t tiles = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (cnt_ints) *cnt_ints = a.ksplit > 1 ? tiles : 0;
  return a.ksplit > 1 ? tiles * a.ksplit * 32 * 32 * kCfgH8[d->cfg].th : 0;  // 16 floats per thread of 64 x th threads
}

}  // namespace rrin

using namespace rrin;

extern "C" int rrin_make_geom_h8(int32_t h, int32_t w, rrin_geom* g) {
  if (!g || h < 1 || w < 1) return RRIN_E_ARG;
  *g = make_geom_h8(h, w);
  return 0;
}

extern "C" int rrin_conv_h8_cfg_count(void) { return kNumCfgH8; }
extern "C" int rrin_conv_h8_cfg_bm(int32_t cfg) {
  return (cfg >= 0 && cfg < kNumCfgH8) ? kCfgH8[cfg].bm : RRIN_E_CONFIG;
}
extern "C" int rrin_conv_h8_cfg_th(int32_t cfg) {
  return (cfg >= 0 && cfg < kNumCfgH8) ? kCfgH8[cfg].th : RRIN_E_CONFIG;
}
// 0: direct form; Winograd tile kind: 1 BM 32 / 4 waves, 3 BM 32 / 8 waves, 4 BM 32 x TH 4 / 4 waves;
// 6 BM 64 x TH 4 and 7 BM 32 x TH 8, register-U tiles (conv_winoc.hip; kind 6 also at fp16,
// conv_winoh.hip); 14 BM 32 x TH 8, the register-U tile in F(4,3) x F(2,3) (conv_winoc42.hip,
// packed by rrin_pack_conv3x3_wino42).  The retired ids (19, 22) report -1.
extern "C" int rrin_conv_h8_cfg_wino(int32_t cfg) {
  return cfg == kWinoCfg      ? 1
         : cfg == kWinoQCfg   ? 3
         : cfg == kWinoQ4Cfg  ? 4
         : cfg == kWinoC2Cfg  ? 6
         : cfg == kWinoC1Cfg  ? 7
         : cfg == kWinoC42Cfg ? 14
         : retired(cfg)       ? -1
                              : 0;
}
// Fused level-0 UNetConvBlock (conv_block0.hip): validate and launch.
extern "C" int rrin_conv_block0_h8_fwd(const rrin_block0_h8_desc* d, void* stream) {
  if (!d || !d->whi_a || !d->bias_a || !d->whi_b || !d->bias_b) return RRIN_E_ARG;
  for (int cfg : {d->cfg_a, d->cfg_b})
    if (cfg < 0 || cfg >= kNumCfgH8 || is_wino(cfg)) return RRIN_E_CONFIG;  // direct-form packs only
  if (d->n < 1 || d->cin < 1 || ((d->cin & 7) && !d->tail_finite)) return RRIN_E_ARG;
  if (!(d->slope >= 0.f && d->slope <= 1.f)) return RRIN_E_ARG;
  const int prec = RRIN_PREC_F16;
  if (!h8_ok(d->src, prec) || !h8_ok(d->dst, prec) || d->src.lo || d->dst.lo) return RRIN_E_SHAPE;
  const int h = d->src.g.h, w = d->src.g.w;
  if (d->dst.g.h != h || d->dst.g.w != w || d->dst.groups < 4 || d->cin > 8 * d->src.groups) return RRIN_E_SHAPE;
  const bool pool = d->pool.hi != nullptr;
  if (pool && (!h8_ok(d->pool, prec) || d->pool.lo || (h & 1) || (w & 1) || d->pool.g.h * 2 != h ||
               d->pool.g.w * 2 != w || d->pool.groups < 4))
    return RRIN_E_SHAPE;
  // 32-bit byte offsets within an image (buffer loads and stores)
  const int64_t lim = (int64_t)1 << 31;
  if (d->src.img_stride * 16 >= lim || d->dst.img_stride * 16 >= lim || (pool && d->pool.img_stride * 16 >= lim))
    return RRIN_E_SHAPE;
  Block0Args a;
  memset(&a, 0, sizeof(a));
  a.src = static_cast<const uint4*>(d->src.hi) + (int64_t)d->src.g_off * d->src.g.plane;
  a.src_img = (int)d->src.img_stride;
  a.src_gp = (int)d->src.g.plane;
  a.src_wp = d->src.g.wp;
  a.src_hp = d->src.g.hp;
  a.cin = d->cin;
  a.ngroups = (d->cin + 7) / 8;
  a.nch = (d->cin + 15) / 16;
  a.wa = static_cast<const uint4*>(d->whi_a);
  a.bma = kCfgH8[d->cfg_a].bm;
  a.ba = d->bias_a;
  a.isa = d->inv_wscale_a;
  a.wb = static_cast<const uint4*>(d->whi_b);
  a.bmb = kCfgH8[d->cfg_b].bm;
  a.bb = d->bias_b;
  a.isb = d->inv_wscale_b;
  a.dst = static_cast<uint4*>(d->dst.hi) + (int64_t)d->dst.g_off * d->dst.g.plane;
  a.dst_img = (int)d->dst.img_stride;
  a.dst_gp = (int)d->dst.g.plane;
  a.dst_wp = d->dst.g.wp;
  if (pool) {
    a.pool = static_cast<uint4*>(d->pool.hi) + (int64_t)d->pool.g_off * d->pool.g.plane;
    a.pool_img = (int)d->pool.img_stride;
    a.pool_gp = (int)d->pool.g.plane;
    a.pool_wp = d->pool.g.wp;
  }
  a.slope = d->slope;
  a.h = h;
  a.w = w;
  a.n = d->n;
  a.tiles_x = (w + kB0TW - 1) / kB0TW;
  a.tiles_y = (h + kB0TH - 1) / kB0TH;
  a.status = d->status;
  if ((int64_t)a.tiles_x * a.tiles_y * a.n > 0x7fffffff) return RRIN_E_SHAPE;
  return launch_block0(a, static_cast<hipStream_t>(stream));
}

extern "C" int rrin_conv_h8_cfg_ok(int32_t cfg, int32_t prec) {
  if (cfg < 0 || cfg >= kNumCfgH8) return 0;
  if (!rec_prec(prec) || retired(cfg)) return 0;
  // Winograd tiles: exact fp32 records; the register-U kind 6 also at fp16 (conv_winoh.hip)
  if (is_wino(cfg) && (prec == RRIN_PREC_F16 ? !is_winoh(cfg) : prec != RRIN_PREC_F32R)) return 0;
  return (planes_of(prec) == 2 ? kCfgH8[cfg].lds2 : kCfgH8[cfg].lds1) <= kMaxLds ? 1 : 0;
}

extern "C" int rrin_conv_h8_cfg_fits(int32_t cfg, int32_t prec, int32_t cin) {
  if (!rrin_conv_h8_cfg_ok(cfg, prec) || cin < 1) return 0;
  const CfgH8& c = kCfgH8[cfg];
  const int nch = (cin + 2 * chans_per_rec(prec) - 1) / (2 * chans_per_rec(prec));
  if (!(c.sched & SCHED_WRES) || nch <= 2) return 1;
  const int planes = planes_of(prec);
  const size_t lds = (planes == 2 ? c.lds2 : c.lds1) + (size_t)(nch - 2) * c.wslab * planes;
  return lds <= kMaxLds ? 1 : 0;
}

static int conv3x3_h8_launch(const rrin_conv_h8_desc* d, const ConvH8Args& a, hipStream_t st);

bool rrin::ring_in_launch_ok(int cfg, int cin, int prec) {
  if (cfg < 0 || cfg >= kNumCfgH8 || retired(cfg) || cin % kFixCi) return false;
  if (is_winoc(cfg)) return prec == RRIN_PREC_F32R;  // kinds 6 / 7 (exact fp32): 256 threads
  if (is_wino(cfg)) return false;                    // kinds 1, 3, 4: the fix-up as a second launch
  return kCfgH8[cfg].nt >= 256;                      // direct-form tiles of 256 / 512 threads
}

extern "C" int rrin_conv3x3_h8_fwd(const rrin_conv_h8_desc* d, void* stream) {
  ConvH8Args a;
  const int rc = h8_prepare(d, a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (a.fix_real > 0) {
    // in the conv's launch (a tile of 256 or 512 threads); otherwise the conv, then the FULL
    // fix-up as its own launch in the same summation order
    if (!ring_in_launch_ok(d->cfg, a.fix.cin, d->prec)) {
      ConvH8Args b = a;
      b.fix_real = 0;
      if (int e = conv3x3_h8_launch(d, b, st)) return e;
      dim3 g((unsigned)a.fix_gx, (unsigned)a.fix_gy, (unsigned)d->n);
      return edge_fix_run(a.fix, g, d->prec, true, nullptr, st, true);  // the in-launch summation order
    }
  }
  return conv3x3_h8_launch(d, a, st);
}

static int conv3x3_h8_launch(const rrin_conv_h8_desc* d, const ConvH8Args& a, hipStream_t st) {
  if (d->cfg == kWinoCfg) return launch_wino(a, d->epi_mode, st);
  if (d->cfg == kWinoQCfg) return launch_winoq(a, d->epi_mode, 8, st);
  if (d->cfg == kWinoQ4Cfg) return launch_winoq(a, d->epi_mode, 4, st);
  if (is_winoh(d->cfg) && d->prec == RRIN_PREC_F16) return launch_winoh(a, d->epi_mode, st);
  if (d->cfg == kWinoC2Cfg) return launch_winoc(a, d->epi_mode, 2, st);
  if (d->cfg == kWinoC1Cfg) return launch_winoc(a, d->epi_mode, 1, st);
  if (d->cfg == kWinoC42Cfg) return launch_winoc42(a, d->epi_mode, st);
  switch (d->cfg) {
#define X(id, nw, wm, wn, sc, pe) \
  case id:                        \
    return launch_h8_cfg<nw, wm, wn, sc>(a, d->prec, d->epi_mode, pe, st);
    RRIN_H8_CFGS(X)
#undef X
  }
  return RRIN_E_CONFIG;
}

#ifdef RRIN_LAB
// Kernel lab (tools/conv_lab.py ablate; built only into librrin_lab.so, `make
// lab`): one F16X3 LEAKY conv of tile config cfg 0, 1 or 6 with the schedule
// knobs `sched` (SCHED_*, ablations included) and grid `persist` (as PE).
template <int NW, int WM, int WN, bool F32>
static int lab_cfg(const ConvH8Args& a, int sched, int persist, hipStream_t st) {
  constexpr int P = F32 ? 1 : 2;
  switch (sched) {
#define L(v) \
  case v:    \
    return launch_h8_k<NW, WM, WN, P, RRIN_EPI_LEAKY, true, v, F32>(a, persist, st);
    L(0) L(1) L(2) L(3) L(4) L(7) L(8) L(11) L(12) L(15) L(16) L(32) L(48) L(64) L(96) L(128) L(144)
#undef L
  }
  return RRIN_E_CONFIG;
}

// F16X3 (cfg 0, 1, 6) or F32R (cfg 0, 1, 3, 4, 5, 6, 16) LEAKY conv with schedule bits
extern "C" int rrin_conv3x3_h8_lab(const rrin_conv_h8_desc* d, int32_t sched, int32_t persist, void* stream) {
  if (d && is_wino(d->cfg) && d->epi_mode == RRIN_EPI_LEAKY) {  // Winograd: sched = ablation bits
    ConvH8Args a;
    const int rc = h8_prepare(d, a);
    if (rc) return rc;
    return launch_wino_lab(a, sched, (hipStream_t)stream);
  }
  if (!d || (d->prec != RRIN_PREC_F16X3 && d->prec != RRIN_PREC_F32R) || d->epi_mode != RRIN_EPI_LEAKY ||
      (d->cin % 8))
    return RRIN_E_ARG;
  if (d->prec == RRIN_PREC_F32R && (sched & SCHED_MFMA16)) return RRIN_E_CONFIG;
  ConvH8Args a;
  const int rc = h8_prepare(d, a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (d->prec == RRIN_PREC_F32R) {
    switch (d->cfg) {
      case 0: return lab_cfg<8, 2, 2, true>(a, sched, persist, st);
      case 1: return lab_cfg<8, 1, 2, true>(a, sched, persist, st);
      case 3: return lab_cfg<4, 1, 4, true>(a, sched, persist, st);
      case 4: return lab_cfg<4, 2, 1, true>(a, sched, persist, st);
      case 5: return lab_cfg<8, 4, 2, true>(a, sched, persist, st);
      case 6: return lab_cfg<4, 1, 2, true>(a, sched, persist, st);
      case 16: return lab_cfg<4, 1, 1, true>(a, sched, persist, st);
    }
    return RRIN_E_CONFIG;
  }
  switch (d->cfg) {
    case 0: return lab_cfg<8, 2, 2, false>(a, sched, persist, st);
    case 1: return lab_cfg<8, 1, 2, false>(a, sched, persist, st);
    case 6: return lab_cfg<4, 1, 2, false>(a, sched, persist, st);
  }
  return RRIN_E_CONFIG;
}
#endif

extern "C" int64_t rrin_pack_conv3x3_h8_halves(int32_t cout, int32_t cin, int32_t bm) {
  if (cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  const int64_t cob = (cout + bm - 1) / bm, nch = (cin + 15) / 16;
  return cob * nch * 9 * 2 * bm * 8;
}

extern "C" int rrin_pack_conv3x3_h8(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                                    const int32_t* perm, int32_t prec, uint16_t* whi, uint16_t* wlo, float* bpack,
                                    float* inv_wscale) {
  if (!w || !b || !whi || !bpack || !inv_wscale || cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  if (prec != RRIN_PREC_F16X3 && prec != RRIN_PREC_F16) return RRIN_E_ARG;
  if (prec == RRIN_PREC_F16X3 && !wlo) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  float mx = 0.f;
  const int64_t nw = (int64_t)cout * cin * 9;
  for (int64_t i = 0; i < nw; ++i) mx = fmaxf(mx, fabsf(w[i]));
  if (!(mx < INFINITY)) return RRIN_E_ARG;
  int s = 0;
  if (mx > 0.f) {
    int e;
    frexpf(mx, &e);  // mx in [2^(e-1), 2^e)
    s = 13 - e;      // scaled max in [2^12, 2^13)
  }
  const float scale = ldexpf(1.0f, s);
  *inv_wscale = ldexpf(1.0f, -s);
  const int cob_n = (cout + bm - 1) / bm, nch = (cin + 15) / 16;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int tap = 0; tap < 9; ++tap)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < bm; ++col)
            for (int e = 0; e < 8; ++e) {
              const int co = cob * bm + col, ch = c * 16 + hh * 8 + e;
              float v = 0.f;
              if (co < cout && ch < cin) v = w[((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9 + tap] * scale;
              const uint16_t hbits = f2h_rne(v);
              whi[o] = hbits;
              if (prec == RRIN_PREC_F16X3) wlo[o] = f2h_rne((v - h2f(hbits)) * 2048.0f);
              ++o;
            }
  for (int co = 0; co < cob_n * bm; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}

extern "C" int64_t rrin_pack_conv3x3_r32_floats(int32_t cout, int32_t cin, int32_t bm) {
  if (cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  const int64_t cob = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  return cob * nch * 9 * 2 * bm * 4;
}

extern "C" int rrin_pack_conv3x3_r32(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                                     const int32_t* perm, float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  const int cob_n = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int tap = 0; tap < 9; ++tap)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < bm; ++col)
            for (int e = 0; e < 4; ++e) {
              const int co = cob * bm + col, ch = c * 8 + hh * 4 + e;
              wpack[o++] = (co < cout && ch < cin) ? w[((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9 + tap] : 0.f;
            }
  for (int co = 0; co < cob_n * bm; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}

extern "C" int64_t rrin_ring_pixels(int32_t h, int32_t w) {
  if (h < 1 || w < 1) return RRIN_E_ARG;
  return ring_pixels(h, w);
}

// Phase-combined weights of conv3x3 o upsample_x2 (see rrin_hip.h).  kR[p][a][k]:
// coefficient of low-res row m+a-1 in upsampled row 2m+p+k-1 (align_corners=False).
extern "C" int rrin_subpixel_weights(const float* w, const float* b, int32_t cout, int32_t cin, float* wsub,
                                     float* bsub) {
  if (!w || !b || !wsub || !bsub || cout < 8 || (cout & 7) || cin < 1) return RRIN_E_ARG;
  static const double kR[2][3][3] = {{{0.75, 0.25, 0.0}, {0.25, 0.75, 0.75}, {0.0, 0.0, 0.25}},
                                     {{0.25, 0.0, 0.0}, {0.75, 0.75, 0.25}, {0.0, 0.25, 0.75}}};
  for (int co = 0; co < cout; ++co)
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
      const int64_t row = (int64_t)(co >> 3) * 32 + ph * 8 + (co & 7);
      bsub[row] = b[co];
      for (int ci = 0; ci < cin; ++ci) {
        const float* src = w + ((int64_t)co * cin + ci) * 9;
        float* dst = wsub + (row * cin + ci) * 9;
        for (int ay = 0; ay < 3; ++ay)
          for (int ax = 0; ax < 3; ++ax) {
            double acc = 0.0;
            for (int ky = 0; ky < 3; ++ky)
              for (int kx = 0; kx < 3; ++kx) acc += kR[py][ay][ky] * kR[px][ax][kx] * (double)src[ky * 3 + kx];
            dst[ay * 3 + ax] = (float)acc;
          }
      }
    }
  return 0;
}

template <int PLANES, int KS, bool F32, bool FULL>
static int edge_fix_launch_m(const EdgeFixArgs& a, dim3 grid, hipStream_t st) {
  constexpr size_t lds = (size_t)KS * kFixSubFloats * sizeof(float);
  static_assert(lds <= 160 * 1024, "edge fix LDS");
  static_assert(kFixSubFloats >= 4 * 256, "K-group sums fit a staging region");
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)edge_fix_h8_kernel<PLANES, KS, F32, FULL>, (int)lds, st)) return e;
  hipLaunchKernelGGL((edge_fix_h8_kernel<PLANES, KS, F32, FULL>), grid, dim3(256 * KS), lds, st, a);
  return hip_code(hipGetLastError());
}

template <int PLANES, int KS, bool F32 = false>
static int edge_fix_launch(const EdgeFixArgs& a, dim3 grid, hipStream_t st, bool full) {
  return full ? edge_fix_launch_m<PLANES, KS, F32, true>(a, grid, st)
              : edge_fix_launch_m<PLANES, KS, F32, false>(a, grid, st);
}

// K groups and K runs of the ring fix-up, by cin and precision only (the
// summation order never depends on batch, size or scratch).  fp32 records: 2
// groups from cin 64 on, never 4 (4 x 256 threads cap a thread at 128 VGPRs and
// the fp32 kernel spills there: 31.6 vs 15.7 us per launch), runs of one chunk per
// group (cin / 64 runs).  fp16: split16 stops at 2 groups (the two-plane kernel
// spills at 4), one run.
static void edge_fix_split(int cin, int prec, int* ks, int* nsl) {
  *nsl = 1;
  if (prec == RRIN_PREC_F32R) {
    *ks = cin % (2 * kFixCi) == 0 ? 2 : 1;
    if (cin % (*ks * kFixCi) == 0) *nsl = cin / (*ks * kFixCi);
    return;
  }
  *ks = cin % (2 * kFixCi) == 0 && cin >= 4 * kFixCi ? 2 : 1;
  if (planes_of(prec) == 1 && cin % (4 * kFixCi) == 0 && cin >= 8 * kFixCi) *ks = 4;
}

// validate d and fill a (everything but the K split); grid: ring tiles x co blocks x images
static int edge_fix_prepare(const rrin_edge_fix_desc* d, EdgeFixArgs& a, dim3& grid) {
  if (!d || (!d->edge && !d->full) || !d->wedge || !d->bias || (d->full != 0 && d->full != 1)) return RRIN_E_ARG;
  if (!rec_prec(d->prec)) return RRIN_E_ARG;
  if (d->n < 1 || d->cin < 8 || (d->cin & 7) || d->cout < 8 || (d->cout & 7)) return RRIN_E_ARG;
  if (d->epi_mode != RRIN_EPI_LINEAR && d->epi_mode != RRIN_EPI_LEAKY) return RRIN_E_ARG;
  if (!h8_ok(d->src, d->prec) || !h8_ok(d->dst, d->prec)) return RRIN_E_SHAPE;
  if (d->dst.g.h != 2 * d->src.g.h || d->dst.g.w != 2 * d->src.g.w) return RRIN_E_SHAPE;
  const int cpr = chans_per_rec(d->prec);
  if (d->cin > cpr * d->src.groups || d->cout > cpr * d->dst.groups) return RRIN_E_ARG;
  const int planes = planes_of(d->prec);
  memset(&a, 0, sizeof(a));
  const int64_t sg = (int64_t)d->src.g_off * d->src.g.plane, dg = (int64_t)d->dst.g_off * d->dst.g.plane;
  a.s_hi = static_cast<const uint4*>(d->src.hi) + sg;
  a.s_lo = planes == 2 ? static_cast<const uint4*>(d->src.lo) + sg : nullptr;
  a.s_img = d->src.img_stride;
  a.s_gp = d->src.g.plane;
  a.s_wp = d->src.g.wp;
  a.sh = d->src.g.h;
  a.sw = d->src.g.w;
  a.cin = d->cin;
  if (d->prec == RRIN_PREC_F32R) {
    a.d_f32 = static_cast<float*>(d->dst.hi) + dg * 4;
  } else {
    a.d_hi = static_cast<_Float16*>(d->dst.hi) + dg * 8;
    a.d_lo = planes == 2 ? static_cast<_Float16*>(d->dst.lo) + dg * 8 : nullptr;
  }
  a.d_img = d->dst.img_stride;
  a.d_gp = d->dst.g.plane;
  a.d_wp = d->dst.g.wp;
  a.cout = d->cout;
  a.edge = d->edge;
  a.wedge = d->wedge;
  a.bias = d->bias;
  a.ring = ring_pixels(d->dst.g.h, d->dst.g.w);
  a.slope = d->slope;
  a.leaky = d->epi_mode == RRIN_EPI_LEAKY;
  a.status = d->status;
  const int H = d->dst.g.h, W = d->dst.g.w;
  a.tiles_row = (W + kFixPx - 1) / kFixPx;
  a.tiles_col = (H - 2 + kFixPx - 1) / kFixPx;
  grid = dim3((unsigned)(2 * a.tiles_row + 2 * a.tiles_col), (unsigned)((d->cout + kFixCo - 1) / kFixCo),
              (unsigned)d->n);
  a.nslices = 1;
  a.cross = 0;
  return 0;
}

// the fix-up as its own launch: K groups / runs by edge_fix_split; the cross-workgroup K split
// where the caller passed its scratch (fp32 records)
// (one_group: one K group, fp32 runs of one chunk -- the order of the in-launch fix-up)
static int edge_fix_run(EdgeFixArgs a, dim3 grid, int prec, bool full, const rrin_edge_fix_desc* d,
                        hipStream_t st, bool one_group) {
  int ks, nsl;
  edge_fix_split(a.cin, prec, &ks, &nsl);
  if (one_group) {
    ks = 1;
    nsl = prec == RRIN_PREC_F32R ? a.cin / kFixCi : 1;
    d = nullptr;
  }
  a.nslices = nsl;
  a.cross = 0;
  dim3 g = grid;
  const int n = (int)grid.z;
  const int64_t tiles = (int64_t)grid.x * grid.y * n;
  if (d && nsl > 1 && d->part && d->cnt && tiles * nsl * 1024 <= d->part_floats && tiles <= d->cnt_len) {
    a.cross = 1;  // one workgroup per K run (same arithmetic as the loop over runs)
    a.part = d->part;
    a.cnt = d->cnt;
    g.z = (unsigned)(n * nsl);
  }
  if (prec == RRIN_PREC_F32R) {
    return ks == 2 ? edge_fix_launch<1, 2, true>(a, g, st, full) : edge_fix_launch<1, 1, true>(a, g, st, full);
  }
  switch (planes_of(prec) * 8 + ks) {
    case 2 * 8 + 2: return edge_fix_launch<2, 2>(a, g, st, full);
    case 2 * 8 + 1: return edge_fix_launch<2, 1>(a, g, st, full);
    case 1 * 8 + 4: return edge_fix_launch<1, 4>(a, g, st, full);
    case 1 * 8 + 2: return edge_fix_launch<1, 2>(a, g, st, full);
    default: return edge_fix_launch<1, 1>(a, g, st, full);
  }
}

extern "C" int rrin_subpixel_edge_fix_h8(const rrin_edge_fix_desc* d, void* stream) {
  EdgeFixArgs a;
  dim3 grid;
  if (int e = edge_fix_prepare(d, a, grid)) return e;
  return edge_fix_run(a, grid, d->prec, d->full == 1, d, (hipStream_t)stream);
}

extern "C" int64_t rrin_edge_fix_split_floats(const rrin_edge_fix_desc* d, int64_t* cnt) {
  if (!d || d->n < 1 || d->cin < 8 || (d->cin & 7) || d->cout < 8 || !rec_prec(d->prec)) return RRIN_E_ARG;
  int ks, nsl;
  edge_fix_split(d->cin, d->prec, &ks, &nsl);
  const int H = d->dst.g.h, W = d->dst.g.w;
  if (H < 2 || W < 1) return RRIN_E_SHAPE;
  const int64_t tiles = (int64_t)(2 * ((W + kFixPx - 1) / kFixPx) + 2 * ((H - 2 + kFixPx - 1) / kFixPx)) *
                        ((d->cout + kFixCo - 1) / kFixCo) * d->n;
  if (cnt) *cnt = nsl > 1 ? tiles : 0;
  return nsl > 1 ? tiles * nsl * 1024 : 0;
}

extern "C" int rrin_upsample2x_h8(const rrin_h8* src, const rrin_h8* dst, int32_t n, int32_t prec, void* stream) {
  if (!src || !dst || n < 1 || !rec_prec(prec)) return RRIN_E_ARG;
  if (!h8_ok(*src, prec) || !h8_ok(*dst, prec)) return RRIN_E_SHAPE;
  if (dst->g.h != 2 * src->g.h || dst->g.w != 2 * src->g.w || dst->groups < src->groups) return RRIN_E_SHAPE;
  const int64_t total = (int64_t)n * src->groups * dst->g.h * dst->g.w;
  const int grid = (int)((total + 255) / 256);
  const int64_t so = (int64_t)src->g_off * src->g.plane, dof = (int64_t)dst->g_off * dst->g.plane;
  const uint4* shi = static_cast<const uint4*>(src->hi) + so;
  uint4* dhi = static_cast<uint4*>(dst->hi) + dof;
  hipStream_t st = (hipStream_t)stream;
  if (prec == RRIN_PREC_F32R) {
    hipLaunchKernelGGL(up2x_r32_kernel, dim3(grid), dim3(256), 0, st, shi, src->img_stride, src->g.plane, src->g.wp,
                       src->g.h, src->g.w, dhi, dst->img_stride, dst->g.plane, dst->g.wp, src->groups, total);
  } else if (planes_of(prec) == 2) {
    hipLaunchKernelGGL(up2x_h8_kernel<2>, dim3(grid), dim3(256), 0, st, shi,
                       static_cast<const uint4*>(src->lo) + so, src->img_stride, src->g.plane, src->g.wp, src->g.h,
                       src->g.w, dhi, static_cast<uint4*>(dst->lo) + dof, dst->img_stride, dst->g.plane, dst->g.wp,
                       src->groups, total);
  } else {
    hipLaunchKernelGGL(up2x_h8_kernel<1>, dim3(grid), dim3(256), 0, st, shi, (const uint4*)nullptr,
                       src->img_stride, src->g.plane, src->g.wp, src->g.h, src->g.w, dhi, (uint4*)nullptr,
                       dst->img_stride, dst->g.plane, dst->g.wp, src->groups, total);
  }
  return hip_code(hipGetLastError());
}

namespace rrin {
// zero channels [c0, c1) of every interior pixel of a record-layout view (H8 hi
// and lo planes, or R32); rrin_unet_fwd clears the channels its PLAIN head
// writes past in_ch so that the next call's first conv never stages them
__global__ void clear_channels_kernel(_Float16* hi, _Float16* lo, float* r32, int64_t img_stride, int64_t gp, int wp,
                                      int c0, int c, int h, int w, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  int64_t t = i / w;
  const int y = (int)(t % h);
  t /= h;
  const int ch = c0 + (int)(t % c);
  const int n = (int)(t / c);
  if (r32) {
    r32[r32_elem_index(img_stride, gp, wp, n, ch, y, x)] = 0.f;
    return;
  }
  const int64_t k = h8_half_index(img_stride, gp, wp, n, ch, y, x);
  hi[k] = (_Float16)0.f;
  if (lo) lo[k] = (_Float16)0.f;
}

int clear_channels_h8(const rrin_h8* v, int32_t n, int32_t c0, int32_t c1, int32_t prec, hipStream_t st) {
  if (!v || n < 1 || c0 < 0 || c1 <= c0 || !rec_prec(prec) || c1 > chans_per_rec(prec) * v->groups) return RRIN_E_ARG;
  const int64_t total = (int64_t)n * (c1 - c0) * v->g.h * v->g.w;
  const int grid = (int)((total + 255) / 256);
  if (prec == RRIN_PREC_F32R) {
    hipLaunchKernelGGL(clear_channels_kernel, dim3(grid), dim3(256), 0, st, (_Float16*)nullptr, (_Float16*)nullptr,
                       static_cast<float*>(v->hi) + (int64_t)v->g_off * v->g.plane * 4, v->img_stride, v->g.plane,
                       v->g.wp, c0, c1 - c0, v->g.h, v->g.w, total);
  } else {
    const int64_t go = (int64_t)v->g_off * v->g.plane * 8;
    hipLaunchKernelGGL(clear_channels_kernel, dim3(grid), dim3(256), 0, st, static_cast<_Float16*>(v->hi) + go,
                       planes_of(prec) == 2 ? static_cast<_Float16*>(v->lo) + go : (_Float16*)nullptr,
                       (float*)nullptr, v->img_stride, v->g.plane, v->g.wp, c0, c1 - c0, v->g.h, v->g.w, total);
  }
  return hip_code(hipGetLastError());
}
}  // namespace rrin

extern "C" int rrin_nchw_to_h8(const float* src, int32_t n, int32_t c, int32_t ch_off, const rrin_h8* dst,
                               int32_t prec, void* stream) {
  if (!src || !dst || n < 1 || c < 1 || ch_off < 0 || !rec_prec(prec)) return RRIN_E_ARG;
  if (ch_off + c > chans_per_rec(prec) * dst->groups) return RRIN_E_ARG;
  if (!h8_ok(*dst, prec)) return RRIN_E_SHAPE;
  const int64_t total = (int64_t)n * c * dst->g.h * dst->g.w;
  const int grid = (int)((total + 255) / 256);
  if (prec == RRIN_PREC_F32R) {
    hipLaunchKernelGGL(nchw_to_r32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src,
                       static_cast<float*>(dst->hi) + (int64_t)dst->g_off * dst->g.plane * 4, dst->img_stride,
                       dst->g.plane, dst->g.wp, ch_off, c, dst->g.h, dst->g.w, total);
    return hip_code(hipGetLastError());
  }
  const int64_t go = (int64_t)dst->g_off * dst->g.plane * 8;
  hipLaunchKernelGGL(nchw_to_h8_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src,
                     static_cast<_Float16*>(dst->hi) + go,
                     planes_of(prec) == 2 ? static_cast<_Float16*>(dst->lo) + go : (_Float16*)nullptr,
                     dst->img_stride, dst->g.plane, dst->g.wp, ch_off, c, dst->g.h, dst->g.w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_h8_to_nchw(const rrin_h8* src, int32_t n, int32_t c, int32_t ch_off, float* dst, int32_t prec,
                               void* stream) {
  if (!src || !dst || n < 1 || c < 1 || ch_off < 0 || !rec_prec(prec)) return RRIN_E_ARG;
  if (ch_off + c > chans_per_rec(prec) * src->groups) return RRIN_E_ARG;
  if (!h8_ok(*src, prec)) return RRIN_E_SHAPE;
  const int64_t total = (int64_t)n * c * src->g.h * src->g.w;
  const int grid = (int)((total + 255) / 256);
  if (prec == RRIN_PREC_F32R) {
    hipLaunchKernelGGL(r32_to_nchw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const float*>(src->hi) + (int64_t)src->g_off * src->g.plane * 4, src->img_stride,
                       src->g.plane, src->g.wp, ch_off, dst, c, src->g.h, src->g.w, total);
    return hip_code(hipGetLastError());
  }
  const int64_t go = (int64_t)src->g_off * src->g.plane * 8;
  hipLaunchKernelGGL(h8_to_nchw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const _Float16*>(src->hi) + go,
                     planes_of(prec) == 2 ? static_cast<const _Float16*>(src->lo) + go : (const _Float16*)nullptr,
                     src->img_stride, src->g.plane, src->g.wp, ch_off, dst, c, src->g.h, src->g.w, total);
  return hip_code(hipGetLastError());
}

template <int COUT, int MODE>
static int head_h8_launch(const HeadH8Args& a, int planes, int grid, hipStream_t st) {
  if (planes == 0)  // F32R
    hipLaunchKernelGGL((head_r32_kernel<COUT, MODE>), dim3(grid), dim3(256), 0, st, a);
  else if (planes == 2)
    hipLaunchKernelGGL((head_h8_kernel<COUT, MODE, 2>), dim3(grid), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((head_h8_kernel<COUT, MODE, 1>), dim3(grid), dim3(256), 0, st, a);
  return hip_code(hipGetLastError());
}

// Validate a head descriptor and turn it into kernel arguments (grid: blocks).
static int head_prepare(const rrin_head_h8_desc* d, HeadH8Args& a, int& grid) {
  if (!d || !d->w || !d->bias || d->cin != 32 || d->n < 1) return RRIN_E_ARG;
  if (!rec_prec(d->prec)) return RRIN_E_ARG;
  if (!h8_ok(d->src, d->prec) || !h8_ok(d->g16, d->prec)) return RRIN_E_SHAPE;
  const int h = d->src.g.h, w = d->src.g.w;
  const int cpr = chans_per_rec(d->prec);
  if (d->g16.g.h != h || d->g16.g.w != w || d->src.groups * cpr < 32) return RRIN_E_SHAPE;
  if (d->mode != RRIN_HEAD_PLAIN) {
    if (d->g16.groups * cpr < 16 || d->g16.g_off != 0 || !d->coef) return RRIN_E_ARG;
  } else if (cpr * d->g16.groups < d->cout) {
    return RRIN_E_ARG;
  }
  if (d->mode == RRIN_HEAD_FINAL && !d->out) return RRIN_E_ARG;
  const int planes = planes_of(d->prec);
  memset(&a, 0, sizeof(a));
  const int64_t sg = (int64_t)d->src.g_off * d->src.g.plane;
  a.src_hi = static_cast<const uint4*>(d->src.hi) + sg;
  a.src_lo = planes == 2 ? static_cast<const uint4*>(d->src.lo) + sg : nullptr;
  a.src_img = d->src.img_stride;
  a.src_gp = d->src.g.plane;
  a.src_wp = d->src.g.wp;
  const int64_t gg = (int64_t)d->g16.g_off * d->g16.g.plane * 8;
  if (d->prec == RRIN_PREC_F32R) {
    a.g32 = static_cast<uint4*>(d->g16.hi) + (int64_t)d->g16.g_off * d->g16.g.plane;
  } else {
    a.g_hi = static_cast<_Float16*>(d->g16.hi) + gg;
    a.g_lo = planes == 2 ? static_cast<_Float16*>(d->g16.lo) + gg : nullptr;
  }
  a.g_img = d->g16.img_stride;
  a.g_gp = d->g16.g.plane;
  a.g_wp = d->g16.g.wp;
  a.w = d->w;
  a.bias = d->bias;
  a.coef = d->coef;
  a.out = d->out;
  a.raw = d->raw_out;
  a.status = d->status;
  if (d->mode == RRIN_HEAD_FLOW && d->flow_raw.hi) {
    if (!h8_ok(d->flow_raw, d->prec) || d->flow_raw.g.h != h || d->flow_raw.g.w != w) return RRIN_E_SHAPE;
    const int64_t fo = (int64_t)d->flow_raw.g_off * d->flow_raw.g.plane * 8;
    if (d->prec == RRIN_PREC_F32R) {
      a.fr32 = static_cast<uint4*>(d->flow_raw.hi) + (int64_t)d->flow_raw.g_off * d->flow_raw.g.plane;
    } else {
      a.fr_hi = static_cast<_Float16*>(d->flow_raw.hi) + fo;
      a.fr_lo = planes == 2 ? static_cast<_Float16*>(d->flow_raw.lo) + fo : nullptr;
    }
    a.fr_img = d->flow_raw.img_stride;
    a.fr_gp = d->flow_raw.g.plane;
    a.fr_wp = d->flow_raw.g.wp;
  }
  a.h = h;
  a.w_ = w;
  a.tiles_x = (w + 31) / 32;
  a.tiles_y = (h + 15) / 16;
  grid = a.tiles_x * a.tiles_y * d->n;
  return 0;
}

extern "C" int rrin_head_h8_fwd(const rrin_head_h8_desc* d, void* stream) {
  HeadH8Args a;
  int grid = 0;
  const int rc = head_prepare(d, a, grid);
  if (rc) return rc;
  const int planes = d->prec == RRIN_PREC_F32R ? 0 : planes_of(d->prec);
  hipStream_t st = (hipStream_t)stream;
  switch (d->mode) {
    case RRIN_HEAD_PLAIN:
      if (d->cout == 2) return head_h8_launch<2, RRIN_HEAD_PLAIN>(a, planes, grid, st);
      if (d->cout == 3) return head_h8_launch<3, RRIN_HEAD_PLAIN>(a, planes, grid, st);
      if (d->cout == 4) return head_h8_launch<4, RRIN_HEAD_PLAIN>(a, planes, grid, st);
      return RRIN_E_ARG;
    case RRIN_HEAD_FLOW:
      return d->cout == 4 ? head_h8_launch<4, RRIN_HEAD_FLOW>(a, planes, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_REFINE:
      return d->cout == 4 ? head_h8_launch<4, RRIN_HEAD_REFINE>(a, planes, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_MASK:
      return d->cout == 2 ? head_h8_launch<2, RRIN_HEAD_MASK>(a, planes, grid, st) : RRIN_E_ARG;
    case RRIN_HEAD_FINAL:
      return d->cout == 3 ? head_h8_launch<3, RRIN_HEAD_FINAL>(a, planes, grid, st) : RRIN_E_ARG;
  }
  return RRIN_E_ARG;
}

extern "C" int rrin_flow_tblend_h8(const rrin_h8* fr, const rrin_h8* g16, const float* coef, int32_t n, int32_t prec,
                                   void* stream) {
  if (!fr || !g16 || !coef || n < 1 || !rec_prec(prec)) return RRIN_E_ARG;
  if (!h8_ok(*fr, prec) || !h8_ok(*g16, prec) || g16->g_off != 0 || g16->groups * chans_per_rec(prec) < 16)
    return RRIN_E_SHAPE;
  if (fr->g.h != g16->g.h || fr->g.w != g16->g.w) return RRIN_E_SHAPE;
  const int h = g16->g.h, w = g16->g.w;
  const int64_t total = (int64_t)n * h * w;
  const int grid = (int)((total + 255) / 256);
  if (prec == RRIN_PREC_F32R) {
    hipLaunchKernelGGL(flow_tblend_r32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const uint4*>(fr->hi) + (int64_t)fr->g_off * fr->g.plane, fr->img_stride,
                       fr->g.wp, static_cast<uint4*>(g16->hi), g16->img_stride, g16->g.plane, g16->g.wp, coef, h, w,
                       total);
    return hip_code(hipGetLastError());
  }
  const int64_t fo = (int64_t)fr->g_off * fr->g.plane * 8;
  const _Float16* fhi = static_cast<const _Float16*>(fr->hi) + fo;
  hipStream_t st = (hipStream_t)stream;
  if (planes_of(prec) == 2)
    hipLaunchKernelGGL(flow_tblend_h8_kernel<2>, dim3(grid), dim3(256), 0, st, fhi,
                       static_cast<const _Float16*>(fr->lo) + fo, fr->img_stride, fr->g.plane, fr->g.wp,
                       static_cast<_Float16*>(g16->hi), static_cast<_Float16*>(g16->lo), g16->img_stride,
                       g16->g.plane, g16->g.wp, coef, h, w, total);
  else
    hipLaunchKernelGGL(flow_tblend_h8_kernel<1>, dim3(grid), dim3(256), 0, st, fhi, (const _Float16*)nullptr,
                       fr->img_stride, fr->g.plane, fr->g.wp, static_cast<_Float16*>(g16->hi), (_Float16*)nullptr,
                       g16->img_stride, g16->g.plane, g16->g.wp, coef, h, w, total);
  return hip_code(hipGetLastError());
}

extern "C" int rrin_pack_g16_h8(const float* i0, const float* i1, int32_t n, const rrin_h8* g16, int32_t prec,
                                void* stream) {
  if (!i0 || !i1 || !g16 || n < 1 || !rec_prec(prec)) return RRIN_E_ARG;
  if (!h8_ok(*g16, prec) || g16->g_off != 0 || g16->groups * chans_per_rec(prec) < 16) return RRIN_E_SHAPE;
  const int64_t total = (int64_t)n * g16->g.h * g16->g.w;
  const int grid = (int)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  if (prec == RRIN_PREC_F32R)
    hipLaunchKernelGGL(pack_g16_r32_kernel, dim3(grid), dim3(256), 0, st, i0, i1, static_cast<uint4*>(g16->hi),
                       g16->img_stride, g16->g.plane, g16->g.wp, g16->g.h, g16->g.w, total);
  else if (planes_of(prec) == 2)
    hipLaunchKernelGGL(pack_g16_h8_kernel<2>, dim3(grid), dim3(256), 0, st, i0, i1, static_cast<uint4*>(g16->hi),
                       static_cast<uint4*>(g16->lo), g16->img_stride, g16->g.plane, g16->g.wp, g16->g.h, g16->g.w,
                       total);
  else
    hipLaunchKernelGGL(pack_g16_h8_kernel<1>, dim3(grid), dim3(256), 0, st, i0, i1, static_cast<uint4*>(g16->hi),
                       (uint4*)nullptr, g16->img_stride, g16->g.plane, g16->g.wp, g16->g.h, g16->g.w, total);
  return hip_code(hipGetLastError());
}
