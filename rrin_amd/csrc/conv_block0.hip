// Fused level-0 UNetConvBlock at fp16 (H8 records): conv a (cin -> 32) + LeakyReLU, conv b
// (32 -> 32) + LeakyReLU (+ the down block's avg_pool2d output) in one launch, conv a's output
// tile kept in LDS.  Replaces unet.py:59-63 (the block's two Conv2d + LeakyReLU) and :46 (the pool
// of down_path[0]) at level 0, where the direct-form pair (conv3x3_h8_kernel twice) is bound by
// HBM: a 32-channel full-resolution fp16 tensor is written by conv a and read back by conv b.
//
// Tile: 8 output rows x 62 output columns x 32 channels of one image.  Conv a runs on the
// 10 x 64 positions conv b needs (the 1-pixel halo is recomputed by the neighbouring tiles:
// 1.29x conv a's MACs), from a 12 x 66 input tile; positions outside the image are set to 0
// (conv b's zero padding).  4 waves, two workgroups per CU:
//   * input: 16-channel chunks (2 record groups) by LDS-DMA (buffer_load ... lds), two stages;
//     conv a's weights straight from L2 into registers (9 records per lane and chunk), a chunk
//     ahead;
//   * conv a: wave wv owns the 5 MFMA tiles (32 co x 32 px) of rows wv/2, wv/2 + 2, ..., column
//     half wv % 2; per chunk and tap one ds_read_b128 per tile (its B operand);
//   * conv a's epilogue (scale, bias, leaky, zero outside the image, one fp16 rounding) writes
//     the 32-channel tile into LDS over the dead input stage Y;
//   * conv b: wave wv owns rows 4 (wv/2) .. + 3 of column half wv % 2 (a pool pair is in one
//     wave), B operands from the LDS tile, weights from L2 into registers;
//   * conv b's epilogue as conv3x3_h8_kernel's (store, range guard, 2x2 average pool).
// The arithmetic is that of two conv3x3_h8_kernel launches at fp16 (same packed weights, chunk
// then tap order of the fp32 accumulation, same epilogue expressions and roundings): the outputs
// are bitwise those of the unfused pair (tests/test_gpu_block0.py).
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "common.hpp"

// Ablation builds only (tools/build_wino_variant.sh NAME -DRRIN_B0_ABL=bits conv_block0; outputs wrong
// by design): 1 no conv-a MFMAs, 2 no conv-b MFMAs, 4 no B-operand LDS reads after a tile's first
// tap, 8 no conv-b epilogue stores, 16 no input DMA after the first tile's, 32 no weight loads
// after the prologue
#ifndef RRIN_B0_ABL
#define RRIN_B0_ABL 0
#endif

namespace rrin {

typedef _Float16 b0h8 __attribute__((ext_vector_type(8)));
typedef _Float16 b0h2 __attribute__((ext_vector_type(2)));
typedef float b0f2 __attribute__((ext_vector_type(2)));
typedef float b0f16 __attribute__((ext_vector_type(16)));

constexpr float kB0F16Max = 65504.0f;

__device__ inline __amdgpu_buffer_rsrc_t b0_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ inline void b0_dma16(__amdgpu_buffer_rsrc_t rs, uint4* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0,
                                           0);
}
__device__ inline b0h8 b0_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff) {
  return __builtin_bit_cast(b0h8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
// 4 fp32 values -> 4 RNE fp16 values (one 8-B record half), as split4 of conv_f16.hip
__device__ inline uint2 b0_pack4(const float* v) {
  const b0h2 h0 = __builtin_convertvector((b0f2){v[0], v[1]}, b0h2);
  const b0h2 h1 = __builtin_convertvector((b0f2){v[2], v[3]}, b0h2);
  return make_uint2(__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1));
}

template <bool POOL>
__global__ __launch_bounds__(256, 2) void conv_block0_h8_kernel(Block0Args a) {
  constexpr int TH = kB0TH, TW = kB0TW, IR = kB0IR, IC = kB0IC, MR = kB0MR, MC = kB0MC;
  constexpr int P = kB0Pieces, STAGE = kB0Stage;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  const int half = wv & 1;  // column half of this wave's MFMA tiles (wave-uniform)
  int bid;
  {  // XCD-aware bijective remap: an XCD's workgroups are consecutive tiles (shared halo rows in its L2)
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.tiles_x * a.tiles_y * a.n;
  int tile = bid;
  if (tile >= ntiles) return;
  const int nch = a.nch;
  // LDS: [conv-a tile (kB0Mid) | stage X (chunks 0, 2, ..) | 64 bias floats]; stage Y (chunks 1,
  // 3, ..) aliases the conv-a tile.  Stage X is free during conv b: the next tile's chunk 0 lands
  // there while conv b and its epilogue run (the grid is persistent: a workgroup walks tiles
  // bid, bid + grid, ...)
  uint4* const stX = smem4 + kB0Mid;
  uint4* const stY = smem4;
  float* const sbias = reinterpret_cast<float*>(smem4 + kB0Mid + STAGE);
  if (tid < 64) sbias[tid] = tid < 32 ? a.ba[tid] : a.bb[tid - 32];  // read after the prologue barrier

  // ---- input tile: rows y0 - 2 .. y0 + 9, cols x0 - 2 .. x0 + 63 of a chunk's two record groups,
  // clamped into the padded plane (a clamped row / column only feeds conv-a positions outside
  // the image, which are zeroed); groups past the input's last read its zero top padding row
  // (the direct kernel's convention); lanes past the tile re-read record 0 into the dummy tail
  uint32_t voff[P];
  auto set_offsets = [&](int x0, int y0) {
#pragma unroll
    for (int it = 0; it < P; ++it) {
      const int idx = tid + 256 * it;
      const bool ok = idx < kB0In;
      const int g = idx >= IR * IC ? 1 : 0;
      const int rem = ok ? idx - g * IR * IC : 0;
      const int r = rem / IC, col = rem - r * IC;
      const int yb = min(max(y0 - 2 + r + 1, 0), a.src_hp - 1);
      const int xr = min(max(x0 - 2 + col + kH8PadLeft, 0), a.src_wp - 1);
      voff[it] = ok ? (uint32_t)(g * a.src_gp + yb * a.src_wp + xr) * 16u : 0u;
    }
  };
  const uint32_t cstride = (uint32_t)(2 * a.src_gp * 16);  // bytes between consecutive chunks' group pairs
  // (a chunk's second group past the input's last -- cin % 16 in 1..8 -- is staged from the
  // first group's position and zeroed in the B operands: compute_a<true>)
  const uint32_t gstride = (uint32_t)(a.src_gp * 16);
  bool first_tile = true;
  auto issue_chunk = [&](const uint4* ibase, int c, uint4* st) {
    if constexpr ((RRIN_B0_ABL & 16) != 0)
      if (!first_tile) return;
    const auto rs = b0_rsrc(ibase);
    const bool past = 2 * c + 1 >= a.ngroups;
#pragma unroll
    for (int it = 0; it < P; ++it) {
      const bool g1 = tid + 256 * it >= IR * IC && tid + 256 * it < kB0In;
      b0_dma16(rs, st + 256 * it + 64 * wv, voff[it] + (uint32_t)c * cstride - (past && g1 ? gstride : 0u));
    }
  };
  // a chunk's second group past the input's last (cin % 16 in 1..8) was staged from the first
  // group's position: once its DMA has landed (after the wait that covers it, before the barrier
  // that publishes it) its records become zeros, the direct kernel's zero-row operands
  auto zero_past = [&](int c, uint4* st) {
    if (2 * c + 1 < a.ngroups) return;
#pragma unroll
    for (int it = 0; it < P; ++it) {
      const int idx = tid + 256 * it;
      if (idx >= IR * IC && idx < kB0In) st[idx] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto tile_pos = [&](int t, int& img, int& x0, int& y0) {
    const int tx = t % a.tiles_x;
    t /= a.tiles_x;
    y0 = (t % a.tiles_y) * TH;
    img = t / a.tiles_y;
    x0 = tx * TW;
  };

  // ---- weights (packing of rrin_pack_conv3x3_h8, co block 0): lane (j, hh) of tap t of chunk c
  // is record ((c * 9 + t) * 2 + hh) * bm + j; from L2 straight into registers.  One set of 9
  // records: after tap t's MFMAs of a chunk, tap t of the next chunk (conv a's next, conv b's
  // first, conv b's second, the next tile's conv-a first) replaces w[t]
  const auto rs_wa = b0_rsrc(a.wa);
  const auto rs_wb = b0_rsrc(a.wb);
  const uint32_t wa_voff = (uint32_t)(hh * a.bma + j) * 16u;
  const uint32_t wb_voff = (uint32_t)(hh * a.bmb + j) * 16u;
  const int wa_tap = 2 * a.bma * 16, wb_tap = 2 * a.bmb * 16;  // bytes per tap
  b0h8 w[9];
  // source of the weights that replace w[] during a chunk: conv (0 a, 1 b), chunk; none if conv < 0
  struct WNext {
    int conv, c;
  };
  auto wload = [&](const WNext& nx, int t) {
    if constexpr ((RRIN_B0_ABL & 32) != 0) return;
    if (nx.conv == 0) w[t] = b0_load16(rs_wa, wa_voff, (nx.c * 9 + t) * wa_tap);
    if (nx.conv == 1) w[t] = b0_load16(rs_wb, wb_voff, (nx.c * 9 + t) * wb_tap);
  };
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };

  // B operand of conv-a tile i (row wv / 2 + 2 i, column half) at tap (ky, kx): input record
  // (group hh, row m + ky, column 32 half + j + kx)
  const int a_base = hh * IR * IC + (wv >> 1) * IC + 32 * half + j;
  b0f16 acc[5];
  // zc (std::true_type for chunk 0): each accumulator's first MFMA takes C = 0 (no zeroing per tile)
  auto compute_a = [&](const uint4* st, const WNext& nx, auto zc) {
    const uint4* base = st + a_base;
    b0h8 b[2][5];
    auto ld = [&](int t, int slot) {
      const int ky = t / 3, kx = t - 3 * (t / 3);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if constexpr ((RRIN_B0_ABL & 4) != 0)
          if (t > 0) continue;
        b[slot][i] = __builtin_bit_cast(b0h8, base[(2 * i + ky) * IC + kx]);
      }
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        if constexpr ((RRIN_B0_ABL & 1) != 0)
          asm volatile("" ::"v"(w[t]), "v"(b[t & 1][i]));
        else
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[t], b[t & 1][i],
                                                         decltype(zc)::value && t == 0 ? b0f16{} : acc[i], 0, 0, 0);
      wload(nx, t);
      fence();  // one weight set live: tap t's replacement issues after tap t's MFMAs
    }
  };

  int img, x0, y0;
  tile_pos(tile, img, x0, y0);
  set_offsets(x0, y0);
  const uint4* ibase = a.src + (size_t)img * a.src_img;
  // prologue of the first tile: chunk 0 (DMA), its weights, chunk 1 (DMA); wait for the first two
  issue_chunk(ibase, 0, stX);
  vm_fence();
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = b0_load16(rs_wa, wa_voff, t * wa_tap);
  vm_fence();
  if (nch > 1) {
    issue_chunk(ibase, 1, stY);
    vm_fence();
    RRIN_VMWAIT(P, 0);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  zero_past(0, stX);
  bar();
  bool bad = false;  // a stored value fp16 cannot hold (range guard)
  for (;;) {
    fence();
    // ---- conv a: chunk c from stage X (c even) / Y (c odd)
    // chunk 0 peeled (its MFMAs start the accumulators from C = 0)
    auto chunk_a = [&](const int c, auto zc) {
      const bool more = c + 1 < nch;
      fence();
      compute_a((c & 1) ? stY : stX, more ? WNext{0, c + 1} : WNext{1, 0}, zc);
      fence();
      if (more) {
        // chunk c + 1 (DMA) landed; every wave done with this chunk's stage
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        zero_past(c + 1, ((c + 1) & 1) ? stY : stX);
        bar();
        if (c + 2 < nch) issue_chunk(ibase, c + 2, (c & 1) ? stY : stX);
      }
      fence();
    };
    chunk_a(0, std::true_type{});
    for (int c = 1; c < nch; ++c) chunk_a(c, std::false_type{});
    bar();  // every wave done reading the stages: Y becomes the conv-a tile, X takes the next tile
    const int ntile = tile + (int)gridDim.x;
    const bool has_next = ntile < ntiles;
    int nimg = img, nx0 = x0, ny0 = y0;
    const uint4* nbase = ibase;
    if (has_next) {
      tile_pos(ntile, nimg, nx0, ny0);
      set_offsets(nx0, ny0);
      nbase = a.src + (size_t)nimg * a.src_img;
      issue_chunk(nbase, 0, stX);
    }

    // ---- conv a's epilogue into the LDS tile [4 groups][MR rows][MC cols].  No range check here:
    // a value past the fp16 range rounds to +-inf and reaches every conv-b output of its window as
    // +-inf or NaN (inf x 0 = NaN), which conv b's epilogue flags; only values in (65504, 65520),
    // which round to 65504, go unflagged where the unfused conv a would flag them
    {
      const float4* bq = reinterpret_cast<const float4*>(sbias) + hh;  // channels 8 q + 4 hh ..
      const int x = x0 - 1 + 32 * half + j;
      const bool xin = x >= 0 && x < a.w;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int m = (wv >> 1) + 2 * i;
        const int y = y0 - 1 + m;
        const bool in = xin && y >= 0 && y < a.h;
#pragma unroll
        for (int qp = 0; qp < 2; ++qp) {  // 8-channel blocks 2 qp, 2 qp + 1
          uint2 pk[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int q = 2 * qp + k;
            const float4 bs = bq[2 * q];
            const float bsa[4] = {bs.x, bs.y, bs.z, bs.w};
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = acc[i][4 * q + e];
              t = t * a.isa + bsa[e];
              v[e] = in ? leaky(t, a.slope) : 0.f;
            }
            pk[k] = b0_pack4(v);
          }
          // whole records: lane (j, hh) writes block 2 qp + hh of its pixel (ds_write_b128, 8
          // contiguous lanes per LDS cycle: no bank conflict; the half-record ds_write_b64 was 2-way)
          smem4[((2 * qp + hh) * MR + m) * MC + 32 * half + j] = halves_to_record(pk[0], pk[1]);
        }
      }
    }
    bar();
    fence();

    // ---- conv b: rows 4 (wv / 2) + i, column half; chunk cb = record groups 2 cb, 2 cb + 1
    b0f16 acc2[4];  // set by chunk 0's first MFMA (C = 0)
    const int b_base = hh * MR * MC + ((wv >> 1) * 4) * MC + 32 * half + j;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const uint4* base = smem4 + b_base + 2 * cb * MR * MC;
      const WNext nx = cb == 0 ? WNext{1, 1} : (has_next ? WNext{0, 0} : WNext{-1, 0});
      b0h8 b[2][4];
      auto ld = [&](int t, int slot) {
        const int ky = t / 3, kx = t - 3 * (t / 3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr ((RRIN_B0_ABL & 4) != 0)
            if (t > 0) continue;
          b[slot][i] = __builtin_bit_cast(b0h8, base[(i + ky) * MC + kx]);
        }
      };
      ld(0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if constexpr ((RRIN_B0_ABL & 2) != 0)
            asm volatile("" ::"v"(w[t]), "v"(b[t & 1][i]));
          else
            acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[t], b[t & 1][i],
                                                          cb == 0 && t == 0 ? b0f16{} : acc2[i], 0, 0, 0);
        wload(nx, t);
        fence();
      }
    }
    fence();

    // ---- conv b's epilogue (conv3x3_h8_kernel's EPI_LEAKY / EPI_LEAKY_POOL expressions); buffer
    // whole-record (16-B) stores, an invalid position's offset past the buffer (dropped)
    {
      constexpr uint32_t kOOB = 0x80000000u;
      const float4* bq = reinterpret_cast<const float4*>(sbias + 32) + hh;
      const int xc = 32 * half + j;  // tile column
      const int x = x0 + xc;
      const bool xok = xc < TW && x < a.w;
      const auto rs_d = b0_rsrc(a.dst + (size_t)img * a.dst_img);
      const auto rs_p = b0_rsrc(POOL ? a.pool + (size_t)img * a.pool_img : a.dst);
      const int yb = y0 + (wv >> 1) * 4;
      const uint32_t d0 = (uint32_t)((yb + 1) * a.dst_wp + x + kH8PadLeft) * 16u;
      const uint32_t p0 = (uint32_t)((yb / 2 + 1) * a.pool_wp + x / 2 + kH8PadLeft) * 16u;
      auto st16 = [&](__amdgpu_buffer_rsrc_t rs, uint4 r, uint32_t off) {
        if constexpr ((RRIN_B0_ABL & 8) == 0)
          __builtin_amdgcn_raw_buffer_store_b128((unsigned __attribute__((ext_vector_type(4)))){r.x, r.y, r.z, r.w},
                                                 rs, off, 0, 0);
      };
      // 8-channel blocks in pairs (2 qp, 2 qp + 1): each lane's two half-records become one whole
      // record (halves_to_record), lane (j, hh) storing block 2 qp + hh: 16-B stores, half as many
#pragma unroll
      for (int qp = 0; qp < 2; ++qp) {
        float v[2][4][4];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int q = 2 * qp + k;
          const float4 bs = bq[2 * q];
          const float bsb[4] = {bs.x, bs.y, bs.z, bs.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = acc2[i][4 * q + e];
              t = t * a.isb + bsb[e];
              v[k][i][e] = leaky(t, a.slope);
            }
            if (xok && yb + i < a.h)
              bad |= !(fmaxf(fmaxf(fabsf(v[k][i][0]), fabsf(v[k][i][1])), fmaxf(fabsf(v[k][i][2]), fabsf(v[k][i][3]))) <=
                       kB0F16Max);
          }
        }
        const int qo = 2 * qp + hh;  // the block this lane stores
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = xok && yb + i < a.h;
          const uint4 rec = halves_to_record(b0_pack4(v[0][i]), b0_pack4(v[1][i]));
          st16(rs_d, rec, ok ? d0 + (uint32_t)(qo * a.dst_gp + i * a.dst_wp) * 16u : kOOB);
        }
        if constexpr (POOL) {
#pragma unroll
          for (int p2 = 0; p2 < 2; ++p2) {
            float s4[2][4];
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float s = v[k][2 * p2][e] + v[k][2 * p2 + 1][e];
                s4[k][e] = 0.25f * (s + __shfl_xor(s, 1));
              }
            const bool ok = !(j & 1) && xok && yb + 2 * p2 < a.h;
#pragma unroll
            for (int k = 0; k < 2; ++k)
              if (ok)
                bad |= !(fmaxf(fmaxf(fabsf(s4[k][0]), fabsf(s4[k][1])), fmaxf(fabsf(s4[k][2]), fabsf(s4[k][3]))) <=
                         kB0F16Max);
            const uint4 rec = halves_to_record(b0_pack4(s4[0]), b0_pack4(s4[1]));
            st16(rs_p, rec, ok ? p0 + (uint32_t)(qo * a.pool_gp + p2 * a.pool_wp) * 16u : kOOB);
          }
        }
      }
    }
    if (!has_next) break;
    // every wave done reading the conv-a tile: the next tile's chunk 1 goes into stage Y; wait for
    // its chunk 0 and chunk-0 weights by counting the younger loads only (loads complete in
    // order among themselves, not in order with the epilogue's stores)
    bar();
    if (nch > 1) {
      vm_fence();
      issue_chunk(nbase, 1, stY);
      vm_fence();
      RRIN_VMWAIT(P, 0);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    zero_past(0, stX);
    bar();
    first_tile = false;
    tile = ntile;
    img = nimg;
    x0 = nx0;
    y0 = ny0;
    ibase = nbase;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (bad && a.status) *a.status = 1;
}

// One tile per workgroup.  The kernel can walk tiles bid, bid + grid, ... with the next tile's
// chunk 0 staged behind the current epilogue, but no build launches fewer workgroups than tiles:
// round 5's persistent grids (RRIN_BLOCK0_BPC, kind 10) lost in the forward and kind 10 ran
// nondeterministically, so the knob is gone and the walk never takes a second tile.
template <bool POOL>
static int launch_block0_k(const Block0Args& a, hipStream_t st) {
  auto k = conv_block0_h8_kernel<POOL>;
  static LdsAttr attr;
  if (int e = attr.ensure((const void*)k, (int)kB0Lds, st)) return e;
  const int64_t tiles = (int64_t)a.tiles_x * a.tiles_y * a.n;
  hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(256), kB0Lds, st, a);
  return hip_code(hipGetLastError());
}

int launch_block0(const Block0Args& a, hipStream_t st) {
  return a.pool ? launch_block0_k<true>(a, st) : launch_block0_k<false>(a, st);
}

}  // namespace rrin
