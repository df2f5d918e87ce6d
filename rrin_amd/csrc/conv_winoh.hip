// fp16 3x3 conv as Winograd F(2x2,3x3) on H8 records (8 fp16 channels per 16-B record):
// the register-U tile of conv_winoc.hip (kind 6) with v_mfma_f32_32x32x16_f16.  Tile
// config kWinoC2Cfg at precision RRIN_PREC_F16 (BASELINE configs C3-C5).
//
// Replaces nn.Conv2d(3, pad=1) + LeakyReLU(0.1) (unet.py:29,59-63), the fused
// avg_pool2d output (unet.py:46), the cat by channel offset (unet.py:93) and the
// sub-pixel form of Upsample + up conv (unet.py:77-78), as the direct-form
// conv3x3_h8_kernel does at fp16.
//
// Arithmetic:
//   * U = G g G^T per (co, ci, point) in double on the host, times the conv's
//     power-of-two weight scale, rounded once to fp16 (rrin_pack_conv3x3_wino_h8);
//   * V = B^T d B in packed fp16 (v_pk_fma_f16 with a +-1 factor = one IEEE add per
//     element, two levels): the fp16 activations d, four at most added per V element;
//   * M[xi] = sum_ci U[xi] V[xi]: exact fp16 products, fp32 accumulation (the MFMA);
//   * the output transform, scale, bias, leaky and pool in fp32; the stores round once
//     to fp16 and flag any value fp16 cannot hold (the range guard of the H8 paths).
// |V| <= 4 max|d|: activations beyond 16376 can overflow V where the direct form would
// not; the inf / NaN then reaches the output check and the forward fails loudly.
//
// Tile (as kind 6): BM = 64 output channels (2 co tiles) x 32 px x TH = 4 NT rows.  Wave yw
// (0-3) owns B^T row yw (points 4 yw .. 4 yw + 3); lane (j, hh): patch j of the 32-patch MFMA
// tile, record group hh of the 16-channel chunk (channels 8 hh .. 8 hh + 7): the B operand
// of 32x32x16 (k = 8 (lane / 32) + e) is the transform of that lane's own records, and the A
// operand the packed U record [xi][hh][co][8].  Per wave and chunk: 8 NT MFMAs, 8 U loads
// (one 16-B record per lane each, from L2 into registers a chunk ahead), 8 NT window reads,
// 32 NT packed-f16 VALU, 2-3 LDS-DMA pieces of the raw tile (3 stages, one barrier).
#include <algorithm>

#include "common.hpp"

// Ablation builds only (tools/build_wino_variant.sh, outputs wrong by design): 1 no U loads
// after the prologue, 2 no raw DMA after the prologue, 4 no transform VALU, 8 no epilogue
// stores, 16 no window reads after the prologue
#ifndef RRIN_WINOH_ABL
#define RRIN_WINOH_ABL 0
#endif

namespace rrin {

typedef _Float16 whx8 __attribute__((ext_vector_type(8)));
typedef _Float16 whx2 __attribute__((ext_vector_type(2)));
typedef float wfx16 __attribute__((ext_vector_type(16)));
typedef float wfx4 __attribute__((ext_vector_type(4)));
typedef float wfx2 __attribute__((ext_vector_type(2)));

constexpr float kWinoHF16Max = 65504.0f;  // largest finite fp16

// LDS position of raw column col (0..33) within its row: even columns first (the stride-2
// window reads of 16 lanes fall on distinct banks), as kinds 1-7
__device__ inline int wh_col(int col) { return (col & 1) * 17 + (col >> 1); }

__device__ inline void wh_dma16(__amdgpu_buffer_rsrc_t rs, uint4* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0,
                                           0);
}
__device__ inline __amdgpu_buffer_rsrc_t wh_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ inline whx8 wh_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff) {
  return __builtin_bit_cast(whx8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
// 4 fp32 values -> 4 RNE fp16 values as one 8-B record half
__device__ inline uint2 wh_pack4(const float* v) {
  const whx2 h0 = __builtin_convertvector((wfx2){v[0], v[1]}, whx2);
  const whx2 h1 = __builtin_convertvector((wfx2){v[2], v[3]}, whx2);
  return make_uint2(__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1));
}

template <int NT>
struct WinoH {
  static constexpr int TH = 4 * NT;
  static constexpr int RG = (TH + 2) * 34;          // raw records per group
  static constexpr int RAW = 2 * RG;                // per chunk (2 groups = 16 channels)
  static constexpr int PIECES = (RAW + 255) / 256;  // DMA pieces per thread (every wave issues all)
  static constexpr int STAGE = PIECES * 256;        // records per LDS stage (the tail is a dummy)
  static constexpr int NS = 3;                      // stages: chunk c + 2 lands while c computes
  static constexpr int XREC = NT * 4 * 8 * 64;      // output-transform exchange, one co tile
  static constexpr size_t LDS = (size_t)(NS * STAGE > XREC ? NS * STAGE : XREC) * 16;
};
static_assert(WinoH<1>::LDS == kWinoCLds1 && WinoH<2>::LDS == kWinoCLds2, "LDS sizes (common.hpp)");

// NT 1 (kind 6 at fp16, the one the library launches): 128 accumulator registers, two blocks per
// CU.  (NT 2, round 5's kind 9 -- each U record on 2 patch tiles, one wave per SIMD -- ran 1.2-2.3x
// kind 6's time per conv and was removed in round 6 with the other rejected kinds)
template <int EPI, int NT>
__global__ __launch_bounds__(256, NT == 1 ? 2 : 1) void conv3x3_winoh_kernel(ConvH8Args a) {
  using G = WinoH<NT>;
  constexpr int CT = 2, BM = 64, TH = G::TH, RG = G::RG, STAGE = G::STAGE, P = G::PIECES;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int yw = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  int bid;
  {  // XCD-aware bijective remap: an XCD's workgroups are consecutive tiles
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
  const int nch = a.nchunks;
  int cob, x0, y0, img;
  {  // groups of cob_group co blocks (U of a group fits an XCD's L2), tile positions within
     // a group, the group's co blocks of a tile position on consecutive workgroups
    const int cpg = a.cob_group > 0 ? a.cob_group : a.co_blocks;
    const int gsz = cpg * (ntiles / a.co_blocks);
    const int g = bid / gsz;
    const int r = bid - g * gsz;
    const int cg = min(cpg, a.co_blocks - g * cpg);
    cob = g * cpg + r % cg;
    int t = r / cg;
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    y0 = (t % a.tiles_y) * TH;
    img = t / a.tiles_y;
  }

  // ---- raw tile: rows y0 - 1 .. y0 + TH, cols x0 - 1 .. x0 + 32 of the chunk's two record
  // groups, by buffer_load ... lds (a lane past the tile re-reads record 0 into the dummy tail)
  const uint4* tbase = a.src_hi + (int64_t)img * a.src_img + (int64_t)y0 * a.src_wp + x0 + (kH8PadLeft - 1);
  uint32_t voff[P];
#pragma unroll
  for (int it = 0; it < P; ++it) {
    const int idx = tid + 256 * it;
    const int g = idx >= RG ? 1 : 0;
    const int rem = idx < G::RAW ? idx - g * RG : 0;
    const int r = rem / 34, pos = rem - r * 34;
    const int col = pos < 17 ? 2 * pos : 2 * (pos - 17) + 1;
    voff[it] = (uint32_t)((idx < G::RAW ? (int64_t)g * a.src_gp : 0) + (int64_t)r * a.src_wp + col) * 16u;
  }
  const int64_t chunk_stride = 2 * a.src_gp;  // records between the group pairs of consecutive chunks
  auto issue_raw_at = [&](const uint4* base, int s) {
    const auto rs = wh_rsrc(base);
#pragma unroll
    for (int it = 0; it < P; ++it) wh_dma16(rs, smem4 + s * STAGE + 256 * it + 64 * yw, voff[it]);
  };
  const uint4* raw_next = tbase + (nch > 2 ? 2 : nch - 1) * chunk_stride;

  // ---- U (A operands) straight into registers: packing [cob][chunk][xi][hh][BM co][8 halves]
  const auto ur = wh_rsrc(a.w_hi + (int64_t)cob * nch * 32 * BM);
  const uint32_t uvoff = (uint32_t)(hh * BM + j) * 16u;
  auto load_u = [&](int c, int x, int t) {
    const int soff = c * (32 * BM * 16) + (4 * yw + (x & 2)) * (2 * BM * 16);
    const int imm = (x & 1) * 2048 + t * 512;
    return wh_load16(ur, uvoff + imm, soff);
  };

  // ---- B operands: lane (j, hh) of N tile nt is patch (pr = 2 nt + (j >> 4), jx), the
  // second patch row's columns rotated by 12 (distinct banks per ds_read_b128 lane group)
  const int jx = (j + 12 * (j >> 4)) & 15;
  const int ra = yw == 0 ? 0 : (yw == 2 ? 2 : 1);
  const int rb = yw == 0 ? 2 : (yw == 1 ? 2 : (yw == 2 ? 1 : 3));
  const _Float16 sgh = yw == 1 ? (_Float16)1.0f : (_Float16)-1.0f;
  const whx8 sg = {sgh, sgh, sgh, sgh, sgh, sgh, sgh, sgh};
  // -1 in every half, opaque to the compiler (it would turn fma(-1, b, a) back into a - b)
  unsigned m1w = 0xBC00BC00u;
  asm volatile("" : "+v"(m1w));
  const whx8 m1 = __builtin_bit_cast(whx8, make_uint4(m1w, m1w, m1w, m1w));
  int pcol[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pcol[k] = hh * RG + (2 * (j >> 4)) * 34 + wh_col(2 * jx + k);
  const int oa = ra * 34, ob = rb * 34;

  wfx16 acc[CT][NT][4];
  // (set by chunk 0's first MFMA of each accumulator: C = 0, no zeroing per tile)
  whx8 u[CT][4];   // U of the chunk being computed (point x reloaded after its MFMAs)
  whx8 v[NT][4];   // B operands of the chunk being computed
  whx8 d[NT][8];   // window records of the N tiles of the next chunk

  auto read_raw = [&](int s, int nt) {
    const uint4* rw = smem4 + s * STAGE + nt * 4 * 34;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[nt][2 * k] = __builtin_bit_cast(whx8, rw[oa + pcol[k]]);
      d[nt][2 * k + 1] = __builtin_bit_cast(whx8, rw[ob + pcol[k]]);
    }
  };
  // B^T row yw of the window, then the 4 points of that row: t_k = d[ra][k] +- d[rb][k],
  // V = (t0 - t2, t1 + t2, t2 - t1, t1 - t3); one fp16 rounding per add
  auto transform = [&](int nt) {
    if constexpr ((RRIN_WINOH_ABL & 4) != 0) {
      v[nt][0] = d[nt][0], v[nt][1] = d[nt][2], v[nt][2] = d[nt][4], v[nt][3] = d[nt][6];
      return;
    }
    whx8 tr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tr[k] = __builtin_elementwise_fma(sg, d[nt][2 * k + 1], d[nt][2 * k]);
    // a - b as fma(-1, b, a): one v_pk_fma_f16 per register (a vector subtraction is
    // split into two v_sub_f16 and a v_pack_b32_f16 by the compiler)
    v[nt][0] = __builtin_elementwise_fma(m1, tr[2], tr[0]);
    v[nt][1] = tr[1] + tr[2];
    v[nt][2] = __builtin_elementwise_fma(m1, tr[1], tr[2]);
    v[nt][3] = __builtin_elementwise_fma(m1, tr[3], tr[1]);
  };
  auto mfma_point = [&](int x, int nt, const bool first) {
#pragma unroll
    for (int t = 0; t < CT; ++t)
      acc[t][nt][x] = __builtin_amdgcn_mfma_f32_32x32x16_f16(u[t][x], v[nt][x], first ? wfx16{} : acc[t][nt][x], 0, 0,
                                                                  0);
  };
  auto reload_u = [&](int c, int x) {
#pragma unroll
    for (int t = 0; t < CT; ++t) u[t][x] = load_u(c, x, t);
  };
  // LDS-DMA of a stage is visible to the other waves after the issuing wave's vmcnt wait and
  // a barrier; the barrier is bare (a __syncthreads() would drain vmcnt to 0)
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };

  // Chunk c (U(c) in u, its B operands in v): the schedule of conv_winoc.hip's chunk --
  // points 0-2, each followed by its U load for chunk c + 1; the wait for raw(c + 1); the
  // barrier; raw(c + 2); per N tile chunk c + 1's window reads, point 3, its transform;
  // point 3's U load.  VMEM order per chunk: U pts 0-2, raw(c + 2), U pt 3.
  auto chunk = [&](int c, int s, const bool more, const bool first) {
#pragma unroll
    for (int x = 0; x < 3; ++x) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) mfma_point(x, nt, first);
      if (more && !(RRIN_WINOH_ABL & 1)) reload_u(c + 1, x);
      fence();
    }
    if (more) {
      RRIN_VMWAIT(0, (RRIN_WINOH_ABL & 1) ? 0 : 4 * CT);
      bar();
      if (!(RRIN_WINOH_ABL & 2)) issue_raw_at(raw_next, s == 0 ? 2 : s - 1);
      if (c + 3 < nch) raw_next += chunk_stride;
    }
    const int s1 = s == 2 ? 0 : s + 1;
    // every N tile's window reads first, then point 3's MFMAs (they cover the reads), then
    // the transforms of chunk c + 1
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      if (more && !(RRIN_WINOH_ABL & 16)) read_raw(s1, nt);
    fence();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) mfma_point(3, nt, first);
    fence();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      if (more) transform(nt);
    if (more && !(RRIN_WINOH_ABL & 1)) reload_u(c + 1, 3);
  };

  // prologue in the steady state's VMEM order: raw(0), U(0) pts 0-2, raw(1), U(0) pt 3
  issue_raw_at(tbase, 0);
  vm_fence();
#pragma unroll
  for (int x = 0; x < 3; ++x) reload_u(0, x);
  vm_fence();
  issue_raw_at(nch > 1 ? tbase + chunk_stride : tbase, 1);
  vm_fence();
  reload_u(0, 3);
  vm_fence();
  RRIN_VMWAIT(P, 4 * CT);
  bar();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    read_raw(0, nt);
    transform(nt);
  }
  {
    int s = 0;
    if (nch > 1) {  // chunk 0 peeled: its MFMAs start the accumulators from C = 0
      chunk(0, s, true, true);
      s = 1;
      for (int c = 1; c + 1 < nch; ++c) {
        chunk(c, s, true, false);
        s = s == 2 ? 0 : s + 1;
      }
      chunk(nch - 1, s, false, false);
    } else {
      chunk(0, s, false, true);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA past the end has landed
  // the epilogue's bias values, loaded now: their latency hides behind the exchange
  float bsv[CT][16];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) bsv[t][i] = a.bias[(CT * cob + t) * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
  __syncthreads();  // every read of the stages done before the exchange reuses the LDS

  // ---- output transform (kind 6's order): Q[c] = sum_x M[x] A[x][c] of this wave's B^T
  // row, Y[0][c] = (Q0 + Q1) + Q2, Y[1][c] = (Q1 - Q2) - Q3 over the four waves, exchanged
  // through LDS one co tile at a time; wave yw then finishes output row r = yw & 1, column
  // cc = yw >> 1 of its patches
  wfx4* X = reinterpret_cast<wfx4*>(smem4);
  const int r = yw & 1, cc = yw >> 1;
  uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
  const float isc = a.inv_wscale;
  bool bad = false;  // a stored value fp16 cannot hold (range guard)
  // 4 channels (lane half hh of an 8-channel record) -> 8-B half hh of record rec
  auto store4 = [&](uint4* base, int64_t rec, const float* vv) {
    if constexpr ((RRIN_WINOH_ABL & 8) != 0) return;
    bad |= !(fmaxf(fmaxf(fabsf(vv[0]), fabsf(vv[1])), fmaxf(fabsf(vv[2]), fabsf(vv[3]))) <= kWinoHF16Max);
    reinterpret_cast<uint2*>(base + rec)[hh] = wh_pack4(vv);
  };
#pragma unroll
  for (int t = 0; t < CT; ++t) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        wfx4 g;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int vi = 4 * k + e, c2 = vi >> 4, i = vi & 15;
          const float m0 = acc[t][nt][0][i], m1 = acc[t][nt][1][i], m2 = acc[t][nt][2][i], m3 = acc[t][nt][3][i];
          g[e] = c2 == 0 ? (m0 + m1) + m2 : (m1 - m2) - m3;
        }
        X[((nt * 4 + yw) * 8 + k) * 64 + lane] = g;
      }
    __syncthreads();
    float yv[NT][16];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const int k = 4 * cc + k4;
        const wfx4 q0 = X[((nt * 4 + 0) * 8 + k) * 64 + lane];
        const wfx4 q1 = X[((nt * 4 + 1) * 8 + k) * 64 + lane];
        const wfx4 q2 = X[((nt * 4 + 2) * 8 + k) * 64 + lane];
        const wfx4 q3 = X[((nt * 4 + 3) * 8 + k) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) yv[nt][4 * k4 + e] = r == 0 ? (q0[e] + q1[e]) + q2[e] : (q1[e] - q2[e]) - q3[e];
      }
    __syncthreads();  // X is rewritten by the next co tile / the pool exchange
    const int cobe = CT * cob + t;  // 32-channel block of this co tile
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int pr = 2 * nt + (j >> 4);
      const int y = y0 + 2 * pr + r, x = x0 + 2 * jx + cc;
      if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
        // rows co' = (co / 8) 32 + phase 8 + co % 8: co tile cobe holds real channels
        // 8 cobe .. + 7 (one record group), i >> 2 its phase (py, px)
        const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
        if (cobe * 32 < a.cout && y < a.h && x < a.w) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int Y = 2 * y + (qq >> 1), XX = 2 * x + (qq & 1);
            const int64_t ri = ring_index(Y, XX, HH, WW);
            if (ri >= 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                a.edge[((int64_t)img * creal + cobe * 8 + 4 * hh + e) * a.ring + ri] = yv[nt][4 * qq + e] * isc;
            } else {
              float vv[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) vv[e] = yv[nt][4 * qq + e] * isc + bsv[t][4 * qq + e];
              store4(dst, (int64_t)cobe * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + XX + kH8PadLeft, vv);
            }
          }
        }
      } else {
        float vv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float tv = yv[nt][i] * isc + bsv[t][i];
          if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
          vv[i] = tv;
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (cobe * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
            const int64_t rec = (int64_t)(cobe * 4 + qq) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
            store4(dst, rec, &vv[4 * qq]);
            if constexpr (EPI == RRIN_EPI_LEAKY_REP) {  // edge replicate into the padding ring
              const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
              const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
              for (int dy = dy0; dy <= dy1; ++dy)
                for (int dx = dx0; dx <= dx1; ++dx)
                  if (dy | dx) store4(dst, rec + (int64_t)dy * a.dst_wp + dx, &vv[4 * qq]);
            }
          }
        }
        if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
          // the patch's four outputs (yw = (r, c)) meet in LDS; wave 0 writes
          // avg = 0.25 ((Y00 + Y10) + (Y01 + Y11)), kind 6's order
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            wfx4 g;
#pragma unroll
            for (int e = 0; e < 4; ++e) g[e] = vv[4 * k + e];
            X[(yw * 4 + k) * 64 + lane] = g;
          }
          __syncthreads();
          if (yw == 0) {
            const int xp = x0 + 2 * jx, yp = y0 + 2 * pr;
            uint4* pdst = a.pool_hi + (int64_t)img * a.pool_img;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
              const wfx4 y00 = X[(0 * 4 + qq) * 64 + lane];
              const wfx4 y10 = X[(1 * 4 + qq) * 64 + lane];
              const wfx4 y01 = X[(2 * 4 + qq) * 64 + lane];
              const wfx4 y11 = X[(3 * 4 + qq) * 64 + lane];
              if (cobe * 32 + 8 * qq < a.cout && yp < a.h && xp < a.w) {
                float s4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) s4[e] = 0.25f * ((y00[e] + y10[e]) + (y01[e] + y11[e]));
                store4(pdst, (int64_t)(cobe * 4 + qq) * a.pool_gp + (int64_t)(yp / 2 + 1) * a.pool_wp + xp / 2 +
                                 kH8PadLeft,
                       s4);
              }
            }
          }
          __syncthreads();
        }
      }
    }
  }
  if (bad && a.status) *a.status = 1;
}


template <int EPI, int NT>
static int launch_winoh_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_winoh_kernel<EPI, NT>;
  static LdsAttr attr;
  constexpr size_t lds = WinoH<NT>::LDS;
  if (int e = attr.ensure((const void*)k, (int)lds, st)) return e;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  return hip_code(hipGetLastError());
}

#ifndef RRIN_WINOH_UGROUP_KB
#define RRIN_WINOH_UGROUP_KB 2048
#endif
// co blocks per workgroup group whose U fits an XCD's L2 share (as winoc_cob_group)
static int winoh_cob_group(const ConvH8Args& a) {
  const int64_t per_cob = (int64_t)a.nchunks * 32 * 64 * 16;  // U bytes of one co block
  if (RRIN_WINOH_UGROUP_KB <= 0 || (int64_t)a.co_blocks * per_cob <= (int64_t)RRIN_WINOH_UGROUP_KB * 1024) return 0;
  int g = 1;
  while (2 * g < a.co_blocks && 2 * g * per_cob <= (int64_t)RRIN_WINOH_UGROUP_KB * 1024) g *= 2;
  return g;
}


template <int NT>
static int launch_winoh_e(const ConvH8Args& b, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_winoh_k<RRIN_EPI_LINEAR, NT>(b, st);
    case RRIN_EPI_LEAKY: return launch_winoh_k<RRIN_EPI_LEAKY, NT>(b, st);
    case RRIN_EPI_LEAKY_POOL: return launch_winoh_k<RRIN_EPI_LEAKY_POOL, NT>(b, st);
    case RRIN_EPI_LEAKY_REP: return launch_winoh_k<RRIN_EPI_LEAKY_REP, NT>(b, st);
    case RRIN_EPI_SUBPIXEL: return launch_winoh_k<RRIN_EPI_SUBPIXEL, NT>(b, st);
  }
  return RRIN_E_ARG;
}


int launch_winoh(const ConvH8Args& a, int epi, hipStream_t st) {
  ConvH8Args b = a;
  b.cob_group = winoh_cob_group(a);
  return launch_winoh_e<1>(b, epi, st);
}

}  // namespace rrin

using namespace rrin;

// ---- packing: [co block of bm][16-channel chunk][point xi][record half][bm co][8 halves] of
// U = G g G^T (double) x 2^s, rounded once to fp16; s puts max |U| in [2^12, 2^13) as the
// direct fp16 packing does for max |g| (rrin_pack_conv3x3_h8), *inv_wscale = 2^-s
extern "C" int64_t rrin_pack_conv3x3_wino_h8_halves(int32_t cout, int32_t cin, int32_t bm) {
  if (cout < 1 || cin < 1 || bm != 64) return RRIN_E_ARG;
  const int64_t cob = (cout + bm - 1) / bm, nch = (cin + 15) / 16;
  return cob * nch * 16 * 2 * bm * 8;
}

extern "C" int rrin_pack_conv3x3_wino_h8(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                                         const int32_t* perm, uint16_t* whi, float* bpack, float* inv_wscale) {
  if (!w || !b || !whi || !bpack || !inv_wscale || cout < 1 || cin < 1 || bm != 64) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  static const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
  const int cob_n = (cout + bm - 1) / bm, nch = (cin + 15) / 16;
  auto u_of = [&](int co, int ch, int xi) {
    const float* g = w + ((int64_t)co * cin + (perm ? perm[ch] : ch)) * 9;
    double u = 0.0;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) u += G[xi >> 2][ky] * G[xi & 3][kx] * (double)g[ky * 3 + kx];
    return u;
  };
  double mx = 0.0;
  for (int co = 0; co < cout; ++co)
    for (int ch = 0; ch < cin; ++ch)
      for (int xi = 0; xi < 16; ++xi) mx = fmax(mx, fabs(u_of(co, ch, xi)));
  if (!(mx < INFINITY)) return RRIN_E_ARG;
  int s = 0;
  if (mx > 0.0) {
    int e;
    frexp(mx, &e);  // mx in [2^(e-1), 2^e)
    s = 13 - e;     // scaled max in [2^12, 2^13)
  }
  const double scale = ldexp(1.0, s);
  *inv_wscale = ldexpf(1.0f, -s);
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int xi = 0; xi < 16; ++xi)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < bm; ++col)
            for (int e = 0; e < 8; ++e) {
              const int co = cob * bm + col, ch = c * 16 + hh * 8 + e;
              const double u = (co < cout && ch < cin) ? u_of(co, ch, xi) * scale : 0.0;
              whi[o++] = __builtin_bit_cast(uint16_t, (_Float16)u);
            }
  for (int co = 0; co < cob_n * bm; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}
