// Exact-fp32 3x3 conv as Winograd F(2x2,3x3) on fp32 records (R32): the
// "register-U" tiles, Winograd kinds 6 and 7 of the record-layout conv table.
// Same arithmetic, in the same order, as conv3x3_winoq_kernel (conv_wino.hip):
// the outputs are bitwise those of configs 18-21.
//
// Replaces nn.Conv2d(3, pad=1) + LeakyReLU(0.1) (unet.py:29,59-63), the fused
// avg_pool2d output (unet.py:46), the cat by channel offset (unet.py:93) and the
// sub-pixel form of Upsample + up conv (unet.py:77-78).
//
// Why this shape (tools/coissue_probe2.py): on gfx950 a
// v_mfma_f32_32x32x2_f32 stream with its accumulators in VGPRs (the compiler's form
// here) pays 6-8 pipe cycles for each VALU op and ~55 for each ds_write of the other
// waves on its SIMD, and vector-memory instructions (global loads, LDS-DMA) do not
// overlap it in either accumulator form; LDS reads and SALU do.  What pays is fewer
// non-MFMA instructions per MFMA:
//   * the A operands (transformed weights U) go straight from L2 into registers
//     (buffer_load_dwordx4: one per 4 MFMAs of a co tile, each record holding 4
//     K steps), loaded a chunk ahead: no LDS-DMA pieces and no LDS reads for U;
//   * only the raw input tile goes through LDS (buffer_load ... lds, 3 stages, one
//     barrier per 8-channel chunk); a wave turns its window records into the B
//     operands of its B^T row (one transform per lane, as kinds 1-4) and feeds them
//     to CT co tiles (kind 6: CT 2) or uses each U record on NT patch tiles
//     (kind 7: NT 2);
//   * 4 waves of 8 accumulators (128 registers) per block, two blocks per CU, so
//     one block's barrier, prologue and epilogue run beside the other's MFMAs.
// Per wave and 8-channel chunk: 32 MFMAs, 4 CT U loads, 8 NT LDS reads, 32 NT VALU,
// 2-3 LDS-DMA pieces (kind 3: 16 MFMAs, 4 + 8 LDS reads, 32 VALU, 3-4 pieces).
//
// Tile: BM = 32 CT output channels x 32 px x TH = 4 NT rows (16 x 2 NT patches).
// Wave yw (0-3) owns B^T row yw (points 4 yw .. 4 yw + 3) of every patch; lane
// (j, hh): patch j of a 32-patch MFMA tile, record half hh (channels 4 hh .. + 3
// of the chunk; MFMA product e contracts channels e and 4 + e).
#include "common.hpp"
#include "edge_fix.hpp"

#ifndef RRIN_WINOC_AGPR
#define RRIN_WINOC_AGPR 0
#endif
// Diagnostic build only (tools/clock_probe.py, never the product library): each
// workgroup stamps s_memtime / s_memrealtime at its start, after its main loop and at
// its end into g_winoc_clk[bid % kClkSlots] (the in-kernel clock: MI355X_MICROARCH.md
// 'DVFS give-back' item 6)
#ifndef RRIN_WINOC_CLOCK
#define RRIN_WINOC_CLOCK 0
#endif
// Ablation builds only (tools/build_wino_variant.sh, outputs wrong by design): 1 no U
// loads after the prologue, 2 no raw DMA after the prologue, 4 no transform VALU,
// 8 no epilogue stores, 16 no window reads after the prologue
#ifndef RRIN_WINOC_ABL
#define RRIN_WINOC_ABL 0
#endif

namespace rrin {

#if RRIN_WINOC_CLOCK
constexpr int kClkSlots = 1 << 16;
__device__ unsigned long long g_winoc_clk[kClkSlots * 4];
#endif

typedef float cfloatx16 __attribute__((ext_vector_type(16)));
typedef float cfloatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));

// LDS position of raw column col (0..33) within its row: even columns first (the
// stride-2 window reads of 16 lanes fall on distinct banks), as kinds 1-4
__device__ inline int wc_col(int col) { return (col & 1) * 17 + (col >> 1); }

// buffer_load_dwordx4 ... lds: one 16-B record per lane at byte offset voff of rsrc into
// the lane-linear LDS image at the wave-uniform base
__device__ inline void buf_dma16(__amdgpu_buffer_rsrc_t rs, uint4* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0,
                                           0);
}
__device__ inline __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ inline cfloatx4 buf_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff) {
  return __builtin_bit_cast(cfloatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

template <int NT>
struct WinoC {
  static constexpr int TH = 4 * NT;
  static constexpr int RG = (TH + 2) * 34;          // raw records per group
  static constexpr int RAW = 2 * RG;                // per chunk (2 groups)
  static constexpr int PIECES = (RAW + 255) / 256;  // DMA pieces per thread (every wave issues all)
  static constexpr int STAGE = PIECES * 256;        // records per LDS stage (the tail is a dummy)
  static constexpr int NS = 3;                      // stages: chunk c + 2 lands while c computes
  static constexpr int XREC = NT * 4 * 8 * 64;      // output-transform exchange, one co tile
  static constexpr size_t LDS = (size_t)(NS * STAGE > XREC ? NS * STAGE : XREC) * 16;
};
static_assert(WinoC<1>::LDS == kWinoCLds1 && WinoC<2>::LDS == kWinoCLds2, "LDS sizes (common.hpp)");
static_assert(2 * WinoC<2>::LDS <= 160 * 1024, "two blocks per CU");

template <int EPI, int CT, int NT>
__global__ __launch_bounds__(256, 2) void conv3x3_winoc_kernel(ConvH8Args a) {
  using G = WinoC<NT>;
  constexpr int BM = 32 * CT, TH = G::TH, RG = G::RG, STAGE = G::STAGE, P = G::PIECES;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int yw = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
    // the ring from scratch in this launch (rrin_conv_h8_desc.ring_full): workgroups [0, nfix)
    // run the FULL fix-up (one K group of 256 threads, fp32 records) and leave
    if ((int)blockIdx.x < a.nfix) {
      const int rr = blockIdx.x;
      if (rr < a.fix_real)
        edge_fix_body<1, 1, true, true>(a.fix, rr % a.fix_gx, (rr / a.fix_gx) % a.fix_gy, rr / (a.fix_gx * a.fix_gy));
      return;
    }
  }
  int bid;
  {  // XCD-aware bijective remap (conv_mfma.hip): an XCD's workgroups are consecutive tiles
     // (nfix, a multiple of 8, keeps each conv workgroup's XCD)
    const int nwg = (int)gridDim.x - a.nfix, q = nwg >> 3, r = nwg & 7;
    const int cb = (int)blockIdx.x - a.nfix;
    const int xcd = cb & 7, slot = cb >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int ntiles = a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if (bid >= ntiles) return;
#if RRIN_WINOC_CLOCK
  const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int nch = a.nchunks;
  int cob, x0, y0, img;
  {  // groups of cob_group co blocks, tile positions within a group, the group's co blocks
     // of a tile position on consecutive workgroups (they share its raw tile)
    const int cpg = a.cob_group > 0 ? a.cob_group : a.co_blocks;
    const int gsz = cpg * (ntiles / a.co_blocks);  // workgroups of a full group
    const int g = bid / gsz;
    const int r = bid - g * gsz;
    const int cg = min(cpg, a.co_blocks - g * cpg);  // co blocks of this group (the last may be short)
    cob = g * cpg + r % cg;
    int t = r / cg;
    x0 = (t % a.tiles_x) * 32;
    t /= a.tiles_x;
    y0 = (t % a.tiles_y) * TH;
    img = t / a.tiles_y;
  }

  // ---- raw tile: rows y0 - 1 .. y0 + TH, cols x0 - 1 .. x0 + 32 of the chunk's two
  // record groups, by buffer_load ... lds from a per-chunk base (byte offsets per lane
  // fixed; a lane past the tile re-reads record 0 into the stage's dummy tail)
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
    const auto rs = buf_rsrc(base);
#pragma unroll
    for (int it = 0; it < P; ++it) buf_dma16(rs, smem4 + s * STAGE + 256 * it + 64 * yw, voff[it]);
  };
  // the group pair of chunk min(c + 2, nch - 1), advanced by one chunk per steady chunk
  const uint4* raw_next = tbase + (nch > 2 ? 2 : nch - 1) * chunk_stride;

  // ---- U (A operands) straight into registers: packing [cob][chunk][xi][hh][BM co][4 ch]
  // (rrin_pack_conv3x3_wino_bm, bm = BM); wave yw reads points 4 yw .. + 3, both halves
  const auto ur = buf_rsrc(a.w_hi + (int64_t)cob * nch * 32 * BM);
  const uint32_t uvoff = (uint32_t)(hh * BM + j) * 16u;
  auto load_u = [&](int c, int x, int t) {
    // byte offset of record (xi = 4 yw + x, hh, co = 32 t + j) of chunk c: the chunk and
    // point part in the scalar offset, the rest < 4 KB in the instruction's offset
    const int soff = c * (32 * BM * 16) + (4 * yw + (CT == 2 ? (x & 2) : 0)) * (2 * BM * 16);
    const int imm = (CT == 2 ? (x & 1) * 2048 : x * 1024) + t * 512;
    return buf_load16(ur, uvoff + imm, soff);
  };

  // ---- B operands: lane (j, hh) of N tile nt is patch (pr = 2 nt + (j >> 4), jx), the
  // second patch row's columns rotated by 12 (distinct banks per ds_read_b128 lane group)
  const int jx = (j + 12 * (j >> 4)) & 15;
  const int ra = yw == 0 ? 0 : (yw == 2 ? 2 : 1);
  const int rb = yw == 0 ? 2 : (yw == 1 ? 2 : (yw == 2 ? 1 : 3));
  const float sg = yw == 1 ? 1.f : -1.f;
  int pcol[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pcol[k] = hh * RG + (2 * (j >> 4)) * 34 + wc_col(2 * jx + k);
  const int oa = ra * 34, ob = rb * 34;

  cfloatx16 acc[CT][NT][4];
  // (set by chunk 0's first MFMA of each accumulator: C = 0, no zeroing per tile)
  cfloatx4 u[CT][4];              // U of the chunk being computed (point x reloaded after its MFMAs)
  cfloatx4 v[NT][4];              // B operands of the chunk being computed
  cfloatx4 d[8];                  // window records of one N tile of the next chunk

  // window records of N tile nt of the chunk in stage s -> d; B^T row yw -> its 4
  // points' B operands v[nt]
  auto read_raw = [&](int s, int nt) {
    const uint4* rw = smem4 + s * STAGE + nt * 4 * 34;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[2 * k] = __builtin_bit_cast(cfloatx4, rw[oa + pcol[k]]);
      d[2 * k + 1] = __builtin_bit_cast(cfloatx4, rw[ob + pcol[k]]);
    }
  };
  auto transform = [&](int nt) {
    if constexpr ((RRIN_WINOC_ABL & 4) != 0) {
      v[nt][0] = d[0], v[nt][1] = d[2], v[nt][2] = d[4], v[nt][3] = d[6];
      return;
    }
    cfloatx4 tr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) tr[k][e] = fmaf(sg, d[2 * k + 1][e], d[2 * k][e]);
    v[nt][0] = tr[0] - tr[2];
    v[nt][1] = tr[1] + tr[2];
    v[nt][2] = tr[2] - tr[1];
    v[nt][3] = tr[1] - tr[3];
  };
  auto mfma_point = [&](int x, int nt, const bool first) {
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[t][nt][x] = __builtin_amdgcn_mfma_f32_32x32x2f32(u[t][x][e], v[nt][x][e],
                                                                first && e == 0 ? cfloatx16{} : acc[t][nt][x], 0, 0, 0);
  };
  auto reload_u = [&](int c, int x) {
#pragma unroll
    for (int t = 0; t < CT; ++t) u[t][x] = load_u(c, x, t);
  };
  // LDS-DMA of a stage is visible to the other waves after the issuing wave's vmcnt
  // wait and a barrier; the barrier is bare (a __syncthreads() would drain vmcnt to 0
  // and wait for the chunk in flight too)
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };

  // Chunk c (U(c) in u, its B operands in v), MORE: it has a successor (a constant at
  // both call sites, folded after inlining).
  //   points 0-2, each followed by the load of its U for chunk c + 1 (into the registers
  //   it just used: three points later it is needed); the wait for raw(c + 1) (issued a
  //   chunk ago; the 4 CT younger U loads stay in flight); the barrier (raw(c + 1)
  //   visible, every read of stage (c + 2) % 3 long done); raw(c + 2) -> that stage;
  //   per N tile: chunk c + 1's window reads, point 3 (covers them), the transform of
  //   chunk c + 1 into v; point 3's U load.  VMEM order per chunk: U pts 0-2, raw(c + 2),
  //   U pt 3 -- the same counts every chunk (the prologue matches it), so the compiler's
  //   own waits for u are 3 CT + P deep and this wait is 4 CT; a chunk past the end is
  //   never loaded: raw(nch) re-reads the last chunk into the free stage.
  auto chunk = [&](int c, int s, const bool more, const bool first) {
#pragma unroll
    for (int x = 0; x < 3; ++x) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) mfma_point(x, nt, first);
      if (more && !(RRIN_WINOC_ABL & 1)) reload_u(c + 1, x);
      fence();
    }
    if (more) {
      RRIN_VMWAIT(0, (RRIN_WINOC_ABL & 1) ? 0 : 4 * CT);
      bar();
      if (!(RRIN_WINOC_ABL & 2)) issue_raw_at(raw_next, s == 0 ? 2 : s - 1);
      if (c + 3 < nch) raw_next += chunk_stride;
    }
    const int s1 = s == 2 ? 0 : s + 1;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (more && !(RRIN_WINOC_ABL & 16)) read_raw(s1, nt);
      fence();
      mfma_point(3, nt, first);
      fence();
      if (more) transform(nt);
    }
    if (more && !(RRIN_WINOC_ABL & 1)) reload_u(c + 1, 3);
  };

  // prologue in the steady state's VMEM order: raw(0), U(0) pts 0-2, raw(1), U(0) pt 3;
  // wait for raw(0); chunk 0's B operands
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
#if RRIN_WINOC_CLOCK
  const unsigned long long clk_t1 = __builtin_amdgcn_s_memtime();
#endif
  // the epilogue's bias values, loaded now: their latency hides behind the exchange
  // instead of stalling the stores (the bias blob is padded to whole BM-row blocks)
  float bsv[CT][16];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) bsv[t][i] = a.bias[(CT * cob + t) * 32 + 8 * (i >> 2) + 4 * hh + (i & 3)];
#if RRIN_WINOC_AGPR
  // A/B: an inline-asm AGPR operand makes the compiler keep MFMA accumulators in AGPRs
  asm volatile("" ::"a"(acc[0][0][0][0]));
#endif
  __syncthreads();  // every read of the stages done before the exchange reuses the LDS

  // ---- output transform (kinds 1-4's order): Q[c] = sum_x M[x] A[x][c] of this wave's
  // B^T row, Y[0][c] = (Q0 + Q1) + Q2, Y[1][c] = (Q1 - Q2) - Q3 over the four waves,
  // exchanged through LDS one co tile at a time; wave yw then finishes output row
  // r = yw & 1, column cc = yw >> 1 of its patches
  cfloatx4* X = reinterpret_cast<cfloatx4*>(smem4);
  const int r = yw & 1, cc = yw >> 1;
  uint4* dst = a.dst_hi + (int64_t)img * a.dst_img;
  auto store4 = [&](int64_t rec, const float* vv) {
    if constexpr ((RRIN_WINOC_ABL & 8) != 0) return;
    dst[rec] = make_uint4(__float_as_uint(vv[0]), __float_as_uint(vv[1]), __float_as_uint(vv[2]), __float_as_uint(vv[3]));
  };
#pragma unroll
  for (int t = 0; t < CT; ++t) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        cfloatx4 g;
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
        const cfloatx4 q0 = X[((nt * 4 + 0) * 8 + k) * 64 + lane];
        const cfloatx4 q1 = X[((nt * 4 + 1) * 8 + k) * 64 + lane];
        const cfloatx4 q2 = X[((nt * 4 + 2) * 8 + k) * 64 + lane];
        const cfloatx4 q3 = X[((nt * 4 + 3) * 8 + k) * 64 + lane];
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
        const int HH = 2 * a.h, WW = 2 * a.w, creal = a.cout >> 2;
        if (cobe * 32 < a.cout && y < a.h && x < a.w) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int Y = 2 * y + (qq >> 1), XX = 2 * x + (qq & 1);
            const int64_t ri = ring_index(Y, XX, HH, WW);
            if (ri >= 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                a.edge[((int64_t)img * creal + cobe * 8 + 4 * hh + e) * a.ring + ri] = yv[nt][4 * qq + e];
            } else {
              float vv[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) vv[e] = yv[nt][4 * qq + e] + bsv[t][4 * qq + e];
              store4((int64_t)(2 * cobe + hh) * a.dst_gp + (int64_t)(Y + 1) * a.dst_wp + XX + kH8PadLeft, vv);
            }
          }
        }
      } else {
        float vv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float tv = yv[nt][i] + bsv[t][i];
          if constexpr (EPI != RRIN_EPI_LINEAR) tv = leaky(tv, a.slope);
          vv[i] = tv;
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (cobe * 32 + 8 * qq < a.cout && y < a.h && x < a.w) {
            const int64_t rec = (int64_t)(cobe * 8 + 2 * qq + hh) * a.dst_gp + (int64_t)(y + 1) * a.dst_wp + x + kH8PadLeft;
            store4(rec, &vv[4 * qq]);
            if constexpr (EPI == RRIN_EPI_LEAKY_REP) {  // edge replicate into the padding ring
              const int dy0 = y == 0 ? -1 : 0, dy1 = y == a.h - 1 ? 1 : 0;
              const int dx0 = x == 0 ? -1 : 0, dx1 = x == a.w - 1 ? 1 : 0;
              for (int dy = dy0; dy <= dy1; ++dy)
                for (int dx = dx0; dx <= dx1; ++dx)
                  if (dy | dx) store4(rec + (int64_t)dy * a.dst_wp + dx, &vv[4 * qq]);
            }
          }
        }
        if constexpr (EPI == RRIN_EPI_LEAKY_POOL) {
          // the patch's four outputs (yw = (r, c)) meet in LDS; wave 0 writes
          // avg = 0.25 ((Y00 + Y10) + (Y01 + Y11)), kinds 1-4's order
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cfloatx4 g;
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
              const cfloatx4 y00 = X[(0 * 4 + qq) * 64 + lane];
              const cfloatx4 y10 = X[(1 * 4 + qq) * 64 + lane];
              const cfloatx4 y01 = X[(2 * 4 + qq) * 64 + lane];
              const cfloatx4 y11 = X[(3 * 4 + qq) * 64 + lane];
              if (cobe * 32 + 8 * qq < a.cout && yp < a.h && xp < a.w) {
                float s4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) s4[e] = 0.25f * ((y00[e] + y10[e]) + (y01[e] + y11[e]));
                const int64_t rec = (int64_t)(cobe * 8 + 2 * qq + hh) * a.pool_gp + (int64_t)(yp / 2 + 1) * a.pool_wp +
                                    xp / 2 + kH8PadLeft;
                pdst[rec] = make_uint4(__float_as_uint(s4[0]), __float_as_uint(s4[1]), __float_as_uint(s4[2]),
                                       __float_as_uint(s4[3]));
              }
            }
          }
          __syncthreads();
        }
      }
    }
  }
#if RRIN_WINOC_CLOCK
  const unsigned long long clk_t2 = __builtin_amdgcn_s_memtime(), clk_r2 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    unsigned long long* g = g_winoc_clk + (size_t)(bid % kClkSlots) * 4;
    g[0] = clk_t2 - clk_t0;  // core clocks, whole workgroup
    g[1] = clk_r2 - clk_r0;  // 100 MHz ticks
    g[2] = clk_t1 - clk_t0;  // core clocks to the end of the main loop
    g[3] = clk_r0;           // start (100 MHz ticks)
  }
#endif
}

template <int EPI, int CT, int NT>
static int launch_winoc_k(const ConvH8Args& a, hipStream_t st) {
  auto k = conv3x3_winoc_kernel<EPI, CT, NT>;
  static LdsAttr attr;
  constexpr size_t lds = WinoC<NT>::LDS;
  constexpr size_t flds = (size_t)kFixSubFloats * sizeof(float);  // the FULL fix-up's staging (one K group)
  constexpr size_t lmax = EPI == RRIN_EPI_SUBPIXEL && flds > lds ? flds : lds;
  if (int e = attr.ensure((const void*)k, (int)lmax, st)) return e;
  const int64_t grid = (int64_t)a.co_blocks * a.tiles_x * a.tiles_y * a.n;
  if constexpr (EPI == RRIN_EPI_SUBPIXEL) {
    if (a.fix_real > 0) {  // ring workgroups at the head of the grid; runs of one 32-channel chunk
      ConvH8Args b = a;
      b.nfix = (a.fix_real + 7) & ~7;
      b.fix.nslices = b.fix.cin / kFixCi;
      b.fix.cross = 0;
      hipLaunchKernelGGL(k, dim3((unsigned)(grid + b.nfix)), dim3(256), lmax, st, b);
      return hip_code(hipGetLastError());
    }
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  return hip_code(hipGetLastError());
}

template <int CT, int NT>
static int launch_winoc_e(const ConvH8Args& a, int epi, hipStream_t st) {
  switch (epi) {
    case RRIN_EPI_LINEAR: return launch_winoc_k<RRIN_EPI_LINEAR, CT, NT>(a, st);
    case RRIN_EPI_LEAKY: return launch_winoc_k<RRIN_EPI_LEAKY, CT, NT>(a, st);
    case RRIN_EPI_LEAKY_POOL: return launch_winoc_k<RRIN_EPI_LEAKY_POOL, CT, NT>(a, st);
    case RRIN_EPI_LEAKY_REP: return launch_winoc_k<RRIN_EPI_LEAKY_REP, CT, NT>(a, st);
    case RRIN_EPI_SUBPIXEL: return launch_winoc_k<RRIN_EPI_SUBPIXEL, CT, NT>(a, st);
  }
  return RRIN_E_ARG;
}

// Workgroup order (XCD-aware remap: an XCD runs a contiguous range of workgroups): a
// workgroup streams its co block's whole U (nchunks x 32 BM records); when the co blocks'
// U does not fit an XCD's 4 MB L2, co blocks of one tile position that started at
// different times each stream U from HBM (PMC: up to 11x the algorithmic bytes on the
// deep convs).  Groups of co blocks whose U fits kWinoCUGroupBytes put each XCD on one
// group (its U read once per XCD, L2-resident) at the price of reading each raw tile
// once per group.  The order does not change any result.
#ifndef RRIN_WINOC_UGROUP_KB
#define RRIN_WINOC_UGROUP_KB 2048
#endif
static int winoc_cob_group(const ConvH8Args& a, int bm) {
  const int64_t per_cob = (int64_t)a.nchunks * 32 * bm * 16;  // U bytes of one co block
  if (RRIN_WINOC_UGROUP_KB <= 0 || (int64_t)a.co_blocks * per_cob <= (int64_t)RRIN_WINOC_UGROUP_KB * 1024) return 0;
  int g = 1;  // the largest power of two of co blocks whose U fits (at least one)
  while (2 * g < a.co_blocks && 2 * g * per_cob <= (int64_t)RRIN_WINOC_UGROUP_KB * 1024) g *= 2;
  return g;
}

int launch_winoc(const ConvH8Args& a, int epi, int ct, hipStream_t st) {
  ConvH8Args b = a;
  b.cob_group = winoc_cob_group(a, 32 * ct);
  return ct == 2 ? launch_winoc_e<2, 1>(b, epi, st) : launch_winoc_e<1, 2>(b, epi, st);
}

}  // namespace rrin

#if RRIN_WINOC_CLOCK
// diagnostic builds only: copy n workgroup stamps (4 x u64 each) to host memory
extern "C" int rrin_winoc_clock_read(unsigned long long* host, int n) {
  if (!host || n < 1 || n > rrin::kClkSlots) return RRIN_E_ARG;
  return rrin::hip_code(hipMemcpyFromSymbol(host, HIP_SYMBOL(rrin::g_winoc_clk), (size_t)n * 4 * 8, 0,
                                            hipMemcpyDeviceToHost));
}
#endif
