// Device side of the sub-pixel up conv's ring fix-up, shared by the standalone fix-up kernel
// (conv_f16.hip edge_fix_h8_kernel) and the conv tiles that run it in extra workgroups of their
// own launch (rrin_conv_h8_desc.ring_full: conv3x3_h8_kernel, conv3x3_winoc_kernel), plus the
// record-layout helpers both need (fp16 hi / lo' split, packed-FP32 experiment switches).
#pragma once
#include "common.hpp"

namespace rrin {

// Packed-FP32 experiment only (Makefile `pk-variants`): the library
// is built without packed FP32 VALU ops; these re-enable them per kernel family.
#if defined(RRIN_PK_CONV)
#define RRIN_PK_CONV_ATTR __attribute__((target("packed-fp32-ops")))
#else
#define RRIN_PK_CONV_ATTR
#endif
#if defined(RRIN_PK_EDGE) || defined(RRIN_PK_EDGE_ASM)
#define RRIN_PK_EDGE_ATTR __attribute__((target("packed-fp32-ops")))
#else
#define RRIN_PK_EDGE_ATTR
#endif
// RRIN_PK_EDGE_ASM: the ring fix-up's FMAs as hand-placed v_pk_fma_f32 (everything
// else unpacked): 1 = src1 an explicit splat pair {u, u}, no op_sel; 2 = the form
// the compiler emits, src1 {x, u} read through op_sel:[0,1,0] (low result takes
// the high half).
#if defined(RRIN_PK_EDGE_ASM)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ inline void pk_fma4(f32x2& a01, f32x2& a23, float4 w, float u) {
  const f32x2 w01 = {w.x, w.y}, w23 = {w.z, w.w};
#if RRIN_PK_EDGE_ASM == 1
  const f32x2 uu = {u, u};
  asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a01) : "v"(w01), "v"(uu));
  asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a23) : "v"(w23), "v"(uu));
#else
  const f32x2 xu = {0.f, u};
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0]" : "+v"(a01) : "v"(w01), "v"(xu));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0]" : "+v"(a23) : "v"(w23), "v"(xu));
#endif
}
#endif

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));


// lo halves are stored pre-scaled by 2^11 so they stay normal fp16 for any
// |v| >= ~1e-4 (unscaled, v - hi ~ 2^-12 v would be subnormal below |v| = 0.125
// and lose its bits): v = hi + lo * 2^-11.
constexpr float kLoScale = 2048.0f;
constexpr float kF16Max = 65504.0f;  // largest finite fp16
constexpr float kLoUnscale = 1.0f / 2048.0f;
__device__ inline _Float16 lo_of(float v, _Float16 hi) { return (_Float16)((v - (float)hi) * kLoScale); }
__device__ inline float join(_Float16 hi, _Float16 lo) { return fmaf((float)lo, kLoUnscale, (float)hi); }

// ---- sub-pixel up conv: ring fix-up -------------------------------------------
// The EPI_SUBPIXEL conv equals conv3x3 over the upsampled image U with edge-
// replicate padding; the reference pads with zeros, so a ring pixel (Y, X) gets
//   out = pre - sum_{outside taps} W[co][ci][ky][kx] * U(clamp(Y+ky-1), clamp(X+kx-1)) + bias.
// Along each boundary line the outside taps of a pixel are the 3 taps of one
// kernel row (top/bottom line) or column (left/right line) applied to U on that
// line: a 1-D conv, done here as a small GEMM per tile of 64 line pixels x 32
// output channels with U (recomputed from the low-res source exactly as
// up2x_h8_kernel does) and the weights staged in LDS.  A corner also has the
// two other taps of its outside column ("extra" slots).  Lines: top row and
// bottom row (corners included), left and right columns without the corners.

// The 4 low-res records (8 halves / 4 floats, both planes) that bilinear x2
// (align_corners = False, edge clamp) blends into U(Y, X), and the blend weights.
template <int PLANES, bool F32 = false>
struct Up8 {
  uint4 q[4][PLANES];
  float wa, wc;
  __device__ void fetch(const EdgeFixArgs& a, const uint4* hi, const uint4* lo, int g, int Y, int X) {
    int ra, rb, ca, cb;
    if (Y & 1) { ra = Y >> 1; rb = min(ra + 1, a.sh - 1); wa = 0.75f; }
    else { rb = Y >> 1; ra = max(rb - 1, 0); wa = 0.25f; }
    if (X & 1) { ca = X >> 1; cb = min(ca + 1, a.sw - 1); wc = 0.75f; }
    else { cb = X >> 1; ca = max(cb - 1, 0); wc = 0.25f; }
    const int64_t base = (int64_t)g * a.s_gp + kH8PadLeft;
    const int64_t r[4] = {base + (int64_t)(ra + 1) * a.s_wp + ca, base + (int64_t)(ra + 1) * a.s_wp + cb,
                          base + (int64_t)(rb + 1) * a.s_wp + ca, base + (int64_t)(rb + 1) * a.s_wp + cb};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[k][0] = hi[r[k]];
      if constexpr (PLANES == 2) q[k][1] = lo[r[k]];
    }
  }
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int p = 0; p < PLANES; ++p) q[k][p] = make_uint4(0u, 0u, 0u, 0u);
    wa = wc = 0.5f;
  }
  __device__ float value(int e) const {  // horizontal then vertical, as upsample_bilinear2d
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (F32) {
        v[k] = __builtin_bit_cast(floatx4, q[k][0])[e];
      } else {
        const half8 h = __builtin_bit_cast(half8, q[k][0]);
        v[k] = (float)h[e];
        if constexpr (PLANES == 2) v[k] = join(h[e], __builtin_bit_cast(half8, q[k][PLANES - 1])[e]);
      }
    }
    const float wb = 1.0f - wa, wd = 1.0f - wc;
    const float top = wc * v[0] + wd * v[1];
    const float bot = wc * v[2] + wd * v[3];
    return wa * top + wb * bot;
  }
};

// K split (template KS): the block is KS groups of 256 threads; group k stages
// and accumulates chunks k, k + KS, ... of the input channels in its own LDS
// region, and group 0 adds the other groups' sums in group order at the end
// (one launch, fixed summation order).  KS > 1 shortens the serial chunk chain
// of the few blocks a small ring has (the deep levels: cin 128-256, 16-64
// blocks at 640x368) and gives each CU more waves to hide LDS latency.
constexpr int kFixSubFloats = kFixCi * (kFixPx + 2) + kFixCi * 4 + 7 * kFixCi * kFixCo;
// FULL (rrin_edge_fix_desc.full): the ring value from scratch -- the conv's in-image taps over
// two staged lines of U (the ring line and the next one inward, zero outside the image), plus
// the bias -- instead of the conv's pre-bias ring value minus the outside taps.  It reads
// nothing the sub-pixel conv writes, so it can run beside that conv (net.hip: side stream).
constexpr int kFixFullFloats = 2 * kFixCi * (kFixPx + 2) + 6 * kFixCi * kFixCo;
static_assert(kFixFullFloats <= kFixSubFloats, "FULL ring staging fits the K group's region");

// The fix-up of one ring workgroup (bx: ring tile, by: co block, bz: image [x K run]); the kernel
// below runs it per block, and the sub-pixel conv can run it in extra workgroups of its own
// launch (conv3x3_h8_kernel, ConvH8Args.nfix) -- KS 256-thread K groups, threadIdx.x < 256 KS
template <int PLANES, int KS, bool F32, bool FULL>
// vgroup >= 0 (KS 1 only): a larger workgroup runs one tile per 256-thread slice (slice vgroup,
// LDS staging region vgroup; every slice passes the same barriers -- the same cin, one run
// structure); active false: the slice has no tile (it computes a dummy one and stores nothing).
__device__ inline void edge_fix_body(const EdgeFixArgs& a, const int bx, const int by, const int bz,
                                     const int vgroup = -1, const bool active = true) {
  constexpr int CPR = F32 ? 4 : 8;            // channels per record
  constexpr int GPC = kFixCi / CPR;           // record groups per ci chunk
  constexpr int NL = FULL ? 2 : 1;            // staged U lines
  extern __shared__ __attribute__((aligned(16))) float s_fix[];
  const int ks = KS == 1 ? 0 : threadIdx.x >> 8;  // K group (wave-uniform)
  float* s_base = s_fix + (vgroup >= 0 ? vgroup : ks) * kFixSubFloats;
  // U: row ci * NL + l (l = 0 the ring line, 1 the next line inward)
  float(*s_u)[kFixPx + 2] = reinterpret_cast<float(*)[kFixPx + 2]>(s_base);
  // corner extras: [left ky_a, left ky_b, right ky_a, right ky_b] (not FULL)
  float(*s_ux)[4] = reinterpret_cast<float(*)[4]>(s_base + NL * kFixCi * (kFixPx + 2));
  // slots 0-2 line taps, 3-6 corner extras; FULL: slot 3 l + k = line l, tap k along the line
  float(*s_w)[kFixCi][kFixCo] = reinterpret_cast<float(*)[kFixCi][kFixCo]>(
      s_base + NL * kFixCi * (kFixPx + 2) + (FULL ? 0 : kFixCi * 4));
  const int tid = threadIdx.x & 255, px = tid & (kFixPx - 1), cg = tid / kFixPx;  // 8 groups of 4 channels
  // (fp16 records always run one K run in one workgroup: compile-time there)
  const bool cross = F32 && a.cross;
  const int nsl = F32 ? a.nslices : 1, img = cross ? bz / nsl : bz, co0 = by * kFixCo;
  const int sl0 = cross ? bz - img * nsl : 0, sl1 = cross ? sl0 + 1 : nsl;
  const int csl = a.cin / nsl;  // channels per run (a multiple of KS * kFixCi)
  const int H = 2 * a.sh, W = 2 * a.sw;
  // line of this tile: 0 top, 1 bottom, 2 left, 3 right
  int t = bx, line;
  if (t < 2 * a.tiles_row) { line = t / a.tiles_row; t -= line * a.tiles_row; }
  else { t -= 2 * a.tiles_row; line = 2 + t / a.tiles_col; t -= (line - 2) * a.tiles_col; }
  const bool row = line < 2;
  const int full = row ? W : H;                 // U positions along the line
  const int first = row ? 0 : 1, count = row ? W : H - 2;
  const int pos0 = first + t * kFixPx;          // line coordinate of pixel px = 0
  const int fixed = row ? (line == 0 ? 0 : H - 1) : (line == 2 ? 0 : W - 1);  // the other coordinate
  const int out_k = (line == 0 || line == 2) ? 0 : 2;                          // outside row/col of the kernel
  // corner extras (row lines only): corner at X = 0 and/or X = W-1 inside this tile
  const bool has_l = row && pos0 == 0, has_r = row && pos0 <= W - 1 && W - 1 < pos0 + kFixPx;
  const bool corners = !FULL && (has_l || has_r);
  const int nslot = FULL ? 6 : corners ? 7 : 3;
  const int inner_d = (line == 0 || line == 2) ? 1 : -1;  // FULL: the second line, one step inward
  // extra slot s (0-1 left corner, 2-3 right): kernel row ky = the (s&1)-th of {0,1,2} minus out_k,
  // column 0 (left) or 2 (right); its U sits at row fixed + ky - 1 of that image column
  auto xky = [&](int sl) { return (sl & 1) + (out_k == 0 ? 1 : 0); };
  const uint4* rhi = a.s_hi + (int64_t)img * a.s_img;
  const uint4* rlo = PLANES == 2 ? a.s_lo + (int64_t)img * a.s_img : nullptr;

  // per-thread staging work of one ci chunk, fetched one chunk ahead
  constexpr int kItems = GPC * NL * (kFixPx + 2);  // U: record groups x lines x line positions
  constexpr int kUIt = (kItems + 255) / 256;
  constexpr int kFixB = F32 ? (FULL ? 2 : 4) : 1;  // channels per batch of LDS reads (fp32 records only)
  Up8<PLANES, F32> ru[kUIt], rx;
  float4 rw[7];
  const int w_ci = tid >> 3, w_cq = (tid & 7) * 4;
  auto fetch = [&](int c0) {
#pragma unroll
    for (int it = 0; it < kUIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kItems) {
        const int u_gl = idx / (NL * (kFixPx + 2)), rem = idx - u_gl * (NL * (kFixPx + 2));
        const int u_l = NL == 1 ? 0 : rem / (kFixPx + 2), u_j = rem - u_l * (kFixPx + 2);
        // correction: positions past the line's ends clamp (the conv's replicate padding);
        // FULL: they are the zero padding of the upsampled image
        const int q = FULL ? pos0 - 1 + u_j : min(max(pos0 - 1 + u_j, 0), full - 1);
        const int o = fixed + u_l * inner_d;
        if (c0 + u_gl * CPR < a.cin && q >= 0 && q < full) ru[it].fetch(a, rhi, rlo, c0 / CPR + u_gl, row ? o : q, row ? q : o);
        else ru[it].zero();
      }
    }
    if (corners && tid < 4 * GPC) {  // 4 extra slots x GPC record groups
      const int sl = tid / GPC, gl = tid % GPC;
      if (c0 + gl * CPR < a.cin) rx.fetch(a, rhi, rlo, c0 / CPR + gl, fixed + xky(sl) - 1, sl < 2 ? 0 : W - 1);
      else rx.zero();
    }
    const bool ok = c0 + w_ci < a.cin && co0 + w_cq < a.cout;
#pragma unroll
    for (int sl = 0; sl < 7; ++sl) {
      rw[sl] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (sl < nslot && ok) {
        // FULL: line l of slot sl is kernel row (row lines) / column (column lines) 1 for the
        // ring line, 2 or 0 for the inner line below / above it; k runs along the line
        const int kk = sl < 3 ? 1 : (inner_d > 0 ? 2 : 0), k3 = sl % 3;
        const int tap = FULL ? (row ? kk * 3 + k3 : k3 * 3 + kk)
                             : sl < 3 ? (row ? out_k * 3 + sl : sl * 3 + out_k) : xky(sl - 3) * 3 + (sl < 5 ? 0 : 2);
        rw[sl] = *reinterpret_cast<const float4*>(a.wedge + ((int64_t)(c0 + w_ci) * 9 + tap) * a.cout + co0 + w_cq);
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int it = 0; it < kUIt; ++it) {
      const int idx = tid + 256 * it;
      if (idx < kItems) {
        const int u_gl = idx / (NL * (kFixPx + 2)), rem = idx - u_gl * (NL * (kFixPx + 2));
        const int u_l = NL == 1 ? 0 : rem / (kFixPx + 2), u_j = rem - u_l * (kFixPx + 2);
#pragma unroll
        for (int e = 0; e < CPR; ++e) s_u[(u_gl * CPR + e) * NL + u_l][u_j] = ru[it].value(e);
      }
    }
    if (corners && tid < 4 * GPC)
#pragma unroll
      for (int e = 0; e < CPR; ++e) s_ux[(tid % GPC) * CPR + e][tid / GPC] = rx.value(e);
#pragma unroll
    for (int sl = 0; sl < 7; ++sl)
      if (sl < nslot) *reinterpret_cast<float4*>(&s_w[sl][w_ci][w_cq]) = rw[sl];
  };

  // acc: the 3 line taps; accx: a corner pixel's 2 extra taps, kept apart so the
  // line-tap loop has no per-thread branch (a branch per ci split the loop into
  // blocks that each waited out their own LDS reads: one wave per SIMD, nothing
  // else to hide the latency) and added at the end of each run
  float acc[4], accx[4], tot[4] = {0.f, 0.f, 0.f, 0.f};
#if defined(RRIN_PK_EDGE_ASM)
  f32x2 acc01, acc23, accx01, accx23;
#define FIX_FMA(A, W_, U_) pk_fma4(A##01, A##23, W_, U_)
#else
#define FIX_FMA(A, W_, U_)             \
  A[0] = fmaf((W_).x, U_, A[0]);       \
  A[1] = fmaf((W_).y, U_, A[1]);       \
  A[2] = fmaf((W_).z, U_, A[2]);       \
  A[3] = fmaf((W_).w, U_, A[3])
#endif
  const int pos = pos0 + px;
  const bool cl = has_l && pos == 0, cr = has_r && pos == W - 1;
  const int sb = cl ? 0 : 2;  // corner extra slots of this thread (used by cl / cr only)
  // the conv's pre-fix ring values and the bias, loaded up front: their latency
  // overlaps the first chunk's instead of following the last one
  const bool live = active && ks == 0 && pos - first < count;
  const int Y = row ? fixed : pos, X = row ? pos : fixed;
  float pre[4] = {0.f, 0.f, 0.f, 0.f}, bco[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_pre = [&]() {
    const int64_t e = ring_index(Y, X, H, W);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + cg * 4 + i;
      if (co < a.cout) {
        if constexpr (!FULL) pre[i] = a.edge[((int64_t)img * a.cout + co) * a.ring + e];
        bco[i] = a.bias[co];
      }
    }
  };
  // fp32 records only (fp16: C3 measured ~0.7 % slower with the preload and the
  // batched loop; its KS 4 variant runs at 128 VGPRs)
  constexpr bool kPre = F32;
  if constexpr (kPre)
    if (live) load_pre();
  // every K group runs the same number of chunks per run (launch: csl % (KS * kFixCi) == 0)
  fetch(sl0 * csl + ks * kFixCi);
  for (int sl = sl0; sl < sl1; ++sl) {
#if defined(RRIN_PK_EDGE_ASM)
    acc01 = acc23 = accx01 = accx23 = f32x2{0.f, 0.f};
#else
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = accx[i] = 0.f;
#endif
    const int cend = (sl + 1) * csl;
    for (int c0 = sl * csl + ks * kFixCi; c0 < cend; c0 += KS * kFixCi) {
      stage();
      __syncthreads();
      // the next chunk of this group, in this run or the next one, is in flight during the FMAs below
      const int nxt = c0 + KS * kFixCi < cend ? c0 + KS * kFixCi : (sl + 1 < sl1 ? cend + ks * kFixCi : -1);
      if (nxt >= 0) fetch(nxt);
      // fp32 records: batches of kFixB channels, every LDS read of a batch issued
      // before its FMAs (the scheduler otherwise waits out each read on its own);
      // fp16 (kFixB 1): the plain unrolled loop measured no slower (C3, same box)
      if constexpr (kFixB == 1) {
#pragma unroll 4
        for (int ci = 0; ci < kFixCi; ++ci)
#pragma unroll
          for (int k = 0; k < 3 * NL; ++k) {
            const float u = s_u[ci * NL + k / 3][px + k % 3];
            const float4 w = *reinterpret_cast<const float4*>(&s_w[k][ci][cg * 4]);
            FIX_FMA(acc, w, u);
          }
      } else
#pragma clang loop unroll(disable)
      for (int cb = 0; cb < kFixCi; cb += kFixB) {
        float u[kFixB][3 * NL];
        float4 w[kFixB][3 * NL];
#pragma unroll
        for (int j = 0; j < kFixB; ++j)
#pragma unroll
          for (int k = 0; k < 3 * NL; ++k) {
            u[j][k] = s_u[(cb + j) * NL + k / 3][px + k % 3];
            w[j][k] = *reinterpret_cast<const float4*>(&s_w[k][cb + j][cg * 4]);
          }
#pragma unroll
        for (int j = 0; j < kFixB; ++j)
#pragma unroll
          for (int k = 0; k < 3 * NL; ++k) {
            FIX_FMA(acc, w[j][k], u[j][k]);
          }
      }
      if (corners) {  // block-uniform; every thread runs it, cl / cr keep the result
#pragma unroll 2
        for (int ci = 0; ci < kFixCi; ++ci)
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const float u = s_ux[ci][sb + m];
            const float4 w = *reinterpret_cast<const float4*>(&s_w[3 + sb + m][ci][cg * 4]);
            FIX_FMA(accx, w, u);
          }
      }
      __syncthreads();
    }
#if defined(RRIN_PK_EDGE_ASM)
    acc[0] = acc01.x; acc[1] = acc01.y; acc[2] = acc23.x; acc[3] = acc23.y;
    accx[0] = accx01.x; accx[1] = accx01.y; accx[2] = accx23.x; accx[3] = accx23.y;
#endif
    if (cl || cr)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] += accx[i];
    if constexpr (KS > 1) {
      // groups 1.. park their run sums in their own (now idle) staging region
      if (ks > 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) s_base[i * 256 + tid] = acc[i];
      }
      __syncthreads();
      if (ks == 0) {
#pragma unroll
        for (int k = 1; k < KS; ++k)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] += s_fix[k * kFixSubFloats + i * 256 + tid];
      }
      __syncthreads();  // the next run's staging overwrites the parked sums
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) tot[i] = sl == sl0 ? acc[i] : tot[i] + acc[i];
  }
#undef FIX_FMA
  if (cross) {
    // split-K seam, sc1 form (as conv3x3_winoq_kernel's SK path): write-through run
    // sums, drain, barrier, one relaxed ticket; the last workgroup reads every run's
    // sums with sc1 loads and adds them in run order
    const int64_t tile = ((int64_t)img * (2 * a.tiles_row + 2 * a.tiles_col) + bx) * ((a.cout + kFixCo - 1) / kFixCo) + by;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(a.part + tile * nsl * 1024, 0, nsl * 1024 * 4, 0x00020000);
    if (ks == 0) {
      const u32x4 v = {__float_as_uint(tot[0]), __float_as_uint(tot[1]), __float_as_uint(tot[2]),
                       __float_as_uint(tot[3])};
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (sl0 * 256 + tid) * 16, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* s_last = reinterpret_cast<int*>(s_fix);  // group 0's staging region is idle now
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == nsl - 1;
      if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      *s_last = last;
    }
    __syncthreads();
    if (!*s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (live) {
#pragma unroll 1
      for (int k = 0; k < nsl; ++k) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (k * 256 + tid) * 16, 0, 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) tot[i] = k == 0 ? __uint_as_float(v[i]) : tot[i] + __uint_as_float(v[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = tot[i];
  if (!live) return;
  if constexpr (!kPre) load_pre();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + cg * 4 + i;
    if (co >= a.cout) break;
    float v = FULL ? acc[i] + bco[i] : (pre[i] - acc[i]) + bco[i];
    if (a.leaky) v = v > 0.f ? v : v * a.slope;
    const int64_t k = (((int64_t)img * a.d_img + (int64_t)(co / CPR) * a.d_gp + (int64_t)(Y + 1) * a.d_wp + X +
                        kH8PadLeft) * CPR) + (co % CPR);
    if constexpr (F32) {
      a.d_f32[k] = v;
    } else {
      if (a.status && !(fabsf(v) <= kF16Max)) *a.status = 1;
      const _Float16 vh = (_Float16)v;
      a.d_hi[k] = vh;
      if constexpr (PLANES == 2) a.d_lo[k] = lo_of(v, vh);
    }
  }
}


}  // namespace rrin
