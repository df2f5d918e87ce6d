// Shared device/host helpers for librrin_hip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/rrin_hip.h"

// Counted wait for LDS-DMA staging: s_waitcnt vmcnt(LDS + LD), declaring that the LDS + LD
// youngest vector-memory loads at this point are LDS younger LDS-DMA pieces and LD register
// loads (stores are not counted: they return out of order with loads and can only make the
// wait stricter).  Loads return in issue order, so every load issued before those -- the
// awaited stage -- has landed.  The count is right only for the VMEM order the source pins with
// sched_barrier fences; `make check-isa` (tools/isa_vmcheck.py) walks every path of the
// compiled gfx950 code back from each declared wait and fails the build on a mismatch.
#define RRIN_VMWAIT(LDS, LD) \
  asm volatile("s_waitcnt vmcnt(%0) ; rrin-vm lds=%1 ld=%2" ::"n"((LDS) + (LD)), "n"(LDS), "n"(LD) : "memory")

// Pins the vector-memory issue order at this point (no VMEM instruction is scheduled across
// it; ALU, MFMA and LDS instructions may move): the fence around each issue group a counted
// RRIN_VMWAIT relies on.  sched_barrier's mask names the instruction classes allowed across --
// here everything but VMEM (0x10 all, 0x20 read, 0x40 write).
// (RRIN_NO_VMFENCE: a check build without the fences, tests/test_isa_check.py only.)
#ifdef RRIN_NO_VMFENCE
#define vm_fence() ((void)0)
#else
#define vm_fence() __builtin_amdgcn_sched_barrier(0x78F)
#endif

namespace rrin {

constexpr int kPadRowsAlign = 16;  // hp = round_up(h,16) + 2
constexpr int kPadColsAlign = 32;  // wp = round_up(w,32) + 64
constexpr int kPadLeft = 32;       // pixel x at column x+32: every 32-px output row segment
                                   // is one whole 128-B line (full-line stores)

__host__ __device__ inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

inline rrin_geom make_geom(int h, int w) {
  rrin_geom g;
  g.h = h;
  g.w = w;
  g.hp = round_up(h, kPadRowsAlign) + 2;
  g.wp = round_up(w, kPadColsAlign) + 2 * kPadLeft;
  g.plane = (int64_t)g.hp * g.wp;
  return g;
}

// Offset (floats) of pixel (y,x) inside a plane.
__host__ __device__ inline int64_t pp_pix(const rrin_geom& g, int y, int x) {
  return (int64_t)(y + 1) * g.wp + (x + kPadLeft);
}

// Pointer to channel c (absolute, view offset applied) of image n.
__host__ __device__ inline float* pp_chan(const rrin_pp& v, int n, int c) {
  return v.base + n * v.img_stride + (int64_t)(v.ch_off + c) * v.g.plane;
}

inline int hip_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// ---- per-device launch caches ------------------------------------------------
// The library keeps no state that affects results.  It caches, per device and
// kernel, facts about launching it (the dynamic-LDS attribute has been set; the
// resident blocks per CU); these caches are keyed by the device of the stream the
// launch goes to (not the calling thread's current device: a C-ABI caller may pass
// another device's stream) and are thread-safe (atomics; a race only repeats an
// idempotent query).
constexpr int kMaxDevices = 64;

// Device of stream st (the null stream: the calling thread's current device).
inline int stream_device(hipStream_t st) {
  int d = -1;
  if (st == nullptr || hipStreamGetDevice(st, &d) != hipSuccess) {
    if (hipGetDevice(&d) != hipSuccess) d = 0;
  }
  return (d >= 0 && d < kMaxDevices) ? d : 0;
}

// Run f() with device dev current on this thread (hipFuncSetAttribute and the
// occupancy query act on the current device), restoring the caller's after.
template <class F>
inline hipError_t on_device(int dev, F f) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = dev;
  if (prev != dev) {
    const hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess) return e;
  }
  const hipError_t r = f();
  if (prev != dev) (void)hipSetDevice(prev);
  return r;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device of st).
struct LdsAttr {
  std::atomic<uint64_t> done{0};
  int ensure(const void* kernel, int lds_bytes, hipStream_t st) {
    const int dev = stream_device(st);
    const uint64_t bit = 1ull << dev;
    if (done.load(std::memory_order_acquire) & bit) return 0;
    hipError_t e = on_device(dev, [&] {
      return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    });
    if (e != hipSuccess) return (int)e;
    done.fetch_or(bit, std::memory_order_release);
    return 0;
  }
};

// Two 8-B record halves per lane -> one whole 16-B record per lane (gfx950 v_permlane32_swap):
// lane (j, hh) holds half hh (channels 4 hh .. 4 hh + 3) of 8-channel block q0 in x and of block
// q1 in y -- the MFMA output layout of the H8 epilogues; returns to lane (j, 0) the whole record
// of block q0 and to lane (j, 1) that of block q1 (dwords in channel order).  Two VALU ops per
// record, no LDS: a 16-lane group of ds_write_b64 half-records at a 16-B stride is a 2-way bank
// conflict, and whole records halve the store instructions.
__device__ inline uint4 halves_to_record(uint2 x, uint2 y) {
  const auto a = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
  return make_uint4(a[0], b[0], a[1], b[1]);
}

// ---- H8 (channel-blocked fp16 records) geometry -----------------------------
constexpr int kH8PadLeft = 8;  // records: pixel x at record x+8 (128-B aligned rows)

inline rrin_geom make_geom_h8(int h, int w) {
  rrin_geom g;
  g.h = h;
  g.w = w;
  g.hp = round_up(h, kPadRowsAlign) + 2;
  g.wp = round_up(w, kPadColsAlign) + 2 * kH8PadLeft;
  g.plane = (int64_t)g.hp * g.wp;
  return g;
}

// ---- backwarp: grid_sample(bilinear, zeros, align_corners=False) ----------
// Sampling position follows the reference grid arithmetic in fp32:
//   x = gx + u;  nx = 2*(x/W - 0.5);  ix = (nx + 1) * (W/2) - 0.5   (CPU unnormalize)
// then bilinear weights nw = s*e, ne = s*w, sw = n*e, se = n*w with zero taps
// outside the frame (PyTorch CPU grid sampler order).
struct WarpTaps {
  int x0, y0;
  float nw, ne, sw, se;
  float wx, wy;  // fractional position: ix - floor(ix), iy - floor(iy) (the backward's weights)
  bool vx0, vx1, vy0, vy1;
};

#pragma clang fp contract(off)
__device__ inline WarpTaps warp_taps(int gx, int gy, float u, float v, int H, int W) {
  WarpTaps t;
  const float x = (float)gx + u;
  const float y = (float)gy + v;
  const float nx = 2.0f * (x / (float)W - 0.5f);
  const float ny = 2.0f * (y / (float)H - 0.5f);
  const float ix = (nx + 1.0f) * ((float)W / 2.0f) - 0.5f;
  const float iy = (ny + 1.0f) * ((float)H / 2.0f) - 0.5f;
  const float fx = floorf(ix);
  const float fy = floorf(iy);
  const float we = ix - fx;  // "w" in the CPU kernel: distance to the west edge
  const float e = 1.0f - we;
  const float n = iy - fy;
  const float s = 1.0f - n;
  t.wx = we;
  t.wy = n;
  t.nw = s * e;
  t.ne = s * we;
  t.sw = n * e;
  t.se = n * we;
  // validity tested in float so that huge / non-finite flows never overflow an int
  t.vx0 = fx >= 0.0f && fx <= (float)(W - 1);
  t.vx1 = fx >= -1.0f && fx <= (float)(W - 2);
  t.vy0 = fy >= 0.0f && fy <= (float)(H - 1);
  t.vy1 = fy >= -1.0f && fy <= (float)(H - 2);
  t.x0 = (t.vx0 || t.vx1) ? (int)fx : 0;
  t.y0 = (t.vy0 || t.vy1) ? (int)fy : 0;
  return t;
}

// plane: channel base; rs: row stride; off: offset of pixel (0,0)
__device__ inline float warp_apply(const WarpTaps& t, const float* plane, int64_t rs, int64_t off) {
  const float* p = plane + off + (int64_t)t.y0 * rs + t.x0;
  const float a = (t.vy0 && t.vx0) ? p[0] : 0.0f;
  const float b = (t.vy0 && t.vx1) ? p[1] : 0.0f;
  const float c = (t.vy1 && t.vx0) ? p[rs] : 0.0f;
  const float d = (t.vy1 && t.vx1) ? p[rs + 1] : 0.0f;
  return a * t.nw + b * t.ne + c * t.sw + d * t.se;
}

// Same, with a value accessor get(y, x) (used for the fp16-split Net buffer).
template <class F>
__device__ inline float warp_apply_f(const WarpTaps& t, F get) {
  const float a = (t.vy0 && t.vx0) ? get(t.y0, t.x0) : 0.0f;
  const float b = (t.vy0 && t.vx1) ? get(t.y0, t.x0 + 1) : 0.0f;
  const float c = (t.vy1 && t.vx0) ? get(t.y0 + 1, t.x0) : 0.0f;
  const float d = (t.vy1 && t.vx1) ? get(t.y0 + 1, t.x0 + 1) : 0.0f;
  return a * t.nw + b * t.ne + c * t.sw + d * t.se;
}
#pragma clang fp contract(on)

// ---- record-layout conv kernels (conv_f16.hip, conv_wino.hip) -------------
// LeakyReLU for 0 <= slope <= 1 (h8_prepare checks): one mul + one max
__device__ inline float leaky(float t, float slope) { return fmaxf(t, t * slope); }

// sub-pixel ring fix-up (conv_f16.hip edge_fix_*): tiles of kFixPx line pixels x kFixCo output
// channels, input channels staged kFixCi at a time
constexpr int kFixPx = 32, kFixCo = 32, kFixCi = 32;

struct EdgeFixArgs {
  const uint4* s_hi;
  const uint4* s_lo;
  int64_t s_img, s_gp;  // records
  int s_wp, sh, sw, cin;
  _Float16* d_hi;
  _Float16* d_lo;
  float* d_f32;  // F32R output (d_hi / d_lo unused)
  int64_t d_img, d_gp;
  int d_wp, cout;
  const float* edge;
  const float* wedge;  // [cin][9][cout]
  const float* bias;
  int64_t ring;
  float slope;
  int leaky;
  int tiles_row, tiles_col;  // tiles per row line / per column line
  int* status;               // optional fp16 range flag
  // K slices: the cin chunks in nslices runs of KS chunks (one per K group) or,
  // fp16, one run; a run's group sums are added in group order, the runs' sums
  // in run order.  cross: one workgroup per (tile, run), partial sums through
  // part (1024 floats per run) and the last workgroup (cnt ticket) adds them in
  // run order -- the same arithmetic as one workgroup looping over the runs.
  int nslices, cross;
  float* part;
  int* cnt;
};

struct ConvH8Args {
  const uint4* src_hi;
  const uint4* src_lo;
  int64_t src_img, src_gp;  // records per image / per group plane
  int src_wp;
  int cin, nchunks;         // chunks of 16 input channels
  uint4* dst_hi;
  uint4* dst_lo;
  int64_t dst_img, dst_gp;
  int dst_wp, cout;
  uint4* pool_hi;
  uint4* pool_lo;
  int64_t pool_img, pool_gp;
  int pool_wp;
  const uint4* w_hi;
  const uint4* w_lo;
  const float* bias;
  float inv_wscale, slope;
  int h, w, co_blocks, tiles_x, tiles_y, n;
  int tail_finite;
  float* edge;  // EPI_SUBPIXEL: [n][cout/4][ring] pre-bias values of the 2h x 2w ring
  int64_t ring;
  int* status;  // optional fp16 range flag (F16X3 / F16)
  // Winograd split-K (ksplit > 1): slice ks of a tile runs chunks [ks * kper, ..), writes its
  // pre-bias outputs to part and counts itself in cnt[tile]; the last slice sums all of them
  // in slice order and runs the epilogue (cnt is reset to 0 by that slice)
  int ksplit, kper;
  float* part;
  int* cnt;
  // EPI_SUBPIXEL ring fold (Winograd kind 3, conv_wino.hip): nring correction blocks at
  // the head of the grid compute the out-of-image taps of every ring segment (nseg per
  // image and co block) into corr; the segment's conv tile and its correction block
  // each count themselves in rcnt, and the later one writes the ring pixels
  int nring, nseg, rstride;  // rstride: workgroups per ring group of 8 (a multiple of 8)
  const float* wedge;     // [cin][9][cout/4] original weights
  const float* bias_raw;  // [cout/4]
  float* corr;            // [n][co_blocks][nseg][512]
  int* rcnt;              // [n][co_blocks][nseg], zero between launches
  // register-U Winograd tiles (conv_winoc.hip): workgroup order in groups of cob_group
  // co blocks (0: one group of all co blocks), tile positions within a group, the
  // group's co blocks fastest -- see launch_winoc
  int cob_group;
  // EPI_SUBPIXEL, the ring from scratch in the same launch (rrin_conv_h8_desc.ring_full): the
  // first nfix workgroups of the grid (a multiple of 8: the conv tiles keep their XCD remap) run
  // the FULL ring fix-up over fix (fix_real of them do work; workgroup r covers ring tile
  // r % fix_gx, co block (r / fix_gx) % fix_gy, image r / (fix_gx fix_gy)); they read only the
  // conv's input and write only the ring pixels of dst, which the conv does not write
  EdgeFixArgs fix;
  int nfix, fix_real, fix_gx, fix_gy;
};

// Ring index of pixel (y, x) of an H x W image (rrin_ring_pixels order: top
// row, bottom row, left column, right column; corners in the rows), -1 inside.
__device__ inline int64_t ring_index(int y, int x, int H, int W) {
  if (y == 0) return x;
  if (y == H - 1) return (int64_t)W + x;
  if (x == 0) return 2 * (int64_t)W + (y - 1);
  if (x == W - 1) return 2 * (int64_t)W + (H - 2) + (y - 1);
  return -1;
}

// LDS-DMA: one 16-byte record per lane straight from global memory into the
// lane-linear LDS image (global_load_lds_dwordx4; LDS address = wave-uniform
// base + lane*16), no VGPRs and no LDS store pass.
__device__ inline void dma16(const uint4* src, uint4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Winograd F(2x2,3x3) exact-fp32 conv (conv_wino.hip): tile config kWinoCfg of
// the record-layout table (F32R only), its LDS bytes per block and launcher.
constexpr size_t kWinoLds = (size_t)(2 * 704 + 2 * 16 * 2 * 32) * 16;
int launch_wino(const ConvH8Args& a, int epi, hipStream_t st);
// zero channels [c0, c1) of a record-layout view (conv_f16.hip)
int clear_channels_h8(const rrin_h8* v, int32_t n, int32_t c0, int32_t c1, int32_t prec, hipStream_t st);
// cfg 18's tile on 8 waves of 4 accumulators (<= 128 VGPRs: 4 waves per SIMD),
// two stages of [raw 680 | U 1024] records (three in A/B builds: two blocks per
// CU would fill 163,584 B)
constexpr size_t kWinoQLds = (size_t)3 * (680 + 1024) * 16;
// th = 8 (cfg 20: 8 waves) or 4 (cfg 21: 4 waves, the same arithmetic on half-height tiles)
int launch_winoq(const ConvH8Args& a, int epi, int th, hipStream_t st);
// register-U Winograd tiles (conv_winoc.hip): 4 waves, two blocks per CU, the U operands
// loaded straight into registers; ct = 2: BM 64 x TH 4 (kind 6), ct = 1: BM 32 x TH 8 (kind 7).
// LDS: max(3 raw stages, the output-transform exchange)
constexpr size_t kWinoCLds1 = (size_t)2048 * 16;  // TH 4: 3 x 512 stage records < 2048 exchange
constexpr size_t kWinoCLds2 = (size_t)4096 * 16;  // TH 8: 3 x 768 < 4096
int launch_winoc(const ConvH8Args& a, int epi, int ct, hipStream_t st);
// the register-U tile in Winograd F(4,3) x F(2,3) (conv_winoc42.hip, kind 14): BM 32 x 32 px x
// TH 8, 4 waves, two blocks per CU; LDS: max(3 raw stages of 768, the 4 x 16 x 65 exchange)
constexpr size_t kWinoC42Lds = (size_t)4160 * 16;
int launch_winoc42(const ConvH8Args& a, int epi, hipStream_t st);
// whether rrin_conv3x3_h8_fwd runs a ring_full fix-up inside the conv's launch for tile config
// cfg, cin input channels and precision prec (else it launches it after the conv) -- conv_f16.hip
bool ring_in_launch_ok(int cfg, int cin, int prec);
// the kind-6 tile at fp16 (conv_winoh.hip): H8 records, v_mfma_f32_32x32x16_f16, packed-f16
// input transform; same LDS as kWinoCLds1
int launch_winoh(const ConvH8Args& a, int epi, hipStream_t st);
// fused level-0 UNetConvBlock at fp16 (conv_block0.hip): conv a (cin -> 32) + leaky, conv b
// (32 -> 32) + leaky (+ pool), conv a's output tile in LDS.  Tile kB0TH x kB0TW outputs; conv a
// runs on (kB0TH + 2) x (kB0TW + 2) positions from a (kB0TH + 4) x (kB0TW + 4) input tile
struct Block0Args {  // strides in records; every image of src / dst / pool spans < 2^31 bytes
  const uint4* src;
  int src_img, src_gp;      // records per image / group plane
  int src_wp, src_hp;       // records per row, rows per plane
  int cin, ngroups, nch;    // input channels, their record groups, 16-channel chunks
  const uint4* wa;          // conv a: rrin_pack_conv3x3_h8 halves (co block 0 of width bma)
  int bma;
  const float* ba;
  float isa;
  const uint4* wb;          // conv b
  int bmb;
  const float* bb;
  float isb;
  uint4* dst;
  int dst_img, dst_gp;
  int dst_wp;
  uint4* pool;              // nullptr: no pool output
  int pool_img, pool_gp;
  int pool_wp;
  float slope;
  int h, w, n, tiles_x, tiles_y;
  int* status;
};
constexpr int kB0TH = 8, kB0TW = 62;
constexpr int kB0IR = kB0TH + 4, kB0IC = kB0TW + 4;  // input tile rows / columns
constexpr int kB0MR = kB0TH + 2, kB0MC = kB0TW + 4;  // conv-a tile rows / columns (64 computed + 2 pad)
constexpr int kB0In = 2 * kB0IR * kB0IC;             // input records per 16-channel chunk
constexpr int kB0Pieces = (kB0In + 255) / 256;       // LDS-DMA pieces per thread and chunk
constexpr int kB0Stage = kB0Pieces * 256;            // records per input stage (tail: dummy)
constexpr int kB0Mid = 4 * kB0MR * kB0MC;            // conv-a tile records (aliases input stage Y)
// LDS: conv-a tile | input stage X | 64 bias floats (stage Y inside the conv-a tile)
constexpr size_t kB0Lds = (size_t)(kB0Mid + kB0Stage + 16) * 16;
static_assert(kB0Stage <= kB0Mid, "stage Y inside the conv-a tile");
static_assert(2 * kB0Lds <= 160 * 1024, "two fused-block workgroups per CU");
int launch_block0(const Block0Args& a, hipStream_t st);
#ifdef RRIN_LAB
int launch_wino_lab(const ConvH8Args& a, int abl, hipStream_t st);  // ablation bits (conv_wino.hip)
#endif

}  // namespace rrin
