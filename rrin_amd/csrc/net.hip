// Native forward schedule of RRIN Net (reference model.py:32-65, unet.py:40-51):
// carves the caller's workspace into padded-planar activation buffers and
// enqueues the 77 MFMA convs + 4 fused head convs + 1 input pack on one stream.
// Also: host-side weight packing, error strings, ABI version.
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "common.hpp"

using namespace rrin;

struct rrin_prof {
  std::vector<hipEvent_t> ev;  // 2 per launch: start (recorded or shared), end
  std::vector<int32_t> start;  // per launch: index in ev of its start event
  std::vector<int32_t> kind;
  std::vector<double> flops;
  int count = 0;
  // within one rrin_net_fwd / rrin_unet_fwd call every launch on its stream is
  // bracketed, so a launch that directly follows the previous one on the same
  // stream starts at that launch's end event: one event record per launch
  bool chain = false;  // last_st / last_slot describe the call's previous launch
  hipStream_t last_st = nullptr;
  int last_slot = -1;
};

namespace {

// The four U-Nets in execution order (model.py:35,42,51,62) with the input
// channel count they read from the 16-channel Net buffer g16 (starting at 0).
struct UNetSpec {
  int in_ch, out_ch, depth, head_mode;
};
constexpr UNetSpec kUNets[4] = {
    {6, 4, 5, RRIN_HEAD_FLOW},     // Flow        = UNet(6, 4, 5)   model.py:28
    {10, 4, 4, RRIN_HEAD_REFINE},  // refine_flow = UNet(10, 4, 4)  model.py:29
    {16, 2, 4, RRIN_HEAD_MASK},    // Mask        = UNet(16, 2, 4)  model.py:27
    {9, 3, 4, RRIN_HEAD_FINAL},    // final       = UNet(9, 3, 4)   model.py:30
};
constexpr int kMaxDepth = 5;

inline int chans(int level) { return 32 << level; }  // unet.py:26, wf=5
inline int convs_of(int depth) { return 2 * depth + 1 + 3 * (depth - 1); }

struct Buf {
  float* base;  // F32: fp32 PP planes; F16* / F32R: (hi) records
  void* lo;     // F16X3: lo records
  int ch;
  int cpr;      // record layouts: channels per 16-B record (8: F16*, 4: F32R)
  rrin_geom g;
};

// What a schedule needs of the caller's scratch (size query, rrin_net_scratch_bytes):
// split-K slabs and tickets of the split convs, the ring fix-up's cross-workgroup K split.
struct ScratchNeed {
  int64_t part_floats = 0, cnt_ints = 0;
  void add(int64_t f, int64_t c) {
    part_floats = f > part_floats ? f : part_floats;
    cnt_ints = c > cnt_ints ? c : cnt_ints;
  }
};

// Workspace plan: offsets are identical in size query and forward.
struct Plan {
  int n, prec;
  rrin_prof* prof;        // the caller's launch profiler of this call (nullable)
  int32_t* status;        // the caller's fp16 range flag (nullable)
  rrin_geom g[kMaxDepth];
  Buf G;                  // 16 ch at level 0
  Buf X[kMaxDepth];       // level input (L >= 1): C_{L-1} ch
  Buf T[kMaxDepth];       // first conv of a block: C_L ch
  Buf CAT[kMaxDepth - 1]; // [up | bridge]: 2 C_L ch  (levels 0..3)
  Buf BOT;                // Flow bottom (level 4) conv-b output: 512 ch
  Buf UPT[kMaxDepth - 1]; // F16*: upsampled input of an up.1 conv, one per level (2 C_L ch).  Not
                          // shared across levels: another level's interior writes would land in
                          // this level's zero padding (the conv halo).
  Buf LRB[kMaxDepth];     // F16*, L >= 1: low-res input of a sub-pixel up conv (C_L ch), written with
                          // edge-replicate padding by its producer (EPI_LEAKY_REP)
  float* EDGE;            // F16*: pre-bias ring values of the current sub-pixel up conv
  Buf FLOWRAW;            // raw 4-ch Flow output, kept for reuse across t (skip_flow)
  // split-K / ring fix-up K-split scratch: the caller's (rrin_net_desc.scratch), not the
  // workspace, so a plan without splits pays nothing for it
  float* PART;            // F32R: split-K slice outputs of the current conv (part_floats)
  int32_t* CNT;           // F32R: split-K tile counters (cnt_ints; zero between convs)
  int64_t part_floats, cnt_ints;
  ScratchNeed* dry;       // non-null: size query only -- record the scratch the schedule
                          // needs, launch nothing (rrin_net_scratch_bytes)
  float* RCORR;           // F32R: ring-fold corrections of the current sub-pixel conv
  int32_t* RCNT;          // F32R: ring-fold segment tickets (zero between convs)
  int64_t rcorr_floats, rcnt_ints;
  int64_t bytes;
};

// Caller-provided scratch (rrin_net_desc.scratch): [tickets | part floats].  The ticket count is
// a function of the schedule (n, h, w, the conv table): at least kScratchTickets, else the
// schedule's largest split conv's tile count rounded up to 1024 (scratch_tickets); the size
// query and the forward derive it the same way, so the part slab starts at the same byte.
constexpr int64_t kScratchTickets = 4096;  // minimum ints at the head of the scratch (16 KB)
// ring fix-up: cross-workgroup K split up to this many workgroups (one per CU;
// RRIN_EDGE_CROSS_MAX: A/B builds)
#ifndef RRIN_EDGE_CROSS_MAX
#define RRIN_EDGE_CROSS_MAX 256
#endif
constexpr int64_t kEdgeCrossMaxGroups = RRIN_EDGE_CROSS_MAX;
// fp16 / split16 sub-pixel up convs: the ring from scratch (ABI 17 ring_full), inside the conv's
// launch where the tile allows it (direct-form tiles of 256 / 512 threads; ring_in_launch_ok),
// else as a second launch in the same summation order: every size class gets the same ring bits.
// Exact fp32 keeps the correction launch (its K-split form on small grids: C2 339.6-339.7 vs
// 334.4-334.6 pairs/s with the ring in the Winograd launch, headline +0.3 %; profiles/r06/ring/).
// RRIN_RING_INLAUNCH=0: the correction launch at every precision (A/B)
#ifndef RRIN_RING_INLAUNCH
#define RRIN_RING_INLAUNCH 1
#endif
constexpr bool kRingInLaunch = RRIN_RING_INLAUNCH != 0;

int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }

void make_plan(int n, int h, int w, int prec, char* base, Plan& p) {
  p.n = n;
  p.prec = prec;
  p.prof = nullptr;
  p.status = nullptr;
  const bool f32 = prec == RRIN_PREC_F32;
  const int planes = prec == RRIN_PREC_F16X3 ? 2 : 1;
  const int cpr = prec == RRIN_PREC_F32R ? 4 : 8;
  int64_t off = 0;
  auto take = [&](int ch, const rrin_geom& g) {
    Buf b;
    // F32: ch fp32 planes; F16*: ch/8 record planes of 16 B (same 4 B/value with lo);
    // F32R: ch/4 record planes of 16 B
    const int64_t bytes = f32 ? (int64_t)n * ch * g.plane * 4 : (int64_t)n * ((ch + cpr - 1) / cpr) * g.plane * 16;
    b.base = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += align256(bytes);
    b.lo = nullptr;
    if (planes == 2) {
      b.lo = base ? static_cast<void*>(base + off) : nullptr;
      off += align256(bytes);
    }
    b.ch = ch;
    b.cpr = cpr;
    b.g = g;
    return b;
  };
  for (int L = 0; L < kMaxDepth; ++L) p.g[L] = f32 ? make_geom(h >> L, w >> L) : make_geom_h8(h >> L, w >> L);
  p.G = take(16, p.g[0]);
  for (int L = 0; L < kMaxDepth; ++L) {
    p.X[L] = L ? take(chans(L - 1), p.g[L]) : Buf{nullptr, nullptr, 0, cpr, p.g[0]};
    p.T[L] = take(chans(L), p.g[L]);
    if (L < kMaxDepth - 1) p.CAT[L] = take(2 * chans(L), p.g[L]);
  }
  p.BOT = take(chans(kMaxDepth - 1), p.g[kMaxDepth - 1]);
  for (int L = 0; L < kMaxDepth - 1; ++L)
    p.UPT[L] = f32 ? Buf{nullptr, nullptr, 0, cpr, p.g[L]} : take(2 * chans(L), p.g[L]);
  int64_t edge_floats = 0;
  for (int L = 0; L < kMaxDepth; ++L) {
    p.LRB[L] = (f32 || L == 0) ? Buf{nullptr, nullptr, 0, cpr, p.g[L]} : take(chans(L), p.g[L]);
    if (L < kMaxDepth - 1) {
      const int64_t hh = h >> L, ww = w >> L;
      const int64_t e = (int64_t)n * chans(L) * (2 * ww + 2 * (hh - 2));
      edge_floats = e > edge_floats ? e : edge_floats;
    }
  }
  p.EDGE = nullptr;
  if (!f32) {
    p.EDGE = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += align256(edge_floats * 4);
  }
  p.FLOWRAW = take(f32 ? 4 : cpr, p.g[0]);
  p.PART = nullptr;
  p.CNT = nullptr;
  p.RCORR = nullptr;
  p.RCNT = nullptr;
  p.rcorr_floats = p.rcnt_ints = 0;
  if (prec == RRIN_PREC_F32R) {
    // ring fold of the sub-pixel up conv into level L (runs on level L + 1's grid, 4 C_L
    // phase rows): 512 floats and one ticket per ring segment, co block and image
    for (int L = 0; L < kMaxDepth - 1; ++L) {
      const int64_t hl = h >> (L + 1), wl = w >> (L + 1);
      const int64_t segs = (int64_t)n * (4 * chans(L) / 32) * (2 * ((wl + 31) / 32) + 2 * ((hl + 7) / 8));
      p.rcnt_ints = segs > p.rcnt_ints ? segs : p.rcnt_ints;
    }
    p.rcorr_floats = 512 * p.rcnt_ints;
    p.RCORR = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += align256(p.rcorr_floats * 4);
    p.RCNT = base ? reinterpret_cast<int32_t*>(base + off) : nullptr;
    off += align256(p.rcnt_ints * 4);
  }
  p.part_floats = p.cnt_ints = 0;
  p.dry = nullptr;
  p.bytes = off;
}

inline int64_t scratch_tickets(int64_t cnt_ints) {
  return cnt_ints <= kScratchTickets ? kScratchTickets : (cnt_ints + 1023) / 1024 * 1024;
}

// The caller's scratch into the plan (F32R only; null / too small: no splits); `tickets` from
// scratch_tickets of the schedule's need.
void attach_scratch(Plan& p, void* scratch, int64_t bytes, int64_t tickets) {
  if (p.prec != RRIN_PREC_F32R || !scratch || bytes < tickets * 4) return;
  p.CNT = reinterpret_cast<int32_t*>(scratch);
  p.cnt_ints = tickets;
  p.PART = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + tickets * 4);
  p.part_floats = (bytes - tickets * 4) / 4;
}

// H8 view of channels [ch_off, ch_off+channels) of a buffer, at geometry g
// (g differs from b.g only for the level-shared UPT buffer).
rrin_h8 hview(const Buf& b, int ch_off, int channels, const rrin_geom& g) {
  rrin_h8 v;
  v.hi = b.base;
  v.lo = b.lo;
  v.img_stride = (int64_t)((b.ch + b.cpr - 1) / b.cpr) * g.plane;
  v.g_off = ch_off / b.cpr;
  v.groups = (channels + b.cpr - 1) / b.cpr;
  v.g = g;
  return v;
}
rrin_h8 hview(const Buf& b, int ch_off, int channels) { return hview(b, ch_off, channels, b.g); }

rrin_pp view(const Buf& b, int n, int ch_off, int channels) {
  rrin_pp v;
  v.base = b.base;
  v.img_stride = (int64_t)b.ch * b.g.plane;
  v.ch_off = ch_off;
  v.channels = channels;
  v.g = b.g;
  (void)n;
  return v;
}

// Bracket one launch with profiler events (no-op without a profiler).
struct ProfScope {
  rrin_prof* p;
  hipStream_t st;
  int slot;
  ProfScope(rrin_prof* p_, hipStream_t s, int kind, double flops) : p(p_), st(s), slot(-1) {
    if (p && p->count < (int)p->kind.size()) {
      slot = p->count++;
      p->kind[slot] = kind;
      p->flops[slot] = flops;
      if (p->chain && slot > 0 && p->last_st == st && p->last_slot == slot - 1) {
        p->start[slot] = 2 * (slot - 1) + 1;  // the previous launch's end on this stream
      } else {
        p->start[slot] = 2 * slot;
        (void)hipEventRecord(p->ev[2 * slot], st);
      }
    }
  }
  ~ProfScope() {
    if (slot >= 0) {
      (void)hipEventRecord(p->ev[2 * slot + 1], st);
      p->chain = true;
      p->last_st = st;
      p->last_slot = slot;
    }
  }
};

int conv(const Plan& p, const rrin_conv_weights& cw, int cin, int cout, int src_mode, int epi,
         const rrin_pp& src, const rrin_pp& dst, const rrin_pp* pool, hipStream_t st) {
  ProfScope ps(p.prof, st, RRIN_KIND_CONV, 2.0 * 9 * cin * cout * (double)dst.g.h * dst.g.w * p.n);
  rrin_conv_desc d;
  memset(&d, 0, sizeof(d));
  d.n = p.n;
  d.cin = cin;
  d.cout = cout;
  d.cfg = cw.cfg;
  d.src_mode = src_mode;
  d.epi_mode = epi;
  d.slope = 0.1f;
  d.src = src;
  d.dst = dst;
  if (pool) d.pool = *pool;
  d.wpack = cw.wpack;
  d.bias = cw.bias;
  return rrin_conv3x3_fwd(&d, st);
}

// Where a U-Net's head sends its results: per-image t coefficients and the
// Net output (Net glue modes), and the optional raw conv output (NCHW).
struct HeadIO {
  const float* coef;
  float* out;
  float* raw;
};

// Debug taps (rrin_net_desc.taps): where U-Net u's raw output goes, or NULL.
float* tap_of(const rrin_net_desc* nd, const UNetSpec& u) {
  if (!nd->taps) return nullptr;
  const int64_t px = (int64_t)nd->n * nd->h * nd->w;
  int64_t off = 0;
  for (const auto& v : kUNets) {
    if (&v == &u) return nd->taps + off;
    off += v.out_ch * px;
  }
  return nullptr;
}

#define RRIN_TRY(x)          \
  do {                       \
    int _rc = (x);           \
    if (_rc != 0) return _rc; \
  } while (0)

// One U-Net (unet.py:40-51) from g16 channels [0, in_ch) to its head.
int run_unet(const Plan& p, const UNetSpec& u, const rrin_conv_weights* cw, const rrin_head_weights& hw,
             const HeadIO& io, hipStream_t st) {
  const int D = u.depth;
  int k = 0;
  // ---- down path (unet.py:42-46)
  for (int L = 0; L < D; ++L) {
    const int C = chans(L);
    const rrin_pp in = L ? view(p.X[L], p.n, 0, chans(L - 1)) : view(p.G, p.n, 0, u.in_ch);
    const int cin = L ? chans(L - 1) : u.in_ch;
    const rrin_pp t = view(p.T[L], p.n, 0, C);
    RRIN_TRY(conv(p, cw[k++], cin, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, in, t, nullptr, st));
    if (L < D - 1) {
      const rrin_pp bridge = view(p.CAT[L], p.n, C, C);  // cat's second half (unet.py:93)
      const rrin_pp pooled = view(p.X[L + 1], p.n, 0, C);
      RRIN_TRY(conv(p, cw[k++], C, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY_POOL, t, bridge, &pooled, st));
    } else {
      const Buf& bot = (L == kMaxDepth - 1) ? p.BOT : p.CAT[L];  // CAT[3] is free at depth 4
      RRIN_TRY(conv(p, cw[k++], C, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, t, view(bot, p.n, 0, C), nullptr, st));
      // midconv + leaky (unet.py:47) back into T[bottom]
      RRIN_TRY(conv(p, cw[k++], C, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, view(bot, p.n, 0, C), t, nullptr, st));
    }
  }
  // ---- up path (unet.py:48-49, 72-95)
  rrin_pp x = view(p.T[D - 1], p.n, 0, chans(D - 1));
  for (int L = D - 2; L >= 0; --L) {
    const int C = chans(L);
    const rrin_pp up = view(p.CAT[L], p.n, 0, C);
    RRIN_TRY(conv(p, cw[k++], chans(L + 1), C, RRIN_SRC_UPSAMPLE2X, RRIN_EPI_LINEAR, x, up, nullptr, st));
    const rrin_pp cat = view(p.CAT[L], p.n, 0, 2 * C);
    const rrin_pp t = view(p.T[L], p.n, 0, C);
    RRIN_TRY(conv(p, cw[k++], 2 * C, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, cat, t, nullptr, st));
    RRIN_TRY(conv(p, cw[k++], C, C, RRIN_SRC_DIRECT, RRIN_EPI_LEAKY, t, up, nullptr, st));  // U_L
    x = up;
  }
  // ---- last conv fused with the Net glue (unet.py:51 + model.py)
  rrin_head_desc hd;
  memset(&hd, 0, sizeof(hd));
  hd.n = p.n;
  hd.cin = 32;
  hd.cout = u.out_ch;
  hd.mode = u.head_mode;
  hd.src = x;
  hd.g16 = view(p.G, p.n, 0, 16);
  hd.w = hw.w;
  hd.bias = hw.bias;
  hd.coef = io.coef;
  hd.out = io.out;
  hd.raw_out = io.raw;
  if (u.head_mode == RRIN_HEAD_FLOW) hd.flow_raw = view(p.FLOWRAW, p.n, 0, 4);
  ProfScope ps(p.prof, st, RRIN_KIND_HEAD, 2.0 * 9 * 32 * u.out_ch * (double)x.g.h * x.g.w * p.n);
  return rrin_head_fwd(&hd, st);
}

int conv_h8(const Plan& p, const rrin_conv_weights& cw, int cin, int cout, int epi, const rrin_h8& src,
            const rrin_h8& dst, const rrin_h8* pool, hipStream_t st, float* edge = nullptr, bool ring_fold = false,
            const rrin_edge_fix_desc* ring_full = nullptr) {
  // algorithmic FLOPs of the conv (a sub-pixel conv has 4 phase rows per real channel): 9
  // multiply-adds per output and input channel in the direct form, 4 in Winograd F(2x2,3x3)
  // (16 per 2x2 patch), 3 in F(4,3) x F(2,3) (kind 14: 24 per 4 x 2 patch)
  const int creal = epi == RRIN_EPI_SUBPIXEL ? cout / 4 : cout;
  const int wkind = rrin_conv_h8_cfg_wino(cw.cfg);
  const int macs = wkind == 14 ? 3 : wkind ? 4 : 9;
  ProfScope ps(p.prof, st, RRIN_KIND_CONV, 2.0 * macs * cin * creal * (double)dst.g.h * dst.g.w * p.n);
  rrin_conv_h8_desc d;
  memset(&d, 0, sizeof(d));
  d.n = p.n;
  d.cin = cin;
  d.cout = cout;
  d.cfg = cw.cfg;
  d.prec = p.prec;
  d.epi_mode = epi;
  d.slope = 0.1f;
  d.inv_wscale = cw.inv_wscale;
  d.tail_finite = 1;  // every src of the schedule: cin % 8 == 0, or g16 whose tail channels are finite
  d.src = src;
  d.dst = dst;
  if (pool) d.pool = *pool;
  d.whi = cw.whi;
  d.wlo = cw.wlo;
  d.bias = cw.bias;
  d.edge = edge;
  d.status = p.status;
  d.ring_full = ring_full;
  if (ring_fold) {
    d.ring_w = cw.wedge;
    d.ring_bias = cw.bias_raw;
    d.ring_corr = p.RCORR;
    d.ring_cnt = p.RCNT;
    int64_t cnt = 0;
    const int64_t need = rrin_conv_h8_ring_floats(&d, &cnt);
    if (need < 0) return (int)need;
    if (need > p.rcorr_floats || cnt > p.rcnt_ints) return RRIN_E_CONFIG;
  }
  if (cw.ksplit > 1 && p.prec == RRIN_PREC_F32R) {
    d.ksplit = cw.ksplit;
    d.part = p.PART;
    d.cnt = p.CNT;
    int64_t cnt = 0;
    const int64_t need = rrin_conv_h8_split_floats(&d, &cnt);
    if (need < 0) return (int)need;
    if (p.dry) {
      p.dry->add(need, cnt);
    } else if (!p.PART || need > p.part_floats || cnt > p.cnt_ints) {
      return RRIN_E_WORKSPACE;  // scratch smaller than rrin_net_scratch_bytes
    }
  }
  if (p.dry) return 0;
  return rrin_conv3x3_h8_fwd(&d, st);
}

// Fused level-0 UNetConvBlock (conv a = ca: cin -> 32, conv b = cb: 32 -> 32, + pool): one
// rrin_conv_block0_h8_fwd launch, bitwise the two conv_h8 calls it replaces
int block0_h8(const Plan& p, const rrin_conv_weights& ca, const rrin_conv_weights& cb, int cin, const rrin_h8& src,
              const rrin_h8& dst, const rrin_h8* pool, hipStream_t st) {
  ProfScope ps(p.prof, st, RRIN_KIND_CONV, 2.0 * 9 * (cin * 32 + 32 * 32) * (double)dst.g.h * dst.g.w * p.n);
  rrin_block0_h8_desc d;
  memset(&d, 0, sizeof(d));
  d.n = p.n;
  d.cin = cin;
  d.cfg_a = ca.cfg;
  d.cfg_b = cb.cfg;
  d.slope = 0.1f;
  d.inv_wscale_a = ca.inv_wscale;
  d.inv_wscale_b = cb.inv_wscale;
  d.tail_finite = 1;  // as conv_h8
  d.src = src;
  d.dst = dst;
  if (pool) d.pool = *pool;
  d.whi_a = ca.whi;
  d.bias_a = ca.bias;
  d.whi_b = cb.whi;
  d.bias_b = cb.bias;
  d.status = p.status;
  if (p.dry) return 0;
  return rrin_conv_block0_h8_fwd(&d, st);
}

// up.1 conv of the up block at level L on the sub-pixel path: low-res x (2C ch,
// edge-replicated) -> CAT[L][0, C), and the ring pixels: fp16 / split16 from scratch in the conv's
// own launch (ring_full), exact fp32 by the correction of the conv's pre-bias ring values (the
// outside taps of the zero-padded upsampled image) as a second launch on the same stream.  Round 5
// measured the ring from scratch beside the conv on a side stream and after it: both lost
// (DESIGN.md §5e).
int upconv_subpixel(const Plan& p, const rrin_conv_weights& cw, int C, const rrin_h8& x, const rrin_h8& up,
                    hipStream_t st) {
  if (cw.subpixel == 2) {  // ring folded into the conv (Winograd kind 3, no split)
    if (!p.RCORR || rrin_conv_h8_cfg_wino(cw.cfg) != 3 || cw.ksplit > 1) return RRIN_E_CONFIG;
    return conv_h8(p, cw, 2 * C, 4 * C, RRIN_EPI_SUBPIXEL, x, up, nullptr, st, p.EDGE, true);
  }
  rrin_edge_fix_desc e;
  memset(&e, 0, sizeof(e));
  e.n = p.n;
  e.cin = 2 * C;
  e.cout = C;
  e.prec = p.prec;
  e.epi_mode = RRIN_EPI_LINEAR;
  e.src = x;
  e.dst = up;
  e.edge = p.EDGE;
  e.wedge = cw.wedge;
  e.bias = cw.bias_raw;
  e.status = p.status;
  e.full = 0;
#ifndef RRIN_SKIP_RING_FIX
  if (kRingInLaunch && p.prec != RRIN_PREC_F32R && (2 * C) % kFixCi == 0) {
    // the ring from scratch (ABI 17 ring_full): where the tile allows, extra workgroups of the
    // conv's own launch -- no separate fix-up launch and no dependency step on this stream (C3:
    // the separate fix-ups cost ~3.5 %, profiles/r06/ring/)
    e.full = 1;
    return conv_h8(p, cw, 2 * C, 4 * C, RRIN_EPI_SUBPIXEL, x, up, nullptr, st, p.EDGE, false, &e);
  }
#endif
  RRIN_TRY(conv_h8(p, cw, 2 * C, 4 * C, RRIN_EPI_SUBPIXEL, x, up, nullptr, st, p.EDGE));
#ifdef RRIN_SKIP_RING_FIX  // ablation build only (the ring pixels stay wrong): the fix-ups' cost bound
  return 0;
#endif
  // F32R plans: the cross-workgroup K split (the same result bit for bit) where the
  // split grid is at most one workgroup per CU -- the latency-bound small grids
  // (640x368 x 1: fix-up 195 -> 129 us per forward); larger grids keep one
  // workgroup per tile, whose extra workgroups only queue behind the other
  // stream's convs (720p x 4 on 2 streams: fix-up span 1.4 -> 3.5 ms per step).
  if (p.prec == RRIN_PREC_F32R) {
    int64_t tk = 0;
    const int64_t nf = rrin_edge_fix_split_floats(&e, &tk);
    if (nf > 0 && nf / 1024 <= kEdgeCrossMaxGroups) {
      if (p.dry) {
        p.dry->add(nf, tk);
      } else if (p.PART && nf <= p.part_floats && tk <= p.cnt_ints) {
        e.part = p.PART;
        e.cnt = p.CNT;
        e.part_floats = p.part_floats;
        e.cnt_len = (int32_t)p.cnt_ints;
      }
    }
  }
  if (p.dry) return 0;
  ProfScope ps(p.prof, st, RRIN_KIND_EDGE, 0.0);
  return rrin_subpixel_edge_fix_h8(&e, st);
}

// conv cw (a level-0 conv a) runs fused with the next conv: fp16, asked for by the table
static bool fused_block0(const Plan& p, const rrin_conv_weights& cw) {
  return p.prec == RRIN_PREC_F16 && cw.fuse_next == 1;
}

// One U-Net on the split-fp16 path: same dataflow as run_unet.  An up conv
// either has sub-pixel weights (upsample folded into the conv; its producer then
// writes the low-res tensor into LRB with edge-replicate padding) or runs after
// an explicit upsample pass into UPT.
int run_unet_h8(const Plan& p, const UNetSpec& u, const rrin_conv_weights* cw, const rrin_head_weights& hw,
                const HeadIO& io, hipStream_t st) {
  const int D = u.depth;
  int k = 0;
  rrin_h8 x;
  for (int L = 0; L < D; ++L) {
    const int C = chans(L);
    const int cin = L ? chans(L - 1) : u.in_ch;
    // level 0 views all 16 staged channels of G (zero past in_ch): Winograd tiles read whole chunks
    const rrin_h8 in = L ? hview(p.X[L], 0, cin) : hview(p.G, 0, 16);
    const rrin_h8 t = hview(p.T[L], 0, C);
    if (L == 0 && D >= 2 && fused_block0(p, cw[k])) {  // down_path[0] in one launch
      const rrin_h8 bridge = hview(p.CAT[0], C, C);
      const rrin_h8 pooled = hview(p.X[1], 0, C);
      RRIN_TRY(block0_h8(p, cw[k], cw[k + 1], cin, in, bridge, &pooled, st));
      k += 2;
      continue;
    }
    RRIN_TRY(conv_h8(p, cw[k++], cin, C, RRIN_EPI_LEAKY, in, t, nullptr, st));
    if (L < D - 1) {
      const rrin_h8 bridge = hview(p.CAT[L], C, C);
      const rrin_h8 pooled = hview(p.X[L + 1], 0, C);
      RRIN_TRY(conv_h8(p, cw[k++], C, C, RRIN_EPI_LEAKY_POOL, t, bridge, &pooled, st));
    } else {
      const Buf& bot = (L == kMaxDepth - 1) ? p.BOT : p.CAT[L];
      RRIN_TRY(conv_h8(p, cw[k++], C, C, RRIN_EPI_LEAKY, t, hview(bot, 0, C), nullptr, st));
      // midconv; cw[k + 1] is the first up conv
      const bool sub = D >= 2 && cw[k + 1].subpixel;
      x = sub ? hview(p.LRB[L], 0, C) : t;
      RRIN_TRY(conv_h8(p, cw[k++], C, C, sub ? RRIN_EPI_LEAKY_REP : RRIN_EPI_LEAKY, hview(bot, 0, C), x, nullptr,
                       st));
    }
  }
  for (int L = D - 2; L >= 0; --L) {
    const int C = chans(L);
    const rrin_h8 up = hview(p.CAT[L], 0, C);
    const rrin_conv_weights& cu = cw[k++];
    if (cu.subpixel) {
      RRIN_TRY(upconv_subpixel(p, cu, C, x, up, st));
    } else {
      const rrin_h8 upin = hview(p.UPT[L], 0, 2 * C);
      if (!p.dry) {
        ProfScope ps(p.prof, st, RRIN_KIND_LAYOUT, 0.0);
        RRIN_TRY(rrin_upsample2x_h8(&x, &upin, p.n, p.prec, st));
      }
      RRIN_TRY(conv_h8(p, cu, 2 * C, C, RRIN_EPI_LINEAR, upin, up, nullptr, st));
    }
    const rrin_h8 cat = hview(p.CAT[L], 0, 2 * C);
    const rrin_h8 t = hview(p.T[L], 0, C);
    if (L == 0 && fused_block0(p, cw[k])) {  // the last up block's conv_block in one launch: its
      // output goes to T[0] (the launch reads all of CAT[0] while it writes)
      RRIN_TRY(block0_h8(p, cw[k], cw[k + 1], 2 * C, cat, t, nullptr, st));
      k += 2;
      x = t;
      continue;
    }
    RRIN_TRY(conv_h8(p, cw[k++], 2 * C, C, RRIN_EPI_LEAKY, cat, t, nullptr, st));
    // conv b; cw[k + 1] is the next level's up conv
    const bool sub = L > 0 && cw[k + 1].subpixel;
    const rrin_h8 out = sub ? hview(p.LRB[L], 0, C) : up;
    RRIN_TRY(conv_h8(p, cw[k++], C, C, sub ? RRIN_EPI_LEAKY_REP : RRIN_EPI_LEAKY, t, out, nullptr, st));
    x = out;
  }
  rrin_head_h8_desc hd;
  memset(&hd, 0, sizeof(hd));
  hd.n = p.n;
  hd.cin = 32;
  hd.cout = u.out_ch;
  hd.mode = u.head_mode;
  hd.prec = p.prec;
  hd.src = x;
  hd.g16 = hview(p.G, 0, 16);
  hd.w = hw.w;
  hd.bias = hw.bias;
  hd.coef = io.coef;
  hd.out = io.out;
  hd.raw_out = io.raw;
  hd.status = p.status;
  if (u.head_mode == RRIN_HEAD_FLOW) hd.flow_raw = hview(p.FLOWRAW, 0, 4);
  if (p.dry) return 0;
  ProfScope ps(p.prof, st, RRIN_KIND_HEAD, 2.0 * 9 * 32 * u.out_ch * (double)x.g.h * x.g.w * p.n);
  return rrin_head_h8_fwd(&hd, st);
}

}  // namespace

extern "C" int rrin_make_geom(int32_t h, int32_t w, rrin_geom* g) {
  if (!g || h < 1 || w < 1) return RRIN_E_ARG;
  *g = make_geom(h, w);
  return 0;
}

extern "C" int rrin_net_conv_count(void) {
  int c = 0;
  for (const auto& u : kUNets) c += convs_of(u.depth);
  return c;
}

extern "C" int64_t rrin_net_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t prec) {
  if (n < 1 || h < 16 || w < 16 || (h % 16) || (w % 16)) return RRIN_E_SHAPE;
  if (prec < RRIN_PREC_F32 || prec > RRIN_PREC_F32R) return RRIN_E_ARG;
  Plan p;
  make_plan(n, h, w, prec, nullptr, p);
  return p.bytes;
}

// Scratch the schedule of d needs (F32R: the split convs' slabs and tickets, the ring
// fix-up's cross-workgroup K split; other precisions 0): the schedule walked with every
// launch skipped.
static int scratch_need_of(int n, int h, int w, int prec, const rrin_conv_weights* convs, const UNetSpec* us, int nu,
                           ScratchNeed& need) {
  Plan p;
  // a stand-in base so the views pass the descriptor checks; never dereferenced
  make_plan(n, h, w, prec, reinterpret_cast<char*>((uintptr_t)1 << 30), p);
  p.dry = &need;
  const rrin_head_weights hw{};
  int k = 0;
  for (int u = 0; u < nu; ++u) {
    RRIN_TRY(run_unet_h8(p, us[u], convs + k, hw, HeadIO{nullptr, nullptr, nullptr}, nullptr));
    k += convs_of(us[u].depth);
  }
  return 0;
}

static int64_t scratch_bytes_of(int n, int h, int w, int prec, const rrin_conv_weights* convs, const UNetSpec* us,
                                int nu) {
  if (prec != RRIN_PREC_F32R) return 0;
  ScratchNeed need;
  RRIN_TRY(scratch_need_of(n, h, w, prec, convs, us, nu, need));
  if (need.part_floats == 0 && need.cnt_ints == 0) return 0;
  return scratch_tickets(need.cnt_ints) * 4 + need.part_floats * 4;
}

// The ticket count of the caller's scratch for this schedule (the layout scratch_bytes_of sized)
static int64_t scratch_tickets_of(int n, int h, int w, int prec, const rrin_conv_weights* convs, const UNetSpec* us,
                                  int nu, const void* scratch) {
  if (prec != RRIN_PREC_F32R || !scratch) return kScratchTickets;
  ScratchNeed need;
  if (scratch_need_of(n, h, w, prec, convs, us, nu, need)) return kScratchTickets;
  return scratch_tickets(need.cnt_ints);
}

extern "C" int64_t rrin_net_scratch_bytes(const rrin_net_desc* d) {
  if (!d || !d->convs) return RRIN_E_ARG;
  if (d->n < 1 || d->h < 16 || d->w < 16 || (d->h % 16) || (d->w % 16)) return RRIN_E_SHAPE;
  if (d->prec < RRIN_PREC_F32 || d->prec > RRIN_PREC_F32R) return RRIN_E_ARG;
  return scratch_bytes_of(d->n, d->h, d->w, d->prec, d->convs, kUNets, 4);
}

extern "C" int rrin_net_fwd(const rrin_net_desc* d, void* stream) {
  if (!d || !d->i0 || !d->i1 || !d->out || !d->coef || !d->convs || !d->heads || !d->workspace)
    return RRIN_E_ARG;
  if (d->n < 1 || d->h < 16 || d->w < 16 || (d->h % 16) || (d->w % 16)) return RRIN_E_SHAPE;
  if (d->prec < RRIN_PREC_F32 || d->prec > RRIN_PREC_F32R) return RRIN_E_ARG;
  Plan p;
  make_plan(d->n, d->h, d->w, d->prec, reinterpret_cast<char*>(d->workspace), p);
  if (d->workspace_bytes < p.bytes) return RRIN_E_WORKSPACE;
  attach_scratch(p, d->scratch, d->scratch_bytes,
                 scratch_tickets_of(d->n, d->h, d->w, d->prec, d->convs, kUNets, 4, d->scratch));
  p.prof = d->prof;  // per call: concurrent calls never share launch state
  if (p.prof) p.prof->chain = false;  // the call's first launch records its own start
  hipStream_t st = (hipStream_t)stream;
  if (d->status && (d->prec == RRIN_PREC_F16X3 || d->prec == RRIN_PREC_F16)) {
    p.status = d->status;
    if (hipError_t e = hipMemsetAsync(d->status, 0, sizeof(int32_t), st)) return (int)e;
  }
  if (d->prec != RRIN_PREC_F32) {
    const rrin_h8 gall = hview(p.G, 0, 16);
    int rc = 0;
    {
      ProfScope ps(p.prof, st, RRIN_KIND_LAYOUT, 0.0);
      // x0, x1 into channels 0-5; channels 6-15 zeroed, so the first convs (cin 6/9/10)
      // can stage whole records (their tail channels are finite and meet zero weights)
      rc = rrin_pack_g16_h8(d->i0, d->i1, d->n, &gall, d->prec, st);
      if (!rc && d->skip_flow) {
        const rrin_h8 fr = hview(p.FLOWRAW, 0, 4);
        rc = rrin_flow_tblend_h8(&fr, &gall, d->coef, d->n, d->prec, st);
      }
    }
    int k = 0;
    for (int u = 0; u < 4 && !rc; ++u) {
      if (!(u == 0 && d->skip_flow))
        rc = run_unet_h8(p, kUNets[u], d->convs + k, d->heads[u], HeadIO{d->coef, d->out, tap_of(d, kUNets[u])}, st);
      k += convs_of(kUNets[u].depth);
    }
    return rc;
  }

  // x = cat(x0, x1) into g16 channels 0-5 (model.py:33)
  const rrin_pp gx0 = view(p.G, p.n, 0, 3);
  const rrin_pp gx1 = view(p.G, p.n, 3, 3);
  int rc = 0;
  {
    ProfScope ps(p.prof, st, RRIN_KIND_LAYOUT, 0.0);
    rc = rrin_nchw_to_pp(d->i0, d->n, 3, &gx0, st);
    if (!rc) rc = rrin_nchw_to_pp(d->i1, d->n, 3, &gx1, st);
    if (!rc && d->skip_flow) {  // Flow U-Net skipped: t-blend of the kept raw Flow
      const rrin_pp fr = view(p.FLOWRAW, p.n, 0, 4);
      const rrin_pp g16 = view(p.G, p.n, 0, 16);
      rc = rrin_flow_tblend_fwd(&fr, &g16, d->coef, d->n, st);
    }
  }
  int k = 0;
  for (int u = 0; u < 4 && !rc; ++u) {
    if (!(u == 0 && d->skip_flow))
      rc = run_unet(p, kUNets[u], d->convs + k, d->heads[u], HeadIO{d->coef, d->out, tap_of(d, kUNets[u])}, st);
    k += convs_of(kUNets[u].depth);
  }
  return rc;
}

// One U-Net alone (reference UNet.forward, unet.py:40-51): NCHW in -> NCHW out,
// the same kernels and workspace plan as the Net (input in the Net buffer's
// channels [0, in_ch), head in PLAIN mode with its raw NCHW output as y).
extern "C" int64_t rrin_unet_conv_count(int32_t depth) {
  return (depth < 2 || depth > kMaxDepth) ? RRIN_E_ARG : convs_of(depth);
}

extern "C" int64_t rrin_unet_scratch_bytes(const rrin_unet_desc* d) {
  if (!d || !d->convs) return RRIN_E_ARG;
  if (d->n < 1 || d->h < 16 || d->w < 16 || (d->h % 16) || (d->w % 16)) return RRIN_E_SHAPE;
  if (d->in_ch < 1 || d->in_ch > 16 || d->out_ch < 2 || d->out_ch > 4 || d->depth < 2 || d->depth > kMaxDepth)
    return RRIN_E_ARG;
  if (d->prec < RRIN_PREC_F32 || d->prec > RRIN_PREC_F32R) return RRIN_E_ARG;
  const UNetSpec u{d->in_ch, d->out_ch, d->depth, RRIN_HEAD_PLAIN};
  return scratch_bytes_of(d->n, d->h, d->w, d->prec, d->convs, &u, 1);
}

extern "C" int rrin_unet_fwd(const rrin_unet_desc* d, void* stream) {
  if (!d || !d->x || !d->y || !d->convs || !d->head.w || !d->head.bias || !d->workspace) return RRIN_E_ARG;
  if (d->n < 1 || d->h < 16 || d->w < 16 || (d->h % 16) || (d->w % 16)) return RRIN_E_SHAPE;
  if (d->in_ch < 1 || d->in_ch > 16 || d->out_ch < 2 || d->out_ch > 4 || d->depth < 2 || d->depth > kMaxDepth)
    return RRIN_E_ARG;
  if (d->prec < RRIN_PREC_F32 || d->prec > RRIN_PREC_F32R) return RRIN_E_ARG;
  Plan p;
  make_plan(d->n, d->h, d->w, d->prec, reinterpret_cast<char*>(d->workspace), p);
  if (d->workspace_bytes < p.bytes) return RRIN_E_WORKSPACE;
  {
    const UNetSpec u{d->in_ch, d->out_ch, d->depth, RRIN_HEAD_PLAIN};
    attach_scratch(p, d->scratch, d->scratch_bytes,
                   scratch_tickets_of(d->n, d->h, d->w, d->prec, d->convs, &u, 1, d->scratch));
  }
  p.prof = d->prof;
  if (p.prof) p.prof->chain = false;
  hipStream_t st = (hipStream_t)stream;
  if (d->status && (d->prec == RRIN_PREC_F16X3 || d->prec == RRIN_PREC_F16)) {
    p.status = d->status;  // fp16 range guard, as rrin_net_fwd
    if (hipError_t e = hipMemsetAsync(d->status, 0, sizeof(int32_t), st)) return (int)e;
  }
  const UNetSpec u{d->in_ch, d->out_ch, d->depth, RRIN_HEAD_PLAIN};
  const HeadIO io{nullptr, nullptr, d->y};
  int rc;
  {
    ProfScope ps(p.prof, st, RRIN_KIND_LAYOUT, 0.0);
    if (d->prec == RRIN_PREC_F32) {
      const rrin_pp gx = view(p.G, p.n, 0, d->in_ch);
      rc = rrin_nchw_to_pp(d->x, d->n, d->in_ch, &gx, st);
    } else {
      const rrin_h8 gx = hview(p.G, 0, 16);
      rc = rrin_nchw_to_h8(d->x, d->n, d->in_ch, 0, &gx, d->prec, st);
      // the PLAIN head writes its out_ch channels into this buffer: past in_ch
      // they would be staged (against zero weights) by the next call's first conv
      if (!rc && d->out_ch > d->in_ch) rc = clear_channels_h8(&gx, d->n, d->in_ch, d->out_ch, d->prec, st);
    }
  }
  if (rc) return rc;
  return d->prec == RRIN_PREC_F32 ? run_unet(p, u, d->convs, d->head, io, st)
                                  : run_unet_h8(p, u, d->convs, d->head, io, st);
}

extern "C" int rrin_prof_create(int32_t capacity, rrin_prof** out) {
  if (!out || capacity < 1) return RRIN_E_ARG;
  rrin_prof* p = new rrin_prof();
  p->ev.resize(2 * (size_t)capacity);
  p->start.resize(capacity);
  p->kind.resize(capacity);
  p->flops.resize(capacity);
  // timing-only events: no system-scope fence (a default event record writes
  // back and invalidates the caches, which the next launch then pays for)
  for (auto& e : p->ev) {
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (r != hipSuccess) {
      delete p;
      return (int)r;
    }
  }
  *out = p;
  return 0;
}

extern "C" int rrin_prof_destroy(rrin_prof* p) {
  if (!p) return RRIN_E_ARG;
  for (auto& e : p->ev)
    if (e) (void)hipEventDestroy(e);
  delete p;
  return 0;
}

extern "C" int rrin_prof_reset(rrin_prof* p) {
  if (!p) return RRIN_E_ARG;
  p->count = 0;
  p->chain = false;
  return 0;
}

extern "C" int rrin_prof_read(rrin_prof* p, int32_t* kinds, float* ms, double* flops, int32_t cap,
                              int32_t* count) {
  if (!p || !count) return RRIN_E_ARG;
  const int n = p->count < cap ? p->count : cap;
  for (int i = 0; i < n; ++i) {
    if (kinds) kinds[i] = p->kind[i];
    if (flops) flops[i] = p->flops[i];
    if (ms) {
      hipError_t r = hipEventElapsedTime(&ms[i], p->ev[p->start[i]], p->ev[2 * i + 1]);
      if (r != hipSuccess) return (int)r;
    }
  }
  *count = n;
  return 0;
}

extern "C" int rrin_prof_read_spans(rrin_prof* p, float* t0_ms, float* t1_ms, int32_t cap, int32_t* count) {
  if (!p || !count || !t0_ms || !t1_ms) return RRIN_E_ARG;
  const int n = p->count < cap ? p->count : cap;
  for (int i = 0; i < n; ++i) {
    hipError_t r = hipEventElapsedTime(&t0_ms[i], p->ev[0], p->ev[p->start[i]]);
    if (r == hipSuccess) r = hipEventElapsedTime(&t1_ms[i], p->ev[0], p->ev[2 * i + 1]);
    if (r != hipSuccess) return (int)r;
  }
  *count = n;
  return 0;
}

// ---- weight packing (host) ------------------------------------------------
// wpack[cob][chunk][ci8][tap][bm]: the slab a block stages per K chunk is
// contiguous; zero rows/cols pad cin to 8 and cout to bm.
extern "C" int64_t rrin_pack_conv3x3_floats(int32_t cout, int32_t cin, int32_t bm) {
  if (cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  const int64_t cob = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  return cob * nch * 8 * 9 * bm;
}

extern "C" int64_t rrin_pack_bias_floats(int32_t cout, int32_t bm) {
  if (cout < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  return (int64_t)((cout + bm - 1) / bm) * bm;
}

extern "C" int rrin_pack_conv3x3(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                                 const int32_t* perm, float* wpack, float* bpack) {
  if (!w || !b || !wpack || !bpack || cout < 1 || cin < 1 || bm < 32 || bm % 32) return RRIN_E_ARG;
  if (perm)
    for (int c = 0; c < cin; ++c)
      if (perm[c] < 0 || perm[c] >= cin) return RRIN_E_ARG;
  const int cob_n = (cout + bm - 1) / bm, nch = (cin + 7) / 8;
  int64_t o = 0;
  for (int cob = 0; cob < cob_n; ++cob)
    for (int c = 0; c < nch; ++c)
      for (int ci = 0; ci < 8; ++ci)
        for (int tap = 0; tap < 9; ++tap)
          for (int col = 0; col < bm; ++col) {
            const int co = cob * bm + col, ch = c * 8 + ci;
            float v = 0.f;
            if (co < cout && ch < cin) {
              const int src_ch = perm ? perm[ch] : ch;
              v = w[((int64_t)co * cin + src_ch) * 9 + tap];
            }
            wpack[o++] = v;
          }
  for (int co = 0; co < cob_n * bm; ++co) bpack[co] = co < cout ? b[co] : 0.f;
  return 0;
}

extern "C" int rrin_abi_version(void) { return RRIN_ABI_VERSION; }

extern "C" const char* rrin_strerror(int code) {
  switch (code) {
    case RRIN_OK:
      return "ok";
    case RRIN_E_SHAPE:
      return "rrin: shape precondition violated (H, W must be multiples of 16; N >= 1; views must match)";
    case RRIN_E_ARG:
      return "rrin: invalid argument (null pointer, mode or channel range)";
    case RRIN_E_WORKSPACE:
      return "rrin: workspace smaller than rrin_net_workspace_bytes() (or scratch smaller than "
             "rrin_net_scratch_bytes())";
    case RRIN_E_CONFIG:
      return "rrin: unknown conv tile config";
  }
  if (code > 0) return hipGetErrorString((hipError_t)code);
  return "rrin: unknown error";
}
