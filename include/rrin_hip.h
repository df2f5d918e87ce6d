/*
 * rrin_hip.h — C ABI of librrin_hip.so, the MI355X (gfx950) kernels of the
 * RRIN inference hot path (reference `Net.forward`, /root/reference/model.py:59-65).
 *
 * Rules of the boundary:
 *   - plain C types only: device pointers, sizes, a hipStream_t passed as void*;
 *   - no allocation inside the library: every buffer (activations, workspace,
 *     packed weights) is owned by the caller (the Python host layer uses the
 *     PyTorch caching allocator);
 *   - every entry returns int: 0 = ok, > 0 = a hipError_t, < 0 = RRIN_E_* for a
 *     violated shape/argument precondition; rrin_strerror() decodes it;
 *   - stateless and stream-ordered: calls only enqueue work on `stream`; no
 *     call's result depends on another call.  Everything a call needs comes in
 *     its arguments (the optional launch profiler of rrin_net_fwd included);
 *     the only process-wide data are thread-safe launch caches keyed by the
 *     device of the stream a launch goes to (a kernel's dynamic-LDS attribute,
 *     resident blocks per CU), so a caller may pass any device's stream from any
 *     host thread.  One rrin_prof must not be shared by concurrent calls.
 *
 * Activation layouts between kernels:
 *   - record layout (the default, every `prec` but RRIN_PREC_F32): per image
 *     and channel group one plane of 16-byte records, hp = round_up(h,16)+2
 *     rows, wp = round_up(w,32)+16 records, pixel (y,x) at record
 *     (y+1)*wp + (x+8).  A record holds 4 fp32 channels (RRIN_PREC_F32R, exact
 *     fp32: "R32") or 8 halves (RRIN_PREC_F16X3 hi / lo planes, RRIN_PREC_F16:
 *     "H8").  rrin_geom / rrin_make_geom_h8 / rrin_h8 describe it.
 *   - padded planar ("PP", RRIN_PREC_F32 only: the round-1 fp32 path kept for
 *     A/B): per image and channel a plane of hp x wp fp32 with
 *     wp = round_up(w,32)+64, pixel (y,x) at (y+1)*wp + (x+32).
 * Padding is zero and is never written (it is the convs' zero padding).
 */
#ifndef RRIN_HIP_H
#define RRIN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RRIN_ABI_VERSION 19

#define RRIN_OK 0
#define RRIN_E_SHAPE (-1)     /* H or W not a multiple of 16, or N < 1          */
#define RRIN_E_ARG (-2)       /* null pointer / bad enum / channel range         */
#define RRIN_E_WORKSPACE (-3) /* workspace smaller than rrin_net_workspace_bytes */
#define RRIN_E_CONFIG (-4)    /* no kernel instance for the requested tile cfg   */

/* ---- Planar geometry --------------------------------------------------- */
typedef struct rrin_geom {
  int32_t h, w;      /* logical size                       */
  int32_t hp, wp;    /* padded plane size (see header)      */
  int64_t plane;     /* hp*wp (floats)                      */
} rrin_geom;

/* Fill a geometry for an h x w level. */
int rrin_make_geom(int32_t h, int32_t w, rrin_geom* g);

/* A PP tensor view: base points at channel 0 of image 0. */
typedef struct rrin_pp {
  float* base;
  int64_t img_stride; /* floats between images   */
  int32_t ch_off;     /* first channel of the view */
  int32_t channels;   /* channels in the view     */
  rrin_geom g;
} rrin_pp;

/* ---- Conv 3x3 (MFMA, exact fp32) ---------------------------------------- */
/* Replaces nn.Conv2d(k=3,pad=1)+bias (unet.py:29,59,62,78), LeakyReLU(0.1)
 * (unet.py:47,60,63), F.avg_pool2d(x,2) (unet.py:46, fused as a second output),
 * nn.Upsample(bilinear,x2) (unet.py:77, fused into the input staging) and
 * torch.cat(up,bridge) (unet.py:93, by channel-offset addressing). */
enum rrin_src_mode { RRIN_SRC_DIRECT = 0, RRIN_SRC_UPSAMPLE2X = 1 };
enum rrin_epi_mode {
  RRIN_EPI_LINEAR = 0,
  RRIN_EPI_LEAKY = 1,
  RRIN_EPI_LEAKY_POOL = 2,
  /* H8 only.  LEAKY_REP: leaky, and the image border is also written into the
   * 1-pixel padding ring (edge replicate) -- for a tensor whose only reader is
   * a sub-pixel up conv.  SUBPIXEL: the conv is the phase-combined form of
   * conv3x3(upsample_x2(src)) (rrin_subpixel_weights, cout = 4 x real cout):
   * linear, outputs pixel-shuffled into dst (2x the size of src); the outermost
   * ring of dst is not written but its pre-bias value goes to `edge` for
   * rrin_subpixel_edge_fix_h8. */
  RRIN_EPI_LEAKY_REP = 3,
  RRIN_EPI_SUBPIXEL = 4
};

typedef struct rrin_conv_desc {
  int32_t n;            /* images                                              */
  int32_t cin, cout;    /* real channel counts                                  */
  int32_t cfg;          /* tile config id (rrin_conv_cfg_bm); pack with same bm */
  int32_t src_mode;     /* rrin_src_mode; UPSAMPLE2X: src is at (h/2, w/2)      */
  int32_t epi_mode;     /* rrin_epi_mode                                        */
  float slope;          /* leaky slope (0.1)                                    */
  rrin_pp src;          /* input view (cin channels from src.ch_off)           */
  rrin_pp dst;          /* output view (cout channels from dst.ch_off), h x w  */
  rrin_pp pool;         /* EPI_LEAKY_POOL: pooled output (h/2 x w/2)           */
  const float* wpack;   /* rrin_pack_conv3x3 output for this cfg              */
  const float* bias;    /* padded bias (rrin_pack_conv3x3 output)              */
} rrin_conv_desc;

int rrin_conv_cfg_count(void);
int rrin_conv_cfg_bm(int32_t cfg);          /* output-channel tile of a config  */
int rrin_conv_cfg_th(int32_t cfg);          /* output-row tile of a config       */
int rrin_conv3x3_fwd(const rrin_conv_desc* d, void* stream);

/* Host-side weight packing (CPU memory).  w: OIHW [cout][cin][3][3] fp32,
 * b: [cout].  perm (nullable): packed input channel c reads reference channel
 * perm[c].  Output sizes from rrin_pack_conv3x3_floats(). */
int64_t rrin_pack_conv3x3_floats(int32_t cout, int32_t cin, int32_t bm);
int64_t rrin_pack_bias_floats(int32_t cout, int32_t bm);
int rrin_pack_conv3x3(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                      const int32_t* perm, float* wpack, float* bpack);

/* ---- Head convs (Cout <= 4) with the fused Net glue ---------------------- */
/* One VALU conv3x3 32->{4,4,2,3} fused with the model.py glue that consumes it:
 *   FLOW   (Flow.last)        : t-blend of flows, model.py:37-39
 *   REFINE (refine_flow.last) : flow residual + two backwarps, model.py:44-48,8-21
 *   MASK   (Mask.last)        : sigmoid + weighted blend, model.py:52-55
 *   FINAL  (final.last)       : residual add + clamp to the NCHW output, model.py:62-63
 * g16 is the 16-channel Net buffer [x0(3) x1(3) Ft0(2) Ft1(2) xt1(3) xt2(3)]. */
enum rrin_head_mode { RRIN_HEAD_PLAIN = 0, RRIN_HEAD_FLOW = 1, RRIN_HEAD_REFINE = 2,
                      RRIN_HEAD_MASK = 3, RRIN_HEAD_FINAL = 4 };

typedef struct rrin_head_desc {
  int32_t n, cin, cout, mode;
  rrin_pp src;           /* cin-channel PP input                              */
  rrin_pp g16;           /* Net buffer (modes FLOW..FINAL); PLAIN: dst view    */
  const float* w;        /* OIHW [cout][cin][3][3] (unpacked)                 */
  const float* bias;     /* [cout]                                            */
  const float* coef;     /* [n][8] per-image t coefficients   */
  float* out;            /* FINAL: NCHW [n][3][h][w] contiguous               */
  rrin_pp flow_raw;      /* FLOW (optional, base NULL = skip): raw 4-ch Flow output kept
                            for reuse across t                    */
  float* raw_out;        /* optional (NULL = off): the head conv's output before any glue,
                            NCHW [n][cout][h][w] fp32 (intermediate-tap parity tests) */
} rrin_head_desc;

int rrin_head_fwd(const rrin_head_desc* d, void* stream);

/* ---- Layout kernels ------------------------------------------------------- */
/* NCHW contiguous [n][c][h][w] <-> PP view (c channels at dst.ch_off). */
int rrin_nchw_to_pp(const float* src, int32_t n, int32_t c, const rrin_pp* dst, void* stream);
int rrin_pp_to_nchw(const rrin_pp* src, int32_t n, int32_t c, float* dst, void* stream);

/* Standalone backwarp (model.py:8-21): out = grid_sample(img, grid(flow)),
 * NCHW contiguous fp32; same device code as the fused REFINE head. */
int rrin_warp_fwd(const float* img, const float* flow, float* out, int32_t n, int32_t c,
                  int32_t h, int32_t w, void* stream);

/* ---- Record-layout paths ("H8" family: 16-byte channel records) ---------- */
/* Precision of a forward / conv:
 *   F32   exact fp32 (v_mfma_f32_32x32x2_f32), PP layout above (planar, legacy);
 *   F32R  exact fp32 (v_mfma_f32_32x32x2_f32, fp32 storage) on the record layout
 *         below with 4 fp32 channels per 16-byte record ("R32"); the kernels,
 *         schedules and fusions of the fp16 paths (persistent grids, sub-pixel
 *         up convs, fused heads) -- the default fp32 path;
 *   F16X3 every fp32 value v is held as hi = f16(v), lo = f16((v - hi) * 2^11)
 *         (v = hi + lo 2^-11 to ~2^-22 |v|; lo stays normal) and every product as
 *         hi*hi + 2^-11 (hi*lo + lo*hi) in v_mfma_f32_32x32x16_f16 with fp32
 *         accumulation: fp32-class accuracy at ~5x the fp32 MFMA rate;
 *   F16   hi only (fp16 storage, fp16 products, fp32 accumulation) for the
 *         fp16 configs of BASELINE.json.
 * H8 layout: per image, per group of 8 channels, an hp x wp plane of 16-byte
 * records (8 halfs, channel-innermost); hp = round_up(h,16)+2,
 * wp = round_up(w,32)+16 records, pixel (y,x) at record (y+1)*wp + x+8.
 * F16X3 keeps two such tensors (hi, lo) with identical geometry. */
enum rrin_prec { RRIN_PREC_F32 = 0, RRIN_PREC_F16X3 = 1, RRIN_PREC_F16 = 2, RRIN_PREC_F32R = 3 };
/* In the record layout a "group" is the channels of one record: 8 (F16X3, F16)
 * or 4 (F32R); g_off / groups of an rrin_h8 view count such groups, and the
 * rrin_*_h8 entry points below accept F32R wherever they take a prec. */

int rrin_make_geom_h8(int32_t h, int32_t w, rrin_geom* g); /* plane in records */

typedef struct rrin_h8 {
  void* hi;           /* records (16 B), group 0 of image 0 of the tensor */
  void* lo;           /* same geometry; NULL for F16                     */
  int64_t img_stride; /* records between images                          */
  int32_t g_off;      /* first 8-channel group of the view               */
  int32_t groups;     /* groups in the view                              */
  rrin_geom g;
} rrin_h8;

typedef struct rrin_conv_h8_desc {
  int32_t n, cin, cout, cfg;   /* cfg: rrin_conv_h8_cfg_* */
  int32_t prec;                /* F16X3 or F16 */
  int32_t epi_mode;            /* rrin_epi_mode */
  float slope;
  float inv_wscale;            /* from rrin_pack_conv3x3_h8: weights were scaled by 1/inv_wscale */
  int32_t tail_finite;         /* 1: the channels [cin, 8*ceil(cin/8)) of src are finite (they meet
                                  zero weights), so the LDS-DMA kernel may stage whole records;
                                  0: cin % 8 != 0 uses the masking register-staged kernel */
  int32_t pad_;
  rrin_h8 src, dst, pool;      /* pool: EPI_LEAKY_POOL only */
  const void* whi;             /* packed halves (rrin_pack_conv3x3_h8) */
  const void* wlo;             /* NULL for F16 */
  const float* bias;           /* padded fp32 bias */
  float* edge;                 /* EPI_SUBPIXEL: [n][cout/4][rrin_ring_pixels(H,W)] fp32 */
  int32_t* status;             /* optional (F16X3 / F16): set to 1 when a stored value does not
                                  fit fp16 (|v| > 65504, inf or NaN) -- see rrin_net_desc.status */
  int32_t ksplit;              /* Winograd kinds 3, 4: > 1 splits the input channels into
                                  ksplit slices of whole 8-channel chunks (fewer if a slice would
                                  be empty), one workgroup per tile and slice; the last slice of a
                                  tile sums the slices' pre-bias outputs in slice order.  0 / 1:
                                  no split.  A fixed split per conv keeps batch == per-sample
                                  outputs bitwise; a different split rounds differently */
  int32_t pad2_;
  float* part;                 /* ksplit > 1: rrin_conv_h8_split_floats() floats, any contents */
  int32_t* cnt;                /* ksplit > 1: one int per tile, zero before the first call; every
                                  call leaves it zero again (one call at a time per cnt) */
  /* EPI_SUBPIXEL ring fold (Winograd kind 3, no split): with ring_w set, the launch
     also writes the 1-pixel ring of the 2h x 2w output (the work of
     rrin_subpixel_edge_fix_h8, which is then not called): correction workgroups at
     the head of the grid, one per ring segment, and the segment's conv tile meet
     through ring_cnt; edge still receives the phase values */
  const float* ring_w;         /* original weights [cin][9][cout/4] fp32 (NULL: no fold) */
  const float* ring_bias;      /* original bias [cout/4] */
  float* ring_corr;            /* rrin_conv_h8_ring_floats() floats, any contents */
  int32_t* ring_cnt;           /* rrin_conv_h8_ring_floats() ints, zero before the first call;
                                  every call leaves it zero again */
  /* ABI 17, EPI_SUBPIXEL: the ring pixels from scratch in the same call -- a rrin_edge_fix_desc
     with full = 1 for this conv's src / dst (its own weights, bias, epi_mode, status); edge is
     still written.  The direct-form tiles of 256 or 512 threads run it in extra workgroups at
     the head of the conv's grid (they read only src and write only dst's ring pixels, which the
     sub-pixel conv never writes) with threads / 256 K groups; other configs launch it after the
     conv.  NULL: the caller runs rrin_subpixel_edge_fix_h8 itself. */
  const struct rrin_edge_fix_desc* ring_full;
} rrin_conv_h8_desc;

/* Fused level-0 UNetConvBlock at fp16 (unet.py:59-63, and :46 for down_path[0]): conv a
 * (cin -> 32) + LeakyReLU, conv b (32 -> 32) + LeakyReLU, optionally the 2x2 average pool of the
 * result, in one launch; conv a's output never reaches memory (an 8 x 62 output tile's conv-a
 * values, 1-pixel halo recomputed, stay in LDS).  The weights are the two convs' own
 * rrin_pack_conv3x3_h8 packs (fp16, the bm of cfg_a / cfg_b, direct-form configs); the outputs
 * are bitwise those of the two rrin_conv3x3_h8_fwd calls (EPI_LEAKY into a 32-channel tensor,
 * then EPI_LEAKY or EPI_LEAKY_POOL) at fp16.  dst must not overlap src.  ABI 14. */
typedef struct rrin_block0_h8_desc {
  int32_t n, cin;              /* conv a: cin -> 32 (cin % 8 == 0 or tail_finite); conv b: 32 -> 32 */
  int32_t cfg_a, cfg_b;        /* rrin_conv_h8 configs the packs were made for (direct form) */
  float slope;                 /* 0 <= slope <= 1 */
  float inv_wscale_a, inv_wscale_b; /* from rrin_pack_conv3x3_h8 */
  int32_t tail_finite;         /* as rrin_conv_h8_desc.tail_finite */
  rrin_h8 src, dst, pool;      /* fp16 records; pool.hi NULL: no pool output */
  const void* whi_a;
  const float* bias_a;
  const void* whi_b;
  const float* bias_b;
  int32_t* status;             /* optional fp16 range flag, as rrin_conv_h8_desc.status */
} rrin_block0_h8_desc;
int rrin_conv_block0_h8_fwd(const rrin_block0_h8_desc* d, void* stream);

int rrin_conv_h8_cfg_count(void);
int rrin_conv_h8_cfg_bm(int32_t cfg);
int rrin_conv_h8_cfg_th(int32_t cfg);
int rrin_conv_h8_cfg_ok(int32_t cfg, int32_t prec); /* 1 if the config fits LDS at prec */
/* 1 if the config can run a conv with cin input channels (a config that keeps
 * every weight chunk resident in LDS needs them to fit) */
int rrin_conv_h8_cfg_fits(int32_t cfg, int32_t prec, int32_t cin);
int rrin_conv3x3_h8_fwd(const rrin_conv_h8_desc* d, void* stream);
/* Scratch of a split-K conv (d->ksplit > 1): returns the floats of d->part and
 * stores the ints of d->cnt (0 and 0 without a split); < 0: the error code */
int64_t rrin_conv_h8_split_floats(const rrin_conv_h8_desc* d, int64_t* cnt_ints);
/* Scratch of a ring-folding sub-pixel conv (d->ring_w set): returns the floats of
 * d->ring_corr and stores the ints of d->ring_cnt; < 0: the error code (RRIN_E_CONFIG:
 * the config cannot fold -- run rrin_subpixel_edge_fix_h8 instead) */
int64_t rrin_conv_h8_ring_floats(const rrin_conv_h8_desc* d, int64_t* cnt_ints);
/* Nonzero if cfg is a Winograd config (not packed by rrin_pack_conv3x3_r32 /
 * rrin_pack_conv3x3_h8): the tile kind.  F(2x2,3x3), packed by
 * rrin_pack_conv3x3_wino_bm with the config's BM (F32R): 1 = BM 32 x TH 8 on 4
 * waves, 3 = BM 32 x TH 8 on 8 waves of 4 accumulators (4 waves per SIMD), 4 =
 * kind 3 on TH 4 tiles (4 waves), 6 = BM 64 x TH 4 and 7 = BM 32 x TH 8 on 4 waves
 * with the U operands loaded straight into registers (cin % 8 == 0 or
 * tail_finite); all give bitwise-equal outputs.  Kinds 3 and 4 take a split-K
 * (rrin_conv_h8_desc.ksplit).  Kind 6 also runs at RRIN_PREC_F16 (packed by
 * rrin_pack_conv3x3_wino_h8; cin % 16 == 0 or tail_finite; no split-K, no ring
 * fold).  0: direct form.  -1: a retired id (19, 22: ABI 16 removed the rejected
 * kinds 2, 5 and 8-13 and their configs 25-30; rrin_conv_h8_cfg_ok reports 0 and
 * rrin_conv3x3_h8_fwd returns RRIN_E_CONFIG).  14 (ABI 18, config 25): BM 32 x TH 8 on
 * 4 waves, register U, Winograd F(4,3) x F(2,3) (patches 4 wide x 2 tall: 0.75x kind 6's
 * MFMAs; a different rounding, not bitwise the F(2x2,3x3) kinds), packed by
 * rrin_pack_conv3x3_wino42; cin % 8 == 0 or tail_finite; no split-K, no ring fold, the
 * ring_full fix-up as a second launch. */
int rrin_conv_h8_cfg_wino(int32_t cfg);
/* ABI 19: kind 14's tile geometry, process-wide: 0 (default) picks per launch the one needing
 * fewer rounds of 512 resident workgroups, and persistent workgroups for short K (<= 8 chunks)
 * on large grids; 1 always 32 px x 8 rows (persistent where eligible); 2 always 16 px x 16 rows;
 * 3 always 32 x 8, one workgroup per tile.  Every policy computes each output from the same patch
 * with the same arithmetic: the outputs are the same bits.  Returns the previous policy,
 * RRIN_E_ARG outside 0-3. */
int rrin_conv_h8_set_wino42_geom(int32_t mode);

/* F32R packing: [co_block][chunk of 8 ci][tap][half][bm][4] fp32 (half hh holds
 * input channels chunk*8 + 4*hh .. +3), unscaled; pass as whi (wlo NULL,
 * inv_wscale ignored).  bpack: rrin_pack_bias_floats(cout, bm) floats. */
int64_t rrin_pack_conv3x3_r32_floats(int32_t cout, int32_t cin, int32_t bm);
int rrin_pack_conv3x3_r32(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                          const int32_t* perm, float* wpack, float* bpack);

/* Winograd packing (F32R, the rrin_conv_h8_cfg_wino configs): U = G g G^T per
 * (co, ci) computed in double and rounded once to fp32, laid out
 * [co_block of bm][chunk of 8 ci][xi 16][half 2][co bm][4 ci] (xi = 4*row + col
 * of the 4x4 transform, G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]; half hh holds
 * input channels chunk*8 + 4*hh .. +3); bm = 32 or 64 (the config's BM).
 * bpack: rrin_pack_bias_floats(cout, bm) floats.  The un-suffixed pair is bm 32. */
int64_t rrin_pack_conv3x3_wino_bm_floats(int32_t cout, int32_t cin, int32_t bm);
int rrin_pack_conv3x3_wino_bm(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                              const int32_t* perm, float* wpack, float* bpack);
/* Kind-14 packing (ABI 18): U(eta, xi) = sum G2[eta][ky] G4[xi][kx] g[ky][kx] in double,
 * rounded once to fp32 (G2 the F(2,3) matrix above, rows; G4 = F(4,3)'s [1/4 0 0; -1/6 -1/6
 * -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1], columns), laid out
 * [co_block of 32][chunk of 8 ci][point 6*eta + xi (24)][half 2][co 32][4 ci].  bpack:
 * rrin_pack_bias_floats(cout, 32) floats. */
int64_t rrin_pack_conv3x3_wino42_floats(int32_t cout, int32_t cin);
int rrin_pack_conv3x3_wino42(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                             float* wpack, float* bpack);
int64_t rrin_pack_conv3x3_wino_floats(int32_t cout, int32_t cin);
int rrin_pack_conv3x3_wino(const float* w, const float* b, int32_t cout, int32_t cin, const int32_t* perm,
                           float* wpack, float* bpack);
/* fp16 Winograd packing (ABI 13; kind 6 at RRIN_PREC_F16): U = G g G^T per (co, ci)
 * in double, times a power of two that puts max|U| in [2^12, 2^13), rounded once to
 * fp16, laid out [co_block of 64][chunk of 16 ci][xi 16][half 2][co 64][8 ci] (half hh
 * holds input channels chunk*16 + 8*hh .. +7); *inv_wscale receives the exact inverse
 * scale (pass it in rrin_conv_h8_desc.inv_wscale).  bm must be 64.  bpack:
 * rrin_pack_bias_floats(cout, 64) floats. */
int64_t rrin_pack_conv3x3_wino_h8_halves(int32_t cout, int32_t cin, int32_t bm);
int rrin_pack_conv3x3_wino_h8(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                              const int32_t* perm, uint16_t* whi, float* bpack, float* inv_wscale);

/* Host packing: [co_block][chunk of 16 ci][tap][half][bm][8] halves, weights
 * pre-scaled by a power of two so max|w| lands in [2^12, 2^13) (keeps lo
 * normal); *inv_wscale receives the exact inverse scale. */
int64_t rrin_pack_conv3x3_h8_halves(int32_t cout, int32_t cin, int32_t bm);
int rrin_pack_conv3x3_h8(const float* w, const float* b, int32_t cout, int32_t cin, int32_t bm,
                         const int32_t* perm, int32_t prec, uint16_t* whi, uint16_t* wlo,
                         float* bpack, float* inv_wscale);

/* ---- Sub-pixel form of the up block's upsample + conv (unet.py:77-78) ------
 * conv3x3(upsample_bilinear_x2(x)) at output pixel (2m+py, 2n+px) equals a 3x3
 * conv of x around (m, n) with phase-combined weights W'_(py,px), provided x is
 * edge-replicated by one pixel; it then equals the conv over the replicate-padded
 * upsampled image, so only the outermost output ring differs from the reference
 * (zero padding) -- by the outside taps, which rrin_subpixel_edge_fix_h8 removes.
 * rrin_subpixel_weights: w [cout][cin][3][3], b [cout] -> wsub [4*cout][cin][3][3],
 * bsub [4*cout] with row co' = (co/8)*32 + (2*py+px)*8 + co%8 (cout % 8 == 0),
 * computed in double. */
int rrin_subpixel_weights(const float* w, const float* b, int32_t cout, int32_t cin, float* wsub, float* bsub);
/* pixels on the outermost ring of an H x W image: top row, bottom row, then the
 * left and right columns without the corners (ring index order). */
int64_t rrin_ring_pixels(int32_t h, int32_t w);
typedef struct rrin_edge_fix_desc {
  int32_t n, cin, cout, prec;  /* cout: real output channels (<= 8*dst.groups), cin <= 256 */
  int32_t epi_mode;            /* LINEAR or LEAKY */
  float slope;
  rrin_h8 src;                 /* low-res input of the sub-pixel conv (h x w)   */
  rrin_h8 dst;                 /* its output (2h x 2w): ring pixels are written */
  const float* edge;           /* pre-bias ring values from the EPI_SUBPIXEL conv */
  const float* wedge;          /* original weights as [cin][9][cout] fp32       */
  const float* bias;           /* original bias [cout]                          */
  int32_t* status;             /* optional: fp16 range flag, as rrin_conv_h8_desc */
  /* ABI 11, optional (zero = one workgroup per tile loops over the K runs; the
   * result is the same bit for bit): scratch for the cross-workgroup K split of
   * fp32 records (cin / 64 runs of 64 channels, one workgroup each; the last one
   * of a tile, by a ticket in cnt, adds the runs in run order).  Used when
   * part_floats / cnt_len cover rrin_edge_fix_split_floats; cnt starts at zero
   * and is left at zero. */
  float* part;
  int32_t* cnt;
  int64_t part_floats;
  int32_t cnt_len;
  /* ABI 15: 1 = the ring value from scratch (bias + the conv's in-image taps of the
   * upsampled src, two staged lines per ring line; `edge` unused, may be NULL): it reads
   * nothing the EPI_SUBPIXEL conv writes (that conv writes ring pixels only to `edge`), so
   * the two may run concurrently (the Net measured both orders slower than the
   * correction, DESIGN.md §5e, and uses 0).  0 = the correction of the conv's `edge` values. */
  int32_t full;
} rrin_edge_fix_desc;
int rrin_subpixel_edge_fix_h8(const rrin_edge_fix_desc* d, void* stream);
/* Scratch floats (return; 0 = this cin / precision does not split) and tickets
 * (*cnt) of the ring fix-up's cross-workgroup K split for d's shapes. */
int64_t rrin_edge_fix_split_floats(const rrin_edge_fix_desc* d, int64_t* cnt);

/* nn.Upsample(bilinear, x2) (unet.py:77) of an H8 view into another H8 view. */
int rrin_upsample2x_h8(const rrin_h8* src, const rrin_h8* dst, int32_t n, int32_t prec, void* stream);
/* x = cat(x0, x1) (model.py:33) into the 16-channel H8 Net buffer: channels
 * 0-5 from the two NCHW frames, channels 6-15 zeroed (whole-record stores). */
int rrin_pack_g16_h8(const float* i0, const float* i1, int32_t n, const rrin_h8* g16, int32_t prec, void* stream);
/* NCHW fp32 <-> H8 view (c channels starting at channel ch_off of the view). */
int rrin_nchw_to_h8(const float* src, int32_t n, int32_t c, int32_t ch_off, const rrin_h8* dst,
                    int32_t prec, void* stream);
int rrin_h8_to_nchw(const rrin_h8* src, int32_t n, int32_t c, int32_t ch_off, float* dst, int32_t prec,
                    void* stream);

typedef struct rrin_head_h8_desc {
  int32_t n, cin, cout, mode, prec, pad_;
  rrin_h8 src;           /* 32-channel input                              */
  rrin_h8 g16;           /* Net buffer (2 groups); PLAIN: dst view          */
  const float* w;        /* OIHW fp32 (unpacked)                          */
  const float* bias;
  const float* coef;
  float* out;            /* FINAL: NCHW fp32 */
  rrin_h8 flow_raw;      /* FLOW (optional, hi NULL = skip): raw 4-ch Flow output */
  float* raw_out;        /* optional: head conv output before the glue, NCHW fp32 */
  int32_t* status;       /* optional: fp16 range flag; FINAL writes NaN pixels when it is set */
} rrin_head_h8_desc;
int rrin_head_h8_fwd(const rrin_head_h8_desc* d, void* stream);

/* Flow reuse across t: Ft0/Ft1 of model.py:38-39 recomputed
 * from a kept raw Flow (4 channels) with new per-image coefficients, written to
 * g16 channels 6-9.  The U-Net output itself does not depend on t (model.py:35). */
int rrin_flow_tblend_fwd(const rrin_pp* flow_raw, const rrin_pp* g16, const float* coef, int32_t n,
                         void* stream);
int rrin_flow_tblend_h8(const rrin_h8* flow_raw, const rrin_h8* g16, const float* coef, int32_t n,
                        int32_t prec, void* stream);

/* ---- Whole forward (native schedule) ------------------------------------- */
/* Per-conv weight table entry, in Net conv order (rrin_net_conv_count). */
typedef struct rrin_conv_weights {
  const float* wpack;   /* F32: packed with bm = rrin_conv_cfg_bm(cfg)        */
  const float* bias;    /* packed bias (bm of the config of this precision)  */
  int32_t cfg;          /* F32: rrin_conv_cfg_*; F16*: rrin_conv_h8_cfg_*     */
  float inv_wscale;     /* F16*: from rrin_pack_conv3x3_h8                    */
  const void* whi;      /* F16*: packed halves                                */
  const void* wlo;      /* F16X3: packed lo halves                            */
  int32_t subpixel;     /* F16*, up convs: 1 = whi/wlo/bias hold the sub-pixel
                           weights (4*cout rows) and the upsample pass is skipped;
                           2 = the same with the ring fix-up folded into the conv
                           launch (F32R Winograd kind 3, ksplit <= 1) */
  int32_t ksplit;       /* F32R Winograd kinds 3, 4: rrin_conv_h8_desc.ksplit (0: none);
                           the forward's workspace holds the split scratch */
  const float* wedge;   /* subpixel: original weights [cin][9][cout] fp32      */
  const float* bias_raw;/* subpixel: original bias [cout]                      */
  int32_t fuse_next;    /* F16, level-0 conv a of a UNetConvBlock: 1 = run it and the next
                           conv as one rrin_conv_block0_h8_fwd launch (ABI 14) */
  int32_t pad_;
} rrin_conv_weights;

typedef struct rrin_head_weights {
  const float* w;       /* OIHW, unpacked */
  const float* bias;
} rrin_head_weights;

/* Optional launch profiler: HIP events recorded around every kernel the
 * schedule enqueues (bench.py uses it to time the MFMA conv kernels inside the
 * timed region).  Opaque; created/destroyed by the caller. */
typedef struct rrin_prof rrin_prof;
enum rrin_launch_kind { RRIN_KIND_CONV = 0, RRIN_KIND_HEAD = 1, RRIN_KIND_LAYOUT = 2, RRIN_KIND_EDGE = 3 };

int rrin_prof_create(int32_t capacity, rrin_prof** out);
int rrin_prof_destroy(rrin_prof* p);
int rrin_prof_reset(rrin_prof* p);
/* After the stream has synchronised: per recorded launch its kind, elapsed
 * milliseconds and algorithmic FLOPs (2*MAC of the conv; 0 for layout). */
int rrin_prof_read(rrin_prof* p, int32_t* kinds, float* ms, double* flops, int32_t cap, int32_t* count);
/* Start / end of every recorded launch in ms after the first recorded event
 * (launches on several streams: the union of their spans is the busy time). */
int rrin_prof_read_spans(rrin_prof* p, float* t0_ms, float* t1_ms, int32_t cap, int32_t* count);

typedef struct rrin_net_desc {
  int32_t n, h, w, pad_;
  const float* i0;      /* NCHW [n][3][h][w] */
  const float* i1;
  float* out;           /* NCHW [n][3][h][w] */
  const float* coef;    /* device [n][8] t coefficients */
  /* 4 UNets in execution order Flow, refine_flow, Mask, final; convs of each
   * in UNet order (down a/b per level, mid, up/a/b per level; `last` excluded) */
  const rrin_conv_weights* convs;  /* host array, rrin_net_conv_count() entries */
  const rrin_head_weights* heads;  /* host array of 4 */
  void* workspace;      /* device, >= rrin_net_workspace_bytes, zero-filled once */
  int64_t workspace_bytes;
  int32_t skip_flow;    /* 1: the pair is the one of the previous call on this workspace:
                           reuse its raw Flow (Flow U-Net skipped, t-blend only)      */
  int32_t prec;         /* rrin_prec of the whole forward */
  rrin_prof* prof;      /* nullable: record events around every launch */
  float* taps;          /* nullable (test / debug): the four U-Nets' raw outputs (their `last`
                           conv, before the model.py glue) as NCHW fp32, concatenated:
                           Flow [n][4][h][w] | refine_flow [n][4] | Mask [n][2] | final [n][3]
                           (unet.py:51 outputs used at model.py:35,42,52,62); n*13*h*w floats */
  int32_t* status;      /* optional device int32 (F16X3 / F16 range guard): zeroed at the start
                           of the forward, set to 1 if any activation stored as fp16 overflows
                           (|v| > 65504, inf, NaN); the output is then all NaN (poisoned) instead
                           of silently wrong.  fp32 paths never set it. */
  void* scratch;        /* nullable (ABI 12): device, rrin_net_scratch_bytes(d) bytes, zero-filled
                           once (its ticket words are left zero by every call); F32R split-K
                           slabs of convs with ksplit > 1 (required for them: RRIN_E_WORKSPACE
                           without) and the ring fix-up's cross-workgroup K split (used only
                           when present; the same bits either way).  Kept out of the workspace
                           so plans without splits pay nothing for it. */
  int64_t scratch_bytes;
} rrin_net_desc;

/* Bytes of rrin_net_desc.scratch the forward of d needs with its conv table
 * (0: none; only n, h, w, prec and convs are read).  One forward at a time per scratch. */
int64_t rrin_net_scratch_bytes(const rrin_net_desc* d);

int rrin_net_conv_count(void);                 /* 77 = 81 convs - 4 heads      */

/* One U-Net alone -- the reference UNet(in_channels, n_classes, depth).forward
 * (unet.py:40-51): x NCHW [n][in_ch][h][w] -> y NCHW [n][out_ch][h][w], with
 * the Net's kernels and workspace plan (rrin_net_workspace_bytes of the same
 * n, h, w, prec); in_ch <= 16, out_ch 2..4, depth 2..5.  convs: the U-Net's
 * rrin_unet_conv_count(depth) body convs in UNet order (down a/b per level,
 * mid, up/a/b per level), packed as for rrin_net_fwd (no input permutation);
 * head: its `last` conv, OIHW.  Channels [in_ch, 16) of the workspace's input
 * buffer must be finite (a zero-filled workspace only ever used for U-Nets of
 * one in_ch keeps them zero). */
typedef struct rrin_unet_desc {
  int32_t n, h, w, in_ch, out_ch, depth, prec, pad_;
  const float* x;
  float* y;
  const rrin_conv_weights* convs;  /* host array */
  rrin_head_weights head;
  void* workspace;
  int64_t workspace_bytes;
  rrin_prof* prof;                 /* nullable */
  int32_t* status;                 /* optional device int32: the F16X3 / F16 range guard, as rrin_net_desc */
  void* scratch;                   /* nullable (ABI 12): as rrin_net_desc.scratch, rrin_unet_scratch_bytes */
  int64_t scratch_bytes;
} rrin_unet_desc;
int64_t rrin_unet_conv_count(int32_t depth);
int64_t rrin_unet_scratch_bytes(const rrin_unet_desc* d);
int rrin_unet_fwd(const rrin_unet_desc* d, void* stream);
int64_t rrin_net_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t prec);
int rrin_net_fwd(const rrin_net_desc* d, void* stream);

/* ---- Training path (autograd): NCHW fp32 kernels ------------------------- */
/* With autograd on (the reference trains through Net.forward, train.py:98, and
 * loss.backward(), train.py:144) rrin_amd.train wraps these in autograd
 * Functions.  All tensors are contiguous NCHW fp32.
 *   rrin_tconv3x3 FWD  : out = conv3x3(x, wt) + bias [, leaky]      (unet.py:29,38,59-63,78)
 *                 DGRAD: out = input gradient of that conv: the conv of
 *                        g' = g * leaky'(y) (leaky: y = the forward output) with
 *                        the flipped, transposed weights; x holds g [n][cout][h][w].
 *   rrin_tconv3x3_wgrad: gw = sum over images and pixels of g' (x) x shifted per
 *                        tap, gb = sum g'; deterministic split-K (work buffer of
 *                        rrin_tconv3x3_wgrad_work_floats floats).
 *   rrin_tpool2_*  : F.avg_pool2d(x, 2) (unet.py:46) and its backward; nc = n*c.
 *   rrin_tup2_*    : nn.Upsample(x2, bilinear) (unet.py:77) and its backward;
 *                    h, w = the low-resolution size.
 *   rrin_twarp_bwd : backward of warp (model.py:8-21; forward = rrin_warp_fwd):
 *                    gimg (scatter, summed exactly in 64-bit fixed point:
 *                    deterministic) and gflow; work >= rrin_twarp_bwd_work_bytes. */
enum rrin_tconv_mode { RRIN_TCONV_FWD = 0, RRIN_TCONV_DGRAD = 1 };
typedef struct rrin_tconv_desc {
  int32_t n, cin, cout, h, w;
  int32_t mode;          /* rrin_tconv_mode                                    */
  int32_t leaky;         /* FWD: leaky output; DGRAD: g' = g * leaky'(y)       */
  float slope;           /* leaky slope, 0 < slope <= 1                        */
  const float* x;        /* FWD: input [n][cin][h][w]; DGRAD: g [n][cout][h][w] */
  const float* y;        /* DGRAD with leaky: forward output [n][cout][h][w]    */
  const float* wt;       /* OIHW [cout][cin][3][3]                              */
  const float* bias;     /* FWD: [cout] (nullable)                              */
  float* out;            /* FWD: [n][cout][h][w]; DGRAD: [n][cin][h][w]         */
} rrin_tconv_desc;
int rrin_tconv3x3(const rrin_tconv_desc* d, void* stream);

typedef struct rrin_twgrad_desc {
  int32_t n, cin, cout, h, w, leaky;
  float slope;
  int32_t pad_;
  const float* x;        /* forward input [n][cin][h][w]                        */
  const float* g;        /* output gradient [n][cout][h][w]                     */
  const float* y;        /* leaky: forward output [n][cout][h][w]               */
  float* gw;             /* [cout][cin][3][3]                                   */
  float* gb;             /* [cout] (nullable)                                   */
  float* work;           /* rrin_tconv3x3_wgrad_work_floats(...) floats         */
} rrin_twgrad_desc;
int64_t rrin_tconv3x3_wgrad_work_floats(int32_t n, int32_t cin, int32_t cout, int32_t h, int32_t w);
int rrin_tconv3x3_wgrad(const rrin_twgrad_desc* d, void* stream);

int rrin_tpool2_fwd(const float* x, float* y, int32_t nc, int32_t h, int32_t w, void* stream);
int rrin_tpool2_bwd(const float* gy, float* gx, int32_t nc, int32_t h, int32_t w, void* stream);
int rrin_tup2_fwd(const float* x, float* y, int32_t nc, int32_t h, int32_t w, void* stream);
int rrin_tup2_bwd(const float* gy, float* gx, int32_t nc, int32_t h, int32_t w, void* stream);
int64_t rrin_twarp_bwd_work_bytes(int32_t n, int32_t c, int32_t h, int32_t w);
/* ABI 12: the Winograd packing of rrin_pack_conv3x3_wino_bm computed on the device (the
 * training path repacks every step), bitwise the host packing.  mode 0: the conv of OIHW
 * w [cout][cin][3][3] (rows cout, channels cin); mode 1: its data-gradient conv, w
 * transposed and flipped (rows cin, channels cout).  wpack: rrin_pack_conv3x3_wino_bm_floats
 * (rows, channels, bm) floats. */
int rrin_tpack_wino(const float* w, int32_t cout, int32_t cin, int32_t bm, int32_t mode, float* wpack, void* stream);
int rrin_twarp_bwd(const float* img, const float* flow, const float* gout, float* gimg, float* gflow,
                   void* work, int64_t work_bytes, int32_t n, int32_t c, int32_t h, int32_t w, void* stream);

/* ---- Misc ---------------------------------------------------------------- */
int rrin_abi_version(void);
const char* rrin_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* RRIN_HIP_H */
