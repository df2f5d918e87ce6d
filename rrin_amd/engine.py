"""HIP execution engine behind ``rrin_amd.Net.forward``.

Responsibilities (host side only — every FLOP runs in librrin_hip.so):

* pack the 77 body convs once per weight version into the MFMA slab layout
  (``rrin_pack_conv3x3``, CPU) and upload them as one device blob; the first
  convs of ``refine_flow`` and ``Mask`` get an input-channel permutation so
  they can read the 16-channel Net buffer in its own order;
* keep one zero-initialised workspace per (device, n, h, w) — the padding
  of every padded-planar buffer stays zero because kernels never write it;
* turn ``t`` into the per-image coefficient table with the reference's own
  rounding (Python-float t: double then fp32; tensor t: fp32 tensor ops);
* call ``rrin_net_fwd`` on torch's current stream.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .unet import _level_of

UNET_ORDER = ("Flow", "refine_flow", "Mask", "final")

# g16 = [x0 0-2 | x1 3-5 | Ft0 6-7 | Ft1 8-9 | xt1 10-12 | xt2 13-15]; reference input orders:
#   refine_flow: cat(Ft0, Ft1, x)            model.py:41
#   Mask:        cat(Ft0, Ft1, x, xt1, xt2)  model.py:50
# perm[c] = reference input channel read by buffer channel c.
FIRST_CONV_PERM = {
    "Flow": None,
    "refine_flow": [4, 5, 6, 7, 8, 9, 0, 1, 2, 3],
    "Mask": [4, 5, 6, 7, 8, 9, 0, 1, 2, 3, 10, 11, 12, 13, 14, 15],
    "final": None,
}


def choose_cfg(cin: int, cout: int, level: int) -> int:
    """Tile config id for one conv (conv_mfma.hip config table), from the
    per-shape sweep of tools/conv_lab.py tune at 1280x720, 4 pairs (see
    profiles/ and DESIGN.md §5)."""
    if cout <= 32:
        return 3        # BM 32 x TH 16: full-res layers, 85-103 TF vs 75-88 at TH 8
    if cout >= 512:
        return 4        # BM 64 x TH 4: 80x45 bottom, more blocks for the small grid
    return 1            # BM 64 x TH 8


# Tile config per conv shape (cin, output rows, level of the grid it runs on)
# of the split-fp16 / fp16 convs: fastest in the sweep of every config on every
# conv of the Net (tools/conv_lab.py tune, 1280x720, 4 pairs;
# profiles/r01_v10/tune_*.txt).  The shapes are fixed by the architecture
# (channels and levels), so the keys hold at every resolution.  Sub-pixel up
# convs run on the low-res grid with 4x the output rows.
H8_TUNED = {
    _lib.PREC_F16X3: {(6, 32, 0): 13, (9, 32, 0): 13, (10, 32, 0): 15, (16, 32, 0): 9, (32, 32, 0): 15,
                      (32, 64, 1): 8, (64, 32, 0): 9, (64, 64, 1): 10, (64, 128, 1): 10, (64, 128, 2): 11,
                      (128, 64, 1): 10, (128, 128, 2): 11, (128, 256, 2): 10, (128, 256, 3): 11,
                      (256, 128, 2): 11, (256, 256, 3): 11, (256, 512, 3): 11, (256, 512, 4): 1,
                      (512, 256, 3): 11, (512, 512, 4): 1},
    # fp16: re-swept in round 3 at the BASELINE C3 part size, 1280x736 x 2
    # (profiles/r03/tune_fp16_1280x736x2.json: schedule sum 4.413 -> 4.283 ms; the 512->256
    # L3 up conv 0.222 -> 0.141 ms); C3 bench 466.6-469.1 -> 470.6-477.7 pairs/s in
    # interleaved runs (profiles/r03/fp16_table_ab.txt)
    _lib.PREC_F16: {(6, 32, 0): 9, (9, 32, 0): 9, (10, 32, 0): 9, (16, 32, 0): 13, (32, 32, 0): 9,
                    (32, 64, 1): 10, (64, 32, 0): 9, (64, 64, 1): 10, (64, 128, 1): 11, (64, 128, 2): 10,
                    (128, 64, 1): 11, (128, 128, 2): 11, (128, 256, 2): 11, (128, 256, 3): 11,
                    (256, 128, 2): 10, (256, 256, 3): 11, (256, 512, 3): 10, (256, 512, 4): 4,
                    (512, 256, 3): 10, (512, 512, 4): 4},
}

# Smaller work per forward part leaves the deep levels with a few dozen BM 64 x
# TH 16 tiles for 256 CUs (the 640x368 L3 grid is 46x80 px: 36 blocks), so the
# same sweep at the smaller workloads picks other tiles — mostly BM 32 x TH 8/16
# persistent (cfg 12/13).  Size classes by pixels per forward part (n*h*w):
# "small" <= SMALL_PX (sweep at 640x368 x 1 = BASELINE config C2, conv sum
# 3.30 -> 2.11 ms; BM 32 x TH 4 (cfg 16) at the deepest levels), "medium" <=
# MEDIUM_PX (1280x720 x 1, 5.79 -> 5.34 ms), else "large" (H8_TUNED).
# profiles/r01_v13/tune_*.txt; split16 only (the fp16 path keeps H8_TUNED at
# every size).
# Exact fp32 on fp32 records (F32R): per-shape choice from the sweep of every
# config on every conv shape at 1280x720, 2 pairs per launch -- the part size of
# the 2-stream bench (tools/conv_lab.py tune --precision fp32 --batch 2,
# profiles/r02/tune_fp32r_1280x720x2.txt).  BM 128 x TH 16 (cfg 5) wins at level
# 2; the 45x80 bottom wants the many small persistent tiles of cfg 16.
H8_TUNED[_lib.PREC_F32R] = {(6, 32, 0): 13, (9, 32, 0): 9, (10, 32, 0): 13, (16, 32, 0): 8, (32, 32, 0): 9,
                            (32, 64, 1): 8, (64, 32, 0): 9, (64, 128, 1): 1, (64, 64, 1): 1, (64, 128, 2): 5,
                            (128, 64, 1): 4, (128, 256, 2): 5, (128, 128, 2): 5, (128, 256, 3): 0,
                            (256, 128, 2): 5, (256, 512, 3): 5, (256, 256, 3): 3, (256, 512, 4): 16,
                            (512, 256, 3): 3, (512, 512, 4): 16}

SMALL_PX = 500_000
MEDIUM_PX = 1_200_000
H8_TUNED_BY_SIZE = {
    "small": {_lib.PREC_F16X3: {(6, 32, 0): 15, (9, 32, 0): 13, (10, 32, 0): 15, (16, 32, 0): 13, (32, 32, 0): 13,
                                (32, 64, 1): 13, (64, 32, 0): 13, (64, 64, 1): 13, (64, 128, 1): 11,
                                (64, 128, 2): 16, (128, 64, 1): 13, (128, 128, 2): 12, (128, 256, 2): 13,
                                (128, 256, 3): 16, (256, 128, 2): 16, (256, 256, 3): 12, (256, 512, 3): 13,
                                (256, 512, 4): 16, (512, 256, 3): 16, (512, 512, 4): 16}},
    "medium": {_lib.PREC_F16X3: {(6, 32, 0): 9, (9, 32, 0): 13, (10, 32, 0): 15, (16, 32, 0): 8, (32, 32, 0): 8,
                                 (32, 64, 1): 10, (64, 32, 0): 12, (64, 64, 1): 10, (64, 128, 1): 12,
                                 (64, 128, 2): 11, (128, 64, 1): 11, (128, 128, 2): 10, (128, 256, 2): 11,
                                 (128, 256, 3): 13, (256, 128, 2): 10, (256, 256, 3): 13, (256, 512, 3): 11,
                                 (256, 512, 4): 13, (512, 256, 3): 13, (512, 512, 4): 13}},
}


LARGE_PX = 2_500_000
XLARGE_PX = 6_000_000
# Bigger forward parts (one stream over 720p x 4, the 4K share of config C5):
# fp32 records "xlarge" = the sweep at 1280x720 x 4 (3.7 Mpx per launch,
# profiles/r02/tune_fp32r_1280x720x4.txt), "xxlarge" = the sweep at 3840x2176 x 1
# (8.4 Mpx, profiles/r02/c5_4k/tune_fp32r_3840x2176x1.txt); fp16 "xxlarge" = the
# C5 4K sweep (profiles/r02/c5_4k/tune_fp16_3840x2176x1.txt).  A class a
# precision has no table for uses H8_TUNED.
# Exact fp32 (F32R) "small" / "medium": the sweeps at 640x368 x 1 (config C2;
# the untuned large table's BM 128 tiles left the 46x80 L3 grid with 8-16 TF/s,
# summed conv time 12.84 -> 5.34 ms) and 1280x720 x 1 (18.12 -> 14.45 ms);
# profiles/r02/tune_fp32r_640x368x1.txt, tune_fp32r_1280x720x1.txt.
H8_TUNED_BY_SIZE["small"][_lib.PREC_F32R] = {
    (6, 32, 0): 15, (9, 32, 0): 15, (10, 32, 0): 1, (16, 32, 0): 9, (32, 32, 0): 9, (32, 64, 1): 1, (64, 32, 0): 9,
    (64, 64, 1): 1, (64, 128, 1): 0, (64, 128, 2): 4, (128, 64, 1): 1, (128, 128, 2): 12, (128, 256, 2): 1,
    (128, 256, 3): 16, (256, 128, 2): 4, (256, 256, 3): 6, (256, 512, 3): 16, (256, 512, 4): 16, (512, 256, 3): 16,
    (512, 512, 4): 16}
H8_TUNED_BY_SIZE["medium"][_lib.PREC_F32R] = {
    (6, 32, 0): 15, (9, 32, 0): 1, (10, 32, 0): 9, (16, 32, 0): 6, (32, 32, 0): 8, (32, 64, 1): 0, (64, 32, 0): 6,
    (64, 64, 1): 0, (64, 128, 1): 9, (64, 128, 2): 0, (128, 64, 1): 0, (128, 128, 2): 0, (128, 256, 2): 5,
    (128, 256, 3): 1, (256, 128, 2): 11, (256, 256, 3): 1, (256, 512, 3): 11, (256, 512, 4): 16, (512, 256, 3): 1,
    (512, 512, 4): 16}
H8_TUNED_BY_SIZE["xlarge"] = {
    _lib.PREC_F32R: {(6, 32, 0): 13, (9, 32, 0): 15, (10, 32, 0): 15, (16, 32, 0): 15, (32, 32, 0): 9,
                     (32, 64, 1): 8, (64, 32, 0): 9, (64, 64, 1): 1, (64, 128, 1): 1, (64, 128, 2): 4,
                     (128, 64, 1): 1, (128, 128, 2): 5, (128, 256, 2): 1, (128, 256, 3): 5, (256, 128, 2): 5,
                     (256, 256, 3): 5, (256, 512, 3): 5, (256, 512, 4): 4, (512, 256, 3): 5, (512, 512, 4): 4}}
H8_TUNED_BY_SIZE["xxlarge"] = {
    _lib.PREC_F32R: {(6, 32, 0): 9, (9, 32, 0): 13, (10, 32, 0): 9, (16, 32, 0): 8, (32, 32, 0): 9,
                     (32, 64, 1): 9, (64, 32, 0): 9, (64, 64, 1): 1, (64, 128, 1): 1, (64, 128, 2): 5,
                     (128, 64, 1): 1, (128, 128, 2): 5, (128, 256, 2): 5, (128, 256, 3): 5, (256, 128, 2): 5,
                     (256, 256, 3): 5, (256, 512, 3): 5, (256, 512, 4): 4, (512, 256, 3): 5, (512, 512, 4): 4},
    _lib.PREC_F16: {(6, 32, 0): 13, (9, 32, 0): 13, (10, 32, 0): 15, (16, 32, 0): 9, (32, 32, 0): 9,
                    (32, 64, 1): 10, (64, 32, 0): 9, (64, 64, 1): 10, (64, 128, 1): 10, (64, 128, 2): 10,
                    (128, 64, 1): 10, (128, 128, 2): 11, (128, 256, 2): 11, (128, 256, 3): 10, (256, 128, 2): 11,
                    (256, 256, 3): 11, (256, 512, 3): 11, (256, 512, 4): 1, (512, 256, 3): 11, (512, 512, 4): 11}}


def size_class(pixels: int) -> str:
    """Tile-table class of a forward part of ``pixels`` = n*h*w output pixels."""
    if pixels <= SMALL_PX:
        return "small"
    if pixels <= MEDIUM_PX:
        return "medium"
    if pixels <= LARGE_PX:
        return "large"
    return "xlarge" if pixels <= XLARGE_PX else "xxlarge"


# Exact fp32 (F32R): Winograd F(2x2,3x3) (conv_wino.hip) for the body convs of
# these size classes -- faster than the best direct-form config on every conv
# shape of the Net but the 6-channel first conv (1280x720 x 2: 1.3-1.7x; 640x368
# x 1: 1.0-1.6x; profiles/r02/wino/tune_*).  WINO = False (A/B) uses the
# direct-form tables below.
WINO = True
WINO_SIZES = ("small", "medium", "large", "xlarge", "xxlarge")
# ... except where the direct form wins: the 6-channel first conv (Flow down0.a,
# unet.py:59 with in_channels 6) has one 8-channel K chunk, so a Winograd tile is
# mostly its prologue and epilogue; the direct form's BM 32 x TH 16 persistent
# tile (cfg 13) is 5-11 % faster (0.020 vs 0.021 ms at 640x368 x 1, 0.096 vs
# 0.108 ms at 1280x720 x 2; profiles/r02/wino/tune_fp32r_*_v3.txt, line 2).
WINO_DIRECT = {(6, 32, 0): 13}


# Winograd tile kind (rrin_conv_h8_cfg_wino).  0 = "auto" (the default since round 4):
# the register-U tile kind 6 (conv_winoc.hip, BM 64 x TH 4, U operands loaded straight
# into registers, each transformed input feeding 2 co tiles; bitwise equal to kind 3)
# where the conv's output rows fill 64-channel blocks -- 0.5-16 % faster per conv
# (profiles/r04/ab_kind3_vs_kind6.log), whole 1280x720 x 4 forward 132.1 -> 142.2-142.8
# pairs/s (profiles/r04/bench_kind_ab.txt) -- else kind 3 = BM 32 x TH 8 on 8 waves of
# 4 accumulators (1-9 % faster than kind 1, profiles/r03/cfgab_18_20.txt); the 32-row
# kind 7 loses to kind 3 on the level-0 32-channel convs (ab_kind3_vs_kind7.log).
# A nonzero value forces that kind everywhere (A/B, bench.py --wino-kind).
WINO_KIND = 0


# the kind of the auto mode's 32-output-channel convs (the level-0 convs).  Round 4-5 measured
# the alternatives (kind 7, the persistent kind 8, register U inside kind 3) slower; the
# rejected kinds 2, 5 and 8-13 (kind 12: kind 6 on a persistent grid, slower in the
# two-stream forward) were removed in round 6 -- DESIGN.md §5b-§5e keep the numbers.
WINO_KIND32 = 3


def wino_kind_for(cout: int) -> int:
    if WINO_KIND != 0:
        return WINO_KIND
    if cout % 64 == 0:
        return 6
    return WINO_KIND32 if cout <= 32 else 3
# ... and kind 4 (the same arithmetic on TH 4 tiles of 4 waves: twice the
# workgroups) on the few-tile deep convs where that wins, (cin, cout rows, grid
# level) per size class as in WINO_DIRECT (a sub-pixel up conv: 4 x cout, the
# low-res grid).  cfg 20 vs 21 on every conv shape of the Net
# (profiles/r03/cfgab_20_21_*.txt): 0.71-0.72 at level 4 and 0.84 for the level-2
# up conv at 640x368 x 1; 0.90-0.97 on the level-4 grid at 1280x720 x 2; 1.00-1.10
# on the rest (more tiles than CUs already: the 8-wave tile's shared U stage wins).
# Whole forward (profiles/r03/bench_th4_ab.txt): 640x368 x 1 +2.8 %, 1280x720 x 1
# +0.8 %; 1280x720 x 4 on two streams (class "large") -0.2 %, noise -- the other
# stream already fills the CUs there, so that class keeps the 8-wave tile.
WINO_TH4 = {"small": {(256, 512, 4), (512, 512, 4), (256, 512, 3)},
            "medium": {(256, 512, 4), (512, 512, 4), (512, 1024, 4)}}


# Split-K of the Winograd convs (rrin_conv_h8_desc.ksplit; kinds 3, 4): the few-tile
# deep convs of small images, where a tile per workgroup leaves most CUs idle.  A split
# conv sums its K slices in slice order, a different rounding from the unsplit conv, so
# the split is chosen from the per-image geometry only (the conv's grid h_l x w_l, its
# input channels and output rows), never from the batch: a pair's bits do not depend on
# its batch size, stream split or shard (tests/test_gpu_net.py::
# test_batch_size_bitwise_640x368).  Rule (geom_split): K >= 256 channels,
# slices of >= 8 chunks, and the kind-4 tiles of one image x slices <= GEOM_SPLIT_WGS.
# 640x368 x 1 per conv (profiles/r04/c2_kinds.log, kind 4 + split vs the kind-6 tile):
# 512->512 L4 0.0423 vs 0.0711 ms, 512->1024 sub-pixel 0.0356 vs 0.0719, 256->512 L4
# 0.0263 vs 0.0391, 512->256 L3 0.0687 vs 0.0717; 720p and larger images never split
# (their kind-4 tiles per image exceed the bound).  Round 3's split by size class
# (n*h*w) made bits depend on the batch and is gone.
GEOM_SPLIT = True
GEOM_SPLIT_WGS = 800
# A/B override: grid level -> slices for every Winograd conv at that level (bench.py
# --wino-split); replaces the geometry rule
WINO_SPLIT_LEVELS = {}


def geom_split(cin: int, rows: int, hl: int, wl: int) -> int:
    """Split-K slices (1 = none) of an exact-fp32 Winograd conv of cin input channels and
    `rows` output rows (4 x cout for a sub-pixel up conv) on an hl x wl grid, one image."""
    nch = (cin + 7) // 8
    if not GEOM_SPLIT or nch < 32:
        return 1
    t4 = -(-hl // 4) * -(-wl // 32) * -(-rows // 32)  # kind-4 tiles (BM 32 x 32 px x TH 4)
    for s in (4, 2):
        if t4 * s <= GEOM_SPLIT_WGS and nch // s >= 8:
            return s
    return 1


# Sub-pixel ring fold (rrin_conv_weights.subpixel = 2): the ring fix-up of an
# exact-fp32 sub-pixel up conv runs inside its Winograd launch (kind 3, no split)
# instead of as rrin_subpixel_edge_fix_h8.  Correct (tests/test_gpu_ringfold.py) but
# slower (profiles/r03/ringfold_ab.txt: 1280x720 x 4 121.6-122.0 vs 128.8-129.3
# pairs/s, conv busy +2 ms per step; 1280x720 x 1 108.2 vs 110.4; 640x368 x 1 equal):
# the correction workgroups hold full conv slots for latency-bound ring work that the
# separate launch runs beside the other stream's convs.  Off; the A/B knob stays.
RING_FOLD = False


def choose_split(level: int, cfg: int, geom: int) -> int:
    """Slices of the split-K for a conv of tile config cfg at grid level `level` whose
    geometry rule gave `geom` (0: none)."""
    if _lib.lib().rrin_conv_h8_cfg_wino(cfg) not in (3, 4):
        return 0
    if WINO_SPLIT_LEVELS:
        return WINO_SPLIT_LEVELS.get(level, 0)
    return geom if geom > 1 else 0


def wino_cfg(kind: int = None) -> int:
    lib = _lib.lib()
    kind = WINO_KIND if kind is None else kind
    return next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == kind)


# fp16 (BASELINE C3-C5): Winograd F(2x2,3x3) with f16 MFMAs (conv_winoh.hip, the kind-6
# register-U tile at fp16) on the convs whose output rows fill 64-channel blocks and whose
# input channels fill 16-channel chunks, at the grid levels in WINO_F16_LEVELS; the rest
# (the 32-channel level-0 convs, the 6-16-channel first convs) stay on the direct-form
# tables.  False: the direct form everywhere (A/B, bench.py --no-wino).
WINO_F16 = True
# Per conv at the C3 part size (1280x736 x 2, profiles/r05/cfgab_fp16_winograd.log) the fp16
# Winograd tile (kind 6) runs 0.77-0.81 of the best direct tile's time at level 4 and 0.92-0.98 at
# level 3; at levels 1-2 1.0-1.5 (the direct form keeps more operand reuse per VMEM instruction
# than Winograd's U stream)
WINO_F16_LEVELS = (4,)
WINO_F16_KIND = 6


# fp16: level-0 UNetConvBlocks (conv a: in -> 32, conv b: 32 -> 32, unet.py:59-63) as one launch
# with conv a's output tile in LDS (conv_block0.hip, rrin_conv_block0_h8_fwd; bitwise the two
# direct-form launches).  0: two launches everywhere; 1: down_path[0] (conv a from the U-Net's
# 6-16-channel input) fused; 2: also the last up block's conv_block (conv a 64 -> 32).  In
# isolation at 1280x736 x 2 the fused down block takes 108 vs 121 us, the fused up block 159 vs
# 150 us (its recomputed halo, 1.29x conv a's MACs, costs more than the HBM round trip it saves;
# profiles/r05/block0/); in round 5's C3 forward (4 streams) mode 2 measured best: 480.0-481.7
# pairs/s vs 478.2-479.6 (mode 1) and 474.5-475.7 (unfused), C5 within noise (56.6-56.9).  On the
# round-6 schedule (2 streams for fp16) mode 1 leads: 514.1-514.9 vs 511.5-512.9 (mode 2) and
# 509.2-509.6 (unfused), one box interleaved (profiles/r06/r06ac/).
FUSE_L0 = 1


MAX_DEFAULT_STREAMS = 4  # the most streams a caller is expected to ask for (workspace cache sizing)


def default_streams(precision: str, batch: int) -> int:
    """HIP streams a forward of `batch` pairs is split over by default: 2 at every precision
    (headline 1280x720 x 4 exact fp32: 158 vs 151 on 1 stream, 153 on 3, 155 on 4,
    profiles/r06/r06n, r06s; fp16 C3 1280x736 x 4: 512.3-512.4 on 2 vs 507.3-507.8 on 4 and
    487.8-488.3 on 3 since round 6's record-conv changes, profiles/r06/r06aa -- round 5 had
    measured 4 ahead).  The output is bitwise that of one stream either way."""
    return max(1, min(batch, 2))


def fused_pairs(convs) -> list:
    """Indices i of the (cin, cout, level, edge) list whose conv and conv i + 1 form a level-0
    UNetConvBlock: conv i (not an up conv) -> 32 channels at level 0, conv i + 1 32 -> 32 at
    level 0."""
    out, i = [], 0
    while i + 1 < len(convs):
        cin, cout, level, edge = convs[i]
        c2, o2, l2, e2 = convs[i + 1]
        if level == 0 and cout == 32 and edge is None and (c2, o2, l2) == (32, 32, 0) and e2 is None:
            out.append(i)
            i += 2
        else:
            i += 1
    return out


# exact fp32: the register-U tile in Winograd F(4,3) x F(2,3) (kind 14, conv_winoc42.hip: 3
# multiply-adds per output and input channel instead of F(2x2,3x3)'s 4, one co tile per
# transform) on the convs of these grid levels (an up conv: its low-res grid) that the geometry
# rule does not split, in every size class (never the class-dependent TH-4 tiles for them), so a
# pair's bits stay batch-invariant.
# Per conv at 1280x720 x 2 (profiles/r06/wino42/): 0.84-0.90 of kind 6's time on every conv of
# levels 1-4 (every epilogue, the sub-pixel up convs included) and 0.87 on the level-0 64->32
# conv vs kind 3; the level-0 32->32 convs even in isolation (0.98-1.04), 16->32 1.08.  Whole
# forward, one box interleaved: 1280x720 x 4 143.1-143.7 -> 157.6-157.8 pairs/s with level 0 from
# cin 64, 640x368 x 1 338.6-339.1 -> 357.0-357.5; every level-0 conv with cin % 8 == 0 on kind 14
# (WINO42_MIN_CIN_L0 16) another +0.5 % / +0.3 % (profiles/r06/r06o/: 152.6-152.7 vs 151.7-151.9
# on a slower box, C2 356.7 vs 355.5).
WINO42_LEVELS = (0, 1, 2, 3, 4)
WINO42_MIN_CIN_L0 = 16


def wino42_ok(cin: int, cout: int, level: int) -> bool:
    return (WINO_KIND == 0 and level in WINO42_LEVELS and cout % 32 == 0 and cin % 8 == 0
            and (level > 0 or cin >= WINO42_MIN_CIN_L0))


def wino_f16_ok(cin: int, cout: int, level: int) -> bool:
    return WINO_F16 and level in WINO_F16_LEVELS and cout % 64 == 0 and cin % 16 == 0


def choose_cfg_h8(cin: int, cout: int, prec: int, level: int = 0, size: str = "large", split: int = 1) -> int:
    """Tile config of the record-layout conv (conv_f16.hip table) for a conv
    running on the grid of U-Net level ``level`` (a sub-pixel up conv runs on the
    low-res grid with 4x the output rows) in a forward part of size class
    ``size``: exact fp32 takes the Winograd config (WINO_SIZES; kind 4 where the
    geometry splits K, ``split`` > 1); otherwise the swept choice (H8_TUNED_BY_SIZE,
    H8_TUNED), else a level rule from the same sweep."""
    if prec == _lib.PREC_F32R and WINO and size in WINO_SIZES:
        c = WINO_DIRECT.get((cin, cout, level))
        if c is not None and _lib.lib().rrin_conv_h8_cfg_fits(c, prec, cin):
            return c
        if split > 1:  # the per-image geometry split-K (kind 4) first: batch-invariant either way
            return wino_cfg(4)
        if wino42_ok(cin, cout, level):
            return wino_cfg(14)
        return wino_cfg(4 if (cin, cout, level) in WINO_TH4.get(size, ()) else wino_kind_for(cout))
    if prec == _lib.PREC_F16 and wino_f16_ok(cin, cout, level):
        return wino_cfg(WINO_F16_KIND)
    table = H8_TUNED_BY_SIZE.get(size, {}).get(prec) or H8_TUNED.get(prec, {})
    cfg = table.get((cin, cout, level))
    if cfg is not None and _lib.lib().rrin_conv_h8_cfg_fits(cfg, prec, cin):
        return cfg
    if level == 0 or cout <= 32:
        return 9 if _lib.lib().rrin_conv_h8_cfg_fits(9, prec, cin) else 13  # BM 32 x TH 16, persistent
    if level >= 4:
        return 1    # BM 32 x TH 16, 8 waves: the 45x80 bottom at 720p
    return 10 if level == 1 else 11  # BM 64 x TH 16, spread DMA issue (persistent at level 1)


def t_coefficients(t, n: int) -> torch.Tensor:
    """[n, 8] fp32: -(1-t)t, t*t, (1-t)^2, t(1-t), 1-t, t, 0, 0 (model.py:38-39,54)."""
    if isinstance(t, torch.Tensor) and t.numel() > 1:
        tt = t.detach().to("cpu", torch.float32).reshape(-1)
        if tt.numel() != n:
            raise ValueError(f"t has {tt.numel()} elements for a batch of {n}")
        one_m = 1 - tt
        cols = [(-one_m) * tt, tt * tt, one_m * one_m, tt * one_m, one_m, tt]
        c = torch.stack(cols + [torch.zeros_like(tt)] * 2, dim=1)
    else:
        tf = float(t.item()) if isinstance(t, torch.Tensor) else float(t)
        if isinstance(t, torch.Tensor):  # 0-dim tensor: fp32 tensor arithmetic
            tt = torch.tensor([tf], dtype=torch.float32)
            one_m = 1 - tt
            row = torch.cat([(-one_m) * tt, tt * tt, one_m * one_m, tt * one_m, one_m, tt,
                             torch.zeros(2)])
        else:  # Python float: double arithmetic, rounded once to fp32 (scalar * tensor)
            row = torch.tensor([-(1 - tf) * tf, tf * tf, (1 - tf) * (1 - tf), tf * (1 - tf),
                                1 - tf, tf, 0.0, 0.0], dtype=torch.float64).float()
        c = row.view(1, 8).expand(n, 8).contiguous()
    return c


class RRINEngine:
    # cached workspaces (one per forward part: (pairs, h, w, stream slot)): two shapes at the
    # largest default stream count stay resident together -- an fp16 4-stream forward alone fills 4
    # slots, and evicting one forces a zero-filled reallocation and drops its reuse_flow state
    # (ADVICE r05).  Eviction is by shape: every part of the least recently used (h, w) goes at once.
    MAX_WORKSPACES = 2 * MAX_DEFAULT_STREAMS

    def __init__(self, net, precision: str = "fp32", subpixel_max_level: int = 2, units=None):
        """``units``: the U-Nets to pack, as (name, UNet, first-conv input permutation);
        default the Net's four in execution order (UNET_ORDER, FIRST_CONV_PERM)."""
        self.lib = _lib.lib()
        self.subpixel_max_level = subpixel_max_level
        if units is None:
            units = [(name, getattr(net, name), FIRST_CONV_PERM[name]) for name in UNET_ORDER]
        self.units = units
        self.expected_convs = sum(2 * u.depth + 1 + 3 * (u.depth - 1) for _, u, _ in units)
        params = list(net.parameters())
        self.device = params[0].device
        if self.device.type != "cuda":
            raise RuntimeError("rrin_amd.Net: move the model to a ROCm device (net.cuda()) before "
                               "forward — the HIP kernels are the only implementation")
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}")
        self.precision = precision
        self.prec = _lib.PRECISIONS[precision]
        L = self.lib
        blobs, meta = [], []
        off = 0
        self.heads_t = []
        if self.prec != _lib.PREC_F32:
            self._init_h8(net)
            return
        self._levels32 = []         # grid level per body conv (fp32 path)
        self._table32_small = None  # small size class: TH 4 tiles at levels >= 1
        for name, unet, first_perm in self.units:
            convs = unet.conv_list()
            for idx, (tag, conv) in enumerate(convs):
                w = conv.weight.detach().to("cpu", torch.float32).contiguous().numpy()
                b = conv.bias.detach().to("cpu", torch.float32).contiguous().numpy()
                cout, cin = w.shape[0], w.shape[1]
                if tag == "last":
                    self.heads_t.append((torch.from_numpy(w.copy()).to(self.device),
                                         torch.from_numpy(b.copy()).to(self.device)))
                    continue
                cfg = choose_cfg(cin, cout, 0)
                self._levels32.append(_level_of(unet, tag))
                bm = L.rrin_conv_cfg_bm(cfg)
                nw = L.rrin_pack_conv3x3_floats(cout, cin, bm)
                nb = L.rrin_pack_bias_floats(cout, bm)
                wp = np.empty(nw, np.float32)
                bp = np.empty(nb, np.float32)
                perm = first_perm if idx == 0 else None
                perm_arr = np.asarray(perm, np.int32) if perm is not None else None
                _lib.check(L.rrin_pack_conv3x3(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                               perm_arr.ctypes.data if perm_arr is not None else None,
                                               wp.ctypes.data, bp.ctypes.data), "rrin_pack_conv3x3")
                meta.append((off, off + nw, cfg))
                blobs += [wp, bp]
                off += nw + nb
                # keep 16-B alignment of every slab
                pad = (-off) % 4
                if pad:
                    blobs.append(np.zeros(pad, np.float32))
                    off += pad
        if len(meta) != self.expected_convs:
            raise RuntimeError(f"packed {len(meta)} convs, expected {self.expected_convs}")
        self.blob = torch.from_numpy(np.concatenate(blobs)).to(self.device)
        base = self.blob.data_ptr()
        self.conv_table = (_lib.ConvWeights * len(meta))()
        for i, (wo, bo, cfg) in enumerate(meta):
            self.conv_table[i].wpack = base + 4 * wo
            self.conv_table[i].bias = base + 4 * bo
            self.conv_table[i].cfg = cfg
        self.head_table = (_lib.HeadWeights * len(self.heads_t))()
        for i, (w, b) in enumerate(self.heads_t):
            self.head_table[i].w = w.data_ptr()
            self.head_table[i].bias = b.data_ptr()
        self.cfgs = [m[2] for m in meta]
        self._scratch = {}
        self._ws = OrderedDict()
        self._flow_valid = {}
        self._sides = []
        self._status = {}
        self._pending_status = []
        self._graphs = {}

    def _init_h8(self, net):
        """Pack for the split-fp16 (F16X3) or fp16 (F16) path: [cob][16-ch chunk][tap][half][bm][8]
        halves (rrin_pack_conv3x3_h8), one device blob of halves + one of fp32 biases per
        tile-table size class (the block of output channels BM of a conv's tile config sets
        its packing); the "large" class is packed here, the others on first use."""
        L = self.lib
        self.edge_t = []  # device tensors referenced by the tables (sub-pixel convs)
        self._h8_convs = []  # (w, b, cin, cout rows, grid level, first-conv perm, edge) per body conv
        for name, unet, first_perm in self.units:
            for idx, (tag, conv) in enumerate(unet.conv_list()):
                w = conv.weight.detach().to("cpu", torch.float32).contiguous().numpy()
                b = conv.bias.detach().to("cpu", torch.float32).contiguous().numpy()
                cout, cin = w.shape[0], w.shape[1]
                if tag == "last":
                    self.heads_t.append((torch.from_numpy(w.copy()).to(self.device),
                                         torch.from_numpy(b.copy()).to(self.device)))
                    continue
                edge = None
                level = _level_of(unet, tag)
                if tag.endswith(".up") and level <= self.subpixel_max_level:
                    level += 1  # runs on the low-res grid
                    # upsample folded into phase-combined weights (rrin_subpixel_weights)
                    ws = np.empty((4 * cout, cin, 3, 3), np.float32)
                    bs = np.empty(4 * cout, np.float32)
                    _lib.check(L.rrin_subpixel_weights(w.ctypes.data, b.ctypes.data, cout, cin, ws.ctypes.data,
                                                       bs.ctypes.data), "rrin_subpixel_weights")
                    edge = (torch.from_numpy(np.ascontiguousarray(w.transpose(1, 2, 3, 0))).to(self.device),
                            torch.from_numpy(b.copy()).to(self.device))
                    self.edge_t.append(edge)
                    w, b, cout = ws, bs, 4 * cout
                perm = first_perm if idx == 0 else None
                perm_arr = np.asarray(perm, np.int32) if perm is not None else None
                self._h8_convs.append((w, b, cin, cout, level, perm_arr, edge))
        if len(self._h8_convs) != self.expected_convs:
            raise RuntimeError(f"packed {len(self._h8_convs)} convs, expected {self.expected_convs}")
        self._block0 = fused_pairs([(cin, cout, level, edge) for (_, _, cin, cout, level, _, edge) in self._h8_convs])
        self.head_table = (_lib.HeadWeights * len(self.heads_t))()
        for i, (w, b) in enumerate(self.heads_t):
            self.head_table[i].w = w.data_ptr()
            self.head_table[i].bias = b.data_ptr()
        self._packs = {}          # size class -> packing
        self._packs_by_cfgs = {}  # tuple of per-conv configs -> packing (shared between classes)
        _, _, self.conv_table, self.cfgs = self._pack_h8("large", None, None)
        self._scratch = {}
        self._ws = OrderedDict()
        self._flow_valid = {}
        self._sides = []
        self._graphs = {}
        self._status = {}           # slot -> device int32 range flag (fp16-stored precisions)
        self._pending_status = []   # (event, pinned host copy) of flags not checked yet

    def _geom_splits(self, h, w):
        """Per body conv: the geometry rule's split-K slices at image size h x w (exact fp32
        Winograd; a tuple of 1s elsewhere or without a size)."""
        if h is None or self.prec != _lib.PREC_F32R or not WINO:
            return (1,) * len(self._h8_convs)
        return tuple(geom_split(cin, cout, h >> level, w >> level)
                     for (_, _, cin, cout, level, _, _) in self._h8_convs)

    def _pack_h8(self, size: str, h: int = None, w: int = None):
        """(halves blob, bias blob, ConvWeights table, cfgs) of size class ``size`` at image
        size h x w (the split-K geometry; None: no split), cached; classes / geometries
        whose tile configs agree share one packing."""
        geo = self._geom_splits(h, w)
        key = (size, geo, FUSE_L0)
        p = self._packs.get(key)
        if p is not None:
            return p
        L = self.lib
        cfgs = [choose_cfg_h8(cin, cout, self.prec, level, size, g)
                for (_, _, cin, cout, level, _, _), g in zip(self._h8_convs, geo)]
        ckey = (tuple(cfgs), FUSE_L0)
        p = self._packs_by_cfgs.get(ckey)
        if p is not None:
            self._packs[key] = self._with_splits(p, geo)
            return self._packs[key]
        halves, biases, meta = [], [], []
        hoff = boff = 0
        f32 = self.prec == _lib.PREC_F32R
        for (w, b, cin, cout, level, perm_arr, edge), cfg in zip(self._h8_convs, cfgs):
            bm = L.rrin_conv_h8_cfg_bm(cfg)
            if f32:  # fp32 records: unscaled fp32 weights (offsets in floats)
                bp = np.empty(L.rrin_pack_bias_floats(cout, bm), np.float32)
                pa = perm_arr.ctypes.data if perm_arr is not None else None
                if L.rrin_conv_h8_cfg_wino(cfg) == 14:  # Winograd F(4,3) x F(2,3)
                    wp = np.empty(L.rrin_pack_conv3x3_wino42_floats(cout, cin), np.float32)
                    _lib.check(L.rrin_pack_conv3x3_wino42(w.ctypes.data, b.ctypes.data, cout, cin, pa,
                                                          wp.ctypes.data, bp.ctypes.data), "rrin_pack_conv3x3_wino42")
                elif L.rrin_conv_h8_cfg_wino(cfg) > 0:  # Winograd F(2x2,3x3): transformed weights
                    wp = np.empty(L.rrin_pack_conv3x3_wino_bm_floats(cout, cin, bm), np.float32)
                    _lib.check(L.rrin_pack_conv3x3_wino_bm(w.ctypes.data, b.ctypes.data, cout, cin, bm, pa,
                                                           wp.ctypes.data, bp.ctypes.data), "rrin_pack_conv3x3_wino_bm")
                else:
                    wp = np.empty(L.rrin_pack_conv3x3_r32_floats(cout, cin, bm), np.float32)
                    _lib.check(L.rrin_pack_conv3x3_r32(w.ctypes.data, b.ctypes.data, cout, cin, bm, pa,
                                                       wp.ctypes.data, bp.ctypes.data), "rrin_pack_conv3x3_r32")
                meta.append((hoff, None, boff, cfg, 1.0, edge))
                halves.append(wp)
                hoff += wp.size
                biases.append(bp)
                boff += bp.size
                continue
            if L.rrin_conv_h8_cfg_wino(cfg) > 0:  # fp16 Winograd: U = G g G^T in fp16 (conv_winoh.hip)
                nh = L.rrin_pack_conv3x3_wino_h8_halves(cout, cin, bm)
                whi = np.empty(nh, np.uint16)
                bp = np.empty(L.rrin_pack_bias_floats(cout, bm), np.float32)
                inv = C.c_float()
                _lib.check(L.rrin_pack_conv3x3_wino_h8(
                    w.ctypes.data, b.ctypes.data, cout, cin, bm,
                    perm_arr.ctypes.data if perm_arr is not None else None, whi.ctypes.data, bp.ctypes.data,
                    C.byref(inv)), "rrin_pack_conv3x3_wino_h8")
                meta.append((hoff, None, boff, cfg, inv.value, edge))
                halves.append(whi)
                hoff += nh
                biases.append(bp)
                boff += bp.size
                continue
            nh = L.rrin_pack_conv3x3_h8_halves(cout, cin, bm)
            whi = np.empty(nh, np.uint16)
            wlo = np.empty(nh, np.uint16) if self.prec == _lib.PREC_F16X3 else None
            bp = np.empty(L.rrin_pack_bias_floats(cout, bm), np.float32)
            inv = C.c_float()
            _lib.check(L.rrin_pack_conv3x3_h8(
                w.ctypes.data, b.ctypes.data, cout, cin, bm,
                perm_arr.ctypes.data if perm_arr is not None else None, self.prec, whi.ctypes.data,
                wlo.ctypes.data if wlo is not None else None, bp.ctypes.data, C.byref(inv)),
                "rrin_pack_conv3x3_h8")
            meta.append((hoff, hoff + nh if wlo is not None else None, boff, cfg, inv.value, edge))
            halves.append(whi)
            hoff += nh
            if wlo is not None:
                halves.append(wlo)
                hoff += nh
            biases.append(bp)
            boff += bp.size
        elem = 4 if f32 else 2  # bytes per packed weight
        cat = np.concatenate(halves)
        blob = torch.from_numpy(cat if f32 else cat.view(np.int16)).to(self.device)
        bias_blob = torch.from_numpy(np.concatenate(biases)).to(self.device)
        hb, bb = blob.data_ptr(), bias_blob.data_ptr()
        table = (_lib.ConvWeights * len(meta))()
        for i, (ho, lo, bo, cfg, inv, edge) in enumerate(meta):
            e = table[i]
            e.whi = hb + elem * ho
            e.wlo = hb + elem * lo if lo is not None else None
            e.bias = bb + 4 * bo
            e.cfg = cfg
            e.inv_wscale = inv
            if edge is not None:
                e.subpixel = 1
                e.wedge = edge[0].data_ptr()
                e.bias_raw = edge[1].data_ptr()
        if FUSE_L0 and self.prec == _lib.PREC_F16:
            for i in self._block0:  # both convs on direct-form packs (the fused kernel's weights)
                if self._h8_convs[i][2] >= 32 and FUSE_L0 < 2:
                    continue  # the up block's conv_block (cat input): unfused below FUSE_L0 = 2
                if not (L.rrin_conv_h8_cfg_wino(cfgs[i]) or L.rrin_conv_h8_cfg_wino(cfgs[i + 1])):
                    table[i].fuse_next = 1
        p = (blob, bias_blob, table, cfgs)
        self._packs_by_cfgs[ckey] = p
        self._packs[key] = self._with_splits(p, geo)
        return self._packs[key]

    def _with_splits(self, p, geo):
        """The packing p with the split-K slices of geometry ``geo`` (per conv) set in a
        copy of its ConvWeights table (the weight blobs stay shared)."""
        if self.prec != _lib.PREC_F32R:
            return p
        blob, bias_blob, table, cfgs = p
        ks = [choose_split(level, cfg, g)
              for (_, _, cin, cout, level, _, _), cfg, g in zip(self._h8_convs, cfgs, geo)]
        if not any(ks):
            self._set_fold(table, cfgs)
            return p
        t2 = (_lib.ConvWeights * len(table))()
        C.memmove(t2, table, C.sizeof(table))
        for i, k in enumerate(ks):
            t2[i].ksplit = k
        self._set_fold(t2, cfgs)
        return (blob, bias_blob, t2, cfgs)

    def _set_fold(self, table, cfgs):
        """subpixel = 2 (ring folded into the conv) where the conv can fold, else 1."""
        for i, cfg in enumerate(cfgs):
            if table[i].subpixel:
                fold = (RING_FOLD and self.prec == _lib.PREC_F32R and table[i].ksplit <= 1
                        and self.lib.rrin_conv_h8_cfg_wino(cfg) == 3)
                table[i].subpixel = 2 if fold else 1

    force_size_class = None  # A/B knob: use this tile-table class for every forward part

    def conv_algorithm(self, n: int, h: int, w: int) -> str:
        """'winograd', 'direct' or 'mixed': the form of the body convs of a forward part."""
        if self.prec == _lib.PREC_F32:
            return "direct"
        t = self.conv_table_for(n, h, w)
        k = sum(1 for i in range(self.expected_convs) if self.lib.rrin_conv_h8_cfg_wino(t[i].cfg))
        return "winograd" if k == self.expected_convs else ("direct" if k == 0 else "mixed")

    def conv_table_for(self, n: int, h: int, w: int):
        """ConvWeights table of a forward part of n pairs at h x w (its tile-table size class)."""
        if self.force_size_class is not None and self.prec != _lib.PREC_F32:
            return self._pack_h8(self.force_size_class, h, w)[2]
        if self.prec == _lib.PREC_F32:
            if size_class(n * h * w) != "small":
                return self.conv_table
            if self._table32_small is None:
                # sweep at 640x368 x 1 (profiles/r01_v13/tune_fp32_640x368x1.txt): BM 64 x TH 4
                # (cfg 4) beats BM 64 x TH 8 (cfg 1) on every level 1-3 conv, 2.18 -> 1.46 ms;
                # same BM, so the same packed weights
                L = self.lib
                if L.rrin_conv_cfg_bm(4) != L.rrin_conv_cfg_bm(1):
                    raise RuntimeError("fp32 small-class tiles need cfg 1 and 4 to share BM")
                t = (_lib.ConvWeights * len(self.cfgs))()
                C.memmove(t, self.conv_table, C.sizeof(self.conv_table))
                for i, lvl in enumerate(self._levels32):
                    if lvl >= 1 and t[i].cfg == 1:
                        t[i].cfg = 4
                self._table32_small = t
            return self._table32_small
        return self._pack_h8(size_class(n * h * w), h, w)[2]

    def workspace(self, n: int, h: int, w: int, slot: int = 0) -> torch.Tensor:
        key = (n, h, w, slot)
        ws = self._ws.get(key)
        if ws is None:
            nbytes = self.lib.rrin_net_workspace_bytes(n, h, w, self.prec)
            if nbytes < 0:
                _lib.check(int(nbytes), "rrin_net_workspace_bytes")
            while len(self._ws) >= self.MAX_WORKSPACES:
                lru = next(iter(self._ws))   # least recently used part: evict its whole shape
                for old in [k for k in self._ws if k[1:3] == lru[1:3]]:
                    del self._ws[old]
                    self._flow_valid.pop(old, None)
                    for sk in [k for k in self._scratch if k[0] == old]:
                        del self._scratch[sk]
            ws = torch.zeros(int(nbytes), dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
            self._flow_valid[key] = False
        else:
            self._ws.move_to_end(key)
        return ws

    def scratch(self, key, desc, query) -> torch.Tensor | None:
        """Split-K / ring fix-up scratch of workspace ``key`` for the conv table of ``desc``
        (rrin_net_scratch_bytes / rrin_unet_scratch_bytes; None when the schedule needs none),
        zero-filled once, cached per workspace and table."""
        sk = (key, C.addressof(desc.convs.contents))
        if sk in self._scratch:
            return self._scratch[sk]
        nbytes = int(query(C.byref(desc)))
        if nbytes < 0:
            _lib.check(nbytes, "rrin_net_scratch_bytes")
        sc = torch.zeros(nbytes, dtype=torch.uint8, device=self.device) if nbytes > 0 else None
        self._scratch[sk] = sc
        return sc

    def _net_scratch(self, n: int, h: int, w: int, slot: int):
        """The scratch of Net forward part (n, h, w, slot) for its conv table (cached)."""
        d = _lib.NetDesc()
        d.n, d.h, d.w, d.prec = n, h, w, self.prec
        d.convs = self.conv_table_for(n, h, w)
        return self.scratch((n, h, w, slot), d, self.lib.rrin_net_scratch_bytes)

    side_priority = 0  # torch.cuda.Stream priority of the side streams (-1: high)

    def _side_streams(self, k: int):
        if len(self._sides) < k:
            self._sides += [torch.cuda.Stream(self.device, priority=self.side_priority)
                            for _ in range(k - len(self._sides))]
        return self._sides[:k]

    def forward(self, i0: torch.Tensor, i1: torch.Tensor, t=0.5, prof=None, reuse_flow: bool = False,
                streams: int | None = 1, split=None, taps: dict | None = None) -> torch.Tensor:
        """One Net.forward.  ``reuse_flow=True`` promises that (i0, i1) is the pair
        of the previous call with the same shape: the Flow U-Net (t-independent,
        model.py:35, 30 % of the FLOPs) is skipped and its kept raw output is
        re-blended for this t.  ``streams > 1`` splits the batch
        into that many contiguous parts, each with its own workspace, enqueued
        on its own HIP stream: the parts' kernels overlap, filling each other's
        launch gaps and last-wave tails (pairs are independent, so the output is
        bitwise the same).  ``split`` gives the part sizes explicitly.  ``streams=None``: the
        precision's default (``default_streams``).

        ``taps`` (test / debug, one stream only): a dict that receives the four
        U-Nets' raw outputs (their ``last`` conv before the model.py glue,
        unet.py:51 as used at model.py:35,42,52,62) as NCHW fp32 tensors under
        "Flow", "refine_flow", "Mask", "final"."""
        if i0.device != self.device or i1.device != self.device:
            raise RuntimeError(f"inputs on {i0.device}/{i1.device}, model on {self.device}")
        if i0.dtype != torch.float32 or i1.dtype != torch.float32:
            raise TypeError("rrin_amd.Net computes in fp32; inputs must be float32")
        if i0.dim() != 4 or i0.shape != i1.shape or i0.shape[1] != 3:
            raise ValueError(f"expected two [N,3,H,W] tensors, got {tuple(i0.shape)} / {tuple(i1.shape)}")
        n, _, h, w = i0.shape
        if h % 16 or w % 16 or n < 1:
            raise RuntimeError(f"H and W must be multiples of 16 (the Flow U-Net pools 4 times); "
                               f"got {h}x{w} (reference fails at model.py:41)")
        if streams is None:
            streams = default_streams(self.precision, n)
        self._poll_range()
        i0 = i0.contiguous()
        i1 = i1.contiguous()
        out = torch.empty_like(i0)
        coef = t_coefficients(t, n).to(self.device, non_blocking=True)
        bounds = self._bounds(n, streams, split)
        k = len(bounds)
        tapbuf = None
        if taps is not None:
            if len(bounds) != 1:
                raise ValueError("taps need a single forward part (streams=1)")
            if reuse_flow:
                raise ValueError("taps need the Flow U-Net to run (reuse_flow=False)")
            tapbuf = torch.full((13 * n * h * w,), float("nan"), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            main = torch.cuda.current_stream(self.device)
            # workspaces and split scratch first: a new one is zero-filled on the main stream,
            # before the fork (a side stream only waits for what main enqueued before it)
            wss = [self.workspace(hi - lo, h, w, j) for j, (lo, hi) in enumerate(bounds)]
            for j, (lo, hi) in enumerate(bounds):
                self._net_scratch(hi - lo, h, w, j)
            sides = self._side_streams(k - 1)
            for s in sides:
                s.wait_stream(main)
            for j, (lo, hi) in enumerate(bounds):
                st = main if j == 0 else sides[j - 1]
                self._forward_part(i0[lo:hi], i1[lo:hi], out[lo:hi], coef[lo:hi], j, wss[j], st, prof, reuse_flow,
                                   tapbuf)
            for s in sides:
                main.wait_stream(s)
        if tapbuf is not None:
            off = 0
            for name, c in zip(UNET_ORDER, (4, 4, 2, 3)):
                taps[name] = tapbuf[off:off + n * c * h * w].view(n, c, h, w)
                off += n * c * h * w
        return out

    def unet_forward(self, x: torch.Tensor) -> torch.Tensor:
        """The single packed U-Net (engine built with one unit) on x [N,C,H,W]:
        rrin_unet_fwd, the reference UNet.forward (unet.py:40-51)."""
        if len(self.units) != 1:
            raise RuntimeError("unet_forward needs an engine built for one U-Net")
        _, unet, _ = self.units[0]
        if x.device != self.device or x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != unet.in_channels:
            raise ValueError(f"expected a float32 [N,{unet.in_channels},H,W] tensor on {self.device}")
        n, c, h, w = x.shape
        if h % 16 or w % 16:
            raise RuntimeError(f"H and W must be multiples of 16, got {h}x{w}")
        x = x.contiguous()
        y = torch.empty((n, unet.n_classes, h, w), dtype=torch.float32, device=self.device)
        d = _lib.UNetDesc()
        d.n, d.h, d.w, d.in_ch, d.out_ch, d.depth, d.prec = n, h, w, c, unet.n_classes, unet.depth, self.prec
        d.x, d.y = x.data_ptr(), y.data_ptr()
        d.convs = self.conv_table_for(n, h, w)
        d.head = self.head_table[0]
        ws = self.workspace(n, h, w, slot=100)   # own workspace: its input channels [C, 16) stay zero
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        sc = self.scratch((n, h, w, 100), d, self.lib.rrin_unet_scratch_bytes)
        if sc is not None:
            d.scratch, d.scratch_bytes = sc.data_ptr(), sc.numel()
        status = self._status_of(100) if self.prec in (_lib.PREC_F16X3, _lib.PREC_F16) else None
        d.status = status.data_ptr() if status is not None else None
        with torch.cuda.device(self.device):
            st = torch.cuda.current_stream(self.device)
            _lib.check(self.lib.rrin_unet_fwd(C.byref(d), C.c_void_p(st.cuda_stream)), "rrin_unet_fwd")
            if status is not None:  # the range guard, checked as the Net's (_poll_range)
                host = torch.empty(1, dtype=torch.int32, pin_memory=True)
                host.copy_(status, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                self._pending_status.append((ev, host))
        return y

    def _bounds(self, n: int, streams, split):
        """Contiguous (lo, hi) pair ranges of the forward parts (one per HIP stream)."""
        if split is not None:  # explicit part sizes (pairs per stream)
            split = [int(c) for c in split]
            if sum(split) != n or min(split) < 1:
                raise ValueError(f"split {split} does not partition a batch of {n}")
            cuts = [0]
            for c in split:
                cuts.append(cuts[-1] + c)
            return list(zip(cuts[:-1], cuts[1:]))
        k = max(1, min(int(streams), n))
        return [(n * j // k, n * (j + 1) // k) for j in range(k)]

    def graph(self, n: int, h: int, w: int, streams: int | None = None, split=None) -> "NetGraph":
        """The forward of n pairs at h x w captured as one HIP graph and cached per (n, h, w, part
        split) on this engine -- the engine is rebuilt when the weights, precision or schedule
        change, so a graph never outlives the packing it captured.  Replaying it enqueues every
        kernel of the forward with one call (no per-launch host work): the launch gaps of a
        small forward part (C2 640x368 x 1: ~150 launches in ~2.9 ms) shrink.  Its inputs, t
        coefficients and output live in static device buffers (``NetGraph.i0 / i1 / out``); the
        bits are those of :meth:`forward` (same launches, same buffers' layout;
        ``tests/test_gpu_graph.py``).  reuse_flow and taps are eager-only."""
        if h % 16 or w % 16 or n < 1:
            raise RuntimeError(f"H and W must be multiples of 16, got {h}x{w}")
        if streams is None:
            streams = default_streams(self.precision, n)
        bounds = self._bounds(n, streams, split)
        key = (n, h, w, tuple(bounds))
        g = self._graphs.get(key)
        if g is None:
            g = NetGraph(self, n, h, w, bounds)
            self._graphs[key] = g
        return g

    def _net_desc(self, i0, i1, out, coef, ws, sc, status, skip, prof, tapbuf):
        n, _, h, w = i0.shape
        d = _lib.NetDesc()
        d.n, d.h, d.w = n, h, w
        d.i0, d.i1, d.out, d.coef = i0.data_ptr(), i1.data_ptr(), out.data_ptr(), coef.data_ptr()
        d.convs = self.conv_table_for(n, h, w)
        d.heads = self.head_table
        d.workspace = ws.data_ptr()
        d.workspace_bytes = ws.numel()
        d.skip_flow = 1 if skip else 0
        d.prec = self.prec
        d.prof = prof
        d.taps = tapbuf.data_ptr() if tapbuf is not None else None
        if sc is not None:
            d.scratch, d.scratch_bytes = sc.data_ptr(), sc.numel()
        d.status = status.data_ptr() if status is not None else None
        return d

    def _queue_status(self, slot, stream):
        """Copy part `slot`'s fp16 range flag to the host behind the work enqueued on `stream`
        (checked by the next forward / check_range without a sync)."""
        st = self._status.get(slot)
        if st is None:
            return
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(stream):
            host.copy_(st, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._pending_status.append((ev, host))

    def _forward_part(self, i0, i1, out, coef, slot, ws, stream, prof, reuse_flow, tapbuf=None):
        n, _, h, w = i0.shape
        key = (n, h, w, slot)
        skip = bool(reuse_flow) and self._flow_valid.get(key, False)
        sc = self._net_scratch(n, h, w, slot)  # allocated (and zero-filled) before the fork
        st = self._status_of(slot) if self.prec in (_lib.PREC_F16X3, _lib.PREC_F16) else None
        d = self._net_desc(i0, i1, out, coef, ws, sc, st, skip, prof, tapbuf)
        _lib.check(self.lib.rrin_net_fwd(C.byref(d), C.c_void_p(stream.cuda_stream)), "rrin_net_fwd")
        self._flow_valid[key] = True
        if st is not None:
            self._queue_status(slot, stream)

    # ---- fp16 range guard (fp32_split16 / fp16) ---------------------------------
    # Activations of these precisions are stored as fp16; a value beyond 65504
    # sets the forward's status flag and poisons its output with NaN (device
    # side, no sync).  The flag is also checked on the host: the next forward
    # raises once the flagged one has finished, and check_range() waits and raises.
    def _status_of(self, slot):
        st = self._status.get(slot)
        if st is None:
            st = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._status[slot] = st
        return st

    def _poll_range(self, wait: bool = False):
        keep = []
        for ev, host in self._pending_status:
            if wait:
                ev.synchronize()
            elif not ev.query():
                keep.append((ev, host))
                continue
            if int(host.item()) != 0:
                self._pending_status = []
                raise RuntimeError(
                    f"rrin_amd: an activation exceeded the fp16 range (|v| > 65504) in precision "
                    f"'{self.precision}'; the affected outputs are NaN.  Use precision='fp32' (exact fp32).")
        self._pending_status = keep

    def check_range(self):
        """Wait for every forward issued so far and raise if one overflowed fp16."""
        self._poll_range(wait=True)


class NetGraph:
    """One captured forward (RRINEngine.graph): static inputs ``i0`` / ``i1`` [n,3,h,w], output
    ``out``, device t coefficients.  :meth:`replay` writes the coefficients of t (only when t
    changes: a pinned host row, copied stream-ordered before the graph) and replays the graph on
    the current stream; ``out`` then holds the frames until the next replay."""

    def __init__(self, eng: RRINEngine, n: int, h: int, w: int, bounds):
        dev = eng.device
        self.eng, self.n, self.h, self.w, self.bounds = eng, n, h, w, bounds
        self.i0 = torch.zeros((n, 3, h, w), dtype=torch.float32, device=dev)
        self.i1 = torch.zeros_like(self.i0)
        self.out = torch.zeros_like(self.i0)
        self.coef = torch.zeros((n, 8), dtype=torch.float32, device=dev)
        self._coef_host = torch.zeros((n, 8), dtype=torch.float32, pin_memory=True)
        self._coef_ev = None
        self._t = None
        with torch.no_grad(), torch.cuda.device(dev):
            # an eager forward of the same parts first: workspaces, scratch, range flags, side
            # streams and the packing are allocated outside the capture (nothing allocates inside)
            eng.forward(self.i0, self.i1, 0.5, split=[hi - lo for lo, hi in bounds])
            eng._poll_range(wait=True)
            torch.cuda.synchronize(dev)
            self.ws = [eng.workspace(hi - lo, h, w, j) for j, (lo, hi) in enumerate(bounds)]
            self.sc = [eng._net_scratch(hi - lo, h, w, j) for j, (lo, hi) in enumerate(bounds)]
            prec16 = eng.prec in (_lib.PREC_F16X3, _lib.PREC_F16)
            self.status = [eng._status_of(j) if prec16 else None for j in range(len(bounds))]
            sides = eng._side_streams(len(bounds) - 1)
            self.graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.graph(self.graph, stream=cap):
                main = torch.cuda.current_stream(dev)
                for s in sides:
                    s.wait_stream(main)
                for j, (lo, hi) in enumerate(bounds):
                    st = main if j == 0 else sides[j - 1]
                    d = eng._net_desc(self.i0[lo:hi], self.i1[lo:hi], self.out[lo:hi], self.coef[lo:hi],
                                      self.ws[j], self.sc[j], self.status[j], False, None, None)
                    _lib.check(eng.lib.rrin_net_fwd(C.byref(d), C.c_void_p(st.cuda_stream)), "rrin_net_fwd (capture)")
                for s in sides:
                    main.wait_stream(s)
            torch.cuda.current_stream(dev).wait_stream(cap)

    def replay(self, t=0.5) -> torch.Tensor:
        eng = self.eng
        eng._poll_range()
        st = torch.cuda.current_stream(eng.device)
        key = t.detach().cpu().numpy().tobytes() if isinstance(t, torch.Tensor) else float(t)
        if key != self._t:
            if self._coef_ev is not None:
                self._coef_ev.synchronize()  # the previous upload has read the pinned row
            self._coef_host.copy_(t_coefficients(t, self.n))
            self.coef.copy_(self._coef_host, non_blocking=True)
            self._coef_ev = torch.cuda.Event()
            self._coef_ev.record(st)
            self._t = key
        self.graph.replay()
        for j, s in enumerate(self.status):
            if s is not None:
                eng._queue_status(j, st)
        return self.out
