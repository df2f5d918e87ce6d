"""ctypes binding of ``librrin_hip.so`` (C ABI declared in include/rrin_hip.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) and
loaded from ``rrin_amd/librrin_hip.so``.  There is no fallback: if the library
is missing or its ABI version differs, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 19
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librrin_hip.so")
# A/B sessions only (tools/sessions/): another build of the same library, e.g. ab/librrin_hip_X.so
if os.environ.get("RRIN_LIB_AB"):
    LIB_PATH = os.path.abspath(os.environ["RRIN_LIB_AB"])

# enums (rrin_hip.h)
SRC_DIRECT, SRC_UPSAMPLE2X = 0, 1
EPI_LINEAR, EPI_LEAKY, EPI_LEAKY_POOL, EPI_LEAKY_REP, EPI_SUBPIXEL = 0, 1, 2, 3, 4
KIND_CONV, KIND_HEAD, KIND_LAYOUT, KIND_EDGE = 0, 1, 2, 3
HEAD_PLAIN, HEAD_FLOW, HEAD_REFINE, HEAD_MASK, HEAD_FINAL = 0, 1, 2, 3, 4
PREC_F32, PREC_F16X3, PREC_F16, PREC_F32R = 0, 1, 2, 3
# "fp32": exact fp32 on the record layout (F32R); "fp32_planar": exact fp32 on the
# planar PP layout (the first implementation, kept for A/B); "fp32_split16":
# fp32-emulated (fp16 hi+lo x3); "fp16"
PRECISIONS = {"fp32": PREC_F32R, "fp32_planar": PREC_F32, "fp32_split16": PREC_F16X3, "fp16": PREC_F16}
RECORD_PRECS = (PREC_F16X3, PREC_F16, PREC_F32R)


def chans_per_record(prec: int) -> int:
    """Channels of one 16-B record of the record layout: 4 fp32 or 8 halves."""
    return 4 if prec == PREC_F32R else 8


class Geom(C.Structure):
    _fields_ = [("h", C.c_int32), ("w", C.c_int32), ("hp", C.c_int32), ("wp", C.c_int32),
                ("plane", C.c_int64)]


class PP(C.Structure):
    _fields_ = [("base", C.c_void_p), ("img_stride", C.c_int64), ("ch_off", C.c_int32),
                ("channels", C.c_int32), ("g", Geom)]


class ConvDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("cfg", C.c_int32),
                ("src_mode", C.c_int32), ("epi_mode", C.c_int32), ("slope", C.c_float),
                ("src", PP), ("dst", PP), ("pool", PP), ("wpack", C.c_void_p), ("bias", C.c_void_p)]


class HeadDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("mode", C.c_int32),
                ("src", PP), ("g16", PP), ("w", C.c_void_p), ("bias", C.c_void_p),
                ("coef", C.c_void_p), ("out", C.c_void_p), ("flow_raw", PP), ("raw_out", C.c_void_p)]


class ConvWeights(C.Structure):
    _fields_ = [("wpack", C.c_void_p), ("bias", C.c_void_p), ("cfg", C.c_int32), ("inv_wscale", C.c_float),
                ("whi", C.c_void_p), ("wlo", C.c_void_p), ("subpixel", C.c_int32), ("ksplit", C.c_int32),
                ("wedge", C.c_void_p), ("bias_raw", C.c_void_p), ("fuse_next", C.c_int32), ("pad_", C.c_int32)]


class H8(C.Structure):
    _fields_ = [("hi", C.c_void_p), ("lo", C.c_void_p), ("img_stride", C.c_int64), ("g_off", C.c_int32),
                ("groups", C.c_int32), ("g", Geom)]


class ConvH8Desc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("cfg", C.c_int32),
                ("prec", C.c_int32), ("epi_mode", C.c_int32), ("slope", C.c_float), ("inv_wscale", C.c_float),
                ("tail_finite", C.c_int32), ("pad_", C.c_int32), ("src", H8), ("dst", H8), ("pool", H8), ("whi", C.c_void_p), ("wlo", C.c_void_p),
                ("bias", C.c_void_p), ("edge", C.c_void_p), ("status", C.c_void_p), ("ksplit", C.c_int32),
                ("pad2_", C.c_int32), ("part", C.c_void_p), ("cnt", C.c_void_p), ("ring_w", C.c_void_p),
                ("ring_bias", C.c_void_p), ("ring_corr", C.c_void_p), ("ring_cnt", C.c_void_p),
                ("ring_full", C.c_void_p)]


class Block0Desc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cfg_a", C.c_int32), ("cfg_b", C.c_int32),
                ("slope", C.c_float), ("inv_wscale_a", C.c_float), ("inv_wscale_b", C.c_float),
                ("tail_finite", C.c_int32), ("src", H8), ("dst", H8), ("pool", H8), ("whi_a", C.c_void_p),
                ("bias_a", C.c_void_p), ("whi_b", C.c_void_p), ("bias_b", C.c_void_p), ("status", C.c_void_p)]


class EdgeFixDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("prec", C.c_int32),
                ("epi_mode", C.c_int32), ("slope", C.c_float), ("src", H8), ("dst", H8),
                ("edge", C.c_void_p), ("wedge", C.c_void_p), ("bias", C.c_void_p), ("status", C.c_void_p),
                ("part", C.c_void_p), ("cnt", C.c_void_p), ("part_floats", C.c_int64), ("cnt_len", C.c_int32),
                ("full", C.c_int32)]


class HeadH8Desc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("mode", C.c_int32),
                ("prec", C.c_int32), ("pad_", C.c_int32), ("src", H8), ("g16", H8), ("w", C.c_void_p),
                ("bias", C.c_void_p), ("coef", C.c_void_p), ("out", C.c_void_p), ("flow_raw", H8),
                ("raw_out", C.c_void_p), ("status", C.c_void_p)]


class HeadWeights(C.Structure):
    _fields_ = [("w", C.c_void_p), ("bias", C.c_void_p)]


class NetDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("pad_", C.c_int32),
                ("i0", C.c_void_p), ("i1", C.c_void_p), ("out", C.c_void_p), ("coef", C.c_void_p),
                ("convs", C.POINTER(ConvWeights)), ("heads", C.POINTER(HeadWeights)),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_int64),
                ("skip_flow", C.c_int32), ("prec", C.c_int32), ("prof", C.c_void_p), ("taps", C.c_void_p),
                ("status", C.c_void_p), ("scratch", C.c_void_p), ("scratch_bytes", C.c_int64)]


class TConvDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("h", C.c_int32), ("w", C.c_int32),
                ("mode", C.c_int32), ("leaky", C.c_int32), ("slope", C.c_float), ("x", C.c_void_p),
                ("y", C.c_void_p), ("wt", C.c_void_p), ("bias", C.c_void_p), ("out", C.c_void_p)]


class TWgradDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("h", C.c_int32), ("w", C.c_int32),
                ("leaky", C.c_int32), ("slope", C.c_float), ("pad_", C.c_int32), ("x", C.c_void_p),
                ("g", C.c_void_p), ("y", C.c_void_p), ("gw", C.c_void_p), ("gb", C.c_void_p),
                ("work", C.c_void_p)]


TCONV_FWD, TCONV_DGRAD = 0, 1


class UNetDesc(C.Structure):
    _fields_ = [("n", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("in_ch", C.c_int32), ("out_ch", C.c_int32),
                ("depth", C.c_int32), ("prec", C.c_int32), ("pad_", C.c_int32), ("x", C.c_void_p), ("y", C.c_void_p),
                ("convs", C.POINTER(ConvWeights)), ("head", HeadWeights), ("workspace", C.c_void_p),
                ("workspace_bytes", C.c_int64), ("prof", C.c_void_p), ("status", C.c_void_p),
                ("scratch", C.c_void_p), ("scratch_bytes", C.c_int64)]


# every symbol include/rrin_hip.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "rrin_make_geom": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(Geom)]),
    "rrin_conv_cfg_count": (C.c_int, []),
    "rrin_conv_cfg_bm": (C.c_int, [C.c_int32]),
    "rrin_conv_cfg_th": (C.c_int, [C.c_int32]),
    "rrin_conv3x3_fwd": (C.c_int, [C.POINTER(ConvDesc), C.c_void_p]),
    "rrin_pack_conv3x3_floats": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_pack_bias_floats": (C.c_int64, [C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_void_p, C.c_void_p, C.c_void_p]),
    "rrin_head_fwd": (C.c_int, [C.POINTER(HeadDesc), C.c_void_p]),
    "rrin_nchw_to_pp": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(PP), C.c_void_p]),
    "rrin_pp_to_nchw": (C.c_int, [C.POINTER(PP), C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "rrin_warp_fwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_net_conv_count": (C.c_int, []),
    "rrin_net_workspace_bytes": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rrin_net_scratch_bytes": (C.c_int64, [C.POINTER(NetDesc)]),
    "rrin_tpack_wino": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "rrin_unet_scratch_bytes": (C.c_int64, [C.POINTER(UNetDesc)]),
    "rrin_make_geom_h8": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(Geom)]),
    "rrin_conv_h8_cfg_count": (C.c_int, []),
    "rrin_conv_h8_cfg_bm": (C.c_int, [C.c_int32]),
    "rrin_conv_h8_cfg_th": (C.c_int, [C.c_int32]),
    "rrin_conv_h8_cfg_ok": (C.c_int, [C.c_int32, C.c_int32]),
    "rrin_conv_h8_cfg_fits": (C.c_int, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_conv3x3_h8_fwd": (C.c_int, [C.POINTER(ConvH8Desc), C.c_void_p]),
    "rrin_conv_block0_h8_fwd": (C.c_int, [C.POINTER(Block0Desc), C.c_void_p]),
    "rrin_conv_h8_cfg_wino": (C.c_int, [C.c_int32]),
    "rrin_conv_h8_split_floats": (C.c_int64, [C.c_void_p, C.c_void_p]),
    "rrin_conv_h8_ring_floats": (C.c_int64, [C.c_void_p, C.c_void_p]),
    "rrin_edge_fix_split_floats": (C.c_int64, [C.c_void_p, C.c_void_p]),
    "rrin_pack_conv3x3_wino_floats": (C.c_int64, [C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3_wino_bm_floats": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3_wino_bm": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                            C.c_void_p, C.c_void_p]),
    "rrin_pack_conv3x3_wino": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                         C.c_void_p]),
    "rrin_pack_conv3x3_wino42_floats": (C.c_int64, [C.c_int32, C.c_int32]),
    "rrin_conv_h8_set_wino42_geom": (C.c_int, [C.c_int32]),
    "rrin_pack_conv3x3_wino42": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
    "rrin_pack_conv3x3_wino_h8_halves": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3_wino_h8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]),
    "rrin_pack_conv3x3_h8_halves": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3_h8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                       C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]),
    "rrin_pack_conv3x3_r32_floats": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rrin_pack_conv3x3_r32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                        C.c_void_p, C.c_void_p]),
    "rrin_subpixel_weights": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                        C.c_void_p]),
    "rrin_ring_pixels": (C.c_int64, [C.c_int32, C.c_int32]),
    "rrin_subpixel_edge_fix_h8": (C.c_int, [C.POINTER(EdgeFixDesc), C.c_void_p]),
    "rrin_upsample2x_h8": (C.c_int, [C.POINTER(H8), C.POINTER(H8), C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_pack_g16_h8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(H8), C.c_int32, C.c_void_p]),
    "rrin_nchw_to_h8": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(H8), C.c_int32,
                                  C.c_void_p]),
    "rrin_h8_to_nchw": (C.c_int, [C.POINTER(H8), C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                  C.c_void_p]),
    "rrin_head_h8_fwd": (C.c_int, [C.POINTER(HeadH8Desc), C.c_void_p]),
    "rrin_flow_tblend_fwd": (C.c_int, [C.POINTER(PP), C.POINTER(PP), C.c_void_p, C.c_int32, C.c_void_p]),
    "rrin_flow_tblend_h8": (C.c_int, [C.POINTER(H8), C.POINTER(H8), C.c_void_p, C.c_int32, C.c_int32,
                                      C.c_void_p]),
    "rrin_net_fwd": (C.c_int, [C.POINTER(NetDesc), C.c_void_p]),
    "rrin_unet_conv_count": (C.c_int64, [C.c_int32]),
    "rrin_unet_fwd": (C.c_int, [C.POINTER(UNetDesc), C.c_void_p]),
    "rrin_prof_create": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    "rrin_prof_destroy": (C.c_int, [C.c_void_p]),
    "rrin_prof_reset": (C.c_int, [C.c_void_p]),
    "rrin_prof_read": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                 C.POINTER(C.c_int32)]),
    "rrin_prof_read_spans": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                       C.POINTER(C.c_int32)]),
    "rrin_tconv3x3": (C.c_int, [C.POINTER(TConvDesc), C.c_void_p]),
    "rrin_tconv3x3_wgrad_work_floats": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rrin_tconv3x3_wgrad": (C.c_int, [C.POINTER(TWgradDesc), C.c_void_p]),
    "rrin_tpool2_fwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_tpool2_bwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_tup2_fwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_tup2_bwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_twarp_bwd_work_bytes": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rrin_twarp_bwd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]),
    "rrin_abi_version": (C.c_int, []),
    "rrin_strerror": (C.c_char_p, [C.c_int]),
}

_LIB = None


class RRINError(RuntimeError):
    pass


def build_id(path: str = LIB_PATH) -> str:
    """First 16 hex digits of the SHA-256 of the library file: names the build a
    measurement came from (profiles/pmc_traffic.json entries carry it; bench.py only
    reports a PMC traffic figure measured on the library it runs)."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def lib():
    """Load (once) and return the library; raises if it is absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RRINError(f"{LIB_PATH} not built: run `make -j16` (or __graft_entry__.build()); "
                            "rrin_amd has no non-HIP fallback")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        # an A/B build of an earlier ABI whose changes since are appends only (RRIN_LIB_AB_ABI=16)
        ok = {ABI_VERSION} | ({int(os.environ.get("RRIN_LIB_AB_ABI", ABI_VERSION))} if os.environ.get("RRIN_LIB_AB") else set())
        if h.rrin_abi_version() not in ok:
            raise RRINError(f"librrin_hip ABI {h.rrin_abi_version()} != expected {ABI_VERSION}")
        _LIB = h
    return _LIB


def check(rc: int, what: str = "rrin"):
    if rc != 0:
        msg = lib().rrin_strerror(rc)
        raise RRINError(f"{what} failed ({rc}): {msg.decode() if msg else '?'}")


def geom(h: int, w: int) -> Geom:
    g = Geom()
    check(lib().rrin_make_geom(h, w, C.byref(g)), "rrin_make_geom")
    return g


def geom_h8(h: int, w: int) -> Geom:
    g = Geom()
    check(lib().rrin_make_geom_h8(h, w, C.byref(g)), "rrin_make_geom_h8")
    return g
