"""CPU: the C-ABI library loads, exports every symbol include/rrin_hip.h
declares, and its host-only entry points (packing, geometry, workspace plan,
error strings) behave.  No kernel is launched here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from rrin_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rrin_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rrin_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_all_declared_symbols():
    lib = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    raw = C.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(raw, s)]
    assert not missing, missing
    # the Python binding covers exactly the declared surface
    assert sorted(_lib.SIGNATURES) == syms
    assert lib.rrin_abi_version() == _lib.ABI_VERSION


def test_strerror_and_geom():
    lib = _lib.lib()
    for code in (0, -1, -2, -3, -4):
        assert lib.rrin_strerror(code)
    g = _lib.geom(720, 1280)
    assert (g.h, g.w, g.hp, g.wp) == (720, 1280, 722, 1344)
    assert g.plane == 722 * 1344
    g = _lib.geom(45, 80)
    assert (g.hp, g.wp) == (50, 160)


def test_conv_counts_and_workspace():
    lib = _lib.lib()
    assert lib.rrin_net_conv_count() == 77  # 81 convs - 4 fused heads
    assert lib.rrin_net_workspace_bytes(1, 720, 1280, 0) > 0
    assert lib.rrin_net_workspace_bytes(1, 72, 80, 0) < 0   # not /16
    assert lib.rrin_net_workspace_bytes(4, 736, 1280, 1) > 3 * lib.rrin_net_workspace_bytes(1, 736, 1280, 1)
    for cfg in range(lib.rrin_conv_cfg_count()):
        assert lib.rrin_conv_cfg_bm(cfg) % 32 == 0
        assert 16 % lib.rrin_conv_cfg_th(cfg) == 0
    assert lib.rrin_conv_cfg_bm(99) < 0


@pytest.mark.parametrize("cout,cin,bm,perm", [(32, 6, 32, None), (64, 32, 64, None),
                                              (256, 512, 128, None), (40, 10, 32, "rev")])
def test_pack_layout(cout, cin, bm, perm):
    lib = _lib.lib()
    rng = np.random.default_rng(0)
    w = rng.standard_normal((cout, cin, 3, 3)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    p = np.arange(cin, dtype=np.int32)[::-1].copy() if perm else None
    nw = lib.rrin_pack_conv3x3_floats(cout, cin, bm)
    nb = lib.rrin_pack_bias_floats(cout, bm)
    wp = np.full(nw, np.nan, np.float32)
    bp = np.full(nb, np.nan, np.float32)
    rc = lib.rrin_pack_conv3x3(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                               p.ctypes.data if p is not None else None, wp.ctypes.data, bp.ctypes.data)
    assert rc == 0
    cob, nch = -(-cout // bm), -(-cin // 8)
    arr = wp.reshape(cob, nch, 8, 9, bm)
    wpad = np.zeros((cob * bm, nch * 8, 3, 3), np.float32)
    src = w[:, p] if p is not None else w
    wpad[:cout, :cin] = src
    ref = wpad.reshape(cob, bm, nch, 8, 9).transpose(0, 2, 3, 4, 1)
    np.testing.assert_array_equal(arr, ref)
    np.testing.assert_array_equal(bp[:cout], b)
    assert not bp[cout:].any()


def test_pack_rejects_bad_args():
    lib = _lib.lib()
    w = np.zeros((32, 6, 3, 3), np.float32)
    b = np.zeros(32, np.float32)
    out = np.zeros(lib.rrin_pack_conv3x3_floats(32, 6, 32), np.float32)
    bo = np.zeros(32, np.float32)
    bad = np.array([0, 1, 2, 3, 4, 9], np.int32)
    assert lib.rrin_pack_conv3x3(w.ctypes.data, b.ctypes.data, 32, 6, 32, bad.ctypes.data,
                                 out.ctypes.data, bo.ctypes.data) == -2
    assert lib.rrin_pack_conv3x3(w.ctypes.data, b.ctypes.data, 32, 6, 48, None,
                                 out.ctypes.data, bo.ctypes.data) == -2


def _h2f(bits):
    return bits.view(np.float16).astype(np.float64)


@pytest.mark.parametrize("cout,cin,bm,prec", [(32, 6, 32, 1), (64, 32, 64, 1), (128, 256, 64, 2), (40, 10, 32, 1)])
def test_pack_h8_layout_and_split(cout, cin, bm, prec):
    """[cob][16-ch chunk][tap][half][bm][8] halves; weights scaled by 2^s with
    max|w|*2^s in [2^12, 2^13); hi+lo reproduces w*2^s to 2^-22 (split mode)."""
    lib = _lib.lib()
    rng = np.random.default_rng(1)
    w = (rng.standard_normal((cout, cin, 3, 3)) * 0.05).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    nh = lib.rrin_pack_conv3x3_h8_halves(cout, cin, bm)
    whi = np.zeros(nh, np.uint16)
    wlo = np.zeros(nh, np.uint16)
    bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
    inv = C.c_float()
    rc = lib.rrin_pack_conv3x3_h8(w.ctypes.data, b.ctypes.data, cout, cin, bm, None, prec, whi.ctypes.data,
                                  wlo.ctypes.data if prec == 1 else None, bp.ctypes.data, C.byref(inv))
    assert rc == 0
    scale = 1.0 / inv.value
    assert scale == 2.0 ** round(np.log2(scale))
    assert 2 ** 12 <= np.abs(w).max() * scale < 2 ** 13
    cob, nch = -(-cout // bm), -(-cin // 16)
    rec = _h2f(whi) + (_h2f(wlo) / 2048.0 if prec == 1 else 0)
    rec = rec.reshape(cob, nch, 9, 2, bm, 8)
    # back to [co][ci][tap]
    got = rec.transpose(0, 4, 1, 3, 5, 2).reshape(cob * bm, nch * 16, 9)[:cout, :cin] / scale
    ref = w.reshape(cout, cin, 9).astype(np.float64)
    tol = 2.0 ** -21 if prec == 1 else 2.0 ** -10
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max()
    np.testing.assert_array_equal(bp[:cout], b)


def test_h8_geometry_and_cfgs():
    lib = _lib.lib()
    g = _lib.geom_h8(720, 1280)
    assert (g.hp, g.wp) == (722, 1296)
    ok = [lib.rrin_conv_h8_cfg_ok(c, 1) for c in range(lib.rrin_conv_h8_cfg_count())]
    assert ok[0] == 1 and ok[1] == 1
    # every config runs fp16, except the Winograd one (exact fp32 on fp32 records only)
    assert all(lib.rrin_conv_h8_cfg_ok(c, 2) != lib.rrin_conv_h8_cfg_wino(c)
               for c in range(lib.rrin_conv_h8_cfg_count()))
    for prec in (0, 1, 2):
        assert lib.rrin_net_workspace_bytes(2, 64, 96, prec) > 0
    # weight-resident configs (all weight chunks in LDS) fit small cin only
    for c in range(lib.rrin_conv_h8_cfg_count()):
        assert lib.rrin_conv_h8_cfg_fits(c, 1, 16) == ok[c]
    assert lib.rrin_conv_h8_cfg_fits(9, 1, 64) == 1 and lib.rrin_conv_h8_cfg_fits(9, 1, 128) == 0
    assert lib.rrin_conv_h8_cfg_fits(8, 1, 512) == 0 and lib.rrin_conv_h8_cfg_fits(0, 1, 512) == 1


def _h8_view(h, w, groups, base=1 << 30):
    hp, wp = (h + 15) // 16 * 16 + 2, (w + 31) // 32 * 32 + 16
    g = _lib.Geom(h, w, hp, wp, hp * wp)
    return _lib.H8(base, None, groups * hp * wp, 0, groups, g)


@pytest.mark.parametrize("wino", [False, True])
def test_h8_dma_source_span_limit(wino):
    """the LDS-DMA staging addresses a source through buffer resources with
    32-bit byte offsets, so a source whose staged span reaches 2 GB must be rejected (RRIN_E_SHAPE)
    instead of staging zeros.  Host-only size query: nothing is launched or dereferenced."""
    lib = _lib.lib()
    ncfg = lib.rrin_conv_h8_cfg_count()
    if wino:   # kind 6 at fp16 (conv_winoh.hip)
        cfg = next(c for c in range(ncfg) if lib.rrin_conv_h8_cfg_wino(c) == 6)
    else:      # a direct-form LDS-DMA tile
        cfg = next(c for c in range(ncfg)
                   if lib.rrin_conv_h8_cfg_wino(c) == 0 and lib.rrin_conv_h8_cfg_ok(c, _lib.PREC_F16) == 1)

    def query(h, w, cin=64):
        d = _lib.ConvH8Desc()
        d.n, d.cin, d.cout, d.cfg, d.prec = 1, cin, 64, cfg, _lib.PREC_F16
        d.epi_mode, d.slope, d.inv_wscale = _lib.EPI_LEAKY, 0.1, 1.0
        d.src, d.dst = _h8_view(h, w, cin // 8), _h8_view(h, w, 8)
        d.whi = d.bias = 1 << 30
        return lib.rrin_conv_h8_split_floats(C.byref(d), None)

    ok = query(736, 1280)
    assert ok >= 0, ok
    # 64 fp16 channels = 8 record groups: the direct form stages all 8 (2.2 GB at 6144x3456)
    assert query(3456, 6144) == (ok if wino else -1)
    # the Winograd tiles stage from one base per tile and chunk: 3 planes must stay below 2 GB
    assert query(11776, 11776) == -1
