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
    assert lib.rrin_net_workspace_bytes(1, 720, 1280) > 0
    assert lib.rrin_net_workspace_bytes(1, 72, 80) < 0   # not /16
    assert lib.rrin_net_workspace_bytes(4, 736, 1280) > 3 * lib.rrin_net_workspace_bytes(1, 736, 1280)
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
