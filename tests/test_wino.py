"""CPU: the Winograd F(2x2, 3x3) form of the exact-fp32 conv (conv_wino.hip).

The host packing (rrin_pack_conv3x3_wino: U = G g G^T per output/input channel
pair, in double, rounded once to fp32) and the kernel's transforms, restated
here in float64 -- input V = B^T d B per 2x2 output patch, per-point channel
contraction, output Y = A^T M A -- must reproduce the direct 3x3 conv (zero
padding, reference unet.py:29) of the same weights.  The GPU tests
(tests/test_gpu_h8.py, the Winograd config in every config sweep) check the
kernel itself against float64."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib

BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)


def pack_wino(w, b, perm=None):
    lib = _lib.lib()
    cout, cin = w.shape[:2]
    wp = np.zeros(lib.rrin_pack_conv3x3_wino_floats(cout, cin), np.float32)
    bp = np.zeros(lib.rrin_pack_bias_floats(cout, 32), np.float32)
    pa = np.asarray(perm, np.int32) if perm is not None else None
    _lib.check(lib.rrin_pack_conv3x3_wino(w.ctypes.data, b.ctypes.data, cout, cin,
                                          pa.ctypes.data if pa is not None else None, wp.ctypes.data,
                                          bp.ctypes.data))
    return wp, bp


def unpack_u(wp, cout, cin):
    """[cob][chunk of 8][xi][half][co32][4] -> U[xi][co][ci] (float64)."""
    cob, nch = (cout + 31) // 32, (cin + 7) // 8
    u = wp.reshape(cob, nch, 16, 2, 32, 4).transpose(2, 0, 4, 1, 3, 5).reshape(16, cob * 32, nch * 8)
    return u[:, :cout, :cin].astype(np.float64)


def wino_conv(x, u, bias):
    """float64 restatement of the kernel's dataflow: x [cin][h][w] (h, w even)."""
    cin, h, w = x.shape
    xp = np.zeros((cin, h + 2, w + 2))
    xp[:, 1:h + 1, 1:w + 1] = x
    # 4x4 windows at stride 2: [cin][ph][pw][4][4]
    win = np.lib.stride_tricks.sliding_window_view(xp, (4, 4), axis=(1, 2))[:, ::2, ::2]
    v = np.einsum("ab,cpqbd,ed->cpqae", BT, win, BT)              # B^T d B
    m = np.einsum("xoc,cpqx->opqx", u.reshape(16, *u.shape[1:]), v.reshape(*v.shape[:3], 16))
    m = m.reshape(*m.shape[:3], 4, 4)
    y = np.einsum("ra,opqab,sb->oprqs", AT, m, AT)                # A^T M A
    co = y.shape[0]
    return y.reshape(co, h, w) + bias[:, None, None]


@pytest.mark.parametrize("cin,cout", [(6, 32), (10, 32), (32, 64), (64, 32)])
def test_wino_packing_reproduces_direct_conv(cin, cout):
    g = torch.Generator().manual_seed(cin * 1000 + cout)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).numpy()
    b = (torch.randn(cout, generator=g) * 0.1).numpy()
    x = (torch.rand(cin, 12, 18, generator=g) * 2 - 1).numpy()
    wp, bp = pack_wino(w, b)
    np.testing.assert_array_equal(bp[:cout], b)
    assert not bp[cout:].any()
    y = wino_conv(x.astype(np.float64), unpack_u(wp, cout, cin), b.astype(np.float64))
    ref = F.conv2d(torch.from_numpy(x[None]).double(), torch.from_numpy(w).double(),
                   torch.from_numpy(b).double(), padding=1)[0].numpy()
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)


def test_wino_packing_layout_and_perm():
    """Padding channels are zero; the input permutation selects reference channels."""
    cout, cin = 40, 10
    rng = np.random.default_rng(3)
    w = rng.standard_normal((cout, cin, 3, 3)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    perm = [4, 5, 6, 7, 8, 9, 0, 1, 2, 3]
    wp, _ = pack_wino(w, b, perm)
    full = wp.reshape(2, 2, 16, 2, 32, 4).transpose(2, 0, 4, 1, 3, 5).reshape(16, 64, 16)
    assert not full[:, cout:].any() and not full[:, :, cin:].any()
    u_perm = unpack_u(wp, cout, cin)
    u_ref = unpack_u(pack_wino(np.ascontiguousarray(w[:, perm]), b)[0], cout, cin)
    np.testing.assert_array_equal(u_perm, u_ref)
    # point xi = (0, 0) is the corner tap g[0][0] itself (G row 0 = [1 0 0])
    np.testing.assert_array_equal(u_ref[0], w[:, perm, 0, 0].astype(np.float64))


def test_wino_config_entry():
    lib = _lib.lib()
    ids = [c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) > 0]
    # kinds 1 (BM 32, 4 waves), 3 (BM 32, 8 waves of 4 accumulators), TH 8; 4 (kind 3's
    # arithmetic on TH 4 tiles, 4 waves); the register-U tiles 6 (BM 64 x TH 4) and 7 (BM 32 x
    # TH 8), 4 waves; kind 14 (ABI 18, id 25): the register-U tile in F(4,3) x F(2,3), BM 32 x
    # TH 8.  Round 6 removed the rejected kinds 2, 5 and 8-13: ids 19 and 22 stay reserved
    # (kind -1, never usable).
    assert sorted(lib.rrin_conv_h8_cfg_wino(c) for c in ids) == [1, 3, 4, 6, 7, 14]
    assert min(ids) == 18  # the direct-form configs keep ids 0-17 (engine tile tables)
    assert lib.rrin_conv_h8_cfg_count() == 26
    assert lib.rrin_conv_h8_cfg_wino(25) == 14
    assert [lib.rrin_conv_h8_cfg_wino(c) for c in (19, 22)] == [-1, -1]
    assert all(lib.rrin_conv_h8_cfg_ok(c, p) == 0 for c in (19, 22) for p in range(4))
    assert {lib.rrin_conv_h8_cfg_wino(c): lib.rrin_conv_h8_cfg_bm(c) for c in ids} == {
        1: 32, 3: 32, 4: 32, 6: 64, 7: 32, 14: 32}
    for c in ids:
        kind = lib.rrin_conv_h8_cfg_wino(c)
        assert lib.rrin_conv_h8_cfg_th(c) == {4: 4, 6: 4}.get(kind, 8)
        assert lib.rrin_conv_h8_cfg_ok(c, _lib.PREC_F32R) == 1
        # split16 never runs a Winograd tile; fp16 runs kind 6 (conv_winoh.hip)
        assert lib.rrin_conv_h8_cfg_ok(c, _lib.PREC_F16X3) == 0
        assert lib.rrin_conv_h8_cfg_ok(c, _lib.PREC_F16) == (1 if kind == 6 else 0)
    assert lib.rrin_pack_conv3x3_wino_floats(33, 5) == 2 * 1 * 16 * 2 * 32 * 4
    assert lib.rrin_pack_conv3x3_wino_floats(0, 5) < 0
    assert lib.rrin_pack_conv3x3_wino_bm_floats(65, 9, 64) == 2 * 2 * 16 * 2 * 64 * 4
    assert lib.rrin_pack_conv3x3_wino_bm_floats(8, 8, 48) < 0
    assert lib.rrin_pack_conv3x3_wino_h8_halves(65, 17, 64) == 2 * 2 * 16 * 2 * 64 * 8
    assert lib.rrin_pack_conv3x3_wino_h8_halves(64, 16, 32) < 0  # BM 64 only
    assert lib.rrin_pack_conv3x3_wino42_floats(33, 9) == 2 * 2 * 24 * 2 * 32 * 4
    assert lib.rrin_pack_conv3x3_wino42_floats(8, 0) < 0


# F(4,3) (x) and F(2,3) (y) Winograd matrices of kind 14 (conv_winoc42.hip)
BT4 = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float64)
G4 = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
               [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], np.float64)
AT4 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], np.float64)
BT2 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64)
G2 = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64)
AT2 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)


@pytest.mark.parametrize("cout,cin,perm", [(32, 8, False), (72, 40, True), (64, 3, False)])
def test_pack_wino42_layout(cout, cin, perm):
    """Kind-14 packing: [cob 32][8-ch chunk][6 eta + xi][half][32 co][4 ci] of
    U = G2 g G4^T (double, rounded once), zero past cout / cin; and the transform pair it
    belongs to reproduces a 3x3 correlation on a 4-tall x 6-wide window (2 x 4 outputs)."""
    lib = _lib.lib()
    rng = np.random.default_rng(cout * cin)
    w = rng.standard_normal((cout, cin, 3, 3)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    pa = rng.permutation(cin).astype(np.int32) if perm else None
    wp = np.zeros(lib.rrin_pack_conv3x3_wino42_floats(cout, cin), np.float32)
    bp = np.zeros(lib.rrin_pack_bias_floats(cout, 32), np.float32)
    _lib.check(lib.rrin_pack_conv3x3_wino42(w.ctypes.data, b.ctypes.data, cout, cin,
                                            pa.ctypes.data if perm else None, wp.ctypes.data, bp.ctypes.data))
    wperm = w[:, pa] if perm else w
    U = np.einsum("ak,oikl,bl->oiab", G2, wperm.astype(np.float64), G4).reshape(cout, cin, 24)
    cob, nch = -(-cout // 32), -(-cin // 8)
    want = np.zeros((cob * 32, nch * 8, 24))
    want[:cout, :cin] = U
    want = want.reshape(cob, 32, nch, 2, 4, 24).transpose(0, 2, 5, 3, 1, 4).reshape(-1)
    np.testing.assert_array_equal(wp, want.astype(np.float32))
    np.testing.assert_array_equal(bp[:cout], b)
    # the transform: Y = AT2 [(G2 g G4^T) * (BT2 d BT4^T)] AT4^T on a 4 x 6 input window
    d = rng.standard_normal((4, 6))
    g = wperm[0, 0].astype(np.float64)
    Y = AT2 @ ((G2 @ g @ G4.T) * (BT2 @ d @ BT4.T)) @ AT4.T
    ref = np.array([[np.sum(d[r:r + 3, c:c + 3] * g) for c in range(4)] for r in range(2)])
    np.testing.assert_allclose(Y, ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("cout,cin", [(64, 16), (72, 40), (128, 32)])
def test_pack_wino_h8_layout(cout, cin):
    """fp16 Winograd packing: [cob 64][16-ch chunk][xi][half][64 co][8 ci] of fp16(U * 2^s),
    U = G g G^T in double, 2^s putting max|U| in [2^12, 2^13), *inv_wscale = 2^-s."""
    lib = _lib.lib()
    rng = np.random.default_rng(cout + cin)
    w = (rng.standard_normal((cout, cin, 3, 3)) * 0.05).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    nh = lib.rrin_pack_conv3x3_wino_h8_halves(cout, cin, 64)
    whi = np.zeros(nh, np.uint16)
    bp = np.zeros(lib.rrin_pack_bias_floats(cout, 64), np.float32)
    inv = C.c_float()
    _lib.check(lib.rrin_pack_conv3x3_wino_h8(w.ctypes.data, b.ctypes.data, cout, cin, 64, None, whi.ctypes.data,
                                             bp.ctypes.data, C.byref(inv)))
    G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64)
    U = np.einsum("ak,oikl,bl->oiab", G, w.astype(np.float64), G).reshape(cout, cin, 16)
    e = np.frexp(np.abs(U).max())[1]
    assert inv.value == 2.0 ** -(13 - e)
    cob, nch = -(-cout // 64), -(-cin // 16)
    want = np.zeros((cob * 64, nch * 16, 16))
    want[:cout, :cin] = U * 2.0 ** (13 - e)
    # [cob][chunk][xi][hh][co][e] <- want[cob*64 + co][chunk*16 + hh*8 + e][xi]
    want = want.reshape(cob, 64, nch, 2, 8, 16).transpose(0, 2, 5, 3, 1, 4).reshape(-1)
    got = whi.view(np.float16).astype(np.float64)
    np.testing.assert_array_equal(got, want.astype(np.float16).astype(np.float64))
    np.testing.assert_array_equal(bp[:cout], b)
    assert not bp[cout:].any()


def test_split_scratch_size():
    """rrin_conv_h8_split_floats: 16 floats per thread of every (tile, slice) workgroup
    (64 x TH threads), one counter per tile; slices are whole chunks and never empty."""
    import ctypes as C

    import torch

    from rrin_amd.pp import H8Tensor
    lib = _lib.lib()
    q8 = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 3)
    q4 = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 4)
    n, cin, cout, h, w = 2, 96, 64, 46, 80
    src = H8Tensor(n, cin, h, w, torch.device("cpu"), _lib.PREC_F32R)
    dst = H8Tensor(n, cout, h, w, torch.device("cpu"), _lib.PREC_F32R)
    for cfg, th in ((q8, 8), (q4, 4)):
        for ks, eff in ((0, 0), (1, 0), (2, 2), (5, 4), (8, 6), (12, 12)):  # 12 chunks: 5 -> 4 slices of 3
            d = _lib.ConvH8Desc()
            d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope = n, cin, cout, cfg, _lib.PREC_F32R, 1, 0.1
            d.src, d.dst, d.whi, d.bias, d.ksplit = src.view(), dst.view(), 1, 1, ks
            cnt = C.c_int64(-1)
            tiles = 2 * 3 * -(-h // th) * n   # co blocks x tiles_x x tiles_y x n
            assert lib.rrin_conv_h8_split_floats(C.byref(d), C.byref(cnt)) == tiles * eff * 64 * th * 16
            assert cnt.value == (tiles if eff else 0)
    d.cfg = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 1)
    d.ksplit = 2
    assert lib.rrin_conv_h8_split_floats(C.byref(d), None) == _lib.RRIN_E_CONFIG if hasattr(_lib, "RRIN_E_CONFIG") \
        else lib.rrin_conv_h8_split_floats(C.byref(d), None) < 0


def test_edge_fix_split_scratch_size():
    """rrin_edge_fix_split_floats: fp32 ring fix-up runs of 64 channels (cin / 64 of
    them), 1024 floats per (tile, co block, image, run), one ticket per (tile, co
    block, image); one run (cin 64, fp16) needs no scratch."""
    import ctypes as C

    import torch

    from rrin_amd.pp import H8Tensor
    lib = _lib.lib()
    n, h, w = 2, 23, 40
    for prec, cin, cout, runs in ((_lib.PREC_F32R, 256, 128, 4), (_lib.PREC_F32R, 128, 64, 2),
                                  (_lib.PREC_F32R, 64, 32, 1), (_lib.PREC_F16, 256, 128, 1)):
        src = H8Tensor(n, cin, h, w, torch.device("cpu"), prec)
        dst = H8Tensor(n, cout, 2 * h, 2 * w, torch.device("cpu"), prec)
        e = _lib.EdgeFixDesc()
        e.n, e.cin, e.cout, e.prec = n, cin, cout, prec
        e.src, e.dst = src.chunk_view(0, cin), dst.view(0, cout)
        tiles = (2 * -(-2 * w // 32) + 2 * -(-(2 * h - 2) // 32)) * -(-cout // 32) * n
        cnt = C.c_int64(-1)
        nf = lib.rrin_edge_fix_split_floats(C.byref(e), C.byref(cnt))
        assert nf == (tiles * runs * 1024 if runs > 1 else 0), (prec, cin)
        assert cnt.value == (tiles if runs > 1 else 0)
    e.cin = 4
    assert lib.rrin_edge_fix_split_floats(C.byref(e), None) < 0


def _net_table(lib, ksplit_at=None):
    """A 77-entry exact-fp32 Winograd conv table in rrin_net_fwd's schedule order (per
    U-Net: down a/b per level, mid, up/a/b per level), sub-pixel up convs at levels 0-2
    (the engine's default), ksplit_at: grid level -> slices."""
    import ctypes as C
    wq = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 3)
    rows = []
    for depth in (5, 4, 4, 4):  # Flow, refine_flow, Mask, final (model.py:27-30)
        for L in range(depth):
            rows += [(L, 0), (L, 0)]
        rows.append((depth - 1, 0))
        for L in range(depth - 2, -1, -1):
            sub = L <= 2
            rows += [(L + 1 if sub else L, int(sub)), (L, 0), (L, 0)]
    t = (_lib.ConvWeights * len(rows))()
    for i, (grid_level, sub) in enumerate(rows):
        t[i].cfg, t[i].subpixel = wq, sub
        t[i].whi, t[i].bias = 1, 1  # never dereferenced by the size query
        if sub:
            t[i].wedge, t[i].bias_raw = 1, 1
        t[i].ksplit = (ksplit_at or {}).get(grid_level, 0)
    return t, C.cast(t, C.POINTER(_lib.ConvWeights))


def test_net_scratch_bytes():
    """rrin_net_scratch_bytes (ABI 12): the split-K / ring fix-up scratch lives outside the
    workspace, sized by the conv table -- none for an unsplit 720p x 4 forward (its ring
    fix-up grids exceed the cross-split limit), the ring fix-up's K split alone for
    640x368 x 1, more with split-K convs; zero for the other precisions (their ring runs
    from scratch in the conv launch, ABI 17)."""
    import ctypes as C
    lib = _lib.lib()
    assert lib.rrin_net_conv_count() == 77

    def need(n, h, w, prec=_lib.PREC_F32R, ks=None):
        t, ptr = _net_table(lib, ks)
        d = _lib.NetDesc()
        d.n, d.h, d.w, d.prec, d.convs = n, h, w, prec, ptr
        return lib.rrin_net_scratch_bytes(C.byref(d))

    assert need(4, 720, 1280) == 0
    base = need(1, 368, 640)
    assert base > 16 * 1024 and base <= 16 * 1024 + 256 * 1024 * 4
    split = need(1, 368, 640, ks={3: 2, 4: 4})
    assert split > base
    assert need(3, 368, 640, ks={3: 2, 4: 4}) > split  # the slabs scale with the batch
    # large batches: the split convs' tickets (one per tile, tiles grow with the batch) outgrow
    # the 4096-int minimum head (RRIN_E_CONFIG from about 11 pairs); the head grows
    n16, n32 = need(16, 368, 640, ks={3: 2, 4: 4}), need(32, 368, 640, ks={3: 2, 4: 4})
    assert n16 > 0 and n32 > n16
    # head = max(4096, tickets rounded up to 1024) ints: the bytes grow by more than the slabs
    # (with no ring fix-up scratch, split's bytes hold the minimum 4096-int head besides the slabs)
    assert n32 - n16 >= 16 * (split - base - (4096 * 4 if base == 0 else 0)) - 1
    assert need(1, 368, 640, prec=_lib.PREC_F16) == 0
    assert need(1, 72, 80) < 0  # not /16
