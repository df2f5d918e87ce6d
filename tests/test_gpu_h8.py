"""GPU: the record-layout paths of librrin_hip.so -- exact fp32 on fp32 records
(R32, the default "fp32" precision), split-fp16 (fp32_split16) and fp16.

R32 is exact fp32 arithmetic (fp32 storage, v_mfma_f32_32x32x2_f32 products,
fp32 accumulation): held to 1e-5 against float64, the Winograd F(2x2,3x3) tiles too.

fp32_split16 holds each fp32 value as fp16 hi+lo and forms each product from
three exact fp16 products with fp32 accumulation (error ~2^-21 relative per
product), so it is held to the fp32 tolerances.  fp16 is held to the SURVEY
§8d fp16 gate: max-abs <= 1e-2 and PSNR >= 45 dB vs the fp32 CPU reference."""
import ctypes as C
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import H8Tensor
from rrin_amd.synthetic import keyed_tensor
from tests import hip_helpers as H
from tests.golden.spec import CONV_CLASSES

pytestmark = pytest.mark.gpu
X3, F16, R32 = _lib.PREC_F16X3, _lib.PREC_F16, _lib.PREC_F32R
PRECS = [R32, X3, F16]
TOL = {X3: dict(rtol=1e-4, atol=1e-4), F16: dict(rtol=2e-2, atol=2e-2), R32: dict(rtol=1e-5, atol=1e-5)}


# Winograd F(4,3) x F(2,3) (kind 14): transform coefficients up to 8 and U entries of 1/24 round
# more than F(2x2,3x3) -- measured max error vs float64 on these sweeps in DESIGN.md §5f
TOL42 = dict(rtol=5e-5, atol=5e-5)


def tol(prec, cfg):
    """Tolerance of config cfg at prec."""
    if prec == R32 and _lib.lib().rrin_conv_h8_cfg_wino(cfg) == 14:
        return TOL42
    return TOL[prec]


def ref_conv(x, w, b, slope=None):
    y = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    return F.leaky_relu(y, slope) if slope is not None else y


def keyed_conv(cin, cout, key="h8"):
    return (keyed_tensor(f"{key}.{cin}.{cout}.w", (cout, cin, 3, 3), cin * 9),
            keyed_tensor(f"{key}.{cin}.{cout}.b", (cout,), cin * 9))


# configs with one output row per wave (WN == 1 in conv_f16.hip's table): a
# wave must own both rows of a pool pair, so they reject the pool epilogue
NO_POOL_CFGS = (4, 16)


def wino_cfgs(cout=32, epi=None):
    """Ids of the Winograd exact-fp32 configs (R32 only): F(2x2,3x3) kinds 1, 3, 4 and the
    register-U kinds 6-7 (every epilogue, any cout)."""
    lib = _lib.lib()
    return tuple(c for c in range(lib.rrin_conv_h8_cfg_count())
                 if lib.rrin_conv_h8_cfg_wino(c) > 0 and lib.rrin_conv_h8_cfg_ok(c, R32))


def cfgs(prec, cout, cin):
    lib = _lib.lib()
    # the Winograd config stages whole records only: cin % 4 != 0 needs tail_finite (test_h8_conv_dma_finite_tail);
    # the register-U kinds 6-7 stage both record groups of every 8-channel chunk: cin % 8 != 0 needs it too
    return [c for c in range(lib.rrin_conv_h8_cfg_count())
            if lib.rrin_conv_h8_cfg_fits(c, prec, cin) and lib.rrin_conv_h8_cfg_bm(c) <= max(32, 2 * cout)
            and not (lib.rrin_conv_h8_cfg_wino(c) and cin % 4)
            and not (lib.rrin_conv_h8_cfg_wino(c) in (6, 7, 14) and cin % 8)
            and not (prec == F16 and lib.rrin_conv_h8_cfg_wino(c) and cin % 16)]  # fp16 kind 6: 16-ch chunks


def pack_h8(w, b, cfg, prec, dev, perm=None):
    lib = _lib.lib()
    w = w.detach().cpu().float().contiguous().numpy()
    b = b.detach().cpu().float().contiguous().numpy()
    cout, cin = w.shape[:2]
    bm = lib.rrin_conv_h8_cfg_bm(cfg)
    pa = np.asarray(perm, np.int32) if perm is not None else None
    if prec == R32 and lib.rrin_conv_h8_cfg_wino(cfg) == 14:  # Winograd F(4,3) x F(2,3)
        wp = np.zeros(lib.rrin_pack_conv3x3_wino42_floats(cout, cin), np.float32)
        bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
        _lib.check(lib.rrin_pack_conv3x3_wino42(w.ctypes.data, b.ctypes.data, cout, cin,
                                                pa.ctypes.data if pa is not None else None, wp.ctypes.data,
                                                bp.ctypes.data))
        wt = torch.from_numpy(wp).to(dev)
        return wt, wt, torch.from_numpy(bp).to(dev), 1.0
    if prec == R32 and lib.rrin_conv_h8_cfg_wino(cfg):  # Winograd: U = G g G^T per point
        wp = np.zeros(lib.rrin_pack_conv3x3_wino_bm_floats(cout, cin, bm), np.float32)
        bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
        _lib.check(lib.rrin_pack_conv3x3_wino_bm(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                                 pa.ctypes.data if pa is not None else None, wp.ctypes.data,
                                                 bp.ctypes.data))
        wt = torch.from_numpy(wp).to(dev)
        return wt, wt, torch.from_numpy(bp).to(dev), 1.0
    if prec == R32:  # fp32 records: unscaled fp32 weights, no lo blob
        wp = np.zeros(lib.rrin_pack_conv3x3_r32_floats(cout, cin, bm), np.float32)
        bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
        _lib.check(lib.rrin_pack_conv3x3_r32(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                             pa.ctypes.data if pa is not None else None, wp.ctypes.data,
                                             bp.ctypes.data))
        wt = torch.from_numpy(wp).to(dev)
        return wt, wt, torch.from_numpy(bp).to(dev), 1.0
    if prec == F16 and lib.rrin_conv_h8_cfg_wino(cfg):  # fp16 Winograd (kind 6): fp16 U, scaled
        whi = np.zeros(lib.rrin_pack_conv3x3_wino_h8_halves(cout, cin, bm), np.uint16)
        bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
        inv = C.c_float()
        _lib.check(lib.rrin_pack_conv3x3_wino_h8(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                                 pa.ctypes.data if pa is not None else None, whi.ctypes.data,
                                                 bp.ctypes.data, C.byref(inv)))
        wt = torch.from_numpy(whi.view(np.int16)).to(dev)
        return wt, wt, torch.from_numpy(bp).to(dev), inv.value
    nh = lib.rrin_pack_conv3x3_h8_halves(cout, cin, bm)
    whi = np.zeros(nh, np.uint16)
    wlo = np.zeros(nh, np.uint16)
    bp = np.zeros(lib.rrin_pack_bias_floats(cout, bm), np.float32)
    inv = C.c_float()
    _lib.check(lib.rrin_pack_conv3x3_h8(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                        pa.ctypes.data if pa is not None else None, prec, whi.ctypes.data,
                                        wlo.ctypes.data, bp.ctypes.data, C.byref(inv)))
    t = lambda a: torch.from_numpy(a.view(np.int16)).to(dev)  # noqa: E731
    return t(whi), t(wlo), torch.from_numpy(bp).to(dev), inv.value


def set_split(d, ksplit, dev, keep):
    """Give desc d a split-K of ksplit slices (Winograd kinds 3, 4) with fresh scratch;
    keep collects the scratch tensors (the counters are checked by test_gpu_split)."""
    if not ksplit:
        return
    d.ksplit = ksplit
    nc = C.c_int64()
    nf = _lib.lib().rrin_conv_h8_split_floats(C.byref(d), C.byref(nc))
    assert nf > 0 and nc.value > 0, nf
    part = torch.full((nf,), float("nan"), device=dev)
    cnt = torch.zeros(nc.value, dtype=torch.int32, device=dev)
    d.part, d.cnt = part.data_ptr(), cnt.data_ptr()
    keep.extend([part, cnt])


def conv_h8(src: H8Tensor, w, b, cfg, prec, epi=_lib.EPI_LINEAR, dst=None, dst_off=0, pool=None, perm=None,
            cin=None, tail_finite=0, ksplit=0, keep=None):
    dev = src.hi.device
    cout, cin_w = w.shape[:2]
    cin = cin or cin_w
    if dst is None:
        dst = H8Tensor(src.n, cout + dst_off, src.h, src.w, dev, prec)
    if epi == _lib.EPI_LEAKY_POOL and pool is None:
        pool = H8Tensor(src.n, cout, src.h // 2, src.w // 2, dev, prec)
    whi, wlo, bp, inv = pack_h8(w, b, cfg, prec, dev, perm)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = src.n, cin, cout, cfg, prec, epi, 0.1, inv
    d.tail_finite = tail_finite
    d.src = src.chunk_view(0, cin)
    d.dst = dst.view(dst_off, cout)
    if pool is not None:
        d.pool = pool.view(0, cout)
    d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr() if prec == X3 else None, bp.data_ptr()
    set_split(d, ksplit, dev, keep if keep is not None else [])
    _lib.check(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv3x3_h8_fwd")
    torch.cuda.synchronize(dev)
    return dst, pool


@pytest.mark.parametrize("prec", PRECS)
def test_h8_roundtrip(gpu, prec):
    x = torch.randn(2, 11, 23, 40, device=gpu) * 3
    t = H8Tensor.from_nchw(x, prec, c_alloc=24, ch_off=3)
    y = t.to_nchw(3, 11)
    rel = {X3: 2.0 ** -21, F16: 2.0 ** -10, R32: 0.0}[prec]
    floor = {X3: 2.0 ** -34, F16: 2.0 ** -24, R32: 0.0}[prec]   # fp16 subnormal floor of lo (x 2^-11) / hi
    assert bool(((y - x).abs() <= rel * x.abs() + floor).all())
    assert not t.hi[:, :, 0].any() and not t.hi[:, :, :, :8].any() and not t.hi[:, :, 24:].any()


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cin,cout", CONV_CLASSES)
def test_h8_conv_golden(gpu, golden, prec, cin, cout):
    if cout % 8:
        pytest.skip("heads (Cout 2-4) run on the VALU head kernel")
    g = golden("ops")
    w = keyed_tensor(f"golden.conv.{cin}.{cout}.weight", (cout, cin, 3, 3), cin * 9)
    b = keyed_tensor(f"golden.conv.{cin}.{cout}.bias", (cout,), cin * 9)
    x = torch.from_numpy(g[f"conv_{cin}_{cout}_in"]).to(gpu)
    for cfg in cfgs(prec, cout, cin):
        dst, _ = conv_h8(H8Tensor.from_nchw(x, prec), w, b, cfg, prec)
        np.testing.assert_allclose(dst.to_nchw().cpu().numpy(), g[f"conv_{cin}_{cout}_out"], **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 32, 40, 72), (1, 128, 64, 46, 80), (1, 256, 256, 12, 20),
                                            (2, 16, 32, 32, 64)])
def test_h8_conv_pool(gpu, prec, n, cin, cout, h, w):
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout)
    ref = ref_conv(x, wt, b, 0.1)
    refp = F.avg_pool2d(ref, 2)
    for cfg in cfgs(prec, cout, cin):
        if cfg in NO_POOL_CFGS:
            continue  # WN == 1: no pool epilogue (rejected with RRIN_E_CONFIG, see test below)
        dst, pool = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, cfg, prec, epi=_lib.EPI_LEAKY_POOL, dst_off=cout,
                            dst=H8Tensor(n, 2 * cout, h, w, gpu, prec))
        np.testing.assert_allclose(dst.to_nchw(cout, cout).cpu().double().numpy(), ref.numpy(), **tol(prec, cfg))
        assert not dst.to_nchw(0, cout).any()
        np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), refp.numpy(), **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")


@pytest.mark.parametrize("prec", PRECS)
def test_h8_conv_partial_channels_and_perm(gpu, prec):
    x = torch.rand(2, 16, 32, 48, device=gpu)
    wt, b = keyed_conv(10, 32, "perm")
    perm = [4, 5, 6, 7, 8, 9, 0, 1, 2, 3]
    ref = ref_conv(torch.cat([x[:, 6:10], x[:, 0:6]], 1), wt, b)
    xx = x.clone()
    xx[:, 10:] = float("nan")  # channels beyond cin must never be read into the sum
    dst, _ = conv_h8(H8Tensor.from_nchw(xx, prec), wt, b, 1, prec, perm=perm, cin=10)
    np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL[prec])


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("n,c,h,w", [(1, 64, 20, 36), (2, 16, 5, 7), (1, 512, 5, 10)])
def test_h8_upsample(gpu, prec, n, c, h, w):
    x = torch.rand(n, c, h, w, device=gpu) * 2 - 1
    src = H8Tensor.from_nchw(x, prec)
    dst = H8Tensor(n, c, 2 * h, 2 * w, gpu, prec)
    sv, dv = src.view(), dst.view()
    _lib.check(_lib.lib().rrin_upsample2x_h8(C.byref(sv), C.byref(dv), n, prec, H.stream(gpu)))
    torch.cuda.synchronize()
    ref = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    tol = 2e-3 if prec == F16 else 1e-6
    np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), rtol=0, atol=tol)


def test_h8_pool_rejected_for_single_row_waves(gpu):
    x = torch.rand(1, 32, 16, 32, device=gpu)
    wt, b = keyed_conv(32, 32)
    with pytest.raises(_lib.RRINError, match="config"):
        conv_h8(H8Tensor.from_nchw(x, X3), wt, b, 4, X3, epi=_lib.EPI_LEAKY_POOL)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cin", [6, 9, 10])
def test_h8_conv_dma_finite_tail(gpu, prec, cin):
    """tail_finite=1: whole records staged by LDS-DMA; the finite tail channels
    meet zero-padded weights (the first convs of the Net)."""
    x = torch.rand(2, 16, 32, 48, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, 32, "tail")
    ref = ref_conv(x[:, :cin], wt, b)
    for cfg in (1, 6) + (wino_cfgs() if prec == R32 else f16_wino_cfgs() if prec == F16 else ()):
        dst, _ = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, cfg, prec, cin=cin, tail_finite=1)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **tol(prec, cfg))
        # a tensor of just cin channels: allocated in whole 2-group chunks, so the
        # Winograd tiles' staging of the chunk's second group stays inside it
        dst, _ = conv_h8(H8Tensor.from_nchw(x[:, :cin], prec), wt, b, cfg, prec, tail_finite=1)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **tol(prec, cfg))


def f16_wino_cfgs():
    lib = _lib.lib()
    return tuple(c for c in range(lib.rrin_conv_h8_cfg_count())
                 if lib.rrin_conv_h8_cfg_wino(c) > 0 and lib.rrin_conv_h8_cfg_ok(c, F16))


@pytest.mark.parametrize("prec,cin", [(F16, 6), (F16, 20), (R32, 9)])
def test_h8_wino_rejects_short_source_view(gpu, prec, cin):
    """A Winograd F(2x2) tile stages both record groups of every K chunk: a source view
    holding cin but not the chunk's last group is rejected (RRIN_E_SHAPE) instead of
    read past."""
    x = torch.rand(1, cin, 16, 32, device=gpu)
    wt, b = keyed_conv(cin, 32, "tail")
    t = H8Tensor.from_nchw(x, prec)
    cfgs_ = list(f16_wino_cfgs() if prec == F16 else wino_cfgs())
    assert cfgs_
    for cfg in cfgs_:
        whi, wlo, bp, inv = pack_h8(wt, b, cfg, prec, gpu)
        dst = H8Tensor(1, 32, 16, 32, gpu, prec)
        d = _lib.ConvH8Desc()
        d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.inv_wscale = 1, cin, 32, cfg, prec, _lib.EPI_LINEAR, inv
        d.slope, d.tail_finite = 0.1, 1
        d.src, d.dst = t.view(0, cin), dst.view(0, 32)  # an odd group count: one short of the chunk
        d.whi, d.wlo, d.bias = whi.data_ptr(), None, bp.data_ptr()
        assert _lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), H.stream(gpu)) == -1, f"cfg {cfg}"
        d.src = t.chunk_view(0, cin)
        _lib.check(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), H.stream(gpu)), f"cfg {cfg}")
        torch.cuda.synchronize()
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref_conv(x, wt, b).numpy(), **tol(prec, cfg))


@pytest.mark.parametrize("prec", PRECS)
def test_pack_g16(gpu, prec):
    i0 = torch.rand(2, 3, 32, 48, device=gpu)
    i1 = torch.rand(2, 3, 32, 48, device=gpu)
    g = H8Tensor(2, 16, 32, 48, gpu, prec)
    g.hi.fill_(7.0)
    if g.lo is not None:
        g.lo.fill_(7.0)
    v = g.view(0, 16)
    _lib.check(_lib.lib().rrin_pack_g16_h8(i0.data_ptr(), i1.data_ptr(), 2, C.byref(v), prec, H.stream(gpu)))
    torch.cuda.synchronize()
    out = g.to_nchw()
    tol = {X3: 2.0 ** -20, F16: 2.0 ** -10, R32: 0.0}[prec]
    assert float((out[:, :3] - i0).abs().max()) <= tol and float((out[:, 3:6] - i1).abs().max()) <= tol
    assert not out[:, 6:].any()


def replicate_ring(t: H8Tensor):
    """Edge-replicate an H8 tensor's interior into its 1-pixel padding ring (what
    EPI_LEAKY_REP writes)."""
    h, w = t.h, t.w
    for a in (t.hi, t.lo):
        if a is None:
            continue
        a[:, :, 0, 8:8 + w] = a[:, :, 1, 8:8 + w]
        a[:, :, h + 1, 8:8 + w] = a[:, :, h, 8:8 + w]
        a[:, :, 0:h + 2, 7] = a[:, :, 0:h + 2, 8]
        a[:, :, 0:h + 2, 8 + w] = a[:, :, 0:h + 2, 7 + w]


@pytest.mark.parametrize("prec", PRECS)
def test_h8_leaky_rep_writes_replicated_ring(gpu, prec):
    x = torch.rand(2, 32, 13, 45, device=gpu) * 2 - 1
    wt, b = keyed_conv(32, 64, "rep")
    ref = ref_conv(x, wt, b, 0.1)
    for cfg in (0, 6) + (wino_cfgs(64, _lib.EPI_LEAKY_REP) if prec == R32 else ()):
        dst, _ = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, cfg, prec, epi=_lib.EPI_LEAKY_REP)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **tol(prec, cfg))
        # the ring must equal the replicated border; everything else in the padding stays zero
        want = SimpleNamespace(h=dst.h, w=dst.w, hi=dst.hi.clone(), lo=dst.lo.clone() if dst.lo is not None else None)
        for a in (want.hi, want.lo):
            if a is not None:
                a[:, :, 0] = 0
                a[:, :, dst.h + 1:] = 0
                a[:, :, :, :8] = 0
                a[:, :, :, 8 + dst.w:] = 0
        replicate_ring(want)
        assert torch.equal(dst.hi, want.hi), f"cfg {cfg}"
        if prec == X3:
            assert torch.equal(dst.lo, want.lo)
        assert dst.hi[:, :, 0, 7:9 + dst.w].any() and dst.hi[:, :, 1:dst.h + 1, 7].any()


def subpixel_upconv(src: H8Tensor, w, b, cfg, prec, dst=None, ksplit=0, keep=None, fold=False, edge_split=False,
                    full=False, inlaunch=False):
    """EPI_SUBPIXEL conv + ring fix-up through the C ABI (the Net's up.1 conv); fold: the
    ring in the conv launch (rrin_conv_h8_desc.ring_w, Winograd kind 3) instead of
    rrin_subpixel_edge_fix_h8; full: the fix-up's from-scratch mode (rrin_edge_fix_desc.full,
    no edge buffer), launched BEFORE the conv -- it must read nothing the conv writes, and the
    conv must write no ring pixel."""
    lib = _lib.lib()
    dev = src.hi.device
    cout, cin = w.shape[:2]
    wn = w.detach().cpu().float().contiguous().numpy()
    bn = b.detach().cpu().float().contiguous().numpy()
    ws = np.empty((4 * cout, cin, 3, 3), np.float32)
    bs = np.empty(4 * cout, np.float32)
    _lib.check(lib.rrin_subpixel_weights(wn.ctypes.data, bn.ctypes.data, cout, cin, ws.ctypes.data, bs.ctypes.data))
    whi, wlo, bp, inv = pack_h8(torch.from_numpy(ws), torch.from_numpy(bs), cfg, prec, dev)
    H_, W_ = 2 * src.h, 2 * src.w
    if dst is None:
        dst = H8Tensor(src.n, cout, H_, W_, dev, prec)
    edge = torch.full((src.n, cout, lib.rrin_ring_pixels(H_, W_)), float("nan"), device=dev)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = (src.n, cin, 4 * cout, cfg, prec,
                                                                            _lib.EPI_SUBPIXEL, 0.1, inv)
    d.src, d.dst = src.chunk_view(0, cin), dst.view(0, cout)
    d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr() if prec == X3 else None, bp.data_ptr()
    d.edge = edge.data_ptr()
    keep = keep if keep is not None else []
    set_split(d, ksplit, dev, keep)
    wedge = torch.from_numpy(np.ascontiguousarray(wn.transpose(1, 2, 3, 0))).to(dev)
    braw = torch.from_numpy(bn.copy()).to(dev)
    if fold:
        d.ring_w, d.ring_bias = wedge.data_ptr(), braw.data_ptr()
        nc = C.c_int64()
        nf = lib.rrin_conv_h8_ring_floats(C.byref(d), C.byref(nc))
        assert nf > 0 and nc.value > 0, nf
        corr = torch.full((nf,), float("nan"), device=dev)
        cnt = torch.zeros(nc.value, dtype=torch.int32, device=dev)
        d.ring_corr, d.ring_cnt = corr.data_ptr(), cnt.data_ptr()
        keep.extend([corr, cnt])
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv3x3_h8_fwd(subpixel, fold)")
        torch.cuda.synchronize(dev)
        return dst
    e = _lib.EdgeFixDesc()
    e.n, e.cin, e.cout, e.prec, e.epi_mode, e.slope = src.n, cin, cout, prec, _lib.EPI_LINEAR, 0.1
    e.src, e.dst = src.chunk_view(0, cin), dst.view(0, cout)
    e.edge, e.wedge, e.bias = (None if full or inlaunch else edge.data_ptr()), wedge.data_ptr(), braw.data_ptr()
    e.full = int(full or inlaunch)
    if inlaunch:  # ABI 17: the ring from scratch with the conv (rrin_conv_h8_desc.ring_full)
        d.ring_full = C.addressof(e)
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv3x3_h8_fwd(subpixel, ring_full)")
        torch.cuda.synchronize(dev)
        return dst
    if not full:
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv3x3_h8_fwd(subpixel)")
    if edge_split:  # cross-workgroup K split of the fix-up (fp32 records)
        nc = C.c_int64(-1)
        nf = lib.rrin_edge_fix_split_floats(C.byref(e), C.byref(nc))
        assert nf >= 0 and nc.value >= 0, nf
        if nf:
            part = torch.full((nf,), float("nan"), device=dev)
            cnt = torch.zeros(nc.value, dtype=torch.int32, device=dev)
            e.part, e.cnt, e.part_floats, e.cnt_len = part.data_ptr(), cnt.data_ptr(), nf, nc.value
            keep.extend([part, cnt])
    _lib.check(lib.rrin_subpixel_edge_fix_h8(C.byref(e), H.stream(dev)), "rrin_subpixel_edge_fix_h8")
    if full:
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv3x3_h8_fwd(subpixel)")
    torch.cuda.synchronize(dev)
    return dst


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 64, 32, 20, 36), (1, 128, 64, 23, 40), (1, 256, 128, 5, 7),
                                              (2, 512, 256, 3, 5), (1, 64, 32, 1, 1)])
def test_h8_subpixel_upconv(gpu, prec, n, cin, cout, sh, sw):
    """conv3x3(upsample_x2(x)) of the up block (unet.py:77-78) as one low-res
    sub-pixel conv + ring fix-up, against upsample-then-conv in float64."""
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, prec)
    replicate_ring(src)
    for cfg in cfgs(prec, 4 * cout, cin):
        dst = subpixel_upconv(src, wt, b, cfg, prec, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
        np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")
        assert not dst.to_nchw(cout, cout).any()           # the bridge half of CAT is untouched
        assert not dst.hi[:, :, 0].any() and not dst.hi[:, :, :, :8].any()  # zero padding kept


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 64, 32, 20, 36), (1, 128, 64, 23, 40), (1, 256, 128, 5, 7),
                                              (2, 512, 256, 3, 5), (1, 64, 32, 1, 1), (1, 256, 128, 1, 2),
                                              (1, 1024, 512, 2, 3)])
def test_h8_subpixel_ring_full(gpu, prec, n, cin, cout, sh, sw):
    """The from-scratch ring (rrin_edge_fix_desc.full; what net.hip runs on a side stream
    beside the sub-pixel conv) launched before the conv: the whole output within the
    tolerance of upsample-then-conv in float64, the bridge half untouched, and every K split
    of the fix-up (fp32 records: one workgroup per run) bit for bit the one-workgroup result."""
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, prec)
    replicate_ring(src)
    cfg = next(c for c in cfgs(prec, 4 * cout, cin) if prec != _lib.PREC_F32R or _lib.lib().rrin_conv_h8_cfg_wino(c))
    dst = subpixel_upconv(src, wt, b, cfg, prec, full=True, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
    np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **tol(prec, cfg))
    assert not dst.to_nchw(cout, cout).any()
    assert not dst.hi[:, :, 0].any() and not dst.hi[:, :, :, :8].any()
    if prec == _lib.PREC_F32R:
        keep = []
        split = subpixel_upconv(src, wt, b, cfg, prec, full=True, keep=keep, edge_split=True,
                                dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
        assert torch.equal(split.hi, dst.hi)
        assert not keep or not keep[1].any()


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 64, 32, 20, 36), (1, 128, 64, 23, 40), (2, 256, 128, 5, 7),
                                              (1, 512, 256, 3, 5), (1, 64, 32, 1, 1), (3, 128, 64, 46, 80)])
def test_h8_subpixel_ring_in_launch(gpu, prec, n, cin, cout, sh, sw):
    """ABI 17 ring_full: the ring from scratch in extra workgroups of the sub-pixel conv's own
    launch (direct-form tiles of 256 / 512 threads; other configs -- the Winograd tiles, 128-thread
    tiles -- run it as a second launch): every config within the tolerance of upsample-then-conv in
    float64, the bridge half and the padding untouched, repeat launches bitwise equal, and the ring
    pixels bit for bit the same under every config (one K group in every ring_full fix-up, in the
    launch or as the fallback's second launch: the Net's size classes stay bitwise)."""
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, prec)
    replicate_ring(src)
    lib = _lib.lib()
    tested, borders = 0, []
    # the sub-pixel configs of the Net's tables (10-13: 512 / 256 threads), a 128-thread tile (7, 17:
    # second launch) and, exact fp32, the Winograd tiles (second launch)
    for cfg in [c for c in cfgs(prec, 4 * cout, cin) if c in (7, 10, 11, 12, 13, 17) or lib.rrin_conv_h8_cfg_wino(c) > 0]:
        out = [subpixel_upconv(src, wt, b, cfg, prec, inlaunch=True, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
               for _ in range(2)]
        dst = out[0]
        np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")
        assert not dst.to_nchw(cout, cout).any()
        assert not dst.hi[:, :, 0].any() and not dst.hi[:, :, :, :8].any()
        assert torch.equal(out[0].hi, out[1].hi)
        o = dst.to_nchw(0, cout)
        border = torch.cat([o[:, :, 0], o[:, :, -1], o[:, :, :, 0], o[:, :, :, -1]], dim=2)
        if borders:
            assert torch.equal(border, borders[0][1]), f"cfg {cfg} vs cfg {borders[0][0]}: ring bits differ"
        borders.append((cfg, border))
        tested += 1
    assert tested


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 20, 36), (1, 256, 128, 5, 7), (2, 512, 256, 3, 5),
                                              (1, 256, 128, 1, 1), (1, 64, 32, 9, 17)])
def test_h8_subpixel_edge_split(gpu, n, cin, cout, sh, sw):
    """fp32 ring fix-up with its cross-workgroup K split (one workgroup per 64-channel
    run, the last one of a tile adds the runs in run order): bit for bit the
    one-workgroup result, tickets back at zero, and within 1e-5 of float64."""
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, _lib.PREC_F32R)
    replicate_ring(src)
    cfg = next(c for c in cfgs(_lib.PREC_F32R, 4 * cout, cin) if _lib.lib().rrin_conv_h8_cfg_wino(c) == 3)
    plain = subpixel_upconv(src, wt, b, cfg, _lib.PREC_F32R, dst=H8Tensor(n, cout, 2 * sh, 2 * sw, gpu, _lib.PREC_F32R))
    keep = []
    split = subpixel_upconv(src, wt, b, cfg, _lib.PREC_F32R, keep=keep, edge_split=True,
                            dst=H8Tensor(n, cout, 2 * sh, 2 * sw, gpu, _lib.PREC_F32R))
    assert torch.equal(plain.hi, split.hi)
    if cin > 64:
        assert len(keep) == 2 and not keep[1].any()  # scratch was used; every ticket back at zero
    else:
        assert not keep                               # cin 64: one run, no scratch
    np.testing.assert_allclose(split.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cin,epi", [(32, _lib.EPI_LEAKY_POOL), (64, _lib.EPI_LEAKY), (32, _lib.EPI_LINEAR)])
def test_h8_conv_many_tiles_per_block(gpu, prec, cin, epi):
    """Shapes with more tiles than a persistent grid holds, so each block loops
    over several tiles (chunk 0 of tile k+1 staged behind tile k's last chunk)."""
    n, cout, h, w = 4, 32, 96, 640
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "many")
    slope = None if epi == _lib.EPI_LINEAR else 0.1
    ref = ref_conv(x, wt, b, slope)
    refp = F.avg_pool2d(ref, 2)
    for cfg in cfgs(prec, cout, cin):
        if epi == _lib.EPI_LEAKY_POOL and cfg in NO_POOL_CFGS:
            continue
        dst, pool = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, cfg, prec, epi=epi)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")
        if pool is not None:
            np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), refp.numpy(), **tol(prec, cfg),
                                       err_msg=f"cfg {cfg} pool")


@pytest.mark.parametrize("prec", PRECS)
def test_h8_subpixel_many_tiles_per_block(gpu, prec):
    """Sub-pixel up conv (ring scratch + phase epilogue) on a grid with several
    tiles per block, every config."""
    n, cin, cout, sh, sw = 4, 64, 32, 48, 320
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "subm")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, prec)
    replicate_ring(src)
    for cfg in cfgs(prec, 4 * cout, cin):
        dst = subpixel_upconv(src, wt, b, cfg, prec, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
        np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **tol(prec, cfg),
                                   err_msg=f"cfg {cfg}")


def head_h8(src: H8Tensor, dst: H8Tensor, w, b, mode, coef=None, out=None, prec=X3):
    dev = src.hi.device
    w_d = w.detach().float().contiguous().to(dev)
    b_d = b.detach().float().contiguous().to(dev)
    d = _lib.HeadH8Desc()
    d.n, d.cin, d.cout, d.mode, d.prec = src.n, 32, w.shape[0], mode, prec
    d.src, d.g16 = src.view(0, 32), dst.view(0, dst.c)
    d.w, d.bias = w_d.data_ptr(), b_d.data_ptr()
    d.coef = coef.data_ptr() if coef is not None else None
    d.out = out.data_ptr() if out is not None else None
    _lib.check(_lib.lib().rrin_head_h8_fwd(C.byref(d), H.stream(dev)), "rrin_head_h8_fwd")
    torch.cuda.synchronize(dev)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cout", [2, 3, 4])
@pytest.mark.parametrize("n,h,w,scale", [(2, 40, 72, 1.0), (1, 20, 50, 1e-3), (3, 16, 32, 300.0)])
def test_h8_head_plain(gpu, prec, cout, n, h, w, scale):
    """MFMA head conv (32 -> cout) against float64: weights split in the kernel
    with a per-channel power-of-two scale (tiny and large weights), ragged tiles."""
    x = torch.rand(n, 32, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(32, cout, "headh8")
    wt = wt * scale
    dst = H8Tensor(n, 16, h, w, gpu, prec)
    head_h8(H8Tensor.from_nchw(x, prec), dst, wt, b, _lib.HEAD_PLAIN, prec=prec)
    ref = ref_conv(x, wt, b)
    tol = {X3: dict(rtol=1e-4, atol=1e-4 * max(scale, 1.0)), R32: dict(rtol=1e-5, atol=1e-5 * max(scale, 1.0)),
           F16: dict(rtol=2e-2, atol=2e-2 * max(scale, 1.0))}[prec]
    np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **tol)
    assert not dst.to_nchw(cout, 16 - cout).any()
