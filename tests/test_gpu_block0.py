"""GPU: the fused level-0 UNetConvBlock at fp16 (rrin_conv_block0_h8_fwd, conv_block0.hip;
unet.py:59-63 and the down block's pool, :46) through the C ABI.

The fused launch must give the bits of the two direct-form rrin_conv3x3_h8_fwd launches it
replaces (conv a -> a 32-channel tensor, conv b -> dst (+ pool)): same packed weights, same
accumulation order, same epilogue roundings -- on ragged tile grids (the 8 x 62 tile does not
divide the image), first convs with a channel tail, both weight packings' co-block widths, a
channel-offset (CAT) destination; and sit within the fp16 gate of float64.  The Net forward with
the fused blocks (engine.FUSE_L0) gives the unfused forward's output bit for bit."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd import engine as engine_mod
from rrin_amd.pp import H8Tensor
from tests import hip_helpers as H
from tests.test_gpu_h8 import conv_h8, keyed_conv, pack_h8

pytestmark = pytest.mark.gpu
F16 = _lib.PREC_F16
TOLF = dict(rtol=2e-2, atol=2e-2)


def direct_cfg(cin, cout, bm=None):
    """The engine's fp16 level-0 config for (cin, cout), or the first direct-form config of
    co-block width bm that runs at fp16 and takes the pool epilogue."""
    lib = _lib.lib()
    if bm is None:
        return engine_mod.choose_cfg_h8(cin, cout, F16, 0, "large")
    from tests.test_gpu_h8 import NO_POOL_CFGS
    return next(c for c in range(lib.rrin_conv_h8_cfg_count())
                if not lib.rrin_conv_h8_cfg_wino(c) and lib.rrin_conv_h8_cfg_ok(c, F16)
                and lib.rrin_conv_h8_cfg_bm(c) == bm and c not in NO_POOL_CFGS)


def block0(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, pool, dst=None, dst_off=0, status=None, tail_finite=0):
    dev = src.hi.device
    n, h, w = src.n, src.h, src.w
    if dst is None:
        dst = H8Tensor(n, 32 + dst_off, h, w, dev, F16)
    pl = H8Tensor(n, 32, h // 2, w // 2, dev, F16) if pool else None
    wha, _, bpa, inva = pack_h8(wa, ba, cfg_a, F16, dev)
    whb, _, bpb, invb = pack_h8(wb, bb, cfg_b, F16, dev)
    d = _lib.Block0Desc()
    d.n, d.cin, d.cfg_a, d.cfg_b, d.slope = n, cin, cfg_a, cfg_b, 0.1
    d.inv_wscale_a, d.inv_wscale_b, d.tail_finite = inva, invb, tail_finite
    d.src = src.chunk_view(0, cin)
    d.dst = dst.view(dst_off, 32)
    if pl is not None:
        d.pool = pl.view(0, 32)
    d.whi_a, d.bias_a, d.whi_b, d.bias_b = wha.data_ptr(), bpa.data_ptr(), whb.data_ptr(), bpb.data_ptr()
    d.status = status.data_ptr() if status is not None else None
    _lib.check(_lib.lib().rrin_conv_block0_h8_fwd(C.byref(d), H.stream(dev)), "rrin_conv_block0_h8_fwd")
    torch.cuda.synchronize(dev)
    return dst, pl


def unfused(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, pool, dst_off=0, tail_finite=0):
    mid, _ = conv_h8(src, wa, ba, cfg_a, F16, epi=_lib.EPI_LEAKY, cin=cin, tail_finite=tail_finite)
    epi = _lib.EPI_LEAKY_POOL if pool else _lib.EPI_LEAKY
    return conv_h8(mid, wb, bb, cfg_b, F16, epi=epi, dst_off=dst_off)


CASES = [  # n, cin, h, w, pool, dst_off
    (2, 16, 40, 130, True, 32),   # down_path[0] of a 16-channel U-Net into a CAT buffer, ragged x
    (1, 6, 24, 62, True, 0),      # 6-channel first conv (one partial record group), one tile column
    (1, 9, 16, 64, True, 0),      # 9 channels: a second, partial record group
    (2, 32, 34, 96, False, 0),    # ragged y (the last tile row half empty)
    (2, 64, 22, 70, False, 0),    # the last up block's conv_block (cat 64 -> 32)
    (1, 32, 13, 37, False, 0),    # odd sizes
    (3, 64, 48, 200, False, 0),
]


@pytest.mark.parametrize("n,cin,h,w,pool,dst_off", CASES)
def test_block0_bitwise_and_parity(gpu, n, cin, h, w, pool, dst_off):
    torch.manual_seed(n * 1000 + cin * 10 + h + w)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wa, ba = keyed_conv(cin, 32, "block0a")
    wb, bb = keyed_conv(32, 32, "block0b")
    src = H8Tensor.from_nchw(x, F16)
    tf = 1 if cin % 8 else 0
    cfg_a, cfg_b = direct_cfg(cin, 32), direct_cfg(32, 32)
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    d0, p0 = unfused(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, pool, dst_off, tail_finite=tf)
    d1, p1 = block0(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, pool, dst_off=dst_off, status=status, tail_finite=tf)
    assert int(status.item()) == 0
    assert torch.equal(d0.hi, d1.hi), "fused block differs from the two launches"  # padding too
    if pool:
        assert torch.equal(p0.hi, p1.hi)
    ref = F.leaky_relu(F.conv2d(F.leaky_relu(F.conv2d(x.double().cpu(), wa.double(), ba.double(), padding=1), 0.1),
                                wb.double(), bb.double(), padding=1), 0.1)
    np.testing.assert_allclose(d1.to_nchw(dst_off, 32).cpu().double().numpy(), ref.numpy(), **TOLF)
    if pool:
        np.testing.assert_allclose(p1.to_nchw().cpu().double().numpy(), F.avg_pool2d(ref, 2).numpy(), **TOLF)
    if dst_off:
        assert not d1.to_nchw(0, dst_off).any()  # the other half of the CAT buffer untouched


@pytest.mark.parametrize("bma,bmb", [(64, 32), (32, 64)])
def test_block0_pack_widths(gpu, bma, bmb):
    """Packs made for 64-channel co blocks (co 32-63 zero) read at their own stride."""
    n, cin, h, w = 1, 32, 24, 80
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wa, ba = keyed_conv(cin, 32, "block0w_a")
    wb, bb = keyed_conv(32, 32, "block0w_b")
    src = H8Tensor.from_nchw(x, F16)
    cfg_a, cfg_b = direct_cfg(cin, 32, bma), direct_cfg(32, 32, bmb)
    d0, p0 = unfused(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, True)
    d1, p1 = block0(src, cin, wa, ba, cfg_a, wb, bb, cfg_b, True)
    assert torch.equal(d0.hi, d1.hi) and torch.equal(p0.hi, p1.hi)


def test_block0_range_guard(gpu):
    """A conv-a value past the fp16 range sets the status flag (as the unfused conv a would)."""
    n, cin, h, w = 1, 16, 16, 64
    x = torch.full((n, cin, h, w), 60000.0, device=gpu)
    wa, ba = torch.ones(32, cin, 3, 3), torch.zeros(32)
    wb, bb = keyed_conv(32, 32, "block0g")
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    block0(H8Tensor.from_nchw(x, F16), cin, wa, ba, direct_cfg(cin, 32), wb, bb, direct_cfg(32, 32), True,
           status=status)
    assert int(status.item()) == 1


def test_block0_rejects(gpu):
    """Winograd configs, a channel tail without tail_finite and a pool of the wrong size are
    refused, nothing launched."""
    lib = _lib.lib()
    n, cin, h, w = 1, 32, 16, 64
    src = H8Tensor(n, cin, h, w, gpu, F16)
    dst = H8Tensor(n, 32, h, w, gpu, F16)
    wa, ba = keyed_conv(cin, 32, "block0r")
    cfg = direct_cfg(cin, 32)
    wh, _, bp, inv = pack_h8(wa, ba, cfg, F16, gpu)

    def desc(**kw):
        d = _lib.Block0Desc()
        d.n, d.cin, d.cfg_a, d.cfg_b, d.slope, d.inv_wscale_a, d.inv_wscale_b = n, cin, cfg, cfg, 0.1, inv, inv
        d.src, d.dst = src.chunk_view(0, cin), dst.view(0, 32)
        d.whi_a = d.whi_b = wh.data_ptr()
        d.bias_a = d.bias_b = bp.data_ptr()
        for k, v in kw.items():
            setattr(d, k, v)
        return lib.rrin_conv_block0_h8_fwd(C.byref(d), H.stream(gpu))

    assert desc() == 0
    # RRIN_E_CONFIG (-4), RRIN_E_ARG (-2), RRIN_E_SHAPE (-1)
    wino = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c))
    assert desc(cfg_a=wino) == -4
    assert desc(cin=30) == -2
    assert desc(pool=H8Tensor(n, 32, h, w, gpu, F16).view(0, 32)) == -1
    torch.cuda.synchronize(gpu)


@pytest.mark.parametrize("h,w,n,mode", [(256, 256, 1, 2), (368, 640, 2, 2), (368, 640, 2, 1)])
def test_net_fused_blocks_bitwise(gpu, h, w, n, mode):
    """Net.forward at fp16 with the level-0 UNetConvBlocks fused gives the unfused forward's
    output bit for bit (engine.FUSE_L0 = 2: 8 fused launches per forward, 4 U-Nets x
    down_path[0] + last up block; 1: the 4 down blocks)."""
    from rrin_amd import Net
    from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    net = net.to(gpu).eval()
    net.precision = "fp16"
    i0, i1 = synthetic_batch(n, h, w, first_index=3)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    lib = _lib.lib()

    def conv_launches(eng):  # conv launches of one forward, from the schedule's launch profiler
        prof = C.c_void_p()
        _lib.check(lib.rrin_prof_create(4096, C.byref(prof)))
        try:
            eng.forward(i0, i1, 0.5, prof=prof, streams=1)
            torch.cuda.synchronize(gpu)
            cap = 4096
            kinds, ms, fl, cnt = (C.c_int32 * cap)(), (C.c_float * cap)(), (C.c_double * cap)(), C.c_int32()
            _lib.check(lib.rrin_prof_read(prof, kinds, ms, fl, cap, C.byref(cnt)))
            return sum(1 for i in range(cnt.value) if kinds[i] == 0), sum(fl[i] for i in range(cnt.value) if kinds[i] == 0)
        finally:
            lib.rrin_prof_destroy(prof)

    saved = engine_mod.FUSE_L0
    try:
        with torch.no_grad():
            engine_mod.FUSE_L0 = 0
            eng = net.engine()
            ref = eng.forward(i0, i1, 0.5, streams=1)
            n0, f0 = conv_launches(eng)
            engine_mod.FUSE_L0 = mode
            t = eng.conv_table_for(n, h, w)
            nf = 8 if mode == 2 else 4
            assert sum(int(t[i].fuse_next) for i in range(eng.expected_convs)) == nf
            out = eng.forward(i0, i1, 0.5, streams=1)
            n1, f1 = conv_launches(eng)
    finally:
        engine_mod.FUSE_L0 = saved
    assert n1 == n0 - nf, (n0, n1)  # the fused launches ran (one per two convs)
    assert abs(f1 - f0) <= 1e-9 * f0  # same algorithmic FLOPs counted
    assert torch.equal(out, ref)
