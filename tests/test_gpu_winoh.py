"""GPU: the register-U Winograd F(2x2,3x3) tile, kind 6 (BM 64 x TH 4, 4 waves, two blocks per
CU), through the C ABI -- at fp16 (conv_winoh.hip, v_mfma_f32_32x32x16_f16) and at exact fp32
(conv_winoc.hip, v_mfma_f32_32x32x2_f32; built with the max-ilp scheduler, Makefile
SCHED_conv_winoc).

Both tiles wait for their LDS-DMA stages with counted vmcnt waits (RRIN_VMWAIT) whose counts hold
only for the VMEM issue order the source pins; `make check-isa` proves the order on the ISA, and
these tests check the results: every epilogue on grids of many tiles against float64, the
sub-pixel up conv against upsample-then-conv, the fp16 range guard, and run-to-run bitwise
equality beside an LDS-DMA + MFMA conv looping on another stream (DESIGN.md §9's hazard class).
Round 6 removed the rejected kinds 9-13 (persistent and LDS-shared-U variants) that this file
used to compare against kind 6."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import H8Tensor
from tests.test_gpu_h8 import (conv_h8, keyed_conv, pack_h8, ref_conv, replicate_ring, subpixel_upconv)

pytestmark = pytest.mark.gpu
F16, R32 = _lib.PREC_F16, _lib.PREC_F32R
TOL = {F16: dict(rtol=2e-2, atol=2e-2), R32: dict(rtol=1e-5, atol=1e-5)}


def kind_cfg(kind, prec):
    lib = _lib.lib()
    return next(c for c in range(lib.rrin_conv_h8_cfg_count())
                if lib.rrin_conv_h8_cfg_wino(c) == kind and lib.rrin_conv_h8_cfg_ok(c, prec))


def test_fp16_winograd_kind6_only():
    lib = _lib.lib()
    kinds = {lib.rrin_conv_h8_cfg_wino(c) for c in range(lib.rrin_conv_h8_cfg_count())
             if lib.rrin_conv_h8_cfg_ok(c, F16) and lib.rrin_conv_h8_cfg_wino(c) > 0}
    assert kinds == {6}
    c = kind_cfg(6, F16)
    assert (lib.rrin_conv_h8_cfg_bm(c), lib.rrin_conv_h8_cfg_th(c)) == (64, 4)


@pytest.mark.parametrize("prec", [F16, R32])
@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_REP, _lib.EPI_LEAKY_POOL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 128, 192, 256), (2, 256, 256, 184, 160), (8, 32, 64, 72, 300)])
def test_kind6_every_epilogue(gpu, prec, epi, n, cin, cout, h, w):
    """Many tiles per CU slot (every stage of the chunk pipeline and its counted waits run,
    ragged right edge at w = 300), each epilogue vs float64."""
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    if prec == F16 and cin % 16:
        pytest.skip("fp16 kind 6: 16-channel chunks")
    torch.manual_seed(n * cin + cout + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winoh")
    ref = ref_conv(x, wt, b, None if epi == _lib.EPI_LINEAR else 0.1)
    kw = {}
    if epi == _lib.EPI_LEAKY_POOL:  # the bridge half of a CAT buffer, as the Net writes it
        kw = dict(dst_off=cout, dst=H8Tensor(n, 2 * cout, h, w, gpu, prec))
    dst, pool = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, kind_cfg(6, prec), prec, epi=epi, **kw)
    got = dst.to_nchw(cout, cout) if epi == _lib.EPI_LEAKY_POOL else dst.to_nchw()
    np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), **TOL[prec])
    if epi == _lib.EPI_LEAKY_POOL:
        np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), F.avg_pool2d(ref, 2).numpy(), **TOL[prec])
        assert not dst.to_nchw(0, cout).any()
    if epi == _lib.EPI_LEAKY_REP:
        assert torch.equal(dst.hi[:, :, 0, 8:8 + w], dst.hi[:, :, 1, 8:8 + w])  # replicated top row


@pytest.mark.parametrize("prec", [F16, R32])
@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 96, 256), (2, 256, 128, 92, 160)])
def test_kind6_subpixel(gpu, prec, n, cin, cout, sh, sw):
    """The sub-pixel up conv (unet.py:77-78) on kind 6 with its ring fix-up, vs upsample-then-conv."""
    torch.manual_seed(cin + sh)
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winoh_sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, prec)
    replicate_ring(src)
    dst = subpixel_upconv(src, wt, b, kind_cfg(6, prec), prec, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, prec))
    np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **TOL[prec])
    assert not dst.to_nchw(cout, cout).any()


def test_kind6_fp16_range_guard(gpu):
    """A value past the fp16 range sets the status flag."""
    from tests import hip_helpers as H
    n, cin, cout, h, w = 1, 64, 128, 64, 256
    x = torch.full((n, cin, h, w), 60000.0, device=gpu)
    wt = torch.full((cout, cin, 3, 3), 1.0)
    b = torch.zeros(cout)
    src = H8Tensor.from_nchw(x, F16)
    cfg = kind_cfg(6, F16)
    dst = H8Tensor(n, cout, h, w, gpu, F16)
    whi, _, bp, inv = pack_h8(wt, b, cfg, F16, gpu)
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, F16, 1, 0.1, inv
    d.src, d.dst = src.chunk_view(0, cin), dst.view(0, cout)
    d.whi, d.bias, d.status = whi.data_ptr(), bp.data_ptr(), status.data_ptr()
    _lib.check(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), H.stream(gpu)))
    torch.cuda.synchronize(gpu)
    assert int(status.item()) == 1


@pytest.mark.parametrize("prec", [F16, R32])
def test_winograd_conv_bitwise_beside_side_stream_conv(gpu, prec):
    """A Winograd conv (cin 256, a 920-tile grid as at the C3 part size's level 3) repeated 32
    times is bitwise the same whether or not an LDS-DMA + MFMA conv loops on another stream (the
    two share CUs): a counted wait that retires the wrong loads reads a stage before it lands and
    shows up here as run-to-run differences (the round-5 max-ilp build: 16/16 repeats differed)."""
    from tests import hip_helpers as H
    from tests.test_gpu_concurrency import side_conv
    n, cin, cout, h, w = 2, 256, 256, 92, 160
    x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=gpu) * 2 - 1, prec)
    wt, b = keyed_conv(cin, cout, "conc")
    cfg = kind_cfg(6, prec)
    ref, _ = conv_h8(x, wt, b, cfg, prec, epi=_lib.EPI_LEAKY)
    lib, d, keep = side_conv(gpu, F16)
    side = torch.cuda.Stream(gpu)
    main = torch.cuda.current_stream(gpu)
    whi, _, bp, inv = pack_h8(wt, b, cfg, prec, gpu)
    outs = [H8Tensor(n, cout, h, w, gpu, prec) for _ in range(8)]
    dd = []
    for o in outs:
        e = _lib.ConvH8Desc()
        e.n, e.cin, e.cout, e.cfg, e.prec, e.epi_mode, e.slope, e.inv_wscale = n, cin, cout, cfg, prec, 1, 0.1, inv
        e.src, e.dst = x.chunk_view(0, cin), o.view(0, cout)
        e.whi, e.wlo, e.bias = whi.data_ptr(), whi.data_ptr(), bp.data_ptr()
        dd.append(e)
    bad = 0
    for _ in range(4):
        side.wait_stream(main)
        st = C.c_void_p(side.cuda_stream)
        for _ in range(200):
            _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))
        for e in dd:
            _lib.check(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(e), H.stream(gpu)))
        torch.cuda.synchronize(gpu)
        bad += sum(int(not torch.equal(o.hi, ref.hi)) for o in outs)
    assert bad == 0, f"{bad}/32 convs differ from the serial result"
