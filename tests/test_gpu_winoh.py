"""GPU: the fp16 Winograd F(2x2,3x3) tiles (rrin_amd/csrc/conv_winoh.hip) and the persistent
exact-fp32 tile (kind 12, conv_winoc.hip) through the C ABI.

Kinds 6 (BM 64 x TH 4, two blocks per CU) and 9 (BM 64 x TH 8, one block per CU) run one tile
per workgroup; kinds 10 and 11 are the same tiles on a persistent grid: each workgroup walks
several tiles, its chunk pipeline loads the next tile's first chunks during the current tile's
last ones, and every epilogue store is an unconditional buffer store (out-of-image positions
dropped).  The persistent kinds must give the bits of their one-tile forms on grids with many
more tiles than workgroups (so that the tile walk, the cross-tile prefetch and the counted
waits all run), for every epilogue; all of them sit within the fp16 gate of float64.

The persistent kinds fall back to their one-tile forms below 2 tiles per workgroup slot (two
slots per CU for kinds 10 and 12, one for kind 11): every size here is above that (checked),
so the tile walk runs.

Kinds 9-11 are built into the lab library only: their tests run against it
(RRIN_LIB_AB=rrin_amd/librrin_lab.so after `make lab`) and skip on the product library."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import H8Tensor
from tests.test_gpu_h8 import (conv_h8, keyed_conv, ref_conv, replicate_ring, subpixel_upconv)

pytestmark = pytest.mark.gpu
F16 = _lib.PREC_F16
TOLF = dict(rtol=2e-2, atol=2e-2)


def kinds():
    lib = _lib.lib()
    return {lib.rrin_conv_h8_cfg_wino(c): c for c in range(lib.rrin_conv_h8_cfg_count())
            if lib.rrin_conv_h8_cfg_ok(c, F16) and lib.rrin_conv_h8_cfg_wino(c)}


PAIRS = [(6, 10), (9, 11)]  # one-tile kind -> its persistent kind


def need_lab_kinds():
    if not {9, 10, 11, 13} <= set(kinds()):
        pytest.skip("fp16 kinds 9-11, 13: lab library only")


def assert_walks(n, cout_rows, h, w, th, slots_per_cu):
    """The grid of this conv has >= 2 tiles per persistent workgroup slot (else the library runs
    the one-tile form and the comparison would test nothing)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    tiles = -(-cout_rows // 64) * -(-w // 32) * -(-h // th) * n
    assert tiles >= 2 * slots_per_cu * cus, (tiles, cus)


def test_fp16_winograd_kinds_present():
    k = kinds()
    assert set(k) in ({6}, {6, 9, 10, 11, 13}), k
    need_lab_kinds()
    lib = _lib.lib()
    for a, b in PAIRS:
        assert lib.rrin_conv_h8_cfg_bm(k[a]) == lib.rrin_conv_h8_cfg_bm(k[b]) == 64
        assert lib.rrin_conv_h8_cfg_th(k[a]) == lib.rrin_conv_h8_cfg_th(k[b])


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_REP, _lib.EPI_LEAKY_POOL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 128, 192, 256), (2, 256, 256, 184, 160), (8, 32, 64, 72, 300)])
def test_persistent_bitwise_and_parity(gpu, epi, n, cin, cout, h, w):
    need_lab_kinds()
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    assert_walks(n, cout, h, w, 4, 2)
    assert_walks(n, cout, h, w, 8, 1)
    torch.manual_seed(n * cin + cout + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winoh")
    slope = None if epi == _lib.EPI_LINEAR else 0.1
    ref = ref_conv(x, wt, b, slope)
    k = kinds()
    for a, p in PAIRS:
        outs = []
        for cfg in (k[a], k[p]):
            kw = {}
            if epi == _lib.EPI_LEAKY_POOL:  # the bridge half of a CAT buffer, as the Net writes it
                kw = dict(dst_off=cout, dst=H8Tensor(n, 2 * cout, h, w, gpu, F16))
            dst, pool = conv_h8(H8Tensor.from_nchw(x, F16), wt, b, cfg, F16, epi=epi, **kw)
            outs.append((dst, pool))
            got = dst.to_nchw(cout, cout) if epi == _lib.EPI_LEAKY_POOL else dst.to_nchw()
            np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), **TOLF, err_msg=f"cfg {cfg}")
            if epi == _lib.EPI_LEAKY_POOL:
                np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), F.avg_pool2d(ref, 2).numpy(),
                                           **TOLF, err_msg=f"cfg {cfg} pool")
                assert not dst.to_nchw(0, cout).any()
        (d0, p0), (d1, p1) = outs
        assert torch.equal(d0.hi, d1.hi), f"kind {p} differs from kind {a}"  # padding / replicated ring too
        if epi == _lib.EPI_LEAKY_POOL:
            assert torch.equal(p0.hi, p1.hi)
        if epi == _lib.EPI_LEAKY_REP:
            ring = d1.hi[:, :, 0, 8:8 + w]  # the replicated top row equals the first image row
            assert torch.equal(ring, d1.hi[:, :, 1, 8:8 + w])


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 96, 256), (2, 256, 128, 92, 160)])
def test_persistent_subpixel(gpu, n, cin, cout, sh, sw):
    """The sub-pixel up conv (unet.py:77-78) on the persistent kinds: ring scratch + interior
    stores, bitwise the one-tile kinds, within the fp16 gate of upsample-then-conv."""
    need_lab_kinds()
    assert_walks(n, 4 * cout, sh, sw, 4, 2)
    assert_walks(n, 4 * cout, sh, sw, 8, 1)
    torch.manual_seed(cin + sh)
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winoh_sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, F16)
    replicate_ring(src)
    k = kinds()
    for a, p in PAIRS:
        d0 = subpixel_upconv(src, wt, b, k[a], F16, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, F16))
        d1 = subpixel_upconv(src, wt, b, k[p], F16, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, F16))
        np.testing.assert_allclose(d1.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **TOLF)
        assert torch.equal(d0.hi, d1.hi), f"kind {p} differs from kind {a}"
        assert not d1.to_nchw(cout, cout).any()


def test_persistent_range_guard(gpu):
    """A value past the fp16 range sets the status flag in the persistent kinds as well."""
    need_lab_kinds()
    import ctypes as C

    from tests import hip_helpers as H
    from tests.test_gpu_h8 import pack_h8
    n, cin, cout, h, w = 1, 64, 128, 64, 256
    x = torch.full((n, cin, h, w), 60000.0, device=gpu)
    wt = torch.full((cout, cin, 3, 3), 1.0)
    b = torch.zeros(cout)
    src = H8Tensor.from_nchw(x, F16)
    for cfg in kinds().values():
        dst = H8Tensor(n, cout, h, w, gpu, F16)
        whi, _, bp, inv = pack_h8(wt, b, cfg, F16, gpu)
        status = torch.zeros(1, dtype=torch.int32, device=gpu)
        d = _lib.ConvH8Desc()
        d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, F16, 1, 0.1, inv
        d.src, d.dst = src.chunk_view(0, cin), dst.view(0, cout)
        d.whi, d.bias, d.status = whi.data_ptr(), bp.data_ptr(), status.data_ptr()
        _lib.check(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), H.stream(gpu)))
        torch.cuda.synchronize(gpu)
        assert int(status.item()) == 1, f"cfg {cfg}"


R32 = _lib.PREC_F32R


def kind_cfg(kind, prec):
    lib = _lib.lib()
    return next(c for c in range(lib.rrin_conv_h8_cfg_count())
                if lib.rrin_conv_h8_cfg_wino(c) == kind and lib.rrin_conv_h8_cfg_ok(c, prec))


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_REP, _lib.EPI_LEAKY_POOL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 128, 192, 256), (2, 256, 256, 184, 160), (8, 32, 64, 72, 300)])
def test_fp32_persistent_bitwise(gpu, epi, n, cin, cout, h, w):
    """Exact fp32: kind 12 (kind 6 on a persistent grid) gives kind 6's bits on grids of many
    tiles per workgroup, for every epilogue, within 1e-5 of float64."""
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    assert_walks(n, cout, h, w, 4, 2)
    torch.manual_seed(n * cin + cout + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winocp")
    ref = ref_conv(x, wt, b, None if epi == _lib.EPI_LINEAR else 0.1)
    outs = []
    for cfg in (kind_cfg(6, R32), kind_cfg(12, R32)):
        kw = {}
        if epi == _lib.EPI_LEAKY_POOL:
            kw = dict(dst_off=cout, dst=H8Tensor(n, 2 * cout, h, w, gpu, R32))
        dst, pool = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg, R32, epi=epi, **kw)
        got = dst.to_nchw(cout, cout) if epi == _lib.EPI_LEAKY_POOL else dst.to_nchw()
        np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
        outs.append((dst, pool))
    assert torch.equal(outs[0][0].hi, outs[1][0].hi)
    if epi == _lib.EPI_LEAKY_POOL:
        assert torch.equal(outs[0][1].hi, outs[1][1].hi)


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 96, 256), (5, 64, 32, 90, 160)])
def test_fp32_persistent_subpixel(gpu, n, cin, cout, sh, sw):
    assert_walks(n, 4 * cout, sh, sw, 4, 2)
    torch.manual_seed(cin + sh)
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winocp_sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, R32)
    replicate_ring(src)
    d0 = subpixel_upconv(src, wt, b, kind_cfg(6, R32), R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32))
    d1 = subpixel_upconv(src, wt, b, kind_cfg(12, R32), R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32))
    np.testing.assert_allclose(d1.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    assert torch.equal(d0.hi, d1.hi)


@pytest.mark.parametrize("prec,kind", [(F16, 6), (F16, 10), (R32, 6), (R32, 12)])
def test_winograd_conv_bitwise_beside_side_stream_conv(gpu, prec, kind):
    """A Winograd conv (cin 256, a 920-tile grid as at the C3 part size's level 3) is bitwise the
    same whether or not an LDS-DMA + MFMA conv loops on another stream (the two share CUs):
    the fp16 tiles' packed-f16 input transform and the persistent tiles' cross-tile pipeline
    beside another kernel (DESIGN.md §9's hazard class)."""
    import ctypes as C

    from tests import hip_helpers as H
    from tests.test_gpu_concurrency import side_conv
    n, cin, cout, h, w = 2, 256, 256, 92, 160
    x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=gpu) * 2 - 1, prec)
    wt, b = keyed_conv(cin, cout, "conc")
    if kind not in kinds() and prec == F16:
        pytest.skip(f"fp16 kind {kind}: lab library only")
    cfg = kind_cfg(kind, prec)
    ref, _ = conv_h8(x, wt, b, cfg, prec, epi=_lib.EPI_LEAKY)
    lib, d, keep = side_conv(gpu, F16)
    side = torch.cuda.Stream(gpu)
    main = torch.cuda.current_stream(gpu)
    from tests.test_gpu_h8 import pack_h8
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


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_REP, _lib.EPI_LEAKY_POOL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 128, 48, 96), (1, 256, 256, 92, 160), (3, 32, 64, 22, 70),
                                            (1, 16, 64, 46, 80)])
def test_kind13_bitwise_kind6(gpu, epi, n, cin, cout, h, w):
    """Kind 13 (two patch tiles per workgroup, U shared through LDS; lab library) gives kind 6's
    bits: the same U, transforms and accumulation order -- ragged tile rows (h % 8), every
    epilogue."""
    need_lab_kinds()
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    torch.manual_seed(n * cin + cout + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winohl")
    slope = None if epi == _lib.EPI_LINEAR else 0.1
    ref = ref_conv(x, wt, b, slope)
    outs = []
    for kind in (6, 13):
        kw = {}
        if epi == _lib.EPI_LEAKY_POOL:
            kw = dict(dst_off=cout, dst=H8Tensor(n, 2 * cout, h, w, gpu, F16))
        dst, pool = conv_h8(H8Tensor.from_nchw(x, F16), wt, b, kind_cfg(kind, F16), F16, epi=epi, **kw)
        got = dst.to_nchw(cout, cout) if epi == _lib.EPI_LEAKY_POOL else dst.to_nchw()
        np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), **TOLF, err_msg=f"kind {kind}")
        outs.append((dst, pool))
    (d0, p0), (d1, p1) = outs
    assert torch.equal(d0.hi, d1.hi)
    if epi == _lib.EPI_LEAKY_POOL:
        assert torch.equal(p0.hi, p1.hi)


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 46, 80), (1, 256, 128, 92, 160)])
def test_kind13_subpixel(gpu, n, cin, cout, sh, sw):
    need_lab_kinds()
    torch.manual_seed(cin + sh)
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "winohl_sub")
    src = H8Tensor.from_nchw(x, F16)
    replicate_ring(src)
    d0 = subpixel_upconv(src, wt, b, kind_cfg(6, F16), F16, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, F16))
    d1 = subpixel_upconv(src, wt, b, kind_cfg(13, F16), F16, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, F16))
    assert torch.equal(d0.hi, d1.hi)
