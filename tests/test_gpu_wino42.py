"""GPU: the register-U Winograd F(4,3) x F(2,3) tile, kind 14 (conv_winoc42.hip: BM 32 x 32 px x
TH 8, patches 4 wide x 2 tall, 24 transform points, v_mfma_f32_32x32x2_f32), through the C ABI.

Every epilogue on grids of many tiles against float64 (ragged right / bottom edges), the sub-pixel
up conv against upsample-then-conv, the Net's shapes at the tolerance DESIGN.md §5f states, and
run-to-run bitwise equality beside an LDS-DMA + MFMA conv looping on another stream (the counted
vmcnt waits: DESIGN.md §9's hazard class)."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import H8Tensor
from tests.test_gpu_h8 import TOL42, conv_h8, keyed_conv, pack_h8, ref_conv, replicate_ring, subpixel_upconv

pytestmark = pytest.mark.gpu
R32 = _lib.PREC_F32R


def cfg42():
    lib = _lib.lib()
    return next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 14)


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_POOL, _lib.EPI_LEAKY_REP])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 64, 90, 160), (2, 256, 128, 46, 82), (1, 512, 96, 24, 300),
                                            (3, 8, 32, 17, 33)])
def test_kind14_every_epilogue(gpu, epi, n, cin, cout, h, w):
    """Many tiles (the 3-stage chunk pipeline and its counted waits), ragged edges (h % 8, w % 32),
    short K (one chunk), each epilogue vs float64 at TOL42."""
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    torch.manual_seed(n * cin + cout + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "w42")
    ref = ref_conv(x, wt, b, None if epi == _lib.EPI_LINEAR else 0.1)
    kw = {}
    if epi == _lib.EPI_LEAKY_POOL:  # the bridge half of a CAT buffer, as the Net writes it
        kw = dict(dst_off=cout, dst=H8Tensor(n, 2 * cout, h, w, gpu, R32))
    dst, pool = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg42(), R32, epi=epi, **kw)
    got = dst.to_nchw(cout, cout) if epi == _lib.EPI_LEAKY_POOL else dst.to_nchw()
    np.testing.assert_allclose(got.cpu().double().numpy(), ref.numpy(), **TOL42)
    if epi == _lib.EPI_LEAKY_POOL:
        np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), F.avg_pool2d(ref, 2).numpy(), **TOL42)
        assert not dst.to_nchw(0, cout).any()
    if epi == _lib.EPI_LEAKY_REP:
        assert torch.equal(dst.hi[:, :, 0, 8:8 + w], dst.hi[:, :, 1, 8:8 + w])  # replicated top row


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 128, 64, 96, 256), (2, 512, 256, 23, 40), (1, 64, 32, 5, 9)])
def test_kind14_subpixel(gpu, n, cin, cout, sh, sw):
    """The sub-pixel up conv (unet.py:77-78) on kind 14 with the ring fix-up, vs upsample-then-conv."""
    torch.manual_seed(cin + sh)
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "w42_sub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, R32)
    replicate_ring(src)
    for inlaunch in (False, True):  # the correction form and ring_full (second launch for kind 14)
        dst = subpixel_upconv(src, wt, b, cfg42(), R32, inlaunch=inlaunch,
                              dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32))
        np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **TOL42)
        assert not dst.to_nchw(cout, cout).any()


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 256, 256, 92, 160), (2, 64, 32, 360, 640)])
def test_kind14_conv_bitwise_beside_side_stream_conv(gpu, n, cin, cout, h, w):
    """A kind-14 conv (cin 256 on a level-3 grid; cin 64 on a level-1 grid: the persistent
    short-K launch, its next tile's prologue in flight under the epilogue) repeated 32 times is
    bitwise the same whether or not an LDS-DMA + MFMA conv loops on another stream: a counted
    wait that retires the wrong loads reads a stage before it lands and shows up as run-to-run
    differences."""
    from tests import hip_helpers as H
    from tests.test_gpu_concurrency import side_conv
    x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=gpu) * 2 - 1, R32)
    wt, b = keyed_conv(cin, cout, "conc42")
    cfg = cfg42()
    ref, _ = conv_h8(x, wt, b, cfg, R32, epi=_lib.EPI_LEAKY)
    lib, d, keep = side_conv(gpu, _lib.PREC_F16)
    side = torch.cuda.Stream(gpu)
    main = torch.cuda.current_stream(gpu)
    whi, _, bp, inv = pack_h8(wt, b, cfg, R32, gpu)
    outs = [H8Tensor(n, cout, h, w, gpu, R32) for _ in range(8)]
    dd = []
    for o in outs:
        e = _lib.ConvH8Desc()
        e.n, e.cin, e.cout, e.cfg, e.prec, e.epi_mode, e.slope, e.inv_wscale = n, cin, cout, cfg, R32, 1, 0.1, inv
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



@pytest.fixture
def geom():
    """Sets kind 14's tile-geometry policy (rrin_conv_h8_set_wino42_geom) and restores auto."""
    lib = _lib.lib()
    yield lambda mode: lib.rrin_conv_h8_set_wino42_geom(mode)
    lib.rrin_conv_h8_set_wino42_geom(0)


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_POOL, _lib.EPI_LEAKY_REP,
                                 _lib.EPI_SUBPIXEL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 256, 64, 46, 82), (1, 64, 32, 17, 50), (2, 512, 64, 46, 80)])
def test_kind14_geometries_bitwise(gpu, geom, epi, n, cin, cout, h, w):
    """The 32 x 8 and 16 x 16 tiles give the same bits (so the launcher's geometry policy may
    follow the grid and the batch without breaking batch invariance), on ragged grids, every
    epilogue; the 16 x 16 result also against float64."""
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    torch.manual_seed(cin + h + epi)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    src = H8Tensor.from_nchw(x, R32)
    sub = epi == _lib.EPI_SUBPIXEL
    wt, b = keyed_conv(cin, cout, "geo_sub" if sub else "geo")
    if sub:
        replicate_ring(src)
    outs = []
    for mode in (1, 2):
        assert geom(mode) in (0, 1, 2)
        if sub:
            dst = subpixel_upconv(src, wt, b, cfg42(), R32, dst=H8Tensor(n, 2 * cout, 2 * h, 2 * w, gpu, R32))
            outs.append([dst.hi.clone()])
            continue
        kw = dict(dst=H8Tensor(n, 2 * cout, h, w, gpu, R32), dst_off=cout) if epi == _lib.EPI_LEAKY_POOL else {}
        dst, pool = conv_h8(src, wt, b, cfg42(), R32, epi=epi, **kw)
        outs.append([dst.hi.clone()] + ([pool.hi.clone()] if epi == _lib.EPI_LEAKY_POOL else []))
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    if epi == _lib.EPI_LEAKY:
        ref = ref_conv(x, wt, b, 0.1)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL42)


def test_kind14_geometry_policy(gpu, geom):
    """The setter returns the previous policy and rejects modes outside 0-3."""
    assert geom(4) < 0 and geom(-1) < 0
    assert geom(2) == 0 and geom(3) == 2 and geom(1) == 3 and geom(0) == 1


@pytest.mark.parametrize("epi", [_lib.EPI_LINEAR, _lib.EPI_LEAKY, _lib.EPI_LEAKY_POOL, _lib.EPI_LEAKY_REP,
                                 _lib.EPI_SUBPIXEL])
@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 32, 360, 640), (2, 32, 64, 183, 650), (1, 8, 32, 720, 1280)])
def test_kind14_persistent_bitwise(gpu, geom, epi, n, cin, cout, h, w):
    """Short K on a large grid runs persistent workgroups (the next tile's first raw chunks in
    flight under this tile's epilogue, two-phase exchange): the same bits as one workgroup per
    tile (policy 3), every epilogue, ragged grids; and the persistent result against float64."""
    if epi == _lib.EPI_LEAKY_POOL and (h % 2 or w % 2):
        pytest.skip("pool needs even sizes")
    torch.manual_seed(cin + h + epi + 7)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    src = H8Tensor.from_nchw(x, R32)
    sub = epi == _lib.EPI_SUBPIXEL
    wt, b = keyed_conv(cin, cout, "pers_sub" if sub else "pers")
    if sub:
        replicate_ring(src)
    outs = []
    for mode in (3, 0):
        assert geom(mode) in (0, 1, 2, 3)
        if sub:
            dst = subpixel_upconv(src, wt, b, cfg42(), R32, dst=H8Tensor(n, 2 * cout, 2 * h, 2 * w, gpu, R32))
            outs.append([dst.hi.clone()])
            continue
        kw = dict(dst=H8Tensor(n, 2 * cout, h, w, gpu, R32), dst_off=cout) if epi == _lib.EPI_LEAKY_POOL else {}
        dst, pool = conv_h8(src, wt, b, cfg42(), R32, epi=epi, **kw)
        outs.append([dst.hi.clone()] + ([pool.hi.clone()] if epi == _lib.EPI_LEAKY_POOL else []))
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    if epi == _lib.EPI_LEAKY and n * h * w <= 2 * 360 * 640:
        ref = ref_conv(x, wt, b, 0.1)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL42)
