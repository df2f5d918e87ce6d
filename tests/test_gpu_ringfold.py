"""GPU: the sub-pixel up conv with its ring fix-up folded into the conv launch
(rrin_conv_h8_desc.ring_w; Winograd kind 3, the Net's exact-fp32 up.1 convs):
conv3x3(upsample_x2(x)) against float64 on the whole 2h x 2w output at the R32
tolerance (1e-5), including 1-pixel and odd low-res grids; the segment tickets are
left at zero; runs agree bitwise; the interior equals the unfolded launch's bit for
bit (only the ring is computed differently)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import H8Tensor
from tests.test_gpu_h8 import R32, TOL, keyed_conv, replicate_ring, subpixel_upconv

pytestmark = pytest.mark.gpu


def kind3():
    lib = _lib.lib()
    return next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) == 3)


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(2, 64, 32, 20, 36), (1, 128, 64, 23, 40), (1, 256, 128, 5, 7),
                                              (2, 256, 128, 45, 80), (1, 64, 32, 1, 1), (1, 64, 32, 9, 33),
                                              (3, 128, 64, 17, 65)])
def test_ring_fold_vs_float64(gpu, n, cin, cout, sh, sw):
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "fold")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, R32)
    replicate_ring(src)
    cfg = kind3()
    keep = []
    dst = subpixel_upconv(src, wt, b, cfg, R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32), fold=True,
                          keep=keep)
    got = dst.to_nchw(0, cout).cpu().double()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), **TOL[R32])
    assert not dst.to_nchw(cout, cout).any()                          # the bridge half of CAT is untouched
    assert not dst.hi[:, :, 0].any() and not dst.hi[:, :, :, :8].any()  # zero padding kept
    assert not keep[1].any(), "segment tickets left nonzero"
    again = subpixel_upconv(src, wt, b, cfg, R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32), fold=True)
    assert torch.equal(again.hi, dst.hi)
    plain = subpixel_upconv(src, wt, b, cfg, R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32))
    inner = (slice(None), slice(None), slice(1, -1), slice(1, -1))
    assert torch.equal(plain.to_nchw(0, cout)[inner], dst.to_nchw(0, cout)[inner])


def test_ring_fold_rejected_elsewhere(gpu):
    """Only the 8-wave Winograd tile folds: other configs and a split report RRIN_E_CONFIG."""
    import ctypes as C
    lib = _lib.lib()
    x = H8Tensor(1, 64, 8, 8, gpu, R32)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.prec, d.epi_mode, d.slope = 1, 64, 128, R32, _lib.EPI_SUBPIXEL, 0.1
    d.src, d.dst = x.view(), H8Tensor(1, 32, 16, 16, gpu, R32).view()
    d.whi, d.bias, d.edge, d.ring_w, d.ring_bias = 1, 1, 1, 1, 1
    for c in range(lib.rrin_conv_h8_cfg_count()):
        if not lib.rrin_conv_h8_cfg_ok(c, R32):
            continue
        d.cfg = c
        r = lib.rrin_conv_h8_ring_floats(C.byref(d), None)
        assert (r > 0) == (c == kind3()), (c, r)
    d.cfg, d.ksplit = kind3(), 2
    assert lib.rrin_conv_h8_ring_floats(C.byref(d), None) < 0
