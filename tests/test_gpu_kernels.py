"""GPU: each HIP kernel of librrin_hip.so against the CPU oracle / goldens.

Tolerances: fp32 kernels vs float64 CPU references; a 3x3 conv with K = 9*Cin
<= 4608 accumulates ~1e-6 relative rounding, so 1e-4 abs/rel is a loose bound
that still catches any indexing error (those are O(1))."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd.pp import PPTensor
from rrin_amd.synthetic import keyed_tensor
from tests import hip_helpers as H
from tests.golden.spec import CONV_CLASSES

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)


def ref_conv(x, w, b, slope=None):
    y = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    return F.leaky_relu(y, slope) if slope is not None else y


def keyed_conv(cin, cout, key="t"):
    w = keyed_tensor(f"{key}.{cin}.{cout}.w", (cout, cin, 3, 3), cin * 9)
    b = keyed_tensor(f"{key}.{cin}.{cout}.b", (cout,), cin * 9)
    return w, b


def cfgs_for(cout):
    lib = _lib.lib()
    return [c for c in range(lib.rrin_conv_cfg_count()) if lib.rrin_conv_cfg_bm(c) <= max(32, 2 * cout)]


def test_layout_roundtrip(gpu):
    x = torch.randn(2, 5, 23, 40, device=gpu)
    pp = PPTensor.from_nchw(x, c_alloc=7, ch_off=1)
    assert torch.equal(pp.to_nchw(1, 5), x)
    t = pp.t
    assert not t[:, 0].any() and not t[:, 6].any()
    assert not t[:, :, 0].any() and not t[:, :, 24:].any()
    assert not t[:, :, :, :32].any() and not t[:, :, :, 72:].any()


@pytest.mark.parametrize("cin,cout", CONV_CLASSES)
def test_conv_golden_classes(gpu, golden, cin, cout):
    g = golden("ops")
    w = keyed_tensor(f"golden.conv.{cin}.{cout}.weight", (cout, cin, 3, 3), cin * 9)
    b = keyed_tensor(f"golden.conv.{cin}.{cout}.bias", (cout,), cin * 9)
    x = torch.from_numpy(g[f"conv_{cin}_{cout}_in"]).to(gpu)
    for cfg in cfgs_for(cout):
        dst, _ = H.conv(PPTensor.from_nchw(x), w, b, cfg)
        np.testing.assert_allclose(dst.to_nchw().cpu().numpy(), g[f"conv_{cin}_{cout}_out"], **TOL,
                                   err_msg=f"cfg {cfg}")


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 64, 32, 40, 72), (1, 128, 64, 23, 40), (2, 32, 64, 16, 96),
                                            (1, 256, 256, 12, 20), (1, 10, 32, 48, 64)])
def test_conv_leaky_random(gpu, n, cin, cout, h, w):
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout)
    ref = ref_conv(x, wt, b, 0.1)
    for cfg in cfgs_for(cout):
        dst, _ = H.conv(PPTensor.from_nchw(x), wt, b, cfg, epi=_lib.EPI_LEAKY)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL, err_msg=f"cfg {cfg}")


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 32, 32, 32, 64), (1, 64, 64, 46, 80), (1, 128, 256, 10, 6)])
def test_conv_pool_epilogue(gpu, n, cin, cout, h, w):
    """conv -> leaky -> (bridge, avg_pool2d) — unet.py:44-46."""
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "pool")
    ref = ref_conv(x, wt, b, 0.1)
    refp = F.avg_pool2d(ref, 2)
    for cfg in cfgs_for(cout):
        # bridge written at channel offset cout of a 2*cout "cat" buffer (unet.py:93)
        dst, pool = H.conv(PPTensor.from_nchw(x), wt, b, cfg, epi=_lib.EPI_LEAKY_POOL, dst_off=cout,
                           dst=PPTensor(n, 2 * cout, h, w, gpu))
        np.testing.assert_allclose(dst.to_nchw(cout, cout).cpu().double().numpy(), ref.numpy(), **TOL)
        assert not dst.to_nchw(0, cout).any()
        np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), refp.numpy(), **TOL,
                                   err_msg=f"cfg {cfg}")


@pytest.mark.parametrize("n,cin,cout,h,w", [(1, 64, 32, 20, 36), (2, 128, 64, 8, 16), (1, 512, 256, 5, 7),
                                            (1, 256, 128, 23, 40)])
def test_conv_upsample_prologue(gpu, n, cin, cout, h, w):
    """nn.Upsample(bilinear, x2) -> conv (no act) — unet.py:76-79."""
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "up")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = ref_conv(up, wt, b)
    for cfg in cfgs_for(cout):
        dst, _ = H.conv(PPTensor.from_nchw(x), wt, b, cfg, upsample=True)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL, err_msg=f"cfg {cfg}")


def test_conv_channel_views(gpu):
    """src channel offset + Cin not a multiple of 8 + permutation (refine's first conv)."""
    x = torch.rand(2, 16, 32, 48, device=gpu)
    wt, b = keyed_conv(10, 32, "perm")
    perm = [4, 5, 6, 7, 8, 9, 0, 1, 2, 3]
    # buffer channels = [x0 x1 Ft0 Ft1 ...]; reference input order = [Ft0 Ft1 x0 x1]
    ref_in = torch.cat([x[:, 6:10], x[:, 0:6]], 1)
    ref = ref_conv(ref_in, wt, b)
    dst, _ = H.conv(PPTensor.from_nchw(x), wt, b, 0, perm=perm, cin=10)
    np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL)


def test_warp_golden(gpu, golden):
    g = golden("ops")
    img = torch.from_numpy(g["warp_img"]).to(gpu)
    lib = _lib.lib()
    for fk, ok in [("warp_flow", "warp_out"), ("warp_flow_far", "warp_out_far")]:
        flow = torch.from_numpy(g[fk]).to(gpu)
        out = torch.empty_like(img)
        _lib.check(lib.rrin_warp_fwd(img.data_ptr(), flow.data_ptr(), out.data_ptr(), 2, 3, 9, 11,
                                     H.stream(gpu)))
        torch.cuda.synchronize()
        np.testing.assert_allclose(out.cpu().numpy(), g[ok], rtol=0, atol=1e-5)


def test_warp_extreme_flows(gpu):
    img = torch.rand(1, 3, 16, 32, device=gpu)
    flow = torch.tensor([1e9, -1e9, float("inf"), 3.5]).repeat(1, 2, 16, 8)[:, :, :, :32].contiguous().to(gpu)
    out = torch.empty_like(img)
    _lib.check(_lib.lib().rrin_warp_fwd(img.data_ptr(), flow.data_ptr(), out.data_ptr(), 1, 3, 16, 32,
                                        H.stream(gpu)))
    torch.cuda.synchronize()
    assert torch.isfinite(out[..., 0::4]).all()


@pytest.mark.parametrize("cout", [2, 3, 4])
def test_head_plain(gpu, cout):
    x = torch.rand(2, 32, 40, 72, device=gpu) * 2 - 1
    wt, b = keyed_conv(32, cout, "head")
    dst = PPTensor(2, 16, 40, 72, gpu)
    H.head(PPTensor.from_nchw(x), dst, wt, b, _lib.HEAD_PLAIN)
    np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref_conv(x, wt, b).numpy(), **TOL)


def test_head_fused_glue(gpu):
    """FLOW, REFINE, MASK, FINAL epilogues vs the oracle's torch-op glue."""
    from oracle.ref_net import warp as ref_warp
    from rrin_amd.engine import t_coefficients
    n, h, w, t = 2, 32, 64, 0.3
    gen = torch.Generator().manual_seed(1)
    x0 = torch.rand(n, 3, h, w, generator=gen)
    x1 = torch.rand(n, 3, h, w, generator=gen)
    feat = [torch.rand(n, 32, h, w, generator=gen) * 2 - 1 for _ in range(4)]
    W = [keyed_conv(32, c, f"glue{k}") for k, c in enumerate([4, 4, 2, 3])]
    W[0] = (W[0][0] * 300, W[0][1])  # large flows: exercise out-of-frame taps
    coef = t_coefficients(t, n).to(gpu)
    g16 = PPTensor(n, 16, h, w, gpu)
    g16.load(x0.to(gpu), 0)
    g16.load(x1.to(gpu), 3)
    # FLOW
    H.head(PPTensor.from_nchw(feat[0].to(gpu)), g16, *W[0], _lib.HEAD_FLOW, coef)
    fl = ref_conv(feat[0], *W[0]).float()
    ft0 = -(1 - t) * t * fl[:, :2] + t * t * fl[:, 2:4]
    ft1 = (1 - t) * (1 - t) * fl[:, :2] - t * (1 - t) * fl[:, 2:4]
    np.testing.assert_allclose(g16.to_nchw(6, 2).cpu().numpy(), ft0.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(g16.to_nchw(8, 2).cpu().numpy(), ft1.numpy(), rtol=1e-4, atol=1e-3)
    # REFINE (start from the kernel's own Ft so only this stage's error is measured)
    ft0 = g16.to_nchw(6, 2).cpu()
    ft1 = g16.to_nchw(8, 2).cpu()
    H.head(PPTensor.from_nchw(feat[1].to(gpu)), g16, *W[1], _lib.HEAD_REFINE, coef)
    r = ref_conv(feat[1], *W[1]).float()
    ft0r, ft1r = ft0 + r[:, :2], ft1 + r[:, 2:4]
    np.testing.assert_allclose(g16.to_nchw(6, 2).cpu().numpy(), ft0r.numpy(), rtol=1e-5, atol=1e-4)
    ft0g = g16.to_nchw(6, 2).cpu()
    ft1g = g16.to_nchw(8, 2).cpu()
    np.testing.assert_allclose(g16.to_nchw(10, 3).cpu().numpy(), ref_warp(x0, ft0g).numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(g16.to_nchw(13, 3).cpu().numpy(), ref_warp(x1, ft1g).numpy(), rtol=0, atol=1e-5)
    # MASK
    xt1 = g16.to_nchw(10, 3).cpu()
    xt2 = g16.to_nchw(13, 3).cpu()
    H.head(PPTensor.from_nchw(feat[2].to(gpu)), g16, *W[2], _lib.HEAD_MASK, coef)
    m = torch.sigmoid(ref_conv(feat[2], *W[2]).float())
    w1, w2 = (1 - t) * m[:, 0:1], t * m[:, 1:2]
    blend = (w1 * xt1 + w2 * xt2) / (w1 + w2 + 1e-8)
    np.testing.assert_allclose(g16.to_nchw(6, 3).cpu().numpy(), blend.numpy(), rtol=0, atol=1e-5)
    # FINAL
    blend_g = g16.to_nchw(6, 3).cpu()
    out = torch.empty(n, 3, h, w, device=gpu)
    H.head(PPTensor.from_nchw(feat[3].to(gpu)), g16, *W[3], _lib.HEAD_FINAL, coef, out=out)
    fin = (ref_conv(feat[3], *W[3]).float() + blend_g).clamp(0, 1)
    np.testing.assert_allclose(out.cpu().numpy(), fin.numpy(), rtol=0, atol=1e-5)
