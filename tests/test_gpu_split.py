"""GPU: split-K of the Winograd exact-fp32 conv (rrin_conv_h8_desc.ksplit; tile kinds 3
and 4).  A split conv sums the K slices' pre-bias outputs in slice order: a
different association of the same fp32 sums, held to the R32 tolerance (1e-5)
against float64 like every record conv, in every epilogue; the tile counters are
left at zero; two runs agree bitwise; the Net with split convs matches the
unsplit Net to fp32 rounding and keeps batch == per-sample bitwise."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib
from rrin_amd import engine as engine_mod
from rrin_amd.pp import H8Tensor
from rrin_amd.synthetic import synthetic_batch
from tests.test_gpu_net import make_net
from tests.test_gpu_h8 import R32, TOL, conv_h8, keyed_conv, ref_conv, replicate_ring, subpixel_upconv

pytestmark = pytest.mark.gpu


def split_cfgs():
    lib = _lib.lib()
    return [c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c) in (3, 4)]


@pytest.mark.parametrize("ksplit", [2, 3, 8])
@pytest.mark.parametrize("epi", [_lib.EPI_LEAKY, _lib.EPI_LEAKY_POOL, _lib.EPI_LINEAR])
def test_split_conv_vs_float64(gpu, ksplit, epi):
    n, cin, cout, h, w = 2, 96, 64, 46, 80   # 12 chunks: slices of 6 / 4 / 2 (8 -> 6 slices of 2)
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "split")
    slope = None if epi == _lib.EPI_LINEAR else 0.1
    ref = ref_conv(x, wt, b, slope)
    for cfg in split_cfgs():
        keep = []
        dst, pool = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg, R32, epi=epi, ksplit=ksplit, keep=keep)
        np.testing.assert_allclose(dst.to_nchw().cpu().double().numpy(), ref.numpy(), **TOL[R32],
                                   err_msg=f"cfg {cfg} ksplit {ksplit}")
        if pool is not None:
            np.testing.assert_allclose(pool.to_nchw().cpu().double().numpy(), F.avg_pool2d(ref, 2).numpy(),
                                       **TOL[R32], err_msg=f"cfg {cfg} pool")
        assert not keep[1].any(), "tile counters left nonzero"
        dst2, _ = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg, R32, epi=epi, ksplit=ksplit, keep=keep)
        assert torch.equal(dst.hi, dst2.hi), f"cfg {cfg}: split conv not deterministic"


def test_split_leaky_rep(gpu):
    n, cin, cout, h, w = 1, 256, 32, 23, 40
    x = torch.rand(n, cin, h, w, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "splitrep")
    for cfg in split_cfgs():
        base, _ = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg, R32, epi=_lib.EPI_LEAKY_REP)
        spl, _ = conv_h8(H8Tensor.from_nchw(x, R32), wt, b, cfg, R32, epi=_lib.EPI_LEAKY_REP, ksplit=4)
        hi0 = base.hi.view(torch.float32) if base.hi.dtype != torch.float32 else base.hi
        hi1 = spl.hi.view(torch.float32) if spl.hi.dtype != torch.float32 else spl.hi
        np.testing.assert_allclose(hi1.cpu().numpy(), hi0.cpu().numpy(), rtol=1e-5, atol=1e-5,
                                   err_msg=f"cfg {cfg}")   # interior and the replicated ring


@pytest.mark.parametrize("n,cin,cout,sh,sw", [(1, 512, 256, 23, 40), (2, 128, 64, 5, 7)])
def test_split_subpixel(gpu, n, cin, cout, sh, sw):
    x = torch.rand(n, cin, sh, sw, device=gpu) * 2 - 1
    wt, b = keyed_conv(cin, cout, "splitsub")
    up = F.interpolate(x.double().cpu(), scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(up, wt.double().cpu(), b.double().cpu(), padding=1)
    src = H8Tensor.from_nchw(x, R32)
    replicate_ring(src)
    for cfg in split_cfgs():
        dst = subpixel_upconv(src, wt, b, cfg, R32, dst=H8Tensor(n, 2 * cout, 2 * sh, 2 * sw, gpu, R32), ksplit=4)
        np.testing.assert_allclose(dst.to_nchw(0, cout).cpu().double().numpy(), ref.numpy(), **TOL[R32],
                                   err_msg=f"cfg {cfg}")


def test_split_net(gpu):
    """Split-K in the Net: the geometry rule (engine.geom_split, the default: 128x192
    images split their level-3/4 convs) and levels 2-4 split by the A/B override with
    every conv on a split-capable tile; each within fp32 rounding of the unsplit Net,
    batch == per-sample bitwise with the split.  The F(2x2,3x3) kinds only (engine.WINO42_LEVELS
    off): kind 14 rounds differently from the split kinds."""
    net = make_net(gpu, stress=True)
    saved = dict(engine_mod.WINO_SPLIT_LEVELS)
    saved_geo, saved_kind = engine_mod.GEOM_SPLIT, engine_mod.WINO_KIND
    saved42 = engine_mod.WINO42_LEVELS
    engine_mod.WINO42_LEVELS = ()
    try:
        i0, i1 = synthetic_batch(2, 128, 192)
        i0, i1 = i0.to(gpu), i1.to(gpu)
        engine_mod.WINO_SPLIT_LEVELS.clear()
        engine_mod.GEOM_SPLIT = False
        with torch.no_grad():
            net._engine = None
            base = net.engine().forward(i0, i1, 0.5).cpu()
        for geo, levels, kind in ((True, {}, saved_kind), (False, {2: 2, 3: 4, 4: 8}, 3)):
            engine_mod.GEOM_SPLIT, engine_mod.WINO_KIND = geo, kind
            engine_mod.WINO_SPLIT_LEVELS.clear()
            engine_mod.WINO_SPLIT_LEVELS.update(levels)
            net._engine = None
            eng = net.engine()
            assert any(t.ksplit > 1 for t in eng.conv_table_for(2, 128, 192))
            with torch.no_grad():
                both = eng.forward(i0, i1, 0.5).cpu()
                one = eng.forward(i0[1:], i1[1:], 0.5).cpu()
            torch.testing.assert_close(both, base, rtol=0, atol=2e-5)
            assert torch.equal(both[1:], one)
    finally:
        engine_mod.WINO_SPLIT_LEVELS.clear()
        engine_mod.WINO_SPLIT_LEVELS.update(saved)
        engine_mod.GEOM_SPLIT, engine_mod.WINO_KIND = saved_geo, saved_kind
        engine_mod.WINO42_LEVELS = saved42
        net._engine = None
