"""GPU: the drop-in ``rrin_amd.Net`` (HIP path, librrin_hip.so) against the
reference goldens and the CPU oracle.  Gate (BASELINE.json north_star):
max-abs <= 1e-3 fp32 per pixel; the default-weight cases also hold 1e-4."""
import numpy as np
import pytest
import torch

from oracle.ref_net import net_forward
from rrin_amd import engine as engine_mod
from rrin_amd import Net
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch

pytestmark = pytest.mark.gpu
GATE = 1e-3


def make_net(dev, stress=False):
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=stress), strict=True)
    return net.to(dev).eval()


@pytest.fixture(scope="module")
def nets(gpu):
    return {"default": make_net(gpu), "stress": make_net(gpu, True)}


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.mark.parametrize("precision", ["fp32", "fp32_planar"])
@pytest.mark.parametrize("which", ["default", "stress"])
def test_net_golden(gpu, golden, nets, which, precision):
    """Exact fp32 (record layout, the default; and the planar layout) against the
    unmodified reference's outputs."""
    g = golden("net_" + which)
    net = nets[which]
    net.precision = precision
    i0, i1 = torch.from_numpy(g["i0"]).to(gpu), torch.from_numpy(g["i1"]).to(gpu)
    tight = 1e-4 if which == "default" else GATE
    with torch.no_grad():
        for t, key in [(0.5, "out_t050"), (0.25, "out_t025"),
                       (torch.from_numpy(g["t_tensor"]).view(-1, 1, 1, 1).to(gpu), "out_ttensor")]:
            out = net(i0, i1, t=t)
            assert out.shape == i0.shape and out.dtype == torch.float32 and out.device == i0.device
            err = maxabs(out.cpu(), g[key])
            assert err <= tight, f"{which} {key}: max-abs {err:.3e}"
    net.precision = "fp32"


def test_net_golden_odd_levels(gpu, golden, nets):
    g = golden("net_odd")  # 80x112: 5x7 at the Flow bottom
    with torch.no_grad():
        out = nets["default"](torch.from_numpy(g["i0"]).to(gpu), torch.from_numpy(g["i1"]).to(gpu), 0.5)
    assert maxabs(out.cpu(), g["out_t050"]) <= 1e-4


@pytest.mark.parametrize("h,w,n,which", [(256, 256, 1, "stress"), (368, 640, 1, "default"),
                                         (720, 1280, 1, "default"), (720, 1280, 1, "stress")])
def test_net_vs_oracle(gpu, nets, h, w, n, which):
    """Larger sizes against the CPU oracle (same torch-op sequence as the reference)."""
    i0, i1 = synthetic_batch(n, h, w, first_index=17)
    sd = {k: v.detach().cpu() for k, v in nets[which].state_dict().items()}
    with torch.no_grad():
        ref = net_forward(sd, i0, i1, 0.5)
        out = nets[which](i0.to(gpu), i1.to(gpu), 0.5).cpu()
    err = maxabs(out, ref)
    assert err <= GATE, f"{h}x{w}: {err:.3e}"
    mse = float(((out.double() - ref.double()) ** 2).mean())
    assert mse == 0 or 10 * np.log10(1.0 / mse) > 80  # PSNR vs CPU ref


def test_batch_equals_per_sample_and_deterministic(gpu, nets):
    i0, i1 = synthetic_batch(3, 64, 96, first_index=3)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    net = nets["stress"]
    with torch.no_grad():
        full = net(i0, i1, 0.5)
        again = net(i0, i1, 0.5)
        parts = torch.cat([net(i0[k:k + 1], i1[k:k + 1], 0.5) for k in range(3)])
    assert torch.equal(full, again)
    assert torch.equal(full, parts)


@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_batch_size_bitwise_640x368(gpu, nets, precision):
    """at 640x368 (BASELINE C2) a pair's bits must not depend on how it is
    batched -- one pair alone (the "small" size class) vs three in one call ("medium")
    vs a 2-stream split -- since the size class follows n*h*w and sharding relies on
    batch == per-sample.  No class may pick a different K association (split-K)."""
    net = nets["stress"]
    net.precision = precision
    try:
        i0, i1 = synthetic_batch(3, 368, 640, first_index=40)
        i0, i1 = i0.to(gpu), i1.to(gpu)
        eng = net.engine()
        with torch.no_grad():
            three = eng.forward(i0, i1, 0.5)
            two_streams = eng.forward(i0, i1, 0.5, streams=2)
            ones = torch.cat([eng.forward(i0[k:k + 1], i1[k:k + 1], 0.5) for k in range(3)])
        assert torch.equal(three, ones)
        assert torch.equal(two_streams, three)
    finally:
        net.precision = "fp32"


def test_batch_size_bitwise_1280x720_fp32(gpu, nets):
    """At the headline size kind 14's launcher picks the 16 x 16 tile for the level-4 convs of a
    two-pair call (480 workgroups, one round) and the 32 x 8 tile for a one-pair call: a pair's
    bits must still not depend on its batch (the geometries are bitwise equal per output)."""
    net = nets["stress"]
    net.precision = "fp32"
    i0, i1 = synthetic_batch(2, 720, 1280, first_index=60)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    eng = net.engine()
    with torch.no_grad():
        two = eng.forward(i0, i1, 0.5, streams=1)
        ones = torch.cat([eng.forward(i0[k:k + 1], i1[k:k + 1], 0.5) for k in range(2)])
    assert torch.equal(two, ones)


@pytest.mark.parametrize("precision", ["fp32_split16", "fp16", "fp32", "fp32_planar"])
def test_streams_split_is_bitwise(gpu, nets, precision):
    """The batch split over several HIP streams (engine.forward(streams=k)) gives the
    single-stream output bit for bit, also when k does not divide the batch."""
    net = nets["stress"]
    net.precision = precision
    i0, i1 = synthetic_batch(5, 64, 96, first_index=21)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    eng = net.engine()
    with torch.no_grad():
        one = eng.forward(i0, i1, 0.5)
        for k in (2, 3):
            assert torch.equal(eng.forward(i0, i1, 0.5, streams=k), one)
        assert torch.equal(eng.forward(i0, i1, 0.5, split=[1, 4]), one)
        net.streams = 1
        assert torch.equal(net(i0, i1, 0.5), one)
        net.streams = 2
        assert torch.equal(net(i0, i1, 0.5), one)
        net.streams = None  # the module default: by precision and batch (engine.default_streams)
        assert torch.equal(net(i0, i1, 0.5), one)
    net.precision = "fp32"


def test_weight_reload_repacks(gpu):
    net = make_net(gpu)
    i0, i1 = synthetic_batch(1, 64, 64)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    with torch.no_grad():
        a = net(i0, i1)
        net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True))
        b = net(i0, i1)
    assert not torch.equal(a, b)


def test_net_errors(gpu, nets):
    net = nets["default"]
    with torch.no_grad():
        with pytest.raises(RuntimeError, match="multiples of 16"):
            net(torch.zeros(1, 3, 72, 72, device=gpu), torch.zeros(1, 3, 72, 72, device=gpu))
        with pytest.raises(TypeError):
            net(torch.zeros(1, 3, 64, 64, device=gpu).half(), torch.zeros(1, 3, 64, 64, device=gpu).half())


@pytest.mark.parametrize("which", ["default", "stress"])
def test_net_golden_split16(gpu, golden, which):
    """fp32_split16: fp32-class accuracy (three fp16 products per fp32 product)."""
    g = golden("net_" + which)
    net = make_net(gpu, which == "stress")
    net.precision = "fp32_split16"
    i0, i1 = torch.from_numpy(g["i0"]).to(gpu), torch.from_numpy(g["i1"]).to(gpu)
    with torch.no_grad():
        for t, key in [(0.5, "out_t050"), (0.25, "out_t025"),
                       (torch.from_numpy(g["t_tensor"]).view(-1, 1, 1, 1).to(gpu), "out_ttensor")]:
            err = maxabs(net(i0, i1, t=t).cpu(), g[key])
            assert err <= (1e-4 if which == "default" else GATE), f"{which} {key}: {err:.3e}"


@pytest.mark.parametrize("h,w", [(64, 96), (368, 640), (720, 1280)])
def test_net_split16_vs_oracle(gpu, nets, h, w):
    net = make_net(gpu)
    net.precision = "fp32_split16"
    i0, i1 = synthetic_batch(1, h, w, first_index=5)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    with torch.no_grad():
        ref = net_forward(sd, i0, i1, 0.5)
        out = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    assert maxabs(out, ref) <= GATE


@pytest.mark.parametrize("which,h,w", [("default", 64, 96), ("stress", 64, 96), ("default", 368, 640)])
def test_net_fp16_gate(gpu, which, h, w):
    """fp16 configs: max-abs <= 1e-2 and PSNR >= 45 dB vs the fp32 CPU reference."""
    net = make_net(gpu, which == "stress")
    net.precision = "fp16"
    i0, i1 = synthetic_batch(2, h, w, first_index=9)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    with torch.no_grad():
        ref = net_forward(sd, i0, i1, 0.5)
        out = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    err = maxabs(out, ref)
    mse = float(((out.double() - ref.double()) ** 2).mean())
    psnr = 10 * np.log10(1.0 / max(mse, 1e-30))
    assert err <= 1e-2 and psnr >= 45, f"max-abs {err:.3e} psnr {psnr:.1f}"


@pytest.mark.parametrize("precision", ["fp32", "fp32_planar", "fp32_split16", "fp16"])
def test_interpolate_reuses_flow(gpu, precision):
    """Net.interpolate == [forward(t) for t in ts] bitwise, with the Flow U-Net run once."""
    net = make_net(gpu, stress=True)
    net.precision = precision
    i0, i1 = synthetic_batch(2, 64, 96, first_index=11)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    ts = [0.25, 0.5, 0.75]
    with torch.no_grad():
        many = net.interpolate(i0, i1, ts)
        single = [net(i0, i1, t) for t in ts]
    for a, b in zip(many, single):
        assert torch.equal(a, b)


@pytest.mark.parametrize("precision", ["fp32", "fp32_split16", "fp16"])
@pytest.mark.parametrize("level", [-1, 0, 3])
def test_subpixel_levels_agree(gpu, golden, precision, level):
    """Folding the upsample into the up convs (sub-pixel levels 0..level) gives the
    reference result at every setting; -1 = explicit upsample pass everywhere.
    The 80x112 golden has odd low-res sizes (5x7 bottom)."""
    g = golden("net_odd")
    net = make_net(gpu, stress=False)
    net.precision = precision
    net.subpixel_max_level = level
    i0, i1 = torch.from_numpy(g["i0"]).to(gpu), torch.from_numpy(g["i1"]).to(gpu)
    with torch.no_grad():
        err = maxabs(net(i0, i1, 0.5).cpu(), g["out_t050"])
    assert err <= (1e-2 if precision == "fp16" else 1e-4), f"level {level}: {err:.3e}"


@pytest.mark.parametrize("precision", ["fp32", "fp32_split16", "fp16"])
def test_size_class_tables_bitwise(gpu, nets, precision):
    """The tile table follows the pixels per forward part (engine.size_class);
    every direct-form config accumulates K in the same order, and every Winograd
    tile kind in the same order as the others, so the output must not depend on which
    class's table (and packing) ran.  The split-K slices follow the image geometry
    only (engine.geom_split), so they are the same in every class."""
    net = nets["stress"]
    net.precision = precision
    try:
        eng = net.engine()
        i0, i1 = synthetic_batch(2, 128, 192)
        i0, i1 = i0.to(gpu), i1.to(gpu)
        outs = {}
        for cls in ("small", "medium", "large", "xlarge", "xxlarge"):
            table = eng._pack_h8(cls, 128, 192)[2]
            eng.conv_table_for = lambda n, h, w, t=table: t
            with torch.no_grad():
                outs[cls] = eng.forward(i0, i1, 0.5).cpu()
            del eng.conv_table_for
        if precision == "fp32" and engine_mod.WINO and "small" not in engine_mod.WINO_SIZES:
            # the direct form: another rounding
            torch.testing.assert_close(outs["small"], outs["large"], rtol=0, atol=2e-5)
        else:
            assert torch.equal(outs["small"], outs["large"])
        assert torch.equal(outs["medium"], outs["large"])
        assert torch.equal(outs["xlarge"], outs["large"]) and torch.equal(outs["xxlarge"], outs["large"])
    finally:
        net.precision = "fp32"


def test_size_class_tables_bitwise_fp32_planar(gpu, nets):
    """Planar exact-fp32 path: the small class swaps BM 64 x TH 8 tiles for BM 64 x
    TH 4 at levels >= 1 (same packing); the output must be bitwise the large class's."""
    net = nets["stress"]
    net.precision = "fp32_planar"
    eng = net.engine()
    i0, i1 = synthetic_batch(2, 128, 192)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    with torch.no_grad():
        small = eng.forward(i0, i1, 0.5).cpu()
        assert any(t.cfg == 4 for t in eng.conv_table_for(2, 128, 192))
        eng.conv_table_for = lambda n, h, w: eng.conv_table
        large = eng.forward(i0, i1, 0.5).cpu()
        del eng.conv_table_for
    net.precision = "fp32"
    assert torch.equal(small, large)


def test_workspace_cache_holds_two_shapes_at_four_streams(gpu):
    """an fp16 4-pair forward takes 4 workspaces (one per stream part); forwards
    alternating between two shapes must keep both shapes' workspaces (no zero-filled
    reallocation, reuse_flow state kept), and a third shape evicts the least recently used
    shape as a whole."""
    net = make_net(gpu)
    net.precision = "fp16"
    eng = net.engine()
    shapes = [(64, 96), (96, 128)]
    with torch.no_grad():
        for h, w in shapes:
            i0, i1 = synthetic_batch(4, h, w, first_index=3)
            eng.forward(i0.to(gpu), i1.to(gpu), 0.5, streams=4)
        ids = {k: v.data_ptr() for k, v in eng._ws.items()}
        assert len(ids) == 8
        for _ in range(2):
            for h, w in shapes:
                i0, i1 = synthetic_batch(4, h, w, first_index=3)
                eng.forward(i0.to(gpu), i1.to(gpu), 0.5, streams=4)
        assert {k: v.data_ptr() for k, v in eng._ws.items()} == ids
        assert all(eng._flow_valid[k] for k in ids)
        i0, i1 = synthetic_batch(4, 32, 64, first_index=3)   # a third shape: (64, 96) goes, whole
        eng.forward(i0.to(gpu), i1.to(gpu), 0.5, streams=4)
        assert sorted({k[1:3] for k in eng._ws}) == [(32, 64), (96, 128)]
    torch.cuda.synchronize(gpu)
