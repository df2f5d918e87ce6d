"""CPU: host-side logic of the drop-in boundary (no kernel launches)."""
import os

import numpy as np
import pytest
import torch

from rrin_amd import Net
from rrin_amd.engine import FIRST_CONV_PERM, t_coefficients
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch, synthetic_pair
from rrin_amd.unet import conv_flops

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_state_dict_keys_match_reference():
    keys = [l.strip() for l in open(os.path.join(GOLDEN, "state_dict_keys.txt"))]
    net = Net()
    sd = net.state_dict()
    assert list(sd.keys()) == keys and len(keys) == 162
    assert tuple(sd["Flow.up_path.0.up.1.weight"].shape) == (256, 512, 3, 3)
    assert sum(v.numel() for v in sd.values()) == 19_194_445
    # a reference-style checkpoint dict loads strict (convert.py:103, train.py:158-161)
    state = {"model": keyed_state_dict(sd), "optim": {}, "epoch": 3}
    net.load_state_dict(state["model"], strict=True)


def test_conv_flops_match_survey():
    net = Net()
    total = sum(conv_flops(getattr(net, u), 736, 1280) for u in ("Flow", "refine_flow", "Mask", "final"))
    assert abs(total / 1e9 - 1635.5) < 0.1
    total720 = sum(conv_flops(getattr(net, u), 720, 1280) for u in ("Flow", "refine_flow", "Mask", "final"))
    assert abs(total720 / 1e9 - 1600.0) < 0.1


def test_autograd_path_matches_golden_and_trains():
    """With autograd on (train.py:98) Net.forward runs the reference math with
    PyTorch operators: equal to the reference's own output (golden,
    written by the unmodified reference) and differentiable."""
    g = np.load(os.path.join(GOLDEN, "net_default.npz"))
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    i0, i1 = torch.from_numpy(g["i0"]), torch.from_numpy(g["i1"])
    out = net(i0, i1, 0.5)
    assert out.requires_grad
    assert torch.allclose(out, torch.from_numpy(g["out_t050"]), atol=1e-6, rtol=0)
    out.mean().backward()
    assert net.Flow.down_path[0].block[0].weight.grad is not None
    assert float(net.final.last.weight.grad.abs().sum()) > 0


def test_unet_forward_paths():
    """UNet.forward: without autograd the HIP engine (CPU tensors raise: no CPU
    fallback); with autograd the torch-op path, equal to the reference UNet's
    own output (golden unet_refine.npz, refine_flow alone, key-seeded weights)."""
    net = Net()
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm device"):
        net.Flow(torch.zeros(1, 6, 16, 16))
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    g = np.load(os.path.join(GOLDEN, "unet_refine.npz"))
    y = net.refine_flow(torch.from_numpy(g["x"]))
    assert y.requires_grad
    assert torch.allclose(y, torch.from_numpy(g["y"]), atol=1e-5, rtol=0)


def test_packed_weights_follow_inplace_edits():
    """The engine's packing is keyed by every parameter's (storage, version):
    an in-place edit (optimizer step, p.copy_, a sub-UNet load_state_dict)
    changes the fingerprint."""
    net = Net()
    fp0 = net._weights_fingerprint()
    with torch.no_grad():
        net.Mask.last.bias.add_(1.0)
    fp1 = net._weights_fingerprint()
    assert fp1 != fp0
    net.Flow.load_state_dict(net.Flow.state_dict())
    assert net._weights_fingerprint() != fp1


def test_forward_requires_rocm_device():
    net = Net()
    x = torch.zeros(1, 3, 16, 16)
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm device"):
        net(x, x)


@pytest.mark.parametrize("t", [0.5, 0.25, 1 / 3, 0.9])
def test_t_coefficients_python_float(t):
    c = t_coefficients(t, 3)
    assert c.shape == (3, 8) and c.dtype == torch.float32
    # scalar*tensor in the reference: the Python double is rounded to fp32 once
    f = torch.ones(1)
    exp = [(-(1 - t) * t * f).item(), (t * t * f).item(), ((1 - t) * (1 - t) * f).item(),
           (t * (1 - t) * f).item(), ((1 - t) * f).item(), (t * f).item()]
    assert c[1, :6].tolist() == exp


def test_t_coefficients_tensor():
    tt = torch.tensor([0.3, 0.7]).view(2, 1, 1, 1)
    c = t_coefficients(tt, 2)
    f = torch.ones(2, 1, 1, 1)
    exp0 = (-(1 - tt) * tt * f).view(-1)
    assert torch.equal(c[:, 0], exp0)
    assert torch.equal(c[:, 3], (tt * (1 - tt) * f).view(-1))
    with pytest.raises(ValueError):
        t_coefficients(torch.tensor([0.1, 0.2, 0.3]), 2)


def test_channel_permutations_are_bijective():
    assert sorted(FIRST_CONV_PERM["refine_flow"]) == list(range(10))
    assert sorted(FIRST_CONV_PERM["Mask"]) == list(range(16))


def test_synthetic_pairs_deterministic():
    a0, a1 = synthetic_pair(32, 48, 5)
    b0, b1 = synthetic_pair(32, 48, 5)
    assert torch.equal(a0, b0) and torch.equal(a1, b1)
    assert torch.all((a0 * 255).round() == a0 * 255)  # ToTensor quantisation
    assert 0 <= a1.min() and a1.max() <= 1
    x0, _ = synthetic_batch(3, 32, 48, first_index=4)
    assert torch.equal(x0[1:2], a0)


def test_bench_union_ms():
    """bench.py's conv busy time: union of launch spans (overlapping streams)."""
    import bench
    assert bench.union_ms([]) == 0.0
    assert bench.union_ms([(0.0, 1.0), (2.0, 3.0)]) == 2.0            # disjoint: the sum
    assert bench.union_ms([(0.0, 2.0), (1.0, 3.0)]) == 3.0            # overlap counted once
    assert bench.union_ms([(1.0, 4.0), (0.0, 5.0), (2.0, 3.0)]) == 5.0  # nested, unsorted
    assert bench.union_ms([(0.0, 1.0), (1.0, 2.0)]) == 2.0            # touching


def test_size_class_tables():
    """Every tuned tile table entry names a config that exists and fits its cin
    (the library's own check), and the size classes split at the documented
    pixel counts."""
    from rrin_amd import _lib, engine
    lib = _lib.lib()
    ncfg = lib.rrin_conv_h8_cfg_count()
    tables = [(p, t) for p, t in engine.H8_TUNED.items()]
    tables += [(p, t) for cls in engine.H8_TUNED_BY_SIZE.values() for p, t in cls.items()]
    for prec, table in tables:
        for (cin, cout, level), cfg in table.items():
            assert 0 <= cfg < ncfg
            assert lib.rrin_conv_h8_cfg_fits(cfg, prec, cin) == 1, (cin, cout, level, cfg)
        # the size-class tables cover the same conv shapes as the large one
        assert set(table) == set(engine.H8_TUNED[prec]) or prec not in engine.H8_TUNED
    assert engine.size_class(640 * 368) == "small"
    assert engine.size_class(1280 * 720) == "medium"
    assert engine.size_class(2 * 1280 * 720) == "large"
    assert engine.size_class(4 * 1280 * 720) == "xlarge"
    assert engine.size_class(3840 * 2176) == "xxlarge"


def test_autograd_stream_follows_tensor_device(monkeypatch):
    """the training kernels launch on the current stream of the tensors'
    device, not of the thread's current device (a model on cuda:1 without set_device)."""
    import torch

    from rrin_amd import autograd as ag
    seen = []

    class _S:
        cuda_stream = 1234

    def fake_current_stream(device=None):
        seen.append(device)
        return _S()

    monkeypatch.setattr(torch.cuda, "current_stream", fake_current_stream)
    st = ag._stream(torch.device("cuda", 1))
    assert st.value == 1234 and seen == [torch.device("cuda", 1)]


def test_geom_split_depends_on_image_geometry_only():
    """Split-K slices (engine.geom_split) come from one image's geometry: the deep convs
    of 640x368 images split, 720p and larger never do, and nothing in the rule sees the
    batch size (the rounding of a pair must not depend on its batch / stream split)."""
    from rrin_amd import engine
    g = engine.geom_split
    assert g(512, 512, 368 >> 4, 640 >> 4) == 4        # 23x40 level-4 grid
    assert g(256, 512, 368 >> 4, 640 >> 4) == 4
    assert g(256, 256, 368 >> 3, 640 >> 3) == 2        # 46x80: 288 kind-4 tiles
    assert g(128, 256, 368 >> 3, 640 >> 3) == 1        # K = 128: never split
    for cin, rows, lvl in ((512, 512, 4), (256, 256, 3), (512, 1024, 3)):
        assert g(cin, rows, 720 >> lvl, 1280 >> lvl) == 1
        assert g(cin, rows, 736 >> lvl, 1280 >> lvl) == 1
    saved = engine.GEOM_SPLIT
    try:
        engine.GEOM_SPLIT = False
        assert g(512, 512, 23, 40) == 1
    finally:
        engine.GEOM_SPLIT = saved
