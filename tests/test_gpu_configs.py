"""GPU parity at the BASELINE.json configs and on the intermediate taps.

* Intermediate taps (SURVEY §8c "so clamp cannot hide errors"): the four
  U-Nets' raw outputs (unet.py:51 as used at model.py:35,42,52,62) captured by
  ``engine.forward(taps=...)`` against the goldens the unmodified reference
  wrote through forward hooks (tests/golden/gen_golden.py).
* Config C3 (1280x736, 4 pairs, fp16) and the per-GPU share of C5 (3840x2176,
  1 pair, fp16): pair 0 against the CPU oracle at the fp16 gate (max-abs 1e-2,
  PSNR 45 dB), the exact-fp32 path at 1e-3; batch == per-sample bitwise.
* Wide-dynamic-range weights: per-layer weight scales 0.05 .. 20 drive
  mid-network activations past 1e4 (checked on the oracle); fp32 and the
  fp32-emulated split16 stay at the 1e-3 gate; past the fp16 range the split16
  output is NaN-poisoned and the range check raises (never silently wrong).
"""
import numpy as np
import pytest
import torch

import oracle.ref_net as ref
from rrin_amd import Net
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch

pytestmark = pytest.mark.gpu
GATE = 1e-3
TAP_KEYS = {"Flow": "unet_Flow", "refine_flow": "unet_refine_flow", "Mask": "unet_Mask", "final": "unet_final"}


def make_net(dev, sd):
    net = Net()
    net.load_state_dict(sd, strict=True)
    return net.to(dev).eval()


def err_psnr(out, ref_out):
    d = out.double() - ref_out.double()
    mse = float((d * d).mean())
    return float(d.abs().max()), (10 * np.log10(1.0 / mse) if mse > 0 else float("inf"))


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("fp32_planar", 1e-4), ("fp32_split16", 1e-4),
                                           ("fp16", 5e-2)])
@pytest.mark.parametrize("which", ["default", "stress"])
def test_unet_taps_golden(gpu, golden, which, precision, tol):
    """Raw U-Net outputs (pre-glue, pre-clamp) vs the reference's hooks, t = 0.5.
    Tolerance relative to each tap's scale (stress Flow reaches ~10 px).  Run
    with the oracle in-container too: the fp32 paths at 1e-4, fp16 at 5e-2."""
    g = golden("net_" + which)
    net = make_net(gpu, keyed_state_dict(Net().state_dict(), stress=which == "stress"))
    net.precision = precision
    i0, i1 = torch.from_numpy(g["i0"]).to(gpu), torch.from_numpy(g["i1"]).to(gpu)
    taps = {}
    with torch.no_grad():
        out = net.engine().forward(i0, i1, 0.5, taps=taps)
    for name, key in TAP_KEYS.items():
        want = torch.from_numpy(g[key])
        got = taps[name].cpu()
        scale = max(1.0, float(want.abs().max()))
        err = float((got.double() - want.double()).abs().max())
        assert err <= tol * scale, f"{which} {precision} {name}: max-abs {err:.3e} (scale {scale:.1f})"
    assert float((out.cpu() - torch.from_numpy(g["out_t050"])).abs().max()) <= (1e-2 if precision == "fp16" else GATE)


def _oracle(sd, i0, i1, t=0.5, taps=None):
    with torch.no_grad():
        return ref.net_forward(sd, i0, i1, t, taps=taps)


@pytest.fixture(scope="module")
def c3_case():
    """Config C3: 1280x736 (padded 720p), 4 pairs; oracle output of every pair (the forward splits
    them over streams: every pair of every stream part is checked against the oracle)."""
    sd = keyed_state_dict(Net().state_dict())
    i0, i1 = synthetic_batch(4, 736, 1280, first_index=40)
    return sd, i0, i1, _oracle(sd, i0, i1)


@pytest.mark.parametrize("precision", ["fp16", "fp32"])
def test_config_c3_1280x736x4(gpu, c3_case, precision):
    sd, i0, i1, ref = c3_case
    net = make_net(gpu, sd)
    net.precision = precision
    with torch.no_grad():
        out = net(i0.to(gpu), i1.to(gpu), 0.5)
        one = net(i0[2:3].to(gpu), i1[2:3].to(gpu), 0.5)
    net.check_range()
    for p in range(4):   # every pair (every stream part of the forward) vs the oracle
        err, psnr = err_psnr(out[p:p + 1].cpu(), ref[p:p + 1])
        if precision == "fp16":
            assert err <= 1e-2 and psnr >= 45, f"C3 fp16 pair {p}: max-abs {err:.3e} psnr {psnr:.1f}"
        else:
            assert err <= GATE, f"C3 fp32 pair {p}: max-abs {err:.3e}"
    assert torch.equal(out[2:3], one)   # batch == per-sample (pairs are independent)


@pytest.fixture(scope="module")
def c5_case():
    """Per-GPU share of config C5: 3840x2176 (padded 4K), 1 pair; oracle output."""
    sd = keyed_state_dict(Net().state_dict(), stress=True)
    i0, i1 = synthetic_batch(1, 2176, 3840, first_index=7)
    return sd, i0, i1, _oracle(sd, i0, i1)


@pytest.mark.parametrize("precision", ["fp16", "fp32"])
def test_config_c5_3840x2176(gpu, c5_case, precision):
    sd, i0, i1, ref0 = c5_case
    net = make_net(gpu, sd)
    net.precision = precision
    with torch.no_grad():
        out = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    net.check_range()
    err, psnr = err_psnr(out, ref0)
    if precision == "fp16":
        assert err <= 1e-2 and psnr >= 45, f"C5 fp16: max-abs {err:.3e} psnr {psnr:.1f}"
    else:
        assert err <= GATE, f"C5 fp32: max-abs {err:.3e}"


def wide_range_sd(first_scale):
    """Per-layer weight scales from 1/first_scale to first_scale: every U-Net's
    first conv x first_scale (activations scale with it: leaky is positively
    homogeneous), the body convs alternately x10 / x0.1, the `last` conv x
    1/first_scale (outputs return to the usual range)."""
    sd = keyed_state_dict(Net().state_dict(), stress=True)
    for u in ("Flow", "refine_flow", "Mask", "final"):
        convs = [k for k in sd if k.startswith(u + ".") and k.endswith(".weight")]
        for j, k in enumerate(convs):
            if k.endswith("down_path.0.block.0.weight"):
                sd[k] = sd[k] * first_scale
            elif k.endswith("last.weight"):
                sd[k] = sd[k] / first_scale
            else:
                sd[k] = sd[k] * (10.0 if j % 2 else 0.1)
    return sd


def _max_activation(sd, i0, i1):
    """Largest |activation| any conv of the oracle produces (via a wrapped _conv)."""
    seen = [0.0]
    orig = ref._conv

    def conv(sd_, name, x):
        y = orig(sd_, name, x)
        if not name.endswith(".last"):
            seen[0] = max(seen[0], float(y.abs().max()))
        return y
    ref._conv = conv
    try:
        out = _oracle(sd, i0, i1)
    finally:
        ref._conv = orig
    return out, seen[0]


@pytest.mark.parametrize("precision", ["fp32", "fp32_split16"])
def test_wide_dynamic_range_weights(gpu, precision):
    sd = wide_range_sd(20.0)   # mid-network activations ~1.1e4 (the oracle check below)
    i0, i1 = synthetic_batch(2, 128, 192, first_index=31)
    ref_out, amax = _max_activation(sd, i0, i1)
    assert 1e3 < amax < 6e4, f"test setup: mid-network activations reach {amax:.3e}"
    net = make_net(gpu, sd)
    net.precision = precision
    with torch.no_grad():
        out = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    net.check_range()
    err, _ = err_psnr(out, ref_out)
    assert err <= GATE, f"{precision}: max-abs {err:.3e} with activations up to {amax:.3e}"


def test_split16_overflow_is_loud(gpu):
    """Activations past the fp16 range: split16 poisons the output with NaN and
    check_range() raises; exact fp32 still matches the oracle."""
    sd = wide_range_sd(1e5)
    i0, i1 = synthetic_batch(1, 64, 96, first_index=2)
    ref_out, amax = _max_activation(sd, i0, i1)
    assert amax > 65504
    net = make_net(gpu, sd)
    net.precision = "fp32_split16"
    with torch.no_grad():
        out = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    assert torch.isnan(out).all()
    with pytest.raises(RuntimeError, match="fp16 range"):
        net.check_range()
    net.precision = "fp32"
    with torch.no_grad():
        out32 = net(i0.to(gpu), i1.to(gpu), 0.5).cpu()
    assert err_psnr(out32, ref_out)[0] <= GATE


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("fp32_planar", 1e-5), ("fp32_split16", 1e-4),
                                           ("fp16", 3e-2)])
def test_unet_alone_golden(gpu, golden, precision, tol):
    """A U-Net called on its own (reference UNet.forward, unet.py:40-51) through
    rrin_unet_fwd: refine_flow on a random 10-channel input against the output the
    unmodified reference wrote (tests/golden/unet_refine.npz)."""
    g = golden("unet_refine")
    net = make_net(gpu, keyed_state_dict(Net().state_dict()))
    net.refine_flow.precision = precision
    with torch.no_grad():
        y = net.refine_flow(torch.from_numpy(g["x"]).to(gpu)).cpu()
    want = torch.from_numpy(g["y"])
    scale = max(1.0, float(want.abs().max()))
    assert y.shape == want.shape
    assert float((y - want).abs().max()) <= tol * scale


@pytest.mark.parametrize("name,cin", [("Flow", 6), ("Mask", 16), ("final", 9)])
def test_unet_alone_vs_oracle(gpu, name, cin):
    """Each U-Net alone (depth 5 and 4, in_ch 6 / 16 / 9) vs the oracle's unet_forward."""
    sd = keyed_state_dict(Net().state_dict(), stress=True)
    net = make_net(gpu, sd)
    x = torch.rand(2, cin, 64, 96, generator=torch.Generator().manual_seed(cin)) * 2 - 1
    with torch.no_grad():
        y = getattr(net, name)(x.to(gpu)).cpu()
        ref_y = ref.unet_forward(sd, name, x)
    scale = max(1.0, float(ref_y.abs().max()))
    assert float((y - ref_y).abs().max()) <= 1e-5 * scale
