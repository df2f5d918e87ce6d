"""CPU: pin the oracle (oracle/) to the golden vectors produced by the
unmodified reference (tests/golden/gen_golden.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import prims_np
from oracle.ref_net import net_forward, unet_forward, warp
from rrin_amd import Net
from rrin_amd.synthetic import keyed_state_dict, keyed_tensor



def _sd(stress=False):
    return keyed_state_dict(Net().state_dict(), stress=stress)


@pytest.mark.parametrize("which", ["default", "stress"])
def test_net_matches_reference(golden, which):
    g = golden("net_" + which)
    sd = _sd(which == "stress")
    i0, i1 = torch.from_numpy(g["i0"]), torch.from_numpy(g["i1"])
    taps = {}
    with torch.no_grad():
        out = net_forward(sd, i0, i1, 0.5, taps)
        np.testing.assert_allclose(out.numpy(), g["out_t050"], rtol=0, atol=1e-6)
        for ours, ref in [("Flow", "unet_Flow"), ("refine", "unet_refine_flow"),
                          ("mask_logits", "unet_Mask"), ("final_unet", "unet_final")]:
            np.testing.assert_allclose(taps[ours].numpy(), g[ref], rtol=0, atol=1e-6)
        out = net_forward(sd, i0, i1, 0.25)
        np.testing.assert_allclose(out.numpy(), g["out_t025"], rtol=0, atol=1e-6)
        tt = torch.from_numpy(g["t_tensor"]).view(-1, 1, 1, 1)
        out = net_forward(sd, i0, i1, tt)
        np.testing.assert_allclose(out.numpy(), g["out_ttensor"], rtol=0, atol=1e-6)


def test_net_odd_size(golden):
    g = golden("net_odd")
    with torch.no_grad():
        out = net_forward(_sd(), torch.from_numpy(g["i0"]), torch.from_numpy(g["i1"]), 0.5)
    np.testing.assert_allclose(out.numpy(), g["out_t050"], rtol=0, atol=1e-6)


def test_unet_refine(golden):
    g = golden("unet_refine")
    with torch.no_grad():
        y = unet_forward(_sd(), "refine_flow", torch.from_numpy(g["x"]))
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=1e-6)


def test_warp_ops(golden):
    g = golden("ops")
    img = torch.from_numpy(g["warp_img"])
    for fk, ok in [("warp_flow", "warp_out"), ("warp_flow_far", "warp_out_far")]:
        out = warp(img, torch.from_numpy(g[fk]))
        np.testing.assert_allclose(out.numpy(), g[ok], rtol=0, atol=1e-6)
        np.testing.assert_allclose(prims_np.warp(g["warp_img"], g[fk]), g[ok], rtol=0, atol=2e-6)
    # zero flow is NOT identity: half-pixel box average with zero border
    z = warp(img, torch.zeros(2, 2, 9, 11))
    np.testing.assert_allclose(z.numpy(), g["warp_out_zero"], rtol=0, atol=1e-6)
    assert np.abs(g["warp_out_zero"] - g["warp_img"]).max() > 0.1


def test_upsample_pool_ops(golden):
    g = golden("ops")
    np.testing.assert_allclose(prims_np.upsample2x(g["up_in"]), g["up_out"], rtol=0, atol=1e-6)
    up = F.interpolate(torch.from_numpy(g["up_in"]), scale_factor=2, mode="bilinear", align_corners=False)
    np.testing.assert_allclose(up.numpy(), g["up_out"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(prims_np.avgpool2(g["pool_in"]), g["pool_out"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("cin,cout", [(6, 32), (32, 4), (64, 32), (128, 128), (512, 256)])
def test_conv_classes_numpy(golden, cin, cout):
    g = golden("ops")
    w = keyed_tensor(f"golden.conv.{cin}.{cout}.weight", (cout, cin, 3, 3), cin * 9).numpy()
    b = keyed_tensor(f"golden.conv.{cin}.{cout}.bias", (cout,), cin * 9).numpy()
    ref = prims_np.conv3x3(g[f"conv_{cin}_{cout}_in"], w, b)
    np.testing.assert_allclose(ref, g[f"conv_{cin}_{cout}_out"], rtol=0, atol=2e-5)
