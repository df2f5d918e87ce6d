"""Generate the golden fixtures in tests/golden/ by running the UNMODIFIED
reference (`/root/reference/model.py`, `/root/reference/unet.py`) on PyTorch-CPU.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

The reference's ``warp`` calls ``.cuda()`` unconditionally (`model.py:11-12`);
as recorded in SURVEY.md §8c the harness shim ``Tensor.cuda = identity`` is set
here, in the generator, before calling ``Net`` — the reference source is not
modified or copied.  Weights come from the key-seeded recipe
(``rrin_amd.synthetic``), so only inputs/outputs are stored.

Fixtures (all float32, np.savez_compressed):
  net_default.npz / net_stress.npz : N=2, 64x96, t in {0.5, 0.25, tensor[0.3,0.7]},
                                     plus the four raw U-Net outputs at t=0.5
  net_odd.npz                      : N=1, 80x112 (odd size at the deepest level), t=0.5
  ops.npz                          : warp (9x11, flows ~N(0,4^2) and far out of frame),
                                     upsample x2 / avgpool on odd sizes, one conv per
                                     shape class (6x10 spatial), UNetConvBlock, UNetUpBlock
  unet_refine.npz                  : refine_flow U-Net alone at 64x96
"""
from __future__ import annotations

import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"

sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
torch.Tensor.cuda = lambda self, *a, **k: self  # harness shim
torch.set_num_threads(8)

import model as ref_model  # noqa: E402  (reference)
import unet as ref_unet    # noqa: E402  (reference)
from rrin_amd.synthetic import keyed_state_dict, keyed_tensor  # noqa: E402

from tests.golden.spec import CONV_CLASSES  # noqa: E402


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def inputs(n, h, w, seed=7):
    g = torch.Generator().manual_seed(seed)
    i0 = torch.rand(n, 3, h, w, generator=g)
    i1 = torch.rand(n, 3, h, w, generator=g)
    return i0, i1


def run_net(stress):
    net = ref_model.Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=stress), strict=True)
    net.eval()
    i0, i1 = inputs(2, 64, 96)
    taps = {}
    hooks = [getattr(net, name).register_forward_hook(
        lambda m, a, o, name=name: taps.__setitem__(name, o.detach().clone()))
        for name in ("Flow", "refine_flow", "Mask", "final")]
    out = {}
    with torch.no_grad():
        out["out_t050"] = f32(net(i0, i1, t=0.5))
        for k, v in taps.items():
            out["unet_" + k] = f32(v)
        for h in hooks:
            h.remove()
        out["out_t025"] = f32(net(i0, i1, t=0.25))
        tt = torch.tensor([0.3, 0.7]).view(2, 1, 1, 1)
        out["out_ttensor"] = f32(net(i0, i1, t=tt))
    out["i0"], out["i1"] = f32(i0), f32(i1)
    out["t_tensor"] = np.array([0.3, 0.7], np.float32)
    return out


def run_odd():
    net = ref_model.Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    net.eval()
    i0, i1 = inputs(1, 80, 112, seed=11)
    with torch.no_grad():
        o = net(i0, i1, t=0.5)
    return {"i0": f32(i0), "i1": f32(i1), "out_t050": f32(o)}


def conv_module(cls, *args, key):
    m = cls(*args)
    sd = m.state_dict()
    def pre(k):
        return k.rsplit(".", 1)[0] if "." in k else ""
    fan = {pre(k): v.shape[1] * 9 for k, v in sd.items() if k.endswith("weight")}
    m.load_state_dict({k: keyed_tensor(f"{key}.{k}", v.shape, fan[pre(k)]) for k, v in sd.items()})
    return m.eval()


def run_ops():
    out = {}
    g = torch.Generator().manual_seed(3)
    # warp: moderate flows, and far out-of-frame flows
    img = torch.rand(2, 3, 9, 11, generator=g)
    flow = torch.randn(2, 2, 9, 11, generator=g) * 4.0
    flow_far = torch.randn(2, 2, 9, 11, generator=g) * 12.0
    with torch.no_grad():
        out["warp_img"], out["warp_flow"], out["warp_flow_far"] = f32(img), f32(flow), f32(flow_far)
        out["warp_out"] = f32(ref_model.warp(img, flow))
        out["warp_out_far"] = f32(ref_model.warp(img, flow_far))
        out["warp_out_zero"] = f32(ref_model.warp(img, torch.zeros_like(flow)))
        # upsample x2 (nn.Upsample of the UpBlock) and avg-pool on odd sizes
        x = torch.rand(2, 5, 7, 9, generator=g)
        out["up_in"] = f32(x)
        out["up_out"] = f32(torch.nn.Upsample(mode="bilinear", scale_factor=2)(x))
        xp = torch.rand(2, 4, 10, 14, generator=g)
        out["pool_in"] = f32(xp)
        out["pool_out"] = f32(torch.nn.functional.avg_pool2d(xp, 2))
        # one conv per shape class (plain Conv2d, weights keyed by class)
        for cin, cout in CONV_CLASSES:
            conv = conv_module(torch.nn.Conv2d, cin, cout, 3, 1, 1, key=f"golden.conv.{cin}.{cout}")
            xi = torch.rand(1, cin, 6, 10, generator=g) * 2 - 1
            out[f"conv_{cin}_{cout}_in"] = f32(xi)
            out[f"conv_{cin}_{cout}_out"] = f32(conv(xi))
        # reference UNetConvBlock and UNetUpBlock
        cb = conv_module(ref_unet.UNetConvBlock, 16, 32, True, key="golden.convblock")
        xi = torch.rand(1, 16, 8, 12, generator=g) * 2 - 1
        out["convblock_in"], out["convblock_out"] = f32(xi), f32(cb(xi))
        ub = conv_module(ref_unet.UNetUpBlock, 64, 32, True, key="golden.upblock")
        xl = torch.rand(1, 64, 4, 6, generator=g) * 2 - 1
        br = torch.rand(1, 32, 8, 12, generator=g) * 2 - 1
        out["upblock_in"], out["upblock_bridge"], out["upblock_out"] = f32(xl), f32(br), f32(ub(xl, br))
    return out


def run_unet():
    net = ref_model.Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    g = torch.Generator().manual_seed(5)
    x = torch.rand(1, 10, 64, 96, generator=g) * 2 - 1
    with torch.no_grad():
        y = net.refine_flow(x)
    return {"x": f32(x), "y": f32(y)}


def main():
    np.savez_compressed(os.path.join(HERE, "net_default.npz"), **run_net(False))
    np.savez_compressed(os.path.join(HERE, "net_stress.npz"), **run_net(True))
    np.savez_compressed(os.path.join(HERE, "net_odd.npz"), **run_odd())
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **run_ops())
    np.savez_compressed(os.path.join(HERE, "unet_refine.npz"), **run_unet())
    keys = list(ref_model.Net().state_dict().keys())
    with open(os.path.join(HERE, "state_dict_keys.txt"), "w") as f:
        for k in keys:
            f.write(k + "\n")
    print("wrote fixtures; state_dict keys:", len(keys), "crc", zlib.crc32("\n".join(keys).encode()))


if __name__ == "__main__":
    main()
