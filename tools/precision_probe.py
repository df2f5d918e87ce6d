#!/usr/bin/env python3
"""GPU precision probe: error of single convs per precision vs a float64 CPU
reference, normalised by sum |w*x| (the natural fp32 error scale of a dot
product).  Localises where a precision path loses bits.

  python tools/precision_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rrin_amd import _lib  # noqa: E402
from rrin_amd.pp import H8Tensor, PPTensor  # noqa: E402
from tests import hip_helpers as H  # noqa: E402
from tests.test_gpu_h8 import conv_h8  # noqa: E402


def stats(out, x, w, b):
    ref = F.conv2d(x.double().cpu(), w.double(), b.double(), padding=1)
    scale = F.conv2d(x.double().abs().cpu(), w.double().abs(), None, padding=1) + b.double().abs().view(1, -1, 1, 1)
    err = (out.double().cpu() - ref).abs()
    r = err / scale.clamp_min(1e-30)
    return float(r.max()), float(r.median()), float(err.max())


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for cin, cout, h, w, center_only, mag in [(16, 32, 16, 32, True, 1.0), (16, 32, 16, 32, False, 1.0),
                                              (64, 64, 32, 32, False, 1.0), (512, 256, 12, 20, False, 1.0),
                                              (64, 64, 32, 32, False, 1e-3), (64, 64, 32, 32, False, 100.0)]:
        x = (torch.rand(1, cin, h, w, device=dev) * 2 - 1) * mag
        wt = (torch.rand(cout, cin, 3, 3) * 2 - 1) / (cin * 9) ** 0.5
        if center_only:
            m = torch.zeros(3, 3)
            m[1, 1] = 1
            wt = wt * m
        b = torch.zeros(cout)
        res = {}
        d, _ = H.conv(PPTensor.from_nchw(x), wt, b, 1 if cout > 32 else 0)
        res["fp32"] = stats(d.to_nchw(), x, wt, b)
        for name, prec in (("split16", _lib.PREC_F16X3), ("fp16", _lib.PREC_F16)):
            d, _ = conv_h8(H8Tensor.from_nchw(x, prec), wt, b, 1 if cout <= 32 else 0, prec)
            res[name] = stats(d.to_nchw(), x, wt, b)
        print(f"cin {cin:3d} cout {cout:3d} center_only {center_only!s:5} |x|~{mag:g}: " +
              "  ".join(f"{k}: max {v[0]:.2e} med {v[1]:.2e} abs {v[2]:.2e}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
