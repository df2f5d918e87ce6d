"""ORACLE — test infrastructure only.  CPU restatement of RRIN ``Net.forward``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``rrin_amd``) never imports it and has no CPU fallback.

This is a functional restatement over a state_dict of the reference op
sequence, written from SURVEY.md §3.2-3.3 (no module code is shared):

* ``unet_forward``  — `/root/reference/unet.py:40-51` (down blocks, bridge +
  avg_pool2d(2) for all but the last level, leaky(midconv), up blocks, last);
  ConvBlock `unet.py:59-63`; UpBlock `unet.py:76-79,82-94` (center_crop is the
  identity at /16 sizes).
* ``warp``          — `/root/reference/model.py:8-21`: fp32 grid
  ``2*((gx+u)/W - 0.5)``, ``F.grid_sample`` defaults (bilinear, zeros,
  align_corners=False).  The meshgrid stays on the CPU (the reference's
  hard-coded ``.cuda()`` is the only thing removed).
* ``net_forward``   — `/root/reference/model.py:32-65`.

Pinning: ``tests/test_oracle.py`` checks this module against the golden vectors
in ``tests/golden/`` that ``tests/golden/gen_golden.py`` produced by importing
the unmodified reference in the build container (≤1e-6 max-abs).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

SLOPE = 0.1


def _conv(sd, name, x):
    return F.conv2d(x, sd[name + ".weight"], sd[name + ".bias"], padding=1)


def _conv_block(sd, name, x):
    x = F.leaky_relu(_conv(sd, name + ".block.0", x), SLOPE)
    return F.leaky_relu(_conv(sd, name + ".block.2", x), SLOPE)


def unet_depth(sd, prefix):
    return sum(1 for k in sd if k.startswith(prefix + ".down_path.") and k.endswith("block.0.weight"))


def unet_forward(sd: Dict[str, torch.Tensor], prefix: str, x: torch.Tensor) -> torch.Tensor:
    depth = unet_depth(sd, prefix)
    bridges = []
    for i in range(depth):
        x = _conv_block(sd, f"{prefix}.down_path.{i}", x)
        if i < depth - 1:
            bridges.append(x)
            x = F.avg_pool2d(x, 2)
    x = F.leaky_relu(_conv(sd, prefix + ".midconv", x), SLOPE)
    for j in range(depth - 1):
        up = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
        up = _conv(sd, f"{prefix}.up_path.{j}.up.1", up)
        x = torch.cat((up, bridges[-j - 1]), 1)
        x = _conv_block(sd, f"{prefix}.up_path.{j}.conv_block", x)
    return _conv(sd, prefix + ".last", x)


def warp(img: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    n, _, h, w = img.shape
    gy, gx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    x = gx.unsqueeze(0).expand(n, h, w).float() + flow[:, 0]
    y = gy.unsqueeze(0).expand(n, h, w).float() + flow[:, 1]
    grid = torch.stack((2 * (x / w - 0.5), 2 * (y / h - 0.5)), dim=3)
    return F.grid_sample(img, grid, mode="bilinear", padding_mode="zeros", align_corners=False)


def net_forward(sd: Dict[str, torch.Tensor], i0: torch.Tensor, i1: torch.Tensor, t=0.5,
                taps: Optional[dict] = None) -> torch.Tensor:
    """RRIN forward on CPU.  ``taps`` (optional dict) receives intermediates:
    Flow, refine (refine_flow output), mask_logits, final_pre (before clamp)."""
    x = torch.cat((i0, i1), 1)
    flow = unet_forward(sd, "Flow", x)
    f01, f10 = flow[:, :2], flow[:, 2:4]
    ft0 = -(1 - t) * t * f01 + t * t * f10
    ft1 = (1 - t) * (1 - t) * f01 - t * (1 - t) * f10
    r = unet_forward(sd, "refine_flow", torch.cat((ft0, ft1, x), 1))
    ft0 = ft0 + r[:, :2]
    ft1 = ft1 + r[:, 2:4]
    xt1 = warp(i0, ft0)
    xt2 = warp(i1, ft1)
    m_logits = unet_forward(sd, "Mask", torch.cat((ft0, ft1, x, xt1, xt2), 1))
    m = torch.sigmoid(m_logits)
    w1, w2 = (1 - t) * m[:, 0:1], t * m[:, 1:2]
    out = (w1 * xt1 + w2 * xt2) / (w1 + w2 + 1e-8)
    final_unet = unet_forward(sd, "final", torch.cat((i0, i1, out), 1))
    final = final_unet + out
    if taps is not None:
        taps.update(Flow=flow, refine=r, mask_logits=m_logits, final_unet=final_unet,
                    final_pre=final,
                    ft0=ft0, ft1=ft1, xt1=xt1, xt2=xt2, blend=out)
    return final.clamp(0, 1)
