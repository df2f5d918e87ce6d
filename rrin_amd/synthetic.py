"""Deterministic synthetic weights and frame pairs.

No checkpoint ships with the reference and there is no network, so every
weight set used by tests and by ``bench.py`` is regenerated from the key-seeded
recipe below; it is reproducible without the reference:

* for every state_dict key ``k`` (Net order), ``g = Generator().manual_seed(crc32(k))``
  and ``W = (rand(shape, g) * 2 - 1) / sqrt(fan_in)`` with ``fan_in = Cin*9`` of
  the owning conv (biases use their weight's fan-in);
* "stress" weights scale the four ``last`` convs (x300 Flow, x100 refine_flow,
  x50 Mask, x5 final) to produce 10-18 px flows, out-of-frame taps and clamping.

Frame pairs follow SURVEY §8d: ``I0 = randint(0,256)/255`` (the quantisation of
``ToTensor``), ``I1 = roll(I0, (3,5)) + U(-2/255, 2/255)`` clamped to [0,1].
Each pair is generated from ``(seed, global_index)`` so that ranks of a sharded
run produce disjoint pairs with no scatter.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict

import torch

STRESS_SCALE = {
    "Flow.last.weight": 300.0,
    "refine_flow.last.weight": 100.0,
    "Mask.last.weight": 50.0,
    "final.last.weight": 5.0,
}


def keyed_tensor(key: str, shape, fan_in: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(zlib.crc32(key.encode()))
    return (torch.rand(tuple(shape), generator=g) * 2 - 1) / math.sqrt(fan_in)


def keyed_state_dict(template: Dict[str, torch.Tensor], stress: bool = False) -> Dict[str, torch.Tensor]:
    """Fill every tensor of ``template`` (a Net state_dict) with the recipe."""
    out = {}
    fan = {}
    for k, v in template.items():
        if k.endswith(".weight"):
            fan[k[: -len(".weight")]] = v.shape[1] * v.shape[2] * v.shape[3]
    for k, v in template.items():
        prefix = k.rsplit(".", 1)[0]
        t = keyed_tensor(k, v.shape, fan[prefix])
        if stress and k in STRESS_SCALE:
            t = t * STRESS_SCALE[k]
        out[k] = t
    return out


def synthetic_pair(h: int, w: int, index: int, seed: int = 1234):
    """One (I0, I1) pair [1,3,h,w] fp32 on CPU for global pair ``index``."""
    g = torch.Generator().manual_seed(seed + 7919 * index)
    i0 = torch.randint(0, 256, (1, 3, h, w), generator=g).float() / 255.0
    noise = (torch.rand((1, 3, h, w), generator=g) * 2 - 1) * (2.0 / 255.0)
    i1 = (torch.roll(i0, shifts=(3, 5), dims=(2, 3)) + noise).clamp_(0.0, 1.0)
    return i0, i1


def synthetic_batch(b: int, h: int, w: int, first_index: int = 0, seed: int = 1234):
    """Pairs ``first_index .. first_index+b-1`` stacked to [b,3,h,w]."""
    pairs = [synthetic_pair(h, w, first_index + i, seed) for i in range(b)]
    return torch.cat([p[0] for p in pairs]), torch.cat([p[1] for p in pairs])
