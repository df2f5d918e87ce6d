"""Drop-in ``Net`` for RRIN inference on MI355X.

Boundary: same class name, no-arg constructor, submodules
``Mask``/``Flow``/``refine_flow``/``final`` (reference `model.py:24-30`), the
same 162 state_dict keys, and ``forward(input0, input1, t=0.5)`` returning a
fresh ``[N,3,H,W]`` tensor on the inputs' device (`model.py:59-65`).

Unlike the reference, the arithmetic of ``forward`` is done entirely by the
hand-written HIP kernels of ``librrin_hip.so`` (see ``rrin_amd.engine``); there
is no PyTorch-operator path.  The HIP path requires:

* inputs on a ROCm device, fp32 (the metric's dtype), NCHW, H % 16 == W % 16 == 0
  (the reference raises at `model.py:41` otherwise — we raise earlier);
* autograd off (``torch.no_grad()`` / ``inference_mode``), as in the production
  caller `convert.py:117`.  Training (`train.py`) needs backward kernels, which
  are out of scope; we raise instead of silently detaching.
"""
from __future__ import annotations

import torch
from torch import nn

from .unet import UNet


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        # model.py:27-30 — construction order fixes the state_dict key order.
        self.Mask = UNet(16, 2, 4)
        self.Flow = UNet(6, 4, 5)
        self.refine_flow = UNet(10, 4, 4)
        self.final = UNet(9, 3, 4)
        self._engine = None
        self._engine_version = -1
        self._weights_version = 0
        # Arithmetic of the HIP path (not part of the reference contract):
        #   "fp32"         exact fp32 MFMA (v_mfma_f32_32x32x2_f32)
        #   "fp32_split16" fp32 values as fp16 hi+lo pairs, 3 f16 MFMA products, fp32 accumulate
        #   "fp16"         fp16 storage and products, fp32 accumulate (BASELINE fp16 configs)
        self.precision = "fp32"
        # fp32_split16 / fp16: up convs whose output level is <= this run as
        # sub-pixel convs on the low-res input (upsample folded into the weights,
        # no upsample pass); -1 = always an explicit upsample pass
        self.subpixel_max_level = 2
        # HIP streams a batch of N >= 2 pairs is split over (pairs are
        # independent: the output is bitwise that of one stream; the parts'
        # kernels fill each other's launch gaps and tails)
        self.streams = 2
        self.register_load_state_dict_post_hook(Net._on_load)

    # Packed weights are rebuilt after load_state_dict / .to() / param edits.
    @staticmethod
    def _on_load(module, incompatible_keys):
        module._weights_version += 1

    def invalidate_packed_weights(self):
        self._weights_version += 1

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._weights_version += 1
        return out

    def engine(self):
        from .engine import RRINEngine
        if (self._engine is None or self._engine_version != self._weights_version
                or self._engine.precision != self.precision
                or self._engine.subpixel_max_level != self.subpixel_max_level):
            self._engine = None  # free the previous packed weights first
            self._engine = RRINEngine(self, self.precision, self.subpixel_max_level)
            self._engine_version = self._weights_version
        return self._engine

    def interpolate(self, input0, input1, ts):
        """All intermediate frames of one (batch of) pair(s): ``[forward(I0, I1, t) for t in ts]``
        with the t-independent Flow U-Net computed once (the
        reference recomputes it per t, convert.py:127-130)."""
        if torch.is_grad_enabled():
            raise RuntimeError("rrin_amd.Net.interpolate is inference-only: use torch.no_grad()")
        eng = self.engine()
        return [eng.forward(input0, input1, t, reuse_flow=(k > 0), streams=self.streams)
                for k, t in enumerate(ts)]

    def forward(self, input0, input1, t=0.5):
        if torch.is_grad_enabled() and (input0.requires_grad or input1.requires_grad or
                                        any(p.requires_grad for p in self.parameters())):
            raise RuntimeError(
                "rrin_amd.Net runs HIP inference kernels only (no backward): call it under "
                "torch.no_grad() or torch.inference_mode(), as convert.py:117 does")
        return self.engine().forward(input0, input1, t, streams=self.streams)
