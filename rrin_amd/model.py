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
  caller `convert.py:117`.

With autograd on (the training caller `train.py:98`) ``forward``
runs the reference graph (`model.py:32-65`) on the HIP training kernels: on a
ROCm device every conv3x3 (+ leaky), avg-pool, upsample and backwarp is an
autograd Function whose forward and backward are HIP kernels
(``rrin_amd.autograd``, ``csrc/train.hip``), the elementwise glue is PyTorch
autograd; on a CPU device the same graph runs with PyTorch operators
(``_forward_autograd``).  That path is never taken for inference, and a
missing or failing HIP library raises.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
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
        self._engine_fp = None
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
        # kernels fill each other's launch gaps and tails); None: by precision
        # and batch (engine.default_streams: 2)
        self.streams = None
        self.register_load_state_dict_post_hook(Net._on_load)

    # Packed weights are rebuilt after load_state_dict / .to() (version bump) and
    # after any in-place parameter edit (optimizer.step, p.copy_, nn.init, a
    # sub-UNet's load_state_dict): engine() compares each parameter's storage
    # pointer and autograd version counter with those the packing was built from.
    @staticmethod
    def _on_load(module, incompatible_keys):
        module._weights_version += 1

    def invalidate_packed_weights(self):
        self._weights_version += 1

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._weights_version += 1
        return out

    def _weights_fingerprint(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def engine(self):
        from .engine import RRINEngine
        fp = self._weights_fingerprint()
        if (self._engine is None or self._engine_version != self._weights_version
                or self._engine_fp != fp
                or self._engine.precision != self.precision
                or self._engine.subpixel_max_level != self.subpixel_max_level):
            self._engine = None  # free the previous packed weights first
            self._engine = RRINEngine(self, self.precision, self.subpixel_max_level)
            self._engine_version = self._weights_version
            self._engine_fp = fp
        return self._engine

    def check_range(self, wait: bool = True):
        """fp32_split16 / fp16: raise if an activation overflowed fp16 in a
        forward issued so far (those outputs are NaN-poisoned on the device).
        ``wait=False`` only looks at the forwards that have already finished.
        A no-op for the fp32 precisions."""
        if self._engine is not None:
            self._engine._poll_range(wait=wait)

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
            if input0.is_cuda:
                from .autograd import net_forward
                return net_forward(self, input0, input1, t)
            return self._forward_autograd(input0, input1, t)
        return self.engine().forward(input0, input1, t, streams=self.streams)

    @staticmethod
    def _backwarp(img, flow):
        """model.py:8-21 with the grid built on the image's device (the reference
        hard-codes .cuda())."""
        n, _, h, w = img.shape
        gy, gx = torch.meshgrid(torch.arange(h, device=img.device), torch.arange(w, device=img.device),
                                indexing="ij")
        x = gx.unsqueeze(0).expand(n, h, w).float() + flow[:, 0]
        y = gy.unsqueeze(0).expand(n, h, w).float() + flow[:, 1]
        grid = torch.stack((2 * (x / w - 0.5), 2 * (y / h - 0.5)), dim=3)
        return F.grid_sample(img, grid, mode="bilinear", padding_mode="zeros", align_corners=False)

    def _forward_autograd(self, input0, input1, t=0.5):
        """Training path on a CPU device (autograd on): model.py:32-65 with PyTorch operators."""
        x = torch.cat((input0, input1), 1)
        flow = self.Flow(x)
        f01, f10 = flow[:, :2], flow[:, 2:4]
        ft0 = -(1 - t) * t * f01 + t * t * f10
        ft1 = (1 - t) * (1 - t) * f01 - t * (1 - t) * f10
        r = self.refine_flow(torch.cat((ft0, ft1, x), 1))
        ft0 = ft0 + r[:, :2]
        ft1 = ft1 + r[:, 2:4]
        xt1 = self._backwarp(input0, ft0)
        xt2 = self._backwarp(input1, ft1)
        m = torch.sigmoid(self.Mask(torch.cat((ft0, ft1, x, xt1, xt2), 1)))
        w1, w2 = (1 - t) * m[:, 0:1], t * m[:, 1:2]
        out = (w1 * xt1 + w2 * xt2) / (w1 + w2 + 1e-8)
        return (self.final(torch.cat((input0, input1, out), 1)) + out).clamp(0, 1)
