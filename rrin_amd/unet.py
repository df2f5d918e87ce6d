"""Parameter tree of one RRIN U-Net, key-compatible with the reference.

The module tree reproduces the reference U-Net's (`/root/reference/unet.py:9-95`)
*parameter naming*: a checkpoint written by the reference `train.py:158-161`
must load with ``load_state_dict(strict=True)`` (`convert.py:103`).  The
arithmetic is done by `rrin_amd.engine`, which walks the tree and launches HIP
kernels with the packed weights: inside ``Net.forward`` for the whole Net, and
for a ``UNet`` called on its own (``UNet.forward`` without autograd ->
``rrin_unet_fwd``, same kernels).  With autograd on, ``UNet.forward`` is the
training path (HIP forward + backward kernels on a ROCm device,
``rrin_amd.autograd``; PyTorch operators on a CPU device).  Attribute paths (the reference key layout):

    down_path.{i}.block.{0,2}.{weight,bias}          unet.py:23-28, 59-63
    midconv.{weight,bias}                            unet.py:29
    up_path.{j}.up.1.{weight,bias}                   unet.py:31-36, 76-79
    up_path.{j}.conv_block.block.{0,2}.{weight,bias} unet.py:80, 59-63
    last.{weight,bias}                               unet.py:38

Channel plan (``wf=5``): level i has ``2**(5+i)`` channels (unet.py:26).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

WF = 5                 # unet.py:15 default width factor
LEAKY_SLOPE = 0.1      # unet.py:47,60,63


def level_channels(i: int) -> int:
    return 2 ** (WF + i)


def _conv3x3(cin: int, cout: int) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, padding=1)


class _TwoConv(nn.Module):
    """conv3x3 -> leaky -> conv3x3 -> leaky; params at ``block.0`` / ``block.2``
    (reference UNetConvBlock, unet.py:54-69)."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.block = nn.Sequential(_conv3x3(cin, cout), nn.LeakyReLU(LEAKY_SLOPE),
                                   _conv3x3(cout, cout), nn.LeakyReLU(LEAKY_SLOPE))


class _UpStage(nn.Module):
    """bilinear x2 -> conv3x3 (no act), concat with bridge, _TwoConv
    (reference UNetUpBlock, unet.py:72-95)."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.up = nn.Sequential(nn.Upsample(mode="bilinear", scale_factor=2),
                                _conv3x3(cin, cout))
        self.conv_block = _TwoConv(cin, cout)


class UNet(nn.Module):
    """Same constructor contract as reference ``UNet(in_channels, n_classes,
    depth, wf=5, padding=True)`` (unet.py:10-17)."""

    def __init__(self, in_channels: int = 1, n_classes: int = 2, depth: int = 5,
                 wf: int = WF, padding: bool = True):
        super().__init__()
        if wf != WF or not padding:
            raise ValueError("RRIN uses wf=5 and padding=True only")
        self.in_channels = in_channels
        self.n_classes = n_classes
        self.depth = depth
        widths = [level_channels(i) for i in range(depth)]
        ins = [in_channels] + widths[:-1]
        self.down_path = nn.ModuleList(_TwoConv(a, b) for a, b in zip(ins, widths))
        self.midconv = _conv3x3(widths[-1], widths[-1])
        self.up_path = nn.ModuleList(
            _UpStage(widths[i + 1], widths[i]) for i in reversed(range(depth - 1)))
        self.last = _conv3x3(widths[0], n_classes)
        # HIP path of a standalone UNet call (not part of the reference contract):
        # arithmetic as Net.precision ("fp32" exact by default)
        self.precision = "fp32"
        self._engine = None
        self._engine_key = None

    def _hip_engine(self):
        from .engine import RRINEngine
        key = (self.precision, tuple((p.data_ptr(), p._version) for p in self.parameters()))
        if self._engine is None or self._engine_key != key:
            self._engine = None
            self._engine = RRINEngine(self, self.precision, units=[("unet", self, None)])
            self._engine_key = key
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine = None  # device / dtype moves repack
        return super()._apply(fn, *args, **kwargs)

    # -- helpers used by the engine --------------------------------------
    def conv_list(self):
        """All convs in execution order with a role tag (used for packing)."""
        out = []
        for i, d in enumerate(self.down_path):
            out.append((f"down{i}.a", d.block[0]))
            out.append((f"down{i}.b", d.block[2]))
        out.append(("mid", self.midconv))
        for j, u in enumerate(self.up_path):
            out.append((f"up{j}.up", u.up[1]))
            out.append((f"up{j}.a", u.conv_block.block[0]))
            out.append((f"up{j}.b", u.conv_block.block[2]))
        out.append(("last", self.last))
        return out

    def forward(self, x):
        """Reference ``UNet.forward`` (unet.py:40-51).  Without autograd: the HIP
        kernels (``rrin_unet_fwd``; the input must be fp32 on a ROCm device, H
        and W multiples of 16).  With autograd on (training): on a ROCm device
        the HIP training Functions (``rrin_amd.autograd.unet_forward``), on a
        CPU device the same math with PyTorch operators."""
        if not torch.is_grad_enabled() or not (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return self._hip_engine().unet_forward(x)
        if x.is_cuda:  # training on the GPU: HIP forward + backward kernels (rrin_amd.autograd)
            from .autograd import unet_forward
            return unet_forward(self, x)
        bridges = []
        for i, d in enumerate(self.down_path):
            x = d.block(x)
            if i < self.depth - 1:
                bridges.append(x)
                x = F.avg_pool2d(x, 2)
        x = F.leaky_relu(self.midconv(x), LEAKY_SLOPE)
        for j, u in enumerate(self.up_path):
            x = u.conv_block.block(torch.cat((u.up(x), bridges[-j - 1]), 1))
        return self.last(x)


def conv_flops(unet: UNet, h: int, w: int) -> int:
    """Algorithmic FLOPs (2*MAC) of one UNet forward at input size h x w."""
    total = 0
    for tag, conv in unet.conv_list():
        lvl = _level_of(unet, tag)
        hh, ww = h >> lvl, w >> lvl
        total += 2 * conv.out_channels * conv.in_channels * 9 * hh * ww
    return total


def _level_of(unet: UNet, tag: str) -> int:
    if tag.startswith("down"):
        return int(tag[4:tag.index(".")])
    if tag == "mid":
        return unet.depth - 1
    if tag.startswith("up"):
        j = int(tag[2:tag.index(".")])
        return unet.depth - 2 - j
    return 0  # last


def conv_work(unet: UNet, h: int, w: int, bytes_per_value: int = 4):
    """Per body conv (head excluded): (tag, algorithmic FLOPs, bytes read, bytes
    written).  Each conv reads its input once and writes its output once; a down
    block's second conv also writes the 2x2-pooled copy; an up conv reads its
    input at low resolution (the x2 upsample is recomputable)."""
    out = []
    for tag, conv in unet.conv_list():
        if tag == "last":
            continue
        lvl = _level_of(unet, tag)
        px = (h >> lvl) * (w >> lvl)
        rd = conv.in_channels * (px // 4 if tag.endswith(".up") else px)
        wr = conv.out_channels * px
        if tag.startswith("down") and tag.endswith(".b") and lvl < unet.depth - 1:
            wr += conv.out_channels * px // 4
        fl = 2 * conv.out_channels * conv.in_channels * 9 * px
        out.append((tag, fl, rd * bytes_per_value, wr * bytes_per_value))
    return out


def conv_bytes(unet: UNet, h: int, w: int, bytes_per_value: int = 4) -> tuple[int, int]:
    """Algorithmic HBM bytes (read, written) of the body convs of one UNet forward."""
    work = conv_work(unet, h, w, bytes_per_value)
    return sum(r for _, _, r, _ in work), sum(wb for _, _, _, wb in work)


def roofline_bound_s(unet: UNet, h: int, w: int, bytes_per_value: int, peak_flops: float, bw: float,
                     flop_scale: float = 1.0) -> float:
    """Per-layer roofline bound T_LB = sum over body convs of max(FLOP/peak, bytes/BW)
    (SURVEY §8d), in seconds for one image.  ``flop_scale``: FLOPs of the algorithm
    the convs run per direct-form FLOP (Winograd F(2x2,3x3): 4/9) -- a number for every
    conv, or a function of (tag, cin, cout, level) when the form differs by conv."""
    convs = dict(unet.conv_list())

    def scale(tag):
        if not callable(flop_scale):
            return flop_scale
        c = convs[tag]
        return flop_scale(tag, c.in_channels, c.out_channels, _level_of(unet, tag))
    return sum(max(scale(tag) * fl / peak_flops, (r + wb) / bw)
               for tag, fl, r, wb in conv_work(unet, h, w, bytes_per_value))
