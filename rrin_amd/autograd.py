"""Training path on MI355X: autograd Functions over the HIP training kernels.

The reference trains through ``Net.forward`` with autograd on (`train.py:98`)
and ``loss.backward()`` (`train.py:144`).  With autograd on and the model on a
ROCm device, ``rrin_amd.Net.forward`` / ``UNet.forward`` run the reference
graph (`model.py:32-65`, `unet.py:40-51`) with these Functions, each a forward
HIP kernel and its backward HIP kernel(s) from ``csrc/train.hip``:

=====================  ==========================================  ===============================
Function               forward (reference op)                       backward
=====================  ==========================================  ===============================
``conv3x3``            Conv2d(3, pad=1) + bias [+ LeakyReLU(0.1)]   dgrad (flipped W, leaky' fused),
                       (unet.py:29,38,59-63,78)                     wgrad + bias grad (split-K)
``avg_pool2``          F.avg_pool2d(x, 2) (unet.py:46)              0.25 spread
``upsample2``          Upsample(x2, bilinear) (unet.py:77)          transposed stencil (gather)
``backwarp``           warp = grid_sample (model.py:8-21)           image (fixed-point scatter) and
                                                                    flow gradients
=====================  ==========================================  ===============================

The glue between them (cat, the flow t-blend, sigmoid, the blend division,
the residual add and clamp; `model.py:33-63`) is elementwise PyTorch autograd.
On a CPU device the model keeps the PyTorch-operator graph (``Net._forward_autograd``).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

LEAKY_SLOPE = 0.1


def _stream(device: torch.device):
    """The current stream of the tensors' device (not the thread's current device: a
    model on cuda:1 without set_device must not launch on device 0's stream)."""
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32 or not t.is_cuda:
        raise TypeError("rrin_amd training kernels take float32 tensors on a ROCm device")
    return t.contiguous()


# Forward and data-gradient convs on the inference path's exact-fp32 Winograd kernels
# (conv_wino*.hip, record layout) instead of csrc/train.hip's general implicit GEMM:
# the weights are packed on the device every call (rrin_tpack_wino: the host packing's
# bits; the dgrad conv is the forward conv of the flipped, transposed weights), the NCHW
# tensors of the autograd graph go through the record layout (rrin_nchw_to_h8 /
# rrin_h8_to_nchw) in per-shape buffers reused in stream order.  False: train.hip for all
# three (A/B).
TRAIN_WINO = True
# Record-layout buffers by (device, stream, shape, role), least recently used first.  A buffer
# is only touched by kernels on its own stream, so reusing it is ordered; an evicted buffer goes
# back to the caching allocator's pool of that stream.  Bounded: training with varying crop
# sizes does not keep every shape's buffers for the life of the process.
_R32_BUFS: "OrderedDict" = None
R32_BUFS_MAX = 96


def _r32_buf(n, c, h, w, device, role):
    """A zero-padded fp32-record buffer of c channels (a multiple of 8) per stream, shape and
    role (the padding and the channel tail are never written, so they stay zero)."""
    from collections import OrderedDict

    from .pp import H8Tensor
    global _R32_BUFS
    if _R32_BUFS is None:
        _R32_BUFS = OrderedDict()
    key = (device, torch.cuda.current_stream(device).cuda_stream, n, c, h, w, role)
    t = _R32_BUFS.get(key)
    if t is None:
        t = H8Tensor(n, c, h, w, device, _lib.PREC_F32R)
        _R32_BUFS[key] = t
        while len(_R32_BUFS) > R32_BUFS_MAX:
            _R32_BUFS.popitem(last=False)
    else:
        _R32_BUFS.move_to_end(key)
    return t


# Per-launch conv timing for bench.py --train: a list to collect (start event, end event,
# algorithmic FLOPs, kind) of every conv kernel launch (forward, dgrad, wgrad) on the
# launch's own stream; None (default): no events.
PROF = None


class _ProfScope:
    def __init__(self, device, flops, kind):
        self.on = PROF is not None
        if self.on:
            self.st = torch.cuda.current_stream(device)
            self.e0, self.e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self.flops, self.kind = flops, kind

    def __enter__(self):
        if self.on:
            self.e0.record(self.st)
        return self

    def __exit__(self, *exc):
        if self.on:
            self.e1.record(self.st)
            PROF.append((self.e0, self.e1, self.flops, self.kind))
        return False


def _wino_conv(x, wpack, bias, rows, cfg, leaky, st, role):
    """y[n, rows] = conv3x3(x) + bias [, leaky] with packed Winograd weights (cfg's BM)."""
    L = _lib.lib()
    n, cin, h, w = x.shape
    c8, r8 = (cin + 7) // 8 * 8, (rows + 7) // 8 * 8
    xb = _r32_buf(n, c8, h, w, x.device, role + "x")
    v = xb.view(0, c8)
    _lib.check(L.rrin_nchw_to_h8(C.c_void_p(x.data_ptr()), n, cin, 0, C.byref(v), _lib.PREC_F32R, st),
               "rrin_nchw_to_h8")
    yb = _r32_buf(n, r8, h, w, x.device, role + "y")
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec = n, cin, r8, cfg, _lib.PREC_F32R
    d.epi_mode = _lib.EPI_LEAKY if leaky else _lib.EPI_LINEAR
    d.slope, d.inv_wscale, d.tail_finite = LEAKY_SLOPE, 1.0, 1  # channels [cin, c8) stay zero
    d.src, d.dst = xb.view(0, c8), yb.view(0, r8)
    d.whi, d.wlo, d.bias = wpack.data_ptr(), wpack.data_ptr(), bias.data_ptr()
    # Winograd F(2x2,3x3): 4 multiply-adds per output, input channel and pixel
    with _ProfScope(x.device, 2.0 * 4 * cin * rows * h * w * n, "fwd" if role == "f" else "dgrad"):
        _lib.check(L.rrin_conv3x3_h8_fwd(C.byref(d), st), "rrin_conv3x3_h8_fwd (training)")
    y = torch.empty((n, rows, h, w), dtype=torch.float32, device=x.device)
    vy = yb.view(0, r8)
    _lib.check(L.rrin_h8_to_nchw(C.byref(vy), n, rows, 0, C.c_void_p(y.data_ptr()), _lib.PREC_F32R, st),
               "rrin_h8_to_nchw")
    return y


def _wino_pack(weight, rows, cols, mode, st):
    """(packed weights, cfg) of the forward (mode 0) or data-gradient (mode 1) conv."""
    from . import engine
    L = _lib.lib()
    kind = 6 if rows % 64 == 0 else 7
    cfg = engine.wino_cfg(kind)
    bm = L.rrin_conv_h8_cfg_bm(cfg)
    wp = torch.empty(int(L.rrin_pack_conv3x3_wino_bm_floats(rows, cols, bm)), dtype=torch.float32,
                     device=weight.device)
    cout, cin = weight.shape[:2]
    _lib.check(L.rrin_tpack_wino(C.c_void_p(weight.data_ptr()), cout, cin, bm, mode, C.c_void_p(wp.data_ptr()), st),
               "rrin_tpack_wino")
    return wp, cfg, bm


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, leaky: bool):
        x, weight = _f32(x), _f32(weight)
        bias = _f32(bias) if bias is not None else None
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        if weight.shape != (cout, cin, 3, 3):
            raise ValueError(f"weight {tuple(weight.shape)} for input {tuple(x.shape)}")
        st = _stream(x.device)
        if TRAIN_WINO:
            wp, cfg, bm = _wino_pack(weight, cout, cin, 0, st)
            bp = torch.zeros(((cout + bm - 1) // bm) * bm, dtype=torch.float32, device=x.device)
            if bias is not None:
                bp[:cout] = bias
            y = _wino_conv(x, wp, bp, cout, cfg, leaky, st, "f")
        else:
            y = torch.empty((n, cout, h, w), dtype=torch.float32, device=x.device)
            d = _lib.TConvDesc(n=n, cin=cin, cout=cout, h=h, w=w, mode=_lib.TCONV_FWD, leaky=int(leaky),
                               slope=LEAKY_SLOPE, x=x.data_ptr(), y=None, wt=weight.data_ptr(),
                               bias=bias.data_ptr() if bias is not None else None, out=y.data_ptr())
            with _ProfScope(x.device, 2.0 * 9 * cin * cout * h * w * n, "fwd"):
                _lib.check(_lib.lib().rrin_tconv3x3(C.byref(d), st), "rrin_tconv3x3 (forward)")
        ctx.leaky = bool(leaky)
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight, y if leaky else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        gy = _f32(gy)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        L = _lib.lib()
        st = _stream(x.device)
        gx = gw = gb = None
        gp = None
        if TRAIN_WINO and ctx.leaky:
            # g' = g * leaky'(pre), the sign of y being the pre-activation's (slope > 0): once,
            # for both gradient convs
            gp = torch.where(y > 0, gy, gy * LEAKY_SLOPE)
        if ctx.needs_input_grad[0] and TRAIN_WINO:
            gp = gy if gp is None else gp
            wp, cfg, bm = _wino_pack(weight, cin, cout, 1, st)
            zb = torch.zeros(((cin + bm - 1) // bm) * bm, dtype=torch.float32, device=x.device)
            gx = _wino_conv(gp, wp, zb, cin, cfg, False, st, "d")
        elif ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            d = _lib.TConvDesc(n=n, cin=cin, cout=cout, h=h, w=w, mode=_lib.TCONV_DGRAD, leaky=int(ctx.leaky),
                               slope=LEAKY_SLOPE, x=gy.data_ptr(), y=y.data_ptr() if ctx.leaky else None,
                               wt=weight.data_ptr(), bias=None, out=gx.data_ptr())
            with _ProfScope(x.device, 2.0 * 9 * cin * cout * h * w * n, "dgrad"):
                _lib.check(L.rrin_tconv3x3(C.byref(d), st), "rrin_tconv3x3 (dgrad)")
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            gw = torch.empty_like(weight)
            gb = torch.empty((cout,), dtype=torch.float32, device=x.device)
            nw = int(L.rrin_tconv3x3_wgrad_work_floats(n, cin, cout, h, w))
            if nw < 0:
                _lib.check(nw, "rrin_tconv3x3_wgrad_work_floats")
            work = torch.empty((nw,), dtype=torch.float32, device=x.device)
            if gp is not None:  # already masked
                d = _lib.TWgradDesc(n=n, cin=cin, cout=cout, h=h, w=w, leaky=0, slope=LEAKY_SLOPE,
                                    x=x.data_ptr(), g=gp.data_ptr(), y=None,
                                    gw=gw.data_ptr(), gb=gb.data_ptr(), work=work.data_ptr())
            else:
                d = _lib.TWgradDesc(n=n, cin=cin, cout=cout, h=h, w=w, leaky=int(ctx.leaky), slope=LEAKY_SLOPE,
                                    x=x.data_ptr(), g=gy.data_ptr(), y=y.data_ptr() if ctx.leaky else None,
                                    gw=gw.data_ptr(), gb=gb.data_ptr(), work=work.data_ptr())
            # direct form: 9 multiply-adds per weight, image and pixel
            with _ProfScope(x.device, 2.0 * 9 * cin * cout * h * w * n, "wgrad"):
                _lib.check(L.rrin_tconv3x3_wgrad(C.byref(d), st), "rrin_tconv3x3_wgrad")
        return gx, gw, (gb if ctx.has_bias else None), None


class _AvgPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _f32(x)
        n, c, h, w = x.shape
        y = torch.empty((n, c, h // 2, w // 2), dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib().rrin_tpool2_fwd(x.data_ptr(), y.data_ptr(), n * c, h, w, _stream(x.device)), "rrin_tpool2_fwd")
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = _f32(gy)
        n, c, h, w = ctx.shape
        gx = torch.empty(ctx.shape, dtype=torch.float32, device=gy.device)
        _lib.check(_lib.lib().rrin_tpool2_bwd(gy.data_ptr(), gx.data_ptr(), n * c, h, w, _stream(gy.device)),
                   "rrin_tpool2_bwd")
        return gx


class _Upsample2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _f32(x)
        n, c, h, w = x.shape
        y = torch.empty((n, c, 2 * h, 2 * w), dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib().rrin_tup2_fwd(x.data_ptr(), y.data_ptr(), n * c, h, w, _stream(x.device)), "rrin_tup2_fwd")
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = _f32(gy)
        n, c, h, w = ctx.shape
        gx = torch.empty(ctx.shape, dtype=torch.float32, device=gy.device)
        _lib.check(_lib.lib().rrin_tup2_bwd(gy.data_ptr(), gx.data_ptr(), n * c, h, w, _stream(gy.device)), "rrin_tup2_bwd")
        return gx


class _Backwarp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, flow):
        img, flow = _f32(img), _f32(flow)
        n, c, h, w = img.shape
        if flow.shape != (n, 2, h, w):
            raise ValueError(f"flow {tuple(flow.shape)} for image {tuple(img.shape)}")
        out = torch.empty_like(img)
        _lib.check(_lib.lib().rrin_warp_fwd(img.data_ptr(), flow.data_ptr(), out.data_ptr(), n, c, h, w, _stream(img.device)),
                   "rrin_warp_fwd")
        ctx.save_for_backward(img, flow)
        return out

    @staticmethod
    def backward(ctx, gout):
        img, flow = ctx.saved_tensors
        gout = _f32(gout)
        n, c, h, w = img.shape
        L = _lib.lib()
        nb = int(L.rrin_twarp_bwd_work_bytes(n, c, h, w))
        if nb < 0:
            _lib.check(nb, "rrin_twarp_bwd_work_bytes")
        work = torch.empty((nb,), dtype=torch.uint8, device=img.device)
        gimg = torch.empty_like(img)
        gflow = torch.empty_like(flow)
        _lib.check(L.rrin_twarp_bwd(img.data_ptr(), flow.data_ptr(), gout.data_ptr(), gimg.data_ptr(),
                                    gflow.data_ptr(), work.data_ptr(), nb, n, c, h, w, _stream(img.device)), "rrin_twarp_bwd")
        return gimg, gflow


def conv3x3(x, conv: torch.nn.Conv2d, leaky: bool = False):
    return _Conv3x3.apply(x, conv.weight, conv.bias, leaky)


def avg_pool2(x):
    return _AvgPool2.apply(x)


def upsample2(x):
    return _Upsample2.apply(x)


def backwarp(img, flow):
    return _Backwarp.apply(img, flow)


def unet_forward(unet, x):
    """Reference UNet.forward (unet.py:40-51) on the HIP training Functions."""
    bridges = []
    for i, d in enumerate(unet.down_path):
        x = conv3x3(x, d.block[0], leaky=True)
        x = conv3x3(x, d.block[2], leaky=True)
        if i < unet.depth - 1:
            bridges.append(x)
            x = avg_pool2(x)
    x = conv3x3(x, unet.midconv, leaky=True)
    for j, u in enumerate(unet.up_path):
        up = conv3x3(upsample2(x), u.up[1], leaky=False)
        x = torch.cat((up, bridges[-j - 1]), 1)
        x = conv3x3(x, u.conv_block.block[0], leaky=True)
        x = conv3x3(x, u.conv_block.block[2], leaky=True)
    return conv3x3(x, unet.last, leaky=False)


def net_forward(net, input0, input1, t=0.5):
    """Reference Net.forward (model.py:32-65) on the HIP training Functions."""
    x = torch.cat((input0, input1), 1)
    flow = unet_forward(net.Flow, x)
    f01, f10 = flow[:, :2], flow[:, 2:4]
    ft0 = -(1 - t) * t * f01 + t * t * f10
    ft1 = (1 - t) * (1 - t) * f01 - t * (1 - t) * f10
    r = unet_forward(net.refine_flow, torch.cat((ft0, ft1, x), 1))
    ft0 = ft0 + r[:, :2]
    ft1 = ft1 + r[:, 2:4]
    xt1 = backwarp(input0, ft0)
    xt2 = backwarp(input1, ft1)
    m = torch.sigmoid(unet_forward(net.Mask, torch.cat((ft0, ft1, x, xt1, xt2), 1)))
    w1, w2 = (1 - t) * m[:, 0:1], t * m[:, 1:2]
    out = (w1 * xt1 + w2 * xt2) / (w1 + w2 + 1e-8)
    return (unet_forward(net.final, torch.cat((input0, input1, out), 1)) + out).clamp(0, 1)
