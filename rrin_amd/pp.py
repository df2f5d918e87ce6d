"""Padded-planar (PP) activation tensors on the device (layout: DESIGN.md §3).

A PP tensor is a torch allocation ``[n, c, hp, wp]`` fp32 with
``hp = round_up(h,16)+2``, ``wp = round_up(w,32)+64`` and pixel (y,x) at
``[.., y+1, x+32]``; the padding is zero and never written by the kernels.
Conversions to/from NCHW run the library's HIP layout kernels.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib


class PPTensor:
    def __init__(self, n: int, c: int, h: int, w: int, device):
        self.n, self.c, self.h, self.w = n, c, h, w
        self.g = _lib.geom(h, w)
        self.t = torch.zeros((n, c, self.g.hp, self.g.wp), dtype=torch.float32, device=device)

    def view(self, ch_off: int = 0, channels: int | None = None) -> _lib.PP:
        v = _lib.PP()
        v.base = self.t.data_ptr()
        v.img_stride = self.c * self.g.plane
        v.ch_off = ch_off
        v.channels = self.c - ch_off if channels is None else channels
        v.g = self.g
        return v

    @classmethod
    def from_nchw(cls, x: torch.Tensor, c_alloc: int | None = None, ch_off: int = 0) -> "PPTensor":
        x = x.contiguous()
        n, c, h, w = x.shape
        pp = cls(n, c_alloc or c + ch_off, h, w, x.device)
        pp.load(x, ch_off)
        return pp

    def load(self, x: torch.Tensor, ch_off: int = 0):
        x = x.contiguous().float()
        v = self.view(ch_off, x.shape[1])
        _lib.check(_lib.lib().rrin_nchw_to_pp(C.c_void_p(x.data_ptr()), x.shape[0], x.shape[1],
                                              C.byref(v), _stream(x.device)), "rrin_nchw_to_pp")

    def to_nchw(self, ch_off: int = 0, channels: int | None = None) -> torch.Tensor:
        channels = self.c - ch_off if channels is None else channels
        out = torch.empty((self.n, channels, self.h, self.w), dtype=torch.float32, device=self.t.device)
        v = self.view(ch_off, channels)
        _lib.check(_lib.lib().rrin_pp_to_nchw(C.byref(v), self.n, channels, C.c_void_p(out.data_ptr()),
                                              _stream(out.device)), "rrin_pp_to_nchw")
        return out


def _stream(device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class H8Tensor:
    """Channel-record activation tensor (record layout, include/rrin_hip.h):
    ``hi`` (and for fp32_split16 ``lo``) are ``[n, ceil(c/8), hp, wp, 8]``
    half tensors (fp32 records, PREC_F32R: ``[n, ceil(c/4), hp, wp, 4]``
    float), pixel (y,x) at ``[.., y+1, x+8, :]``; padding zero.  The group count is
    rounded up to whole 2-group chunks: the Winograd tiles stage both record groups of
    every K chunk (``chunk_view``), past ``c`` against zero weights."""

    def __init__(self, n: int, c: int, h: int, w: int, device, prec: int):
        self.n, self.c, self.h, self.w, self.prec = n, c, h, w, prec
        self.g = _lib.geom_h8(h, w)
        self.cpr = _lib.chans_per_record(prec)
        self.groups = (c + 2 * self.cpr - 1) // (2 * self.cpr) * 2
        shape = (n, self.groups, self.g.hp, self.g.wp, self.cpr)
        dt = torch.float32 if prec == _lib.PREC_F32R else torch.float16
        self.hi = torch.zeros(shape, dtype=dt, device=device)
        self.lo = torch.zeros(shape, dtype=torch.float16, device=device) if prec == _lib.PREC_F16X3 else None

    def view(self, ch_off: int = 0, channels: int | None = None) -> _lib.H8:
        channels = self.c - ch_off if channels is None else channels
        if ch_off % self.cpr:
            raise ValueError("record views start on a record group")
        v = _lib.H8()
        v.hi = self.hi.data_ptr()
        v.lo = self.lo.data_ptr() if self.lo is not None else None
        v.img_stride = self.groups * self.g.plane
        v.g_off = ch_off // self.cpr
        v.groups = (channels + self.cpr - 1) // self.cpr
        v.g = self.g
        return v

    def chunk_view(self, ch_off: int = 0, channels: int | None = None) -> _lib.H8:
        """``view`` widened to whole 2-group chunks (within the allocation): the source
        view of a conv, which may stage groups past ``channels`` (conv_f16.hip h8_prepare)."""
        v = self.view(ch_off, channels)
        v.groups = min((v.groups + 1) // 2 * 2, self.groups - v.g_off)
        return v

    @classmethod
    def from_nchw(cls, x: torch.Tensor, prec: int, c_alloc: int | None = None, ch_off: int = 0) -> "H8Tensor":
        n, c, h, w = x.shape
        t = cls(n, c_alloc or c + ch_off, h, w, x.device, prec)
        t.load(x, ch_off)
        return t

    def load(self, x: torch.Tensor, ch_off: int = 0):
        x = x.contiguous().float()
        v = self.view(0, self.c)
        _lib.check(_lib.lib().rrin_nchw_to_h8(C.c_void_p(x.data_ptr()), x.shape[0], x.shape[1], ch_off,
                                              C.byref(v), self.prec, _stream(x.device)), "rrin_nchw_to_h8")

    def to_nchw(self, ch_off: int = 0, channels: int | None = None) -> torch.Tensor:
        channels = self.c - ch_off if channels is None else channels
        out = torch.empty((self.n, channels, self.h, self.w), dtype=torch.float32, device=self.hi.device)
        v = self.view(0, self.c)
        _lib.check(_lib.lib().rrin_h8_to_nchw(C.byref(v), self.n, channels, ch_off, C.c_void_p(out.data_ptr()),
                                              self.prec, _stream(out.device)), "rrin_h8_to_nchw")
        return out
