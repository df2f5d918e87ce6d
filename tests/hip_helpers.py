"""Test helpers: drive single kernels of librrin_hip.so through the C ABI."""
import ctypes as C

import numpy as np
import torch

from rrin_amd import _lib
from rrin_amd.pp import PPTensor


def stream(dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def pack(w: torch.Tensor, b: torch.Tensor, cfg: int, perm=None, dev="cuda"):
    lib = _lib.lib()
    w = w.detach().cpu().float().contiguous().numpy()
    b = b.detach().cpu().float().contiguous().numpy()
    cout, cin = w.shape[:2]
    bm = lib.rrin_conv_cfg_bm(cfg)
    wp = np.empty(lib.rrin_pack_conv3x3_floats(cout, cin, bm), np.float32)
    bp = np.empty(lib.rrin_pack_bias_floats(cout, bm), np.float32)
    pa = np.asarray(perm, np.int32) if perm is not None else None
    _lib.check(lib.rrin_pack_conv3x3(w.ctypes.data, b.ctypes.data, cout, cin, bm,
                                     pa.ctypes.data if pa is not None else None, wp.ctypes.data,
                                     bp.ctypes.data))
    return torch.from_numpy(wp).to(dev), torch.from_numpy(bp).to(dev)


def conv(src: PPTensor, w, b, cfg, *, src_off=0, dst=None, dst_off=0, upsample=False, epi=_lib.EPI_LINEAR,
         pool=None, perm=None, cin=None):
    """Run rrin_conv3x3_fwd; returns (dst PPTensor, pool PPTensor or None)."""
    dev = src.t.device
    cout, cin_w = w.shape[:2]
    cin = cin or cin_w
    h, wd = (src.h * 2, src.w * 2) if upsample else (src.h, src.w)
    if dst is None:
        dst = PPTensor(src.n, cout + dst_off, h, wd, dev)
    if epi == _lib.EPI_LEAKY_POOL and pool is None:
        pool = PPTensor(src.n, cout, h // 2, wd // 2, dev)
    wp, bp = pack(w, b, cfg, perm, dev)
    d = _lib.ConvDesc()
    d.n, d.cin, d.cout, d.cfg = src.n, cin, cout, cfg
    d.src_mode = _lib.SRC_UPSAMPLE2X if upsample else _lib.SRC_DIRECT
    d.epi_mode = epi
    d.slope = 0.1
    d.src = src.view(src_off, cin)
    d.dst = dst.view(dst_off, cout)
    if pool is not None:
        d.pool = pool.view(0, cout)
    d.wpack, d.bias = wp.data_ptr(), bp.data_ptr()
    _lib.check(_lib.lib().rrin_conv3x3_fwd(C.byref(d), stream(dev)), "rrin_conv3x3_fwd")
    torch.cuda.synchronize(dev)
    return dst, pool


def head(src: PPTensor, g16: PPTensor, w, b, mode, coef=None, out=None):
    dev = src.t.device
    d = _lib.HeadDesc()
    d.n, d.cin, d.cout, d.mode = src.n, 32, w.shape[0], mode
    d.src = src.view(0, 32)
    d.g16 = g16.view(0, g16.c)
    wd = w.detach().float().contiguous().to(dev)
    bd = b.detach().float().contiguous().to(dev)
    d.w, d.bias = wd.data_ptr(), bd.data_ptr()
    if coef is not None:
        d.coef = coef.data_ptr()
    if out is not None:
        d.out = out.data_ptr()
    _lib.check(_lib.lib().rrin_head_fwd(C.byref(d), stream(dev)), "rrin_head_fwd")
    torch.cuda.synchronize(dev)
