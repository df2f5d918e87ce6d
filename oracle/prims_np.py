"""ORACLE — test infrastructure only.  Closed-form numpy restatements of the
hot-path primitives, independent of PyTorch's kernels (float64):

* ``conv3x3``     — nn.Conv2d(k=3, pad=1) + bias (`unet.py:29,38,59,62,78`)
* ``avgpool2``    — F.avg_pool2d(x, 2) (`unet.py:46`)
* ``upsample2x``  — bilinear x2, align_corners=False: out[2i] = .75 in[i] + .25 in[i-1],
                    out[2i+1] = .75 in[i] + .25 in[i+1], edge clamp (`unet.py:77`)
* ``warp``        — grid_sample(bilinear, zeros, align_corners=False) of the
                    reference grid: samples at (x+u-0.5, y+v-0.5) (`model.py:8-21`)

Only tests may import this (see oracle/ref_net.py header).
"""
from __future__ import annotations

import numpy as np


def conv3x3(x, w, b, slope=None):
    n, cin, h, wd = x.shape
    xp = np.zeros((n, cin, h + 2, wd + 2), np.float64)
    xp[:, :, 1:-1, 1:-1] = x
    out = np.zeros((n, w.shape[0], h, wd), np.float64)
    for ky in range(3):
        for kx in range(3):
            patch = xp[:, :, ky:ky + h, kx:kx + wd]
            out += np.einsum("oc,nchw->nohw", w[:, :, ky, kx].astype(np.float64), patch)
    out += b.astype(np.float64)[None, :, None, None]
    if slope is not None:
        out = np.where(out >= 0, out, slope * out)
    return out


def avgpool2(x):
    n, c, h, w = x.shape
    return x.reshape(n, c, h // 2, 2, w // 2, 2).mean(axis=(3, 5))


def _up1d(a, axis):
    n = a.shape[axis]
    idx = np.arange(n)
    lo = np.take(a, np.maximum(idx - 1, 0), axis=axis)
    hi = np.take(a, np.minimum(idx + 1, n - 1), axis=axis)
    even = 0.75 * a + 0.25 * lo
    odd = 0.75 * a + 0.25 * hi
    shp = list(a.shape)
    shp[axis] = 2 * n
    out = np.empty(shp, np.float64)
    sl_e = [slice(None)] * a.ndim
    sl_o = [slice(None)] * a.ndim
    sl_e[axis] = slice(0, None, 2)
    sl_o[axis] = slice(1, None, 2)
    out[tuple(sl_e)] = even
    out[tuple(sl_o)] = odd
    return out


def upsample2x(x):
    return _up1d(_up1d(x.astype(np.float64), 2), 3)


def warp(img, flow):
    n, c, h, w = img.shape
    img = img.astype(np.float64)
    gy, gx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    sx = gx[None] + flow[:, 0].astype(np.float64) - 0.5
    sy = gy[None] + flow[:, 1].astype(np.float64) - 0.5
    x0 = np.floor(sx).astype(np.int64)
    y0 = np.floor(sy).astype(np.int64)
    fx = sx - x0
    fy = sy - y0
    out = np.zeros((n, c, h, w), np.float64)
    for dy, wy in ((0, 1 - fy), (1, fy)):
        for dx, wx in ((0, 1 - fx), (1, fx)):
            xi = x0 + dx
            yi = y0 + dy
            ok = (xi >= 0) & (xi < w) & (yi >= 0) & (yi < h)
            xc = np.clip(xi, 0, w - 1)
            yc = np.clip(yi, 0, h - 1)
            for bi in range(n):
                v = img[bi][:, yc[bi], xc[bi]]
                out[bi] += v * (wx[bi] * wy[bi] * ok[bi])[None]
    return out
