"""Sub-pixel form of the up block (unet.py:77-78: bilinear x2 upsample, then a
3x3 conv) on the CPU: the phase-combined weights of ``rrin_subpixel_weights``
applied to the edge-replicated low-res input, pixel-shuffled, plus the ring
correction that ``edge_fix_h8_kernel`` applies, must equal
conv2d(upsample(x)) with zero padding.  Pure host code, no GPU."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import _lib


def subpixel_weights(w, b):
    cout, cin = w.shape[:2]
    ws = np.zeros((4 * cout, cin, 3, 3), np.float32)
    bs = np.zeros(4 * cout, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    rc = _lib.lib().rrin_subpixel_weights(w.ctypes.data, b.ctypes.data, cout, cin, ws.ctypes.data, bs.ctypes.data)
    assert rc == 0
    return ws, bs


def ring(h, w):
    """Ring pixels in rrin_ring_pixels order."""
    pts = [(0, x) for x in range(w)] + [(h - 1, x) for x in range(w)]
    pts += [(y, 0) for y in range(1, h - 1)] + [(y, w - 1) for y in range(1, h - 1)]
    return pts


def subpixel_forward(x, w, b):
    """Restatement of the GPU path in float64: EPI_SUBPIXEL conv + ring fix-up."""
    cout = w.shape[0]
    ws, bs = subpixel_weights(w, b)
    xr = F.pad(x, (1, 1, 1, 1), mode="replicate")
    n, _, sh, sw = x.shape
    out = torch.zeros(n, cout, 2 * sh, 2 * sw, dtype=torch.float64)
    for ph in range(4):
        py, px = ph >> 1, ph & 1
        rows = [(co // 8) * 32 + ph * 8 + co % 8 for co in range(cout)]
        y = F.conv2d(xr, torch.from_numpy(ws[rows]).double(), torch.from_numpy(bs[rows]).double())
        out[:, :, py::2, px::2] = y
    up = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    H, W = 2 * sh, 2 * sw
    wt = torch.from_numpy(w).double()
    for (Y, X) in ring(H, W):
        for t in range(9):
            yy, xx = Y + t // 3 - 1, X + t % 3 - 1
            if 0 <= yy < H and 0 <= xx < W:
                continue
            u = up[:, :, min(max(yy, 0), H - 1), min(max(xx, 0), W - 1)]   # [n, cin]
            out[:, :, Y, X] -= u @ wt[:, :, t // 3, t % 3].T
    return out


@pytest.mark.parametrize("cin,cout,sh,sw", [(3, 8, 5, 7), (16, 16, 4, 4), (8, 24, 2, 3), (5, 8, 1, 1)])
def test_subpixel_equals_upsample_conv(cin, cout, sh, sw):
    g = torch.Generator().manual_seed(cin * 100 + sh)
    x = torch.randn(2, cin, sh, sw, generator=g, dtype=torch.float64)
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.2).numpy()
    b = (torch.randn(cout, generator=g) * 0.1).numpy()
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False),
                   torch.from_numpy(w).double(), torch.from_numpy(b).double(), padding=1)
    got = subpixel_forward(x, w, b)
    # weights rounded to fp32 once (computed in double): ~1e-7 relative
    assert (got - ref).abs().max().item() < 2e-6


def test_subpixel_weights_phase_sums():
    """Each phase's weights sum (over taps) to the original tap sum: bilinear
    weights are a partition of unity."""
    w = np.random.default_rng(0).standard_normal((16, 4, 3, 3)).astype(np.float32)
    ws, bs = subpixel_weights(w, np.arange(16, dtype=np.float32))
    for co in range(16):
        for ph in range(4):
            r = (co // 8) * 32 + ph * 8 + co % 8
            np.testing.assert_allclose(ws[r].sum(axis=(1, 2)), w[co].sum(axis=(1, 2)), rtol=1e-5, atol=1e-5)
            assert bs[r] == co


def test_ring_pixels_count():
    L = _lib.lib()
    for h, w in [(2, 2), (4, 6), (90, 160), (720, 1280)]:
        assert L.rrin_ring_pixels(h, w) == len(ring(h, w)) == 2 * w + 2 * (h - 2)
    assert L.rrin_subpixel_weights(None, None, 8, 1, None, None) != 0
    w = np.zeros((12, 1, 3, 3), np.float32)
    assert L.rrin_subpixel_weights(w.ctypes.data, w.ctypes.data, 12, 1, w.ctypes.data, w.ctypes.data) != 0  # cout % 8
