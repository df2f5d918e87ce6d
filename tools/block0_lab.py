#!/usr/bin/env python3
"""Time the fused level-0 UNetConvBlock (rrin_conv_block0_h8_fwd) against the two direct-form
launches it replaces, at fp16 on the Net's level-0 shapes (down_path[0]: cin -> 32 -> 32 + pool;
the last up block's conv_block: 64 -> 32 -> 32), one launch stream, HIP events around `reps`
back-to-back launches, median over `rounds`.

  python tools/block0_lab.py [--height 736 --width 1280 --n 2 --cins 16,64]

With RRIN_LIB_AB=ab/librrin_hip_X.so (tools/build_wino_variant.sh X -DRRIN_B0_ABL=... conv_block0)
the fused column times that build (ablations: outputs wrong by design)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from rrin_amd import _lib  # noqa: E402
from rrin_amd import engine as engine_mod  # noqa: E402
from rrin_amd.pp import H8Tensor  # noqa: E402

F16 = _lib.PREC_F16


def pack(w, b, cfg, dev):
    lib = _lib.lib()
    cout, cin = w.shape[:2]
    bm = lib.rrin_conv_h8_cfg_bm(cfg)
    whi = np.empty(lib.rrin_pack_conv3x3_h8_halves(cout, cin, bm), np.uint16)
    bp = np.empty(lib.rrin_pack_bias_floats(cout, bm), np.float32)
    inv = C.c_float()
    w, b = np.ascontiguousarray(w, np.float32), np.ascontiguousarray(b, np.float32)
    _lib.check(lib.rrin_pack_conv3x3_h8(w.ctypes.data, b.ctypes.data, cout, cin, bm, None, F16, whi.ctypes.data,
                                        None, bp.ctypes.data, C.byref(inv)))
    return torch.from_numpy(whi.view(np.int16)).to(dev), torch.from_numpy(bp).to(dev), inv.value


def timed(fn, reps, rounds, dev):
    out = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        out.append(e0.elapsed_time(e1) / reps)
    return float(np.median(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=736)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--cins", default="16,64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rng = np.random.default_rng(0)
    h, w, n = a.height, a.width, a.n
    for cin in [int(c) for c in a.cins.split(",")]:
        pool = cin != 64
        wa = (rng.standard_normal((32, cin, 3, 3)) / np.sqrt(9 * cin)).astype(np.float32)
        wb = (rng.standard_normal((32, 32, 3, 3)) / np.sqrt(9 * 32)).astype(np.float32)
        ba = (rng.standard_normal(32) * 0.1).astype(np.float32)
        bb = (rng.standard_normal(32) * 0.1).astype(np.float32)
        cfg_a = engine_mod.choose_cfg_h8(cin, 32, F16, 0, "large")
        cfg_b = engine_mod.choose_cfg_h8(32, 32, F16, 0, "large")
        pa, pb = pack(wa, ba, cfg_a, dev), pack(wb, bb, cfg_b, dev)
        src = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, F16)
        mid = H8Tensor(n, 32, h, w, dev, F16)
        dst = H8Tensor(n, 32, h, w, dev, F16)
        pl = H8Tensor(n, 32, h // 2, w // 2, dev, F16) if pool else None
        d = _lib.Block0Desc()
        d.n, d.cin, d.cfg_a, d.cfg_b, d.slope = n, cin, cfg_a, cfg_b, 0.1
        d.inv_wscale_a, d.inv_wscale_b, d.tail_finite = pa[2], pb[2], 1
        d.src, d.dst = src.chunk_view(0, cin), dst.view(0, 32)
        if pl is not None:
            d.pool = pl.view(0, 32)
        d.whi_a, d.bias_a, d.whi_b, d.bias_b = pa[0].data_ptr(), pa[1].data_ptr(), pb[0].data_ptr(), pb[1].data_ptr()

        def conv(cfg, p, s, o, ci, epi, poolv=None):
            e = _lib.ConvH8Desc()
            e.n, e.cin, e.cout, e.cfg, e.prec, e.epi_mode, e.slope, e.inv_wscale = n, ci, 32, cfg, F16, epi, 0.1, p[2]
            e.tail_finite = 1
            e.src, e.dst = s.chunk_view(0, ci), o.view(0, 32)
            if poolv is not None:
                e.pool = poolv.view(0, 32)
            e.whi, e.bias = p[0].data_ptr(), p[1].data_ptr()
            return e

        ea = conv(cfg_a, pa, src, mid, cin, _lib.EPI_LEAKY)
        eb = conv(cfg_b, pb, mid, dst, 32, _lib.EPI_LEAKY_POOL if pool else _lib.EPI_LEAKY, pl)
        fused = timed(lambda: _lib.check(lib.rrin_conv_block0_h8_fwd(C.byref(d), stream)), a.reps, a.rounds, dev)
        ta = timed(lambda: _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(ea), stream)), a.reps, a.rounds, dev)
        tb = timed(lambda: _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(eb), stream)), a.reps, a.rounds, dev)
        flops = 2.0 * 9 * (cin * 32 + 32 * 32) * h * w * n
        print(f"cin {cin:3d} {'pool' if pool else '    '} {n}x{h}x{w}: fused {fused * 1e3:7.1f} us "
              f"({flops / fused / 1e9:6.1f} TF)  conv a {ta * 1e3:6.1f} + conv b {tb * 1e3:6.1f} = "
              f"{(ta + tb) * 1e3:6.1f} us  ratio {fused / (ta + tb):.3f}", flush=True)


if __name__ == "__main__":
    main()
