#!/usr/bin/env python3
"""In-kernel clock of the register-U Winograd conv (MI355X_MICROARCH.md 'DVFS
give-back' item 6; cdna_hip_programming.md rule 28): a diagnostic build
(tools/build_wino_variant.sh clk "-DRRIN_WINOC_CLOCK=1" conv_winoc ->
ab/librrin_hip_clk.so) stamps s_memtime / s_memrealtime per workgroup.  Each shape
runs back to back for --seconds on random data, then the last launch's stamps give
the clock the chip held (median over workgroups, Δmemtime / Δmemrealtime x 100 MHz),
the share of a workgroup's time spent before the end of its main loop, and -- with
the launch time from HIP events -- the MFMA efficiency at the held clock:
Winograd TF/s / (clock x 256 CUs x 4 SIMDs x 64 FLOP per cycle).

  python3 tools/clock_probe.py --shapes 256:256:3:1,64:64:1:3 --batch 2
"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from rrin_amd import _lib  # noqa: E402
from rrin_amd.pp import H8Tensor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "ab", "librrin_hip_clk.so"))
    ap.add_argument("--shapes", default="256:256:3:1,128:64:1:1,64:64:1:3,512:512:4:1")
    ap.add_argument("--cfg", type=int, default=23)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--seconds", type=float, default=2.5)
    ap.add_argument("--kernel", default="winoc", choices=["winoc", "winoq"],
                    help="winoq: the kind-3 tile's phase stamps (ab/librrin_hip_qclk.so, RRIN_WINOQ_CLOCK=1): "
                         "chunk 0 landed / main loop done / stores done, and the start-time spread")
    a = ap.parse_args()
    if a.kernel == "winoq" and a.lib.endswith("librrin_hip_clk.so"):
        a.lib = os.path.join(REPO, "ab", "librrin_hip_qclk.so")
    from tests.test_gpu_h8 import pack_h8
    lib = C.CDLL(os.path.abspath(a.lib))
    lib.rrin_conv3x3_h8_fwd.argtypes = [C.POINTER(_lib.ConvH8Desc), C.c_void_p]
    lib.rrin_conv3x3_h8_fwd.restype = C.c_int
    rd = lib.rrin_winoq_clock_read if a.kernel == "winoq" else lib.rrin_winoc_clock_read
    rd.argtypes = [C.c_void_p, C.c_int]
    rd.restype = C.c_int
    nf = 6 if a.kernel == "winoq" else 4
    dev = torch.device("cuda:0")
    prec = _lib.PREC_F32R
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    print(f"{'shape':>24s} {'ms':>7s} {'TF(wino)':>8s} {'clock GHz':>9s} {'eff@clock':>9s} {'loop share':>10s} wgs")
    for spec in a.shapes.split(","):
        cin, cout, L, epi = (int(v) for v in spec.split(":")[:4])
        n, h, w = a.batch, a.height >> L, a.width >> L
        if epi == 4:
            h, w = h // 2, w // 2
        torch.manual_seed(0)
        x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
        whi, wlo, bp, inv = pack_h8(torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5), torch.randn(cout) * 0.1,
                                    a.cfg, prec, dev)
        dst = H8Tensor(n, cout // 4, 2 * h, 2 * w, dev, prec) if epi == 4 else H8Tensor(n, cout, h, w, dev, prec)
        pool = H8Tensor(n, cout, h // 2, w // 2, dev, prec) if epi == 2 else None
        d = _lib.ConvH8Desc()
        d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, a.cfg, prec, epi, 0.1, inv
        d.tail_finite = 1
        d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout // 4 if epi == 4 else cout)
        if pool is not None:
            d.pool = pool.view(0, cout)
        ring = None
        if epi == 4:
            ring = torch.zeros(n * (cout // 4) * (2 * (2 * w) + 2 * (2 * h - 2)), device=dev)
            d.edge = ring.data_ptr()
        d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
        bm, th = _lib.lib().rrin_conv_h8_cfg_bm(a.cfg), _lib.lib().rrin_conv_h8_cfg_th(a.cfg)
        wgs = ((cout + bm - 1) // bm) * ((w + 31) // 32) * ((h + th - 1) // th) * n
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))
        torch.cuda.synchronize()
        # back to back for a.seconds, timing the last 20 launches
        t_end = time.time() + a.seconds
        while time.time() < t_end:
            for _ in range(20):
                lib.rrin_conv3x3_h8_fwd(C.byref(d), st)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib.rrin_conv3x3_h8_fwd(C.byref(d), st)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 20
        k = min(wgs, 1 << 16)
        buf = np.zeros((k, nf), np.uint64)
        _lib.check(rd(buf.ctypes.data, k), "clock read")
        tf = 2 * 4 * cin * cout * h * w * n / (ms * 1e-3) / 1e12
        if a.kernel == "winoq":
            f = buf.astype(np.float64)
            ok = f[:, 3] > 0
            cyc = f[ok, 2]
            ghz = float(np.median(cyc / f[ok, 3])) * 0.1
            eff = tf / (ghz * 65.536)
            pro, loop, epl = np.median(f[ok, 0]), np.median(f[ok, 1] - f[ok, 0]), np.median(f[ok, 2] - f[ok, 1])
            life_us = np.median(f[ok, 3]) / 100.0
            t0 = f[ok, 4] - f[ok, 4].min()
            span_us = (f[ok, 5].max() - f[ok, 4].min()) / 100.0
            print(f"{cin:5d}->{cout:5d} L{L} epi{epi} n{n} {ms:7.4f} {tf:8.1f} {ghz:9.3f} {eff:9.3f} wgs {wgs} | "
                  f"wg life {life_us:6.2f} us: chunk0 {pro / (ghz * 1e3):5.2f} loop {loop / (ghz * 1e3):5.2f} "
                  f"epilogue+stores {epl / (ghz * 1e3):5.2f} us | launch span {span_us:7.1f} us, "
                  f"start p50/p90 {np.median(t0) / 100:6.1f}/{np.percentile(t0, 90) / 100:6.1f} us", flush=True)
            continue
        cyc, ticks, loop = buf[:, 0].astype(np.float64), buf[:, 1].astype(np.float64), buf[:, 2].astype(np.float64)
        ok = ticks > 0
        ghz = float(np.median(cyc[ok] / ticks[ok])) * 0.1
        share = float(np.median(loop[ok] / cyc[ok]))
        eff = tf / (ghz * 65.536)
        print(f"{cin:5d}->{cout:5d} L{L} epi{epi} n{n} {ms:7.4f} {tf:8.1f} {ghz:9.3f} {eff:9.3f} {share:10.3f} {wgs}",
              flush=True)


if __name__ == "__main__":
    main()
