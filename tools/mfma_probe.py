#!/usr/bin/env python3
"""Issue rate of v_mfma_f32_32x32x2_f32: one dependent chain vs K accumulators
(tools/mfma_probe.hip, built to tools/mfma_probe.so)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(REPO, "tools", "mfma_probe.so"))
lib.probe_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
iters = 2000
for waves in (4, 8):
    for k in (1, 2, 4, 8):
        ms = C.c_float()
        assert lib.probe_run(k, iters, waves, 256, C.byref(ms)) == 0
        mf = 256 * waves * iters * 16
        simd_cyc = ms.value * 1e-3 * 2.4e9  # at 2.4 GHz, per SIMD
        per = simd_cyc / (mf / 1024)        # cycles per MFMA per SIMD
        tf = mf * 4096 / (ms.value * 1e-3) / 1e12
        print(f"waves/block {waves} ({waves // 4}/SIMD) acc {k}: {ms.value:.3f} ms  {tf:.1f} TF  "
              f"{per:.1f} cyc/MFMA/SIMD @2.4GHz", flush=True)
