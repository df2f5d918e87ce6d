#!/usr/bin/env python3
"""Co-issue probe for v_mfma_f32_32x32x2_f32 (tools/coissue_probe.hip, built to
tools/coissue_probe.so): does another wave's VALU / LDS read / LDS-DMA issue
overlap an MFMA stream on the same SIMD, and how many own VALU ops fit between
a wave's MFMAs?  Prints T(mfma alone), T(other alone), T(both) per kind."""
import ctypes as C
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(REPO, "tools", "coissue_probe.so"))
lib.pair_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
lib.self_run.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_float)]


def pair(other, roles, im, io):
    ms = C.c_float()
    rc = lib.pair_run(other, roles, im, io, C.byref(ms))
    assert rc == 0, rc
    return ms.value


names = {1: "v_fma_f32", 2: "ds_read_b128", 3: "LDS-DMA 16B", 4: "wino chunk mix"}
IM = 1000  # 16k MFMAs per wave: 1.02 M cycles at 64 / MFMA
tm = pair(1, 1, IM, 0)
print(f"mfma alone ({IM * 16} per wave, 1 wave/SIMD): {tm:.3f} ms = {tm * 2.4e6 / (IM * 16):.1f} cyc/MFMA @2.4GHz",
      flush=True)
for other, ios in ((1, (1000, 4000, 8000)), (2, (250, 1000, 2000)), (3, (100, 400, 800)), (4, (500, 2000, 4000))):
    for io in ios:
        to = pair(other, 2, IM, io)
        tb = pair(other, 3, IM, io)
        print(f"{names[other]:>15} x{io:5d}: other alone {to:.3f}  mfma alone {tm:.3f}  both {tb:.3f}  "
              f"max {max(tm, to):.3f} sum {tm + to:.3f}  overlap {(tm + to - tb) / max(1e-9, min(tm, to)):.2f}",
              flush=True)
IT = 1000
for k in (0, 2, 4, 8, 12, 16, 24):
    ms = C.c_float()
    assert lib.self_run(k, IT, C.byref(ms)) == 0
    print(f"self: 1 MFMA + {k:2d} own v_fma_f32: {ms.value:.3f} ms = {ms.value * 2.4e6 / (IT * 16):.1f} cyc/MFMA",
          flush=True)
