#!/usr/bin/env python3
"""SIMD-time price of each instruction kind beside a v_mfma_f32_32x32x2_f32 stream
(tools/coissue_probe2.hip -> tools/coissue_probe2.so).  For each kind: T(mfma alone),
T(other alone), T(both); the extra cycles per instruction = (T(both) - T(mfma alone))
x 2.4 GHz / instructions per wave."""
import ctypes as C
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(REPO, "tools", "coissue_probe2.so"))
lib.run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
lib.self_run.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
NAMES = {1: "v_fma_f32", 2: "v_mov_b32", 3: "ds_read_b32", 4: "ds_read_b64", 5: "ds_read_b128",
         6: "ds_write_b128", 7: "global_load_dwordx4", 8: "LDS-DMA 16B", 9: "s_add_u32", 10: "s_nop 0"}


def run(kind, accv, roles, im, io):
    ms = C.c_float()
    rc = lib.run(kind, accv, roles, im, io, C.byref(ms))
    assert rc == 0, rc
    return ms.value


IM = 1000
for accv in (0, 1):
    tm = run(1, accv, 1, IM, 0)
    print(f"acc in {'VGPR' if accv else 'AGPR'}: mfma alone {tm:.3f} ms = {tm * 2.4e6 / (IM * 16):.1f} cyc/MFMA",
          flush=True)
    for kind in range(1, 11):
        for io in (250, 1000):
            to = run(kind, accv, 2, IM, io)
            tb = run(kind, accv, 3, IM, io)
            n = io * 16
            print(f"  {NAMES[kind]:>20} x{n:6d} ({n / (IM * 16):.2f}/MFMA): alone {to:.3f}  both {tb:.3f}  "
                  f"extra {max(0.0, tb - tm) * 2.4e6 / n:6.1f} cyc/instr  (alone {to * 2.4e6 / n:6.1f})",
                  flush=True)
for kind, ns in ((1, (0, 1, 2, 4)), (5, (1, 2, 4)), (8, (1, 2))):
    for n in ns:
        ms = C.c_float()
        assert lib.self_run(kind, n, IM, C.byref(ms)) == 0
        cyc = ms.value * 2.4e6 / (IM * 16)
        print(f"self: MFMA + {n} own {NAMES[kind]}: {cyc:.1f} cyc per MFMA", flush=True)
