#!/usr/bin/env python3
"""Conv kernel lab (GPU).

  python tools/conv_lab.py breakdown [--batch 4 --height 720 --width 1280]
      per-launch time / TFLOP/s of one Net.forward in schedule order (HIP events)
  python tools/conv_lab.py tune [--batch 4 ...] [--out gpurun_out/tune.json]
      every tile config on every distinct conv shape of the Net; best per shape
  python tools/conv_lab.py ablate [--reps 7]
      split16 conv schedule variants and ablations (librrin_lab.so, `make lab`):
      interleaved rounds in one process, median per variant; the schedule
      variants are checked bitwise against the product kernel
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rrin_amd import Net, _lib  # noqa: E402
from rrin_amd.pp import PPTensor  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402

UNETS = [("Flow", 6, 5), ("refine_flow", 10, 4), ("Mask", 16, 4), ("final", 9, 4)]


def schedule(h, w, h8=False, sub_max_level=2):
    """(unet, tag, cin, cout, level, src_mode, epi) in rrin_net_fwd launch order.
    h8 (split/fp16 path): an up conv at level <= sub_max_level is a sub-pixel
    conv on the low-res input (src 2, epi 4, cout = real channels) followed by
    its ring fix-up, and its producer writes edge-replicated (epi 3); other up
    convs follow an explicit upsample pass."""
    out = [("-", "pack", 0, 0, 0, -1, -1)]
    for name, cin0, D in UNETS:
        sub = [h8 and L <= sub_max_level for L in range(D)]
        for L in range(D):
            C_ = 32 << L
            cin = (32 << (L - 1)) if L else cin0
            out.append((name, f"down{L}.a", cin, C_, L, 0, 1))
            if L < D - 1:
                out.append((name, f"down{L}.b", C_, C_, L, 0, 2))
            else:
                out.append((name, f"down{L}.b", C_, C_, L, 0, 1))
                out.append((name, "mid", C_, C_, L, 0, 3 if sub[D - 2] else 1))
        for L in range(D - 2, -1, -1):
            C_ = 32 << L
            if sub[L]:
                out.append((name, f"up{L}.sub", 2 * C_, C_, L, 2, 4))
                out.append((name, f"up{L}.ring", 0, 0, L, -3, -3))
            else:
                if h8:
                    out.append((name, f"up{L}.ups", 0, 0, L, -1, -1))
                out.append((name, f"up{L}.up", 2 * C_, C_, L, 0 if h8 else 1, 0))
            out.append((name, f"up{L}.a", 2 * C_, C_, L, 0, 1))
            out.append((name, f"up{L}.b", C_, C_, L, 0, 3 if (L > 0 and sub[L - 1]) else 1))
        out.append((name, "head", 32, 0, 0, -2, -2))
    return out


def breakdown(args):
    dev = torch.device("cuda:0")
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()))
    net = net.to(dev).eval()
    net.precision = args.precision
    eng = net.engine()
    if args.first_cfg is not None:
        # the first conv of each U-Net is entry 0 of its block of the table; a config
        # with the same BM shares the weight packing, so it can be swapped in place
        k = 0
        for name, _, D in UNETS:
            e = eng.conv_table[k]
            if _lib.lib().rrin_conv_h8_cfg_bm(e.cfg) == _lib.lib().rrin_conv_h8_cfg_bm(args.first_cfg):
                e.cfg = args.first_cfg
                eng.cfgs[k] = args.first_cfg
            k += 2 * D + 1 + 3 * (D - 1)
    lib = _lib.lib()
    i0, i1 = synthetic_batch(args.batch, args.height, args.width)
    i0, i1 = i0.to(dev), i1.to(dev)
    with torch.no_grad():
        for _ in range(2):
            eng.forward(i0, i1)
    torch.cuda.synchronize()
    cap = 128
    h = C.c_void_p()
    _lib.check(lib.rrin_prof_create(cap, C.byref(h)))
    reps = args.reps
    tot = {}
    for r in range(reps):
        lib.rrin_prof_reset(h)
        with torch.no_grad():
            eng.forward(i0, i1, prof=h.value)
        torch.cuda.synchronize()
        kinds = (C.c_int32 * cap)()
        ms = (C.c_float * cap)()
        fl = (C.c_double * cap)()
        cnt = C.c_int32()
        _lib.check(lib.rrin_prof_read(h, kinds, ms, fl, cap, C.byref(cnt)))
        for i in range(cnt.value):
            tot.setdefault(i, []).append((kinds[i], ms[i], fl[i]))
    lib.rrin_prof_destroy(h)
    sch = schedule(args.height, args.width, args.precision != "fp32_planar", net.subpixel_max_level)
    rows = []
    conv_i = 0
    for i, entry in enumerate(sch):
        vals = sorted(tot[i], key=lambda v: v[1])
        k, ms_, fl_ = vals[len(vals) // 2]
        cfg = None
        if entry[5] >= 0:
            cfg = eng.cfgs[conv_i]
            conv_i += 1
        rows.append(dict(unet=entry[0], tag=entry[1], cin=entry[2], cout=entry[3], level=entry[4],
                         src=entry[5], epi=entry[6], cfg=cfg, ms=ms_, tflops=fl_ / (ms_ * 1e-3) / 1e12 if ms_ else 0))
    total = sum(r["ms"] for r in rows)
    for r in rows:
        print(f"{r['unet']:12s} {r['tag']:10s} {r['cin']:4d}->{r['cout']:4d} L{r['level']} src{r['src']:2d} "
              f"epi{r['epi']:2d} cfg {str(r['cfg']):4s} {r['ms']:8.3f} ms {r['tflops']:7.1f} TF "
              f"{100 * r['ms'] / total:5.1f}%")
    print(f"total {total:.3f} ms per forward (B={args.batch})")
    agg = {}
    for r in rows:
        key = f"L{r['level']} src{r['src']} epi{r['epi']}"
        a = agg.setdefault(key, [0.0, 0.0])
        a[0] += r["ms"]
        a[1] += r["tflops"] * r["ms"]
    for k, (m, tw) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:20s} {m:8.3f} ms  {tw / m if m else 0:6.1f} TF")
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


def tune_h8(args):
    from rrin_amd.pp import H8Tensor
    from tests.test_gpu_h8 import pack_h8
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    prec = _lib.PRECISIONS[args.precision]
    shapes = sorted({(e[2], e[3], e[4], e[5], e[6]) for e in schedule(args.height, args.width, True) if e[5] >= 0})
    n = args.batch
    results = []
    for cin, cout, L, src, epi in shapes:
        h, w = args.height >> L, args.width >> L
        kout = 4 * cout if epi == 4 else cout          # sub-pixel: 4 phase rows per channel, low-res grid
        hs, ws_ = (h // 2, w // 2) if epi == 4 else (h, w)
        x = H8Tensor.from_nchw(torch.rand(n, cin, hs, ws_, device=dev) * 2 - 1, prec)
        dst = H8Tensor(n, cout, h, w, dev, prec)
        pool = H8Tensor(n, cout, h // 2, w // 2, dev, prec) if epi == 2 else None
        edge = torch.zeros(n, cout, lib.rrin_ring_pixels(h, w), device=dev) if epi == 4 else None
        wt = torch.randn(kout, cin, 3, 3) / (3 * cin ** 0.5)
        b = torch.zeros(kout)
        best, line = None, []
        for cfg in range(lib.rrin_conv_h8_cfg_count()):
            if not lib.rrin_conv_h8_cfg_fits(cfg, prec, cin) or lib.rrin_conv_h8_cfg_bm(cfg) > max(32, 2 * kout):
                continue
            whi, wlo, bp, inv = pack_h8(wt, b, cfg, prec, dev)
            d = _lib.ConvH8Desc()
            d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, kout, cfg, prec, epi, 0.1, inv
            d.tail_finite = 1  # channels past cin are zero (as the Net's g16 buffer): whole-record staging
            d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout)
            if edge is not None:
                d.edge = edge.data_ptr()
            if pool is not None:
                d.pool = pool.view(0, cout)
            d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            if lib.rrin_conv3x3_h8_fwd(C.byref(d), st) != 0:
                continue
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            tf = 2 * 9 * cin * cout * h * w * n / (ms * 1e-3) / 1e12
            line.append(f"cfg{cfg}:{ms:.3f}ms/{tf:.0f}TF")
            results.append(dict(cin=cin, cout=cout, level=L, src=src, epi=epi, cfg=cfg, ms=ms, tflops=tf))
            if best is None or ms < best[1]:
                best = (cfg, ms, tf)
        print(f"{cin:4d}->{cout:4d} L{L} epi{epi}: best cfg{best[0]} {best[2]:.0f} TF | " + " ".join(line), flush=True)
    if args.out:
        json.dump(results, open(args.out, "w"), indent=1)


def tune(args):
    if args.precision != "fp32_planar":
        return tune_h8(args)
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    ncfg = lib.rrin_conv_cfg_count()
    shapes = sorted({(e[2], e[3], e[4], e[5], e[6]) for e in schedule(args.height, args.width) if e[5] >= 0})
    n = args.batch
    results = []
    for cin, cout, L, src, epi in shapes:
        h, w = args.height >> L, args.width >> L
        hs, ws_ = (h // 2, w // 2) if src == 1 else (h, w)
        x = PPTensor.from_nchw(torch.rand(n, cin, hs, ws_, device=dev) * 2 - 1)
        dst = PPTensor(n, cout, h, w, dev)
        pool = PPTensor(n, cout, h // 2, w // 2, dev) if epi == 2 else None
        wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
        b = torch.zeros(cout)
        best = None
        line = []
        for cfg in range(ncfg):
            bm = lib.rrin_conv_cfg_bm(cfg)
            if bm > max(32, 2 * cout):
                continue
            from tests.hip_helpers import pack
            wp, bp = pack(wt, b, cfg, dev=dev)
            d = _lib.ConvDesc()
            d.n, d.cin, d.cout, d.cfg, d.src_mode, d.epi_mode, d.slope = n, cin, cout, cfg, src, epi, 0.1
            d.src, d.dst = x.view(0, cin), dst.view(0, cout)
            if pool is not None:
                d.pool = pool.view(0, cout)
            d.wpack, d.bias = wp.data_ptr(), bp.data_ptr()
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            for _ in range(2):
                _lib.check(lib.rrin_conv3x3_fwd(C.byref(d), st))
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(lib.rrin_conv3x3_fwd(C.byref(d), st))
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            fl = 2 * 9 * cin * cout * h * w * n
            tf = fl / (ms * 1e-3) / 1e12
            line.append(f"cfg{cfg}:{ms:.3f}ms/{tf:.0f}TF")
            results.append(dict(cin=cin, cout=cout, level=L, src=src, epi=epi, cfg=cfg, ms=ms, tflops=tf))
            if best is None or ms < best[1]:
                best = (cfg, ms, tf)
        print(f"{cin:4d}->{cout:4d} L{L} src{src} epi{epi}: best cfg{best[0]} {best[2]:.0f} TF | " + " ".join(line),
              flush=True)
    if args.out:
        json.dump(results, open(args.out, "w"), indent=1)


def single(args):
    """Run one conv shape/config --reps times (for rocprofv3 --pmc)."""
    from rrin_amd.pp import H8Tensor
    from tests.test_gpu_h8 import pack_h8
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    prec = _lib.PRECISIONS[args.precision]
    cin, cout, L, epi, cfg = args.shape
    n, h, w = args.batch, args.height >> L, args.width >> L
    if args.precision == "fp32_planar":  # exact-fp32 PP conv; --src 1 = fused upsample of a half-size input
        from tests.hip_helpers import pack
        src = args.src
        hs, ws_ = (h // 2, w // 2) if src == 1 else (h, w)
        x = PPTensor.from_nchw(torch.rand(n, cin, hs, ws_, device=dev) * 2 - 1)
        dst = PPTensor(n, cout, h, w, dev)
        pool = PPTensor(n, cout, h // 2, w // 2, dev) if epi == 2 else None
        wp, bp = pack(torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5), torch.zeros(cout), cfg, dev=dev)
        d = _lib.ConvDesc()
        d.n, d.cin, d.cout, d.cfg, d.src_mode, d.epi_mode, d.slope = n, cin, cout, cfg, src, epi, 0.1
        d.src, d.dst = x.view(0, cin), dst.view(0, cout)
        if pool is not None:
            d.pool = pool.view(0, cout)
        d.wpack, d.bias = wp.data_ptr(), bp.data_ptr()
        if args.sched is None:
            fwd = lambda st: _lib.check(lib.rrin_conv3x3_fwd(C.byref(d), st))  # noqa: E731
        else:  # lab build with ablation bits (librrin_lab32.so)
            lab = C.CDLL(os.path.join(REPO, "rrin_amd", "librrin_lab32.so"))
            lab.rrin_conv3x3_lab32.argtypes = [C.POINTER(_lib.ConvDesc), C.c_int32, C.c_void_p]
            fwd = lambda st: _lib.check(lab.rrin_conv3x3_lab32(C.byref(d), args.sched, st))  # noqa: E731
    else:
        fwd = None
    if fwd is not None:
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fwd(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fwd(st)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(f"{cin}->{cout} L{L} src{args.src} epi{epi} cfg{cfg} fp32_planar: {ms:.4f} ms "
              f"{2 * 9 * cin * cout * h * w * n / (ms * 1e-3) / 1e12:.1f} TF")
        return
    x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
    dst = H8Tensor(n, cout, h, w, dev, prec)
    pool = H8Tensor(n, cout, h // 2, w // 2, dev, prec) if epi == 2 else None
    wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
    whi, wlo, bp, inv = pack_h8(wt, torch.zeros(cout), cfg, prec, dev)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, prec, epi, 0.1, inv
    d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout)
    if pool is not None:
        d.pool = pool.view(0, cout)
    d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if args.sched is not None:  # lab build: schedule / ablation bits, persistent grid factor
        lab = C.CDLL(os.path.join(REPO, "rrin_amd", "librrin_lab.so"))
        lab.rrin_conv3x3_h8_lab.argtypes = [C.POINTER(_lib.ConvH8Desc), C.c_int32, C.c_int32, C.c_void_p]
        run = lambda: _lib.check(lab.rrin_conv3x3_h8_lab(C.byref(d), args.sched, args.persist, st))  # noqa: E731
    else:
        run = lambda: _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))  # noqa: E731
    run()
    if args.sched is not None and args.check:  # lab variant vs the product kernel, bitwise
        ref = H8Tensor(n, cout, h, w, dev, prec)
        d2 = _lib.ConvH8Desc.from_buffer_copy(d)
        d2.dst = ref.view(0, cout)
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d2), st))
        torch.cuda.synchronize()
        same = torch.equal(dst.to_nchw(), ref.to_nchw())
        print(f"check sched {args.sched} vs product: {'bitwise equal' if same else 'DIFFERENT'}")
        if not same:
            sys.exit(3)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        run()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    print(f"{cin}->{cout} L{L} epi{epi} cfg{cfg} {args.precision}: {ms:.4f} ms "
          f"{2 * 9 * cin * cout * h * w * n / (ms * 1e-3) / 1e12:.1f} TF")


# (name, SCHED_* knobs of conv_f16.hip, persistent grid) -- the lab build's variants
LAB_VARIANTS = [("base", 0, 0), ("persist", 0, 1), ("spread", 16, 0), ("persist+spread", 16, 1),
                ("stagger", 64, 0), ("persist+stagger", 64, 1), ("wres", 32, 0), ("persist+wres", 32, 1),
                ("persist+wres+spread", 48, 1), ("persist+wres+stagger", 96, 1),
                ("mfma16", 128, 0), ("spread+mfma16", 144, 0), ("persist+spread+mfma16", 144, 1),
                ("noW", 1, 0), ("noIn", 2, 0), ("noLoads", 3, 0), ("noMfma", 4, 0), ("ldsOnly", 7, 0),
                ("noEpi", 8, 0)]
LAB_SHAPES = [(32, 32, 0, 6), (64, 32, 0, 6), (64, 32, 0, 1), (64, 64, 1, 0), (128, 64, 1, 0), (128, 128, 2, 0),
              (256, 128, 2, 0), (256, 256, 3, 0), (512, 256, 3, 0), (512, 512, 4, 0)]


# fp32 records (--precision fp32): the tuned config of each shape (engine.H8_TUNED)
LAB_SHAPES_R32 = [(32, 32, 0, 6), (64, 32, 0, 1), (64, 64, 1, 1), (128, 64, 1, 4), (128, 128, 2, 5),
                  (256, 128, 2, 5), (256, 256, 3, 3), (512, 512, 4, 16)]
LAB_VARIANTS_R32 = [("base", 0, 0), ("persist", 0, 1), ("spread", 16, 0), ("persist+spread", 16, 1),
                    ("noW", 1, 0), ("noIn", 2, 0), ("noLoads", 3, 0), ("noMfma", 4, 0), ("noEpi", 8, 0),
                    ("noLoads+noEpi", 11, 0), ("persist+noLoads+noEpi", 11, 1)]


def ablate(args):
    from rrin_amd.pp import H8Tensor
    from tests.test_gpu_h8 import pack_h8
    lab = C.CDLL(os.path.join(REPO, "rrin_amd", "librrin_lab.so"))
    fn = lab.rrin_conv3x3_h8_lab
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(_lib.ConvH8Desc), C.c_int32, C.c_int32, C.c_void_p]
    lib = _lib.lib()
    dev = torch.device("cuda:0")
    r32 = args.precision == "fp32"
    prec = _lib.PREC_F32R if r32 else _lib.PREC_F16X3
    variants = LAB_VARIANTS_R32 if r32 else LAB_VARIANTS
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    results = []
    for cin, cout, L, cfg in (LAB_SHAPES_R32 if r32 else LAB_SHAPES):
        n, h, w = args.batch, args.height >> L, args.width >> L
        torch.manual_seed(cin * 1000 + cout)
        x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
        dst = H8Tensor(n, cout, h, w, dev, prec)
        wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
        whi, wlo, bp, inv = pack_h8(wt, torch.randn(cout) * 0.1, cfg, prec, dev)
        d = _lib.ConvH8Desc()
        d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = (n, cin, cout, cfg, prec,
                                                                                _lib.EPI_LEAKY, 0.1, inv)
        d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout)
        d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
        _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))
        torch.cuda.synchronize()
        ref = (dst.hi.clone(), dst.lo.clone() if dst.lo is not None else None)
        fl = 2 * 9 * cin * cout * h * w * n
        ok, times = {}, {}
        for name, sched, pers in variants:
            dst.hi.zero_()
            if dst.lo is not None:
                dst.lo.zero_()
            rc = fn(C.byref(d), sched, pers, st)
            torch.cuda.synchronize()
            if rc != 0:
                ok[name] = f"rc{rc}"
                continue
            if sched & 143 == 0:
                same = torch.equal(dst.hi, ref[0]) and (dst.lo is None or torch.equal(dst.lo, ref[1]))
                ok[name] = "ok" if same else "MISMATCH"
            times[name] = []
        for _ in range(args.reps):  # interleaved rounds (guide rule 24)
            for name, sched, pers in variants:
                if name not in times:
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    fn(C.byref(d), sched, pers, st)
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / 3)
        base = sorted(times["base"])[len(times["base"]) // 2]
        line = []
        for name, sched, pers in variants:
            if name not in times:
                line.append(f"{name}:{ok.get(name)}")
                continue
            ms = sorted(times[name])[len(times[name]) // 2]
            results.append(dict(cin=cin, cout=cout, level=L, cfg=cfg, variant=name, sched=sched, persist=pers, ms=ms,
                                tflops=fl / (ms * 1e-3) / 1e12, check=ok.get(name, "-")))
            tag = "" if ok.get(name, "ok") == "ok" else "(" + ok[name] + ")"
            line.append(f"{name}:{ms:.3f}({ms / base:.2f}){tag}")
        print(f"{cin:4d}->{cout:4d} L{L} cfg{cfg} base {base:.3f} ms {fl / (base * 1e-3) / 1e12:.0f} TF | "
              + " ".join(line), flush=True)
    if args.out:
        json.dump(results, open(args.out, "w"), indent=1)


LAB32_VARIANTS = [("base", 0), ("noDma", 1), ("noMfma", 2), ("noDma+noMfma", 3), ("noEpi", 4), ("noSync", 8),
                  ("noDma+noSync", 9), ("noEpi+noSync", 12), ("noDma+noEpi+noSync", 13)]
LAB32_SHAPES = [(32, 32, 0, 0), (64, 64, 1, 4), (128, 64, 1, 4), (128, 128, 2, 1), (256, 256, 3, 4), (512, 256, 3, 5),
                (512, 512, 4, 4)]


def ablate32(args):
    """Exact-fp32 conv ablations (librrin_lab32.so): interleaved rounds, median per variant."""
    from tests.hip_helpers import pack
    lab = C.CDLL(os.path.join(REPO, "rrin_amd", "librrin_lab32.so"))
    fn = lab.rrin_conv3x3_lab32
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(_lib.ConvDesc), C.c_int32, C.c_void_p]
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    results = []
    for cin, cout, L, cfg in LAB32_SHAPES:
        n, h, w = args.batch, args.height >> L, args.width >> L
        torch.manual_seed(cin * 1000 + cout)
        x = PPTensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1)
        dst = PPTensor(n, cout, h, w, dev)
        wp, bp = pack(torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5), torch.randn(cout) * 0.1, cfg, dev=dev)
        d = _lib.ConvDesc()
        d.n, d.cin, d.cout, d.cfg, d.src_mode, d.epi_mode, d.slope = n, cin, cout, cfg, 0, _lib.EPI_LEAKY, 0.1
        d.src, d.dst = x.view(0, cin), dst.view(0, cout)
        d.wpack, d.bias = wp.data_ptr(), bp.data_ptr()
        fl = 2 * 9 * cin * cout * h * w * n
        times = {name: [] for name, _ in LAB32_VARIANTS}
        for name, sched in LAB32_VARIANTS:
            _lib.check(fn(C.byref(d), sched, st), f"lab32 {name}")
        torch.cuda.synchronize()
        for _ in range(args.reps):
            for name, sched in LAB32_VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    fn(C.byref(d), sched, st)
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / 3)
        base = sorted(times["base"])[len(times["base"]) // 2]
        line = []
        for name, sched in LAB32_VARIANTS:
            ms = sorted(times[name])[len(times[name]) // 2]
            results.append(dict(cin=cin, cout=cout, level=L, cfg=cfg, variant=name, ms=ms,
                                tflops=fl / (ms * 1e-3) / 1e12))
            line.append(f"{name}:{ms:.3f}({ms / base:.2f})")
        print(f"{cin:4d}->{cout:4d} L{L} cfg{cfg} base {base:.3f} ms {fl / (base * 1e-3) / 1e12:.0f} TF | "
              + " ".join(line), flush=True)
    if args.out:
        json.dump(results, open(args.out, "w"), indent=1)


def abconv(args):
    """A/B of the record-layout conv of two library builds (--lib vs --lib-b) on
    the shapes of --shapes (cin:cout:level:epi:cfg,...), interleaved rounds in one
    process, outputs compared bitwise; median ms per build."""
    from rrin_amd.pp import H8Tensor
    from tests.test_gpu_h8 import pack_h8
    dev = torch.device("cuda:0")
    paths = [args.lib or _lib.LIB_PATH] + args.lib_b.split(",")
    libs = [C.CDLL(os.path.abspath(p)) for p in paths]
    for L_ in libs:
        L_.rrin_conv3x3_h8_fwd.argtypes = [C.POINTER(_lib.ConvH8Desc), C.c_void_p]
        L_.rrin_conv3x3_h8_fwd.restype = C.c_int
    prec = _lib.PRECISIONS[args.precision]
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    bad = 0
    for spec in args.shapes.split(","):
        cin, cout, L, epi, cfg = (int(v) for v in spec.split(":"))
        n, h, w = args.batch, args.height >> L, args.width >> L
        if epi == 4:  # sub-pixel: the conv runs on the low-res grid, 4 x cout phase rows
            h, w = h // 2, w // 2
        torch.manual_seed(0)
        x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
        wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
        whi, wlo, bp, inv = pack_h8(wt, torch.randn(cout) * 0.1, cfg, prec, dev)
        outs, descs, keep = [], [], []
        for _ in libs:
            if epi == 4:
                dst = H8Tensor(n, cout // 4, 2 * h, 2 * w, dev, prec)
            else:
                dst = H8Tensor(n, cout, h, w, dev, prec)
            pool = H8Tensor(n, cout, h // 2, w // 2, dev, prec) if epi == 2 else None
            d = _lib.ConvH8Desc()
            d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, prec, epi, 0.1, inv
            d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout // 4 if epi == 4 else cout)
            if pool is not None:
                d.pool = pool.view(0, cout)
            if epi == 4:
                ring = torch.zeros(n * (cout // 4) * (2 * (2 * w) + 2 * (2 * h - 2)), device=dev)
                d.edge = ring.data_ptr()
                keep.append(ring)
            d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
            outs.append((dst, pool))
            descs.append(d)
        times = [[] for _ in libs]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i, L_ in enumerate(libs):
            _lib.check(L_.rrin_conv3x3_h8_fwd(C.byref(descs[i]), st))
        torch.cuda.synchronize()
        same = True
        for k in range(1, len(libs)):
            same = same and torch.equal(outs[0][0].to_nchw(), outs[k][0].to_nchw())
            if epi == 2:
                same = same and torch.equal(outs[0][1].to_nchw(), outs[k][1].to_nchw())
            if epi == 4:
                same = same and torch.equal(keep[0], keep[k])
        for _ in range(args.rounds):
            for i, L_ in enumerate(libs):
                e0.record()
                for _ in range(args.reps):
                    L_.rrin_conv3x3_h8_fwd(C.byref(descs[i]), st)
                e1.record()
                e1.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.reps)
        med = [sorted(t)[len(t) // 2] for t in times]
        wf = 2 * 4 * cin * cout * h * w * n  # Winograd work (4/9 of direct)
        rel = "  ".join(f"{chr(66 + k)} {med[k + 1]:.4f} ({med[k + 1] / med[0]:.3f})" for k in range(len(libs) - 1))
        print(f"{cin:4d}->{cout:4d} L{L} epi{epi} cfg{cfg} n{n}: A {med[0]:.4f} ms  {rel}  "
              f"best {wf / (min(med) * 1e-3) / 1e12:.1f} TF(wino)  {'bitwise equal' if same else 'DIFFERENT'}",
              flush=True)
        bad += 0 if same else 1
    if bad and args.check:
        sys.exit(3)


def cfgab(args):
    """Tile configs of the product library on the same conv (each with its own
    packing), interleaved timing, medians relative to the first.  --cfgs A,B[,C...];
    a variant "21s4" runs config 21 with a split-K of 4 slices (kinds 3, 4).
    Variants without a split are compared bitwise with the first unsplit one; split
    variants report their max-abs difference (a split rounds differently).  Shapes
    as abconv without the cfg field: cin:cout:level:epi."""
    from rrin_amd.pp import H8Tensor
    from tests.test_gpu_h8 import pack_h8, set_split
    dev = torch.device("cuda:0")
    L_ = _lib.lib()
    prec = _lib.PRECISIONS[args.precision]
    variants = []
    for v in args.cfgs.split(","):
        c, _, k = v.partition("s")
        variants.append((int(c), int(k) if k else 0))
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    bad = 0
    for spec in args.shapes.split(","):
        cin, cout, L, epi = (int(v) for v in spec.split(":")[:4])
        n, h, w = args.batch, args.height >> L, args.width >> L
        if epi == 4:
            h, w = h // 2, w // 2
        torch.manual_seed(0)
        x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
        wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
        bias = torch.randn(cout) * 0.1
        outs, descs, keep, ok = [], [], [], []
        for cfg, ks in variants:
            if not L_.rrin_conv_h8_cfg_fits(cfg, prec, cin):
                ok.append(False)
                outs.append(None)
                descs.append(None)
                continue
            whi, wlo, bp, inv = pack_h8(wt, bias, cfg, prec, dev)
            dst = H8Tensor(n, cout // 4, 2 * h, 2 * w, dev, prec) if epi == 4 else H8Tensor(n, cout, h, w, dev, prec)
            pool = H8Tensor(n, cout, h // 2, w // 2, dev, prec) if epi == 2 else None
            d = _lib.ConvH8Desc()
            d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, prec, epi, 0.1, inv
            d.tail_finite = 1  # channels past cin are zero (as the Net's g16 buffer)
            d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout // 4 if epi == 4 else cout)
            if pool is not None:
                d.pool = pool.view(0, cout)
            ring = None
            if epi == 4:
                ring = torch.zeros(n * (cout // 4) * (2 * (2 * w) + 2 * (2 * h - 2)), device=dev)
                d.edge = ring.data_ptr()
            d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
            set_split(d, ks, dev, keep)
            keep.append((whi, wlo, bp, ring))
            outs.append((dst, pool, ring))
            descs.append(d)
            ok.append(_lib.lib().rrin_conv3x3_h8_fwd(C.byref(d), st) == 0)
        torch.cuda.synchronize()
        ref = next(i for i, (c, k) in enumerate(variants) if ok[i] and not k)
        notes = []
        for i, (c, k) in enumerate(variants):
            if not ok[i] or i == ref:
                continue
            a, b = outs[ref][0].to_nchw(), outs[i][0].to_nchw()
            if k:
                notes.append(f"{c}s{k} maxdiff {float((a - b).abs().max()):.1e}")
            else:
                same = torch.equal(a, b)
                if epi == 2:
                    same = same and torch.equal(outs[ref][1].to_nchw(), outs[i][1].to_nchw())
                if epi == 4:
                    same = same and torch.equal(outs[ref][2], outs[i][2])
                bad += 0 if same else 1
                notes.append(f"{c} {'bitwise' if same else 'DIFFERENT'}")
        times = [[] for _ in variants]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for i, d in enumerate(descs):
                if not ok[i]:
                    continue
                e0.record()
                for _ in range(args.reps):
                    L_.rrin_conv3x3_h8_fwd(C.byref(d), st)
                e1.record()
                e1.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.reps)
        med = [sorted(t)[len(t) // 2] if t else float("nan") for t in times]
        wf = 2 * 4 * cin * cout * h * w * n
        cols = "  ".join(f"{c}{'s%d' % k if k else ''} {med[i]:.4f} ({med[i] / med[0]:.3f})"
                         for i, (c, k) in enumerate(variants))
        best = min(m for m in med if m == m)
        print(f"{cin:4d}->{cout:4d} L{L} epi{epi} n{n}: {cols}  best {wf / (best * 1e-3) / 1e12:.1f} TF(wino)  "
              + "; ".join(notes), flush=True)
    if bad and args.check:
        sys.exit(3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["breakdown", "tune", "single", "ablate", "ablate32", "abconv", "cfgab"])
    ap.add_argument("--cfgs", default="20,23", help="cfgab: tile configs, e.g. 20,21,23,21s4 (s: split-K slices)")
    ap.add_argument("--lib", default=None, help="abconv: library A (default: the in-tree product library)")
    ap.add_argument("--lib-b", default=None, help="abconv: libraries B, C, ... (comma-separated)")
    ap.add_argument("--shapes", default="256:256:3:1:18,64:32:0:1:18,32:32:0:1:18,128:64:1:1:18",
                    help="abconv: cin:cout:level:epi:cfg list")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shape", type=int, nargs=5, default=[512, 256, 3, 1, 0],
                    help="single: cin cout level epi cfg")
    ap.add_argument("--check", action="store_true", help="single, lab: compare with the product kernel bitwise")
    ap.add_argument("--src", type=int, default=0, help="single, fp32: src mode (1 = fused upsample)")
    ap.add_argument("--sched", type=int, default=None,
                    help="single: lab schedule / ablation bits (fp32_planar: librrin_lab32.so; records: librrin_lab.so)")
    ap.add_argument("--persist", type=int, default=0, help="single, records + --sched: persistent grid factor")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--first-cfg", type=int, default=None,
                    help="breakdown: run the first conv of every U-Net with this H8 config (same BM only)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32_planar", "fp32_split16", "fp16"])
    args = ap.parse_args()
    {"breakdown": breakdown, "tune": tune, "single": single, "ablate": ablate, "ablate32": ablate32,
     "abconv": abconv, "cfgab": cfgab}[args.mode](args)


if __name__ == "__main__":
    main()
