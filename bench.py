#!/usr/bin/env python3
"""RRIN inference throughput on MI355X (BASELINE.json metric).

One step = one ``Net.forward`` over this rank's batch of synthetic 1280x720
fp32 frame pairs (inputs already resident in HBM) in exact fp32 arithmetic
(``--precision fp32``, the default: fp32 storage, v_mfma_f32_32x32x2_f32
products, fp32 accumulation) + the RCCL all-gather that
reassembles the interpolated frames of all ranks (rrin_amd.shard); the gather
of step k runs on RCCL's stream while step k+1 computes, and every gather has
completed before the clock stops.  Weak scaling: every rank owns ``--batch``
pairs per step.

  python bench.py [--gpus N --steps K --warmup W --batch B --height H --width W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

Rank 0 prints one JSON line.  ``roofline`` is for the dominant kernel (the
MFMA conv3x3 family): algorithmic conv FLOPs / the family's busy time (union of
its launch spans — the batch runs as ``--streams`` parts whose launches
overlap), measured live with HIP events recorded around every launch of the
timed steps; ``unprofiled`` re-times the same K steps without those events
(their records cost ~1 % of the rate at 720p x4 and ~15 % at 640x368 x1, so
``value`` is the conservative, profiled figure); ``cpu_baseline`` times the CPU oracle (oracle/, a restatement of
the reference op sequence) on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

# HIP hardware queues per process (HIP's default is 4).  The forward's two
# streams must land on different hardware queues to overlap; with RCCL's own
# streams in the process (N > 1) four queues are not enough and HIP maps the two
# onto one queue: 72.3 vs 78.3 pairs/s with the RCCL gather at world size 1
# (profiles/r02/hw_queues_ab.txt).  Set before the first HIP call.
os.environ["GPU_MAX_HW_QUEUES"] = (sys.argv[sys.argv.index("--hw-queues") + 1]
                                   if "--hw-queues" in sys.argv else "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from rrin_amd import Net, _lib  # noqa: E402
from rrin_amd import engine as engine_mod  # noqa: E402
from rrin_amd.shard import GatherPipeline, verify_gather  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402
from rrin_amd.unet import conv_bytes, conv_flops, conv_work, roofline_bound_s  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (MFMA 32x32x2 f32 = VALU rate), MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2500.0   # dense f16 MFMA (v_mfma_f32_32x32x16_f16), no sparsity
HBM_PEAK_GBS = 8000.0
# Roofline peak in fp32-equivalent TFLOP/s per precision: the split path spends
# three f16 MFMA products on every fp32 product.
PEAK = {"fp32": FP32_PEAK_TFLOPS, "fp32_planar": FP32_PEAK_TFLOPS, "fp32_split16": F16_PEAK_TFLOPS / 3,
        "fp16": F16_PEAK_TFLOPS}
MFMA_PRODUCTS = {"fp32": 1, "fp32_planar": 1, "fp32_split16": 3, "fp16": 1}
# Only "fp32" is fp32 arithmetic (the BASELINE metric); split16 emulates fp32 with fp16 products.
PREC_LABEL = {"fp32": "fp32", "fp32_planar": "fp32", "fp32_split16": "fp32-emulated (fp16 hi+lo x3)",
              "fp16": "fp16"}
KERNEL = {"fp32": "conv3x3_h8_kernel on fp32 records (77 body convs, v_mfma_f32_32x32x2_f32)",
          "fp32_planar": "conv3x3_mfma_kernel, planar fp32 (77 body convs, v_mfma_f32_32x32x2_f32)",
          "fp32_split16": "conv3x3_h8_kernel (77 body convs, v_mfma_f32_32x32x16_f16 x3)",
          "fp16": "conv3x3_h8_kernel (77 body convs, v_mfma_f32_32x32x16_f16)"}
# Winograd F(2x2,3x3) tiles by kind (rrin_conv_h8_cfg_wino; engine.wino_kind_for)
WINO_KERNELS = {1: "conv3x3_wino_kernel (BM 32 x TH 8, 4 waves of 8 accumulators)",
                3: "conv3x3_winoq_kernel (BM 32 x TH 8, 8 waves of 4 accumulators)",
                4: "conv3x3_winoq_kernel (BM 32 x TH 4, 4 waves)",
                6: "conv3x3_winoc_kernel (register-U, BM 64 x TH 4, 4 waves of 2 co tiles)",
                7: "conv3x3_winoc_kernel (register-U, BM 32 x TH 8, 4 waves of 2 patch tiles)",
                14: "conv3x3_winoc42_kernel (register-U, Winograd F(4,3) x F(2,3), BM 32 x TH 8, 4 waves)"}
# fp16 Winograd tiles (conv_winoh.hip)
WINO_KERNELS_F16 = {6: "conv3x3_winoh_kernel (register-U, BM 64 x TH 4)"}


def kernel_wino(eng, n, h, w):
    """The body convs' kernels of a forward part of n pairs at h x w, with counts."""
    lib = _lib.lib()
    t = eng.conv_table_for(n, h, w)
    kinds = [lib.rrin_conv_h8_cfg_wino(t[i].cfg) for i in range(eng.expected_convs)]
    if eng.precision == "fp16":
        parts = [f"{WINO_KERNELS_F16.get(k, f'kind {k}')} x {kinds.count(k)}" for k in sorted(set(kinds)) if k]
        fused = sum(int(t[i].fuse_next) for i in range(eng.expected_convs))
        if fused:
            parts.append(f"conv_block0_h8_kernel (fused level-0 UNetConvBlock, conv a's tile in LDS) x {fused} "
                         f"(= {2 * fused} convs)")
        if kinds.count(0) - 2 * fused:
            parts.append(f"conv3x3_h8_kernel direct form x {kinds.count(0) - 2 * fused}")
        return ("Winograd F(2x2,3x3) on fp16 records, packed-fp16 input transform, v_mfma_f32_32x32x16_f16 "
                "contraction per transform point, fp32 output transform: " + "; ".join(parts))
    parts = [f"{WINO_KERNELS.get(k, f'kind {k}')} x {kinds.count(k)}" for k in sorted(set(kinds)) if k]
    if kinds.count(0):
        parts.append(f"conv3x3_h8_kernel direct form x {kinds.count(0)}")
    return ("Winograd F(2x2,3x3) on fp32 records, fp32 input/output transforms, v_mfma_f32_32x32x2_f32 "
            "contraction per transform point: " + "; ".join(parts))


DTYPE = {"fp32": "f32", "fp32_planar": "f32",
         "fp32_split16": "f16x3 (fp32-emulated: fp16 hi+lo split, 3 f16 MFMA products, f32 accumulate)",
         "fp16": "f16"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4, help="frame pairs per GPU per step")
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--t", type=float, default=0.5)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32_planar", "fp32_split16", "fp16"],
                    help="fp32: exact fp32 (v_mfma_f32_32x32x2_f32, fp32 storage) -- the BASELINE metric; "
                         "fp32_split16: fp32-EMULATED (values as fp16 hi+lo, 3 fp16 products per fp32 "
                         "product, fp32 accumulate); fp16: fp16 storage/products")
    ap.add_argument("--no-prof", action="store_true", help="skip the per-launch event profiler")
    ap.add_argument("--no-alt", action="store_true",
                    help="N=1: skip the secondary line (fp32 run: the fp32-emulated split16 path; "
                         "other precisions: the exact-fp32 path)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo only to rehearse N ranks on fewer GPUs")
    ap.add_argument("--cpu-pairs", type=int, default=2, help="pairs timed on the CPU baseline")
    ap.add_argument("--cpu-all-threads", action="store_true",
                    help="also time one CPU pair on os.cpu_count() threads (beyond the job's CPU quota)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the rank's pairs are split over (their kernels overlap, filling each "
                         "other's launch gaps and last-wave tails; outputs are bitwise those of one stream); "
                         "default engine.default_streams: 2")
    ap.add_argument("--dist-init", action="store_true",
                    help="initialise torch.distributed and run the all-gather path even at WORLD_SIZE 1 "
                         "(exercises RCCL / the gather check on a single GPU)")
    ap.add_argument("--hw-queues", default="8", help="GPU_MAX_HW_QUEUES for this process (read before HIP init)")
    ap.add_argument("--side-priority", type=int, default=0,
                    help="stream priority of the forward's side streams (torch.cuda.Stream priority; -1 = high)")
    ap.add_argument("--size-class", default=None, choices=["small", "medium", "large", "xlarge", "xxlarge"],
                    help="A/B: force the tile table of this size class for every forward part")
    ap.add_argument("--no-wino", action="store_true",
                    help="A/B: the direct-form conv (one MFMA product per tap) instead of Winograd F(2x2,3x3), "
                         "exact fp32 and fp16")
    ap.add_argument("--fuse-l0", type=int, default=None, choices=[0, 1, 2],
                    help="fp16: level-0 UNetConvBlocks as one fused launch: 0 none, 1 down_path[0], "
                         "2 also the last up block's; default engine.FUSE_L0")
    ap.add_argument("--wino-f16-levels", default=None,
                    help="A/B: grid levels of the fp16 Winograd convs, e.g. '2,3,4' (engine.WINO_F16_LEVELS)")
    ap.add_argument("--wino-kind", type=int, default=None,
                    help="A/B: Winograd tile kind of the exact-fp32 body convs (rrin_conv_h8_cfg_wino; "
                         "0 = auto: kind 6 where cout %% 64 == 0, else 3; default engine.WINO_KIND)")
    ap.add_argument("--wino-split", default=None,
                    help="A/B: split-K slices per grid level for every Winograd conv, e.g. '2:2,3:4,4:8' "
                         "(engine.WINO_SPLIT_LEVELS, replaces the geometry rule); 'none' disables split-K (engine.GEOM_SPLIT)")
    ap.add_argument("--no-ring-fold", action="store_true",
                    help="A/B: run the sub-pixel ring fix-up as its own launch (engine.RING_FOLD = False)")
    ap.add_argument("--wino42-levels", default=None,
                    help="exact fp32: grid levels whose convs run Winograd F(4,3) x F(2,3) (kind 14), e.g. "
                         "'2,3' or 'none' (engine.WINO42_LEVELS)")
    ap.add_argument("--wino42-min-cin-l0", type=int, default=None,
                    help="A/B: smallest cin of a level-0 conv on kind 14 (engine.WINO42_MIN_CIN_L0)")
    ap.add_argument("--wino42-geom", type=int, default=None, choices=(0, 1, 2, 3),
                    help="A/B: kind 14's tile geometry (rrin_conv_h8_set_wino42_geom: 0 auto, 1 32x8, 2 16x16, "
                         "3 32x8 one workgroup per tile; the same output bits)")
    ap.add_argument("--wino-kind32", type=int, default=None,
                    help="A/B: Winograd kind of the 32-output-channel convs in the auto mode "
                         "(engine.WINO_KIND32: 3 or 7)")
    ap.add_argument("--no-wino-th4", action="store_true",
                    help="A/B: no TH-4 Winograd tiles on the deep convs (engine.WINO_TH4)")
    ap.add_argument("--split", default=None,
                    help="explicit pairs per stream, e.g. 1,3 (overrides --streams' even split)")
    ap.add_argument("--graph", action="store_true",
                    help="time HIP-graph replays of the forward (RRINEngine.graph: one captured graph per part "
                         "split, static inputs / t coefficients / output); the roofline then comes from an "
                         "eager profiled pass of the same K steps (per-launch events cannot be read per replay)")
    ap.add_argument("--train", action="store_true",
                    help="training step instead (SURVEY §8f f4, train.py:98,142-145): Net.forward under "
                         "autograd on the HIP training kernels + charbonnier loss + backward + AdamW step; "
                         "default size 640x368 x 2 pairs")
    a = ap.parse_args()
    a.batch_given = "--batch" in sys.argv
    a.height_given = "--height" in sys.argv
    a.width_given = "--width" in sys.argv
    return a


def host_cpu_share():
    """(threads to use, description): the CPUs this process may run on -- the
    cgroup CPU quota when one is set (a GPU box gives each 1-GPU job a share of
    a larger host), else the affinity mask."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    threads = min(aff, quota) if quota else aff
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env:
        threads = min(threads, env) if quota else env
    return threads, {"host_cpus": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "omp_num_threads": env or None}


CPU_ALL_THREADS = False


def cpu_baseline(sd, h, w, pairs, t, gpu_out0, alt_out0=None):
    """Time the CPU oracle on pair 0 and compare its output with the GPU's."""
    from oracle.ref_net import net_forward  # checker / baseline only
    threads, host = host_cpu_share()
    torch.set_num_threads(threads)
    i0, i1 = synthetic_batch(1, h, w, first_index=0)
    with torch.no_grad():
        net_forward(sd, i0[:, :, :64, :64].contiguous(), i1[:, :, :64, :64].contiguous(), t)  # warm
        t0 = time.perf_counter()
        for _ in range(pairs):
            ref = net_forward(sd, i0, i1, t)
        dt = time.perf_counter() - t0
    def compare(o):
        d = (o.double() - ref.double())
        mse = float((d * d).mean())
        return {"pair": 0, "max_abs": float(d.abs().max()),
                "psnr_db": (10 * math.log10(1.0 / mse)) if mse > 0 else float("inf"), "gate_max_abs": 1e-3}
    parity = compare(gpu_out0)
    if alt_out0 is not None:
        parity["alt"] = compare(alt_out0)
    res = {"value": pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
           "sample": f"{pairs} x Net.forward {w}x{h} N=1 fp32 on PyTorch-CPU (oracle/ref_net.py), {dt:.1f} s",
           "host": host,
           "cores_note": "threads used = the CPUs this job may use (cgroup quota / affinity / OMP_NUM_THREADS); "
                         "host_cpus = every CPU of the machine"}
    allc = os.cpu_count() or threads
    if allc > threads:
        # the job may use `threads` of the host's `allc` CPUs (cgroup quota): a
        # linear projection to every core is the upper bound the CPU reference
        # could reach on this host -- reported beside, never as `value`
        res["projected_all_host_cores"] = {
            "value": res["value"] * allc / threads, "cores": allc,
            "note": "linear scaling of the measured rate to os.cpu_count() cores (upper bound, not measured)"}
    if CPU_ALL_THREADS and allc > threads:
        # measured on os.cpu_count() threads: oversubscribes the job's quota
        # (on the GPU box 256 threads on 16 CPUs: 0.015 pairs/s)
        torch.set_num_threads(allc)
        with torch.no_grad():
            t0 = time.perf_counter()
            net_forward(sd, i0, i1, t)
            dt_all = time.perf_counter() - t0
        torch.set_num_threads(threads)
        res["all_host_threads"] = {"value": 1.0 / dt_all, "threads": allc, "sample": f"1 pair, {dt_all:.1f} s"}
        if 1.0 / dt_all > res["value"]:
            res.update(value=1.0 / dt_all, cores=allc, sample=res["sample"] + f"; best: {allc} threads")
    return res, parity


def union_ms(spans):
    """Length of the union of [t0, t1] intervals (ms)."""
    tot, end = 0.0, None
    for a, b in sorted(spans):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def time_steps(eng, i0, i1, t, steps, dev, prof=None, streams=1):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out = None
    with torch.no_grad():
        for _ in range(steps):
            out = eng.forward(i0, i1, t, prof=prof, streams=streams)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, out


def read_prof(lib, prof, cap):
    kinds = (C.c_int32 * cap)()
    ms = (C.c_float * cap)()
    fl = (C.c_double * cap)()
    cnt = C.c_int32()
    _lib.check(lib.rrin_prof_read(prof, kinds, ms, fl, cap, C.byref(cnt)), "rrin_prof_read")
    n = cnt.value
    t0s, t1s = (C.c_float * cap)(), (C.c_float * cap)()
    _lib.check(lib.rrin_prof_read_spans(prof, t0s, t1s, cap, C.byref(cnt)), "rrin_prof_read_spans")
    conv = [i for i in range(n) if kinds[i] == 0]
    # conv busy time (union of spans), conv FLOPs, launches
    return union_ms([(t0s[i], t1s[i]) for i in conv]), sum(fl[i] for i in conv), len(conv)


def train_main(args):
    """One training step per iteration (train.py:98-145 without its VGG perceptual loss,
    whose weights need the network): forward of the rank's pairs under autograd on the
    HIP training kernels (rrin_amd.autograd), charbonnier loss (losses.py:39-42) against
    a synthetic target frame, backward, AdamW (lr 1e-4, train.py:49).  Prints one JSON
    line: pairs/s and the conv work of the step (forward, dgrad and wgrad) over the
    whole step time -- a lower bound on the conv kernels' rate; their own launch times
    come from the rocprofv3 family summary (profiles/)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch if args.batch_given else 2
    H = args.height if args.height_given else 368
    W = args.width if args.width_given else 640
    net = Net()
    sd = keyed_state_dict(net.state_dict())
    net.load_state_dict(sd, strict=True)
    net = net.to(dev).train()
    i0, i1 = synthetic_batch(B, H, W, first_index=0)
    i0, i1, tgt = i0.to(dev), i1.to(dev), (0.5 * (i0 + i1)).to(dev)
    opt = torch.optim.AdamW(net.parameters(), lr=1e-4)

    def step():
        opt.zero_grad(set_to_none=True)
        out = net(i0, i1, args.t)
        loss = torch.sum(torch.sqrt((out - tgt).pow(2) + 1e-6)) / B  # charbonnierLoss, losses.py:39-42
        loss.backward()
        opt.step()
        return loss

    from rrin_amd import autograd as ag
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ag.PROF = []  # per-launch conv events (forward, dgrad, wgrad) on each launch's stream
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    events, ag.PROF = ag.PROF, None
    # conv busy time = the union of the conv launch spans, on one clock: every event's time
    # from the first start event
    ref = events[0][0]
    spans = [(ref.elapsed_time(e0), ref.elapsed_time(e1)) for e0, e1, _, _ in events]
    busy_ms = union_ms(spans)
    conv_fl = sum(f for _, _, f, _ in events)
    by_kind = {}
    for (a, b), (_, _, f, k) in zip(spans, events):
        kk = by_kind.setdefault(k, [0, 0.0, 0.0])
        kk[0] += 1
        kk[1] += b - a
        kk[2] += f
    ach = conv_fl / (busy_ms * 1e-3) / 1e12
    step_ach = conv_fl / el / 1e12
    wino = ag.TRAIN_WINO
    kernel = ("forward and dgrad: the exact-fp32 Winograd F(2x2,3x3) register-U tiles (conv3x3_winoc_kernel, "
              "kinds 6/7, v_mfma_f32_32x32x2_f32; weights packed on the device by rrin_tpack_wino, dgrad = the "
              "forward conv of the flipped transposed weights); wgrad: csrc/train.hip row-tiled MFMA "
              "(conv3x3 wgrad, v_mfma_f32_32x32x2_f32, direct form, deterministic split-K)" if wino else
              "csrc/train.hip implicit GEMM for forward / dgrad / wgrad (v_mfma_f32_32x32x2_f32, direct form)")
    basis = ("FLOPs of the algorithm each launch runs: Winograd F(2x2,3x3) = 2*4*Cin*Cout*H*W per image for the "
             "forward and dgrad convs, direct form 2*9*Cin*Cout*H*W for wgrad" if wino else
             "direct-form conv FLOPs 2*9*Cin*Cout*H*W per image for forward, dgrad and wgrad")
    res = {
        "metric": f"training steps at {W}x{H} fp32 (Net forward + backward + AdamW, frame pairs/s)",
        "value": round(B * args.steps / el, 3), "unit": "pairs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (key-seeded weights, randint/255 frame pairs, target = their mean)",
        "config": {"workload": f"RRIN training step {W}x{H} fp32, {B} pairs: forward under autograd (HIP training "
                               "kernels), charbonnierLoss, backward, AdamW lr 1e-4 (train.py:98,142-145; no VGG loss)",
                   "global_batch": B, "height": H, "width": W, "parallelism": "single GPU"},
        "roofline": {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / FP32_PEAK_TFLOPS, 4), "traffic": None,
                     "kernel": kernel, "flops_basis": basis,
                     "conv_tflop_per_step": round(conv_fl / args.steps / 1e12, 4),
                     "conv_busy_ms_per_step": round(busy_ms / args.steps, 3),
                     "launches_per_step": {k: v[0] // args.steps for k, v in by_kind.items()},
                     "tflops_by_kind": {k: round(v[2] / (v[1] * 1e-3) / 1e12, 2) for k, v in by_kind.items()},
                     "frac_basis": "algorithmic conv FLOPs of every conv launch (the 81 forward convs incl. the "
                                   "heads, their dgrads but Flow's first, every wgrad) / conv busy time = union of "
                                   "the launch spans (HIP events recorded on each launch's own stream)",
                     "whole_step_tflops": round(step_ach, 2)},
        "loss": float(loss.item()),
        "cpu_baseline": None,
    }
    print(json.dumps(res), flush=True)


def main():
    args = parse()
    if args.train:
        train_main(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    local = local % max(torch.cuda.device_count(), 1)  # rehearsal: several ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.dist_init
    if distributed:
        if args.dist_init and world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    if args.no_wino:
        engine_mod.WINO = False
        engine_mod.WINO_F16 = False
    if args.fuse_l0 is not None:
        engine_mod.FUSE_L0 = args.fuse_l0
    if args.wino_f16_levels is not None:
        engine_mod.WINO_F16_LEVELS = tuple(int(v) for v in args.wino_f16_levels.split(",") if v)
    if args.wino_kind is not None:
        engine_mod.WINO_KIND = args.wino_kind
    if args.wino_split == "none":
        engine_mod.GEOM_SPLIT = False
    elif args.wino_split:
        engine_mod.WINO_SPLIT_LEVELS.update({int(k): int(v) for k, v in
                                             (kv.split(":") for kv in args.wino_split.split(","))})
    if args.no_ring_fold:
        engine_mod.RING_FOLD = False
    if args.no_wino_th4:
        engine_mod.WINO_TH4 = {}
    if args.wino42_levels is not None:
        engine_mod.WINO42_LEVELS = tuple(int(v) for v in args.wino42_levels.split(",") if v and v != "none")
    if args.wino42_min_cin_l0 is not None:
        engine_mod.WINO42_MIN_CIN_L0 = args.wino42_min_cin_l0
    if args.wino_kind32 is not None:
        engine_mod.WINO_KIND32 = args.wino_kind32
    if args.wino42_geom is not None:
        _lib.lib().rrin_conv_h8_set_wino42_geom(args.wino42_geom)
    net = Net()
    sd = keyed_state_dict(net.state_dict())
    net.load_state_dict(sd, strict=True)
    net = net.to(dev).eval()
    net.precision = args.precision
    B, H, W = args.batch, args.height, args.width
    i0, i1 = synthetic_batch(B, H, W, first_index=rank * B)
    i0, i1 = i0.to(dev), i1.to(dev)
    # the all-gather of step k overlaps the compute of step k+1 (double-buffered outputs)
    gather = GatherPipeline((world * B, 3, H, W), torch.float32, dev) if distributed else None
    eng = net.engine()
    eng.side_priority = args.side_priority
    eng.force_size_class = args.size_class
    lib = _lib.lib()
    split = [int(c) for c in args.split.split(",")] if args.split else None
    if split:
        args.streams = len(split)
    elif args.streams is None:
        args.streams = engine_mod.default_streams(args.precision, B)

    last_gather = [None]
    ngraph = None
    if args.graph:
        ngraph = eng.graph(B, H, W, streams=args.streams, split=split)
        ngraph.i0.copy_(i0)
        ngraph.i1.copy_(i1)

    def step(prof=None):
        with torch.no_grad():
            if ngraph is not None and prof is None:
                out = ngraph.replay(args.t)
                if gather is not None:
                    out = out.clone()  # the next replay rewrites the static output
            else:
                out = eng.forward(i0, i1, args.t, prof=prof, streams=args.streams, split=split)
            if gather is not None:
                last_gather[0] = (out, gather.submit(out)[0])
        return out

    for _ in range(args.warmup):
        step()
    if gather is not None:
        gather.drain()
    torch.cuda.synchronize(dev)
    last = [None]

    prof = None
    cap = 0
    if not args.no_prof:
        cap = 100 * args.steps * max(1, args.streams)
        h = C.c_void_p()
        _lib.check(lib.rrin_prof_create(cap, C.byref(h)), "rrin_prof_create")
        prof = h.value

    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last[0] = step(None if ngraph is not None else prof)
    if gather is not None:
        gather.drain()  # every step's gather is inside the timed region
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # the same K steps again without the per-launch events (their records cost
    # ~1 % of the rate at 720p x4, ~15 % at 640x368 x1): reported beside `value`
    unprofiled = None
    if prof is not None:
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        u0 = time.perf_counter()
        for _ in range(args.steps):
            step(prof if ngraph is not None else None)
        if gather is not None:
            gather.drain()
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        uel = time.perf_counter() - u0
        if distributed:
            tt = torch.tensor([uel], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            uel = float(tt.item())
        unprofiled = {"value": round(world * B * args.steps / uel, 3),
                      "ms_per_step": round(1e3 * uel / args.steps, 3),
                      "note": "same K steps, no per-launch HIP events"}
        if ngraph is not None:
            unprofiled["note"] = ("the same K steps as eager forwards with the per-launch HIP events the "
                                  "roofline is read from (value: HIP-graph replays, no events)")
            unprofiled = {"eager_profiled": unprofiled}

    roofline = None
    conv_ms_step = head_ms_step = None
    if prof is not None:
        kinds = (C.c_int32 * cap)()
        ms = (C.c_float * cap)()
        fl = (C.c_double * cap)()
        cnt = C.c_int32()
        _lib.check(lib.rrin_prof_read(prof, kinds, ms, fl, cap, C.byref(cnt)), "rrin_prof_read")
        n = cnt.value
        conv_ms = sum(ms[i] for i in range(n) if kinds[i] == 0)
        conv_fl = sum(fl[i] for i in range(n) if kinds[i] == 0)
        head_ms = sum(ms[i] for i in range(n) if kinds[i] == 1)
        other_ms = sum(ms[i] for i in range(n) if kinds[i] == 2)
        edge_ms = sum(ms[i] for i in range(n) if kinds[i] == 3)
        conv_launches = sum(1 for i in range(n) if kinds[i] == 0)
        # busy time of the conv family = union of its launch spans (launches of
        # the --streams parts overlap; with one stream this is the sum)
        t0s, t1s = (C.c_float * cap)(), (C.c_float * cap)()
        cnt2 = C.c_int32()
        _lib.check(lib.rrin_prof_read_spans(prof, t0s, t1s, cap, C.byref(cnt2)), "rrin_prof_read_spans")
        conv_busy = union_ms([(t0s[i], t1s[i]) for i in range(cnt2.value) if kinds[i] == 0])
        lib.rrin_prof_destroy(prof)
        conv_ms_step = conv_ms / args.steps
        head_ms_step = head_ms / args.steps
        achieved = conv_fl / (conv_busy * 1e-3) / 1e12
        peak = PEAK[args.precision]
        algo = eng.conv_algorithm(B // max(1, args.streams), H, W)
        units = ("Flow", "refine_flow", "Mask", "final")
        direct_fl = args.steps * B * sum(fl for u in units for _, fl, _, _ in conv_work(getattr(net, u), H, W))
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1),
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                    "mfma_issued_tflops": round(achieved * MFMA_PRODUCTS[args.precision], 1),
                    "kernel": (kernel_wino(eng, B // max(1, args.streams), H, W)
                               if algo in ("winograd", "mixed") and args.precision in ("fp32", "fp16")
                               else KERNEL[args.precision]),
                    "conv_algorithm": algo,
                    "flops_basis": ("FLOPs of the algorithm the convs run: Winograd F(2x2,3x3) = 16 multiply-adds "
                                    "per 2x2 output patch and channel pair (4/9 of the direct form's)"
                                    + (f"; F(4,3) x F(2,3) (kind 14, grid levels {list(engine_mod.WINO42_LEVELS)}) = 24 "
                                       "per 4x2 patch (3/9)" if args.precision == "fp32" and engine_mod.WINO42_LEVELS
                                       else "")
                                    + (("; the 6-channel first conv runs the direct form (engine.WINO_DIRECT) and counts "
                                        "its direct-form FLOPs" if args.precision == "fp32" else
                                        "; the direct-form convs (engine.wino_f16_ok false: level 0, cout 32, cin % 16) "
                                        "count their direct-form FLOPs") if algo == "mixed" else "")
                                    if algo in ("winograd", "mixed") else "direct-form conv FLOPs (2*9*Cin*Cout*H*W)"),
                    "direct_equivalent_tflops": round(direct_fl / (conv_busy * 1e-3) / 1e12, 2),
                    # round-5 comparable rate: every conv priced at F(2x2,3x3)'s 4/9 of the direct
                    # FLOPs (kind 14 runs 3/9, so its own-algorithm `achieved` reads lower)
                    "f2x2_basis_tflops": (round(direct_fl * 4 / 9 / (conv_busy * 1e-3) / 1e12, 2)
                                          if algo in ("winograd", "mixed") else None),
                    "flops_per_launch_avg": conv_fl / max(conv_launches, 1),
                    "avg_launch_ms": conv_ms / max(conv_launches, 1),
                    "conv_busy_ms_per_step": round(conv_busy / args.steps, 3),
                    "frac_basis": ("algorithmic conv FLOPs / conv busy time = union of the conv launch spans "
                                   "(HIP events on each launch's own stream; the --streams parts overlap)"),
                    "launch_overlap": round(conv_ms / conv_busy, 3),
                    "streams": args.streams,
                    "conv_ms_per_step": round(conv_ms_step, 3),
                    "head_ms_per_step": round(head_ms_step, 3),
                    "layout_upsample_ms_per_step": round(other_ms / args.steps, 3),
                    "subpixel_ring_fix_ms_per_step": round(edge_ms / args.steps, 3)}
        # SURVEY §8d per-layer bound: sum_l max(FLOP_l / peak, bytes_l / 8 TB/s) over the body convs
        bpv = 2 if args.precision == "fp16" else 4
        fscale = 4.0 / 9.0 if algo in ("winograd", "mixed") else 1.0
        if args.precision == "fp16" and algo == "mixed":
            # per conv: Winograd where engine.wino_f16_ok puts it (an up conv runs on the
            # low-res grid with 4 x cout rows), else the direct form
            def fscale(tag, cin, cout, lvl):
                up = tag.endswith(".up") and lvl <= eng.subpixel_max_level
                ok = engine_mod.wino_f16_ok(cin, 4 * cout if up else cout, lvl + 1 if up else lvl)
                return 4.0 / 9.0 if ok else 1.0
        if args.precision == "fp32" and algo in ("winograd", "mixed") and engine_mod.WINO42_LEVELS:
            def fscale(tag, cin, cout, lvl):  # kind 14 where engine.wino42_ok puts it
                up = tag.endswith(".up") and lvl <= eng.subpixel_max_level
                ok = engine_mod.wino42_ok(cin, 4 * cout if up else cout, lvl + 1 if up else lvl)
                return 3.0 / 9.0 if ok else 4.0 / 9.0
        tlb = B * sum(roofline_bound_s(getattr(net, u), H, W, bpv, peak * 1e12, HBM_PEAK_GBS * 1e9, fscale)
                      for u in ("Flow", "refine_flow", "Mask", "final"))
        roofline["t_lb_conv_ms_per_step"] = round(1e3 * tlb, 3)
        roofline["t_lb_frac_of_conv_time"] = round(1e3 * tlb / (conv_busy / args.steps), 4)

    if roofline is not None:
        # HBM bytes per conv launch from the PMC passes of the same command
        # (tools/gpu_check.sh pmc -> tools/pmc_summary.py; rocprofv3 cannot
        # collect counters inside this process's timed region)
        tab = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
        # exact fp32: "fp32" = the Winograd kernel, "fp32-direct" = the direct form (--no-wino)
        kp = args.precision + ("-direct" if args.precision == "fp32" and roofline["conv_algorithm"] == "direct" else "")
        key = f"{kp}@{W}x{H}x{B}" + (f"s{args.streams}" if args.streams > 1 else "")
        build = _lib.build_id()
        roofline["traffic_build"] = build
        if os.path.exists(tab):
            ent = json.load(open(tab)).get(key)
            if ent is not None and ent.get("build") != build:
                # measured on another build of the kernels: no stale figure in the line
                roofline["traffic_note"] = (f"profiles/pmc_traffic.json[{key}] is from build {ent.get('build')}, "
                                            f"this library is {build}: traffic not measured for this build")
                ent = None
            if ent is not None:
                roofline["traffic"] = round(ent["hbm_bytes_per_launch"])
                roofline["traffic_unit"] = "bytes/launch"
                roofline["traffic_per_step_gb"] = round(ent["hbm_bytes_per_step"] / 1e9, 2)
                bpv = 2 if args.precision == "fp16" else 4  # split16 stores hi+lo halves
                alg = sum(sum(conv_bytes(getattr(net, u), H, W, bpv))
                          for u in ("Flow", "refine_flow", "Mask", "final"))
                roofline["algorithmic_bytes_per_step_gb"] = round(B * alg / 1e9, 2)
                roofline["traffic_source"] = f"profiles/pmc_traffic.json[{key}], build {build}"
                roofline["traffic_kernels"] = ent.get("kernel_family")

    eng.check_range()  # fp16-stored precisions: no activation left the fp16 range (raises otherwise)
    gather_check = None
    if distributed:
        # the gathered output of the last step holds every rank's own shard in rank
        # order, bit for bit (rrin_amd.shard.verify_gather: own slice by equality,
        # every slice's CRC-32 against its owner's)
        gather.drain()
        gather_check = verify_gather(last_gather[0][0], last_gather[0][1])
        if not gather_check["ok"]:
            raise RuntimeError("all-gathered output does not match the ranks' shards")

    graph_info = None
    if ngraph is not None:
        # the replayed output against an eager forward of the same inputs (bit for bit)
        with torch.no_grad():
            eager = eng.forward(i0, i1, args.t, streams=args.streams, split=split)
            torch.cuda.synchronize(dev)
            graph_info = {"mode": "HIP graph replay (RRINEngine.graph: one captured forward, static inputs, "
                                  "device-resident t coefficients)",
                          "bitwise_equal_eager": bool(torch.equal(last[0], eager))}
        if not graph_info["bitwise_equal_eager"]:
            raise RuntimeError("graph replay output differs from the eager forward")
    pairs = world * B * args.steps
    value = pairs / elapsed
    res = {
        "metric": f"interpolated frames/sec at {W}x{H} {PREC_LABEL[args.precision]} (Net.forward, frame pairs/s)",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPE[args.precision],
        "data": "synthetic (key-seeded weights, randint/255 frame pairs; SURVEY §8c-d)",
        "config": {"workload": f"RRIN Net.forward {W}x{H} {PREC_LABEL[args.precision]}, {B} pairs/GPU/step, "
                               f"t={args.t}" + (f", + all-gather of outputs ({'RCCL' if args.dist_backend == 'nccl' else 'gloo'})"
                                                  if distributed else ""),
                   "global_batch": world * B, "height": H, "width": W,
                   "parallelism": f"frame-batch dp{world}",
                   "gflop_per_pair": round(sum(conv_flops(getattr(net, u), H, W)
                                               for u in ("Flow", "refine_flow", "Mask", "final")) / 1e9, 1)},
        "roofline": roofline,
        "unprofiled": unprofiled,
        "graph": graph_info,
        "gather_check": gather_check,
        "cpu_baseline": None,
        "parity": None,
    }
    alt_out = None
    alt_key = None
    if world == 1 and not args.no_alt:
        # secondary line on the same inputs: an fp32 run reports the fp32-emulated
        # split16 path beside it; any other precision reports the exact-fp32 path
        alt = "fp32_split16" if args.precision in ("fp32", "fp32_planar") else "fp32"
        alt_key = "fp32_emulated_split16" if alt == "fp32_split16" else "fp32_exact"
        net.precision = alt
        eng2 = net.engine()
        with torch.no_grad():
            for _ in range(max(1, args.warmup)):
                eng2.forward(i0, i1, args.t, streams=args.streams)
        cap2 = 100 * args.steps * max(1, args.streams)
        h2 = C.c_void_p()
        _lib.check(lib.rrin_prof_create(cap2, C.byref(h2)), "rrin_prof_create")
        el2, o2 = time_steps(eng2, i0, i1, args.t, args.steps, dev, h2.value, args.streams)
        eng2.check_range()
        cbusy, cfl, _ = read_prof(lib, h2.value, cap2)
        lib.rrin_prof_destroy(h2.value)
        alt_out = o2[0:1].cpu()
        tf = cfl / (cbusy * 1e-3) / 1e12
        res[alt_key] = {"value": round(B * args.steps / el2, 3), "ms_per_step": round(1e3 * el2 / args.steps, 3),
                        "dtype": DTYPE[alt], "metric": f"interpolated frames/sec at {W}x{H} {PREC_LABEL[alt]}",
                        "conv_tflops": round(tf, 2), "peak": round(PEAK[alt], 1),
                        "conv_algorithm": eng2.conv_algorithm(B // max(1, args.streams), H, W),
                        "conv_frac_of_peak": round(tf / PEAK[alt], 4),
                        "kernel": KERNEL[alt],
                        "streams": args.streams}
        del eng2
        net.precision = args.precision
    if rank == 0 and args.cpu_baseline == "auto":
        # every line carries parity (rank 0's pair 0 = global pair 0 vs the CPU
        # oracle) and the CPU baseline; at N > 1 the timed CPU sample is that one
        # parity pair, so the other ranks wait only seconds at the final barrier
        global CPU_ALL_THREADS
        CPU_ALL_THREADS = args.cpu_all_threads and world == 1
        res["cpu_baseline"], res["parity"] = cpu_baseline({k: v.detach().cpu() for k, v in sd.items()}, H, W,
                                                          args.cpu_pairs if world == 1 else 1, args.t,
                                                          last[0][0:1].cpu(), alt_out)
        if alt_key in res:
            res[alt_key]["parity"] = res["parity"].pop("alt")
    if rank == 0:
        print(json.dumps(res), flush=True)
    if distributed:
        dist.barrier()  # rank 0's CPU baseline / parity pass ends before any rank leaves
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
