#!/usr/bin/env python3
"""Aggregate a rocprofv3 --stats kernel_stats.csv by kernel family (template
instantiations of one kernel summed), to compare the conv family's average
launch duration with the one bench.py measures with HIP events.

  python tools/kernel_family_stats.py kernel_stats.csv [kernel_trace.csv STEPS [FAMILY ...]]
        [--parts P] [--ms-per-step MS]

With a kernel_trace.csv, also each FAMILY's busy time per step = the union of its
dispatch spans (the quantity bench.py's roofline divides by when the batch is split
over several streams).  STEPS is the number of bench steps the trace holds, or
"auto": the dispatches of the once-per-forward-part kernel (pack_g16_*: one per
stream part) / P (= bench --streams, default 2).  A profiled `bench.py --steps K
--warmup W` runs W + K steps plus bench's unprofiled re-run of the K steps: "auto"
counts them all.  With --ms-per-step (the bench line's own ms_per_step), a family
whose union per step exceeds it is an error (exit 2): a union longer than the step
means the step count is wrong.

--profiled-log LOG: the log of the profiled command itself (a bench.py JSON line): its own
ms_per_step and launch_overlap are printed beside the trace's, and an all-kernel union per step
above that step (5 % slack for the warm-up steps) is an error (exit 2) -- the step count or the
trace is wrong.  --live-log LOG: the unprofiled bench line the numbers are quoted for; its step
and launch_overlap are printed beside the profiled ones, and a profiled step more than 15 %
slower is flagged ("profile not of the benched regime": per-kernel averages from such a trace do
not describe the benched forward).
"""
import json
import argparse
import csv
import re
import sys
from collections import defaultdict

MARKER = re.compile(r"^pack_g16_(r32|h8)_kernel$")


def family(name):
    m = re.search(r"rrin::(\w+?)(<|\()", name)
    return m.group(1) if m else name[:48]


def stats(path):
    fam = defaultdict(lambda: [0, 0.0])
    for row in csv.DictReader(open(path)):
        f = fam[family(row["Name"])]
        f[0] += int(row["Calls"])
        f[1] += float(row["TotalDurationNs"])
    total = sum(v[1] for v in fam.values())
    print(f"{'family':32s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'share':>6s}")
    for k, (n, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:32s} {n:6d} {ns / 1e6:10.3f} {ns / 1e6 / n:9.4f} {100 * ns / total:5.1f}%")


def union_ns(spans):
    tot, end = 0, None
    for a, b in sorted(spans):
        if end is None or a > end:
            tot, end = tot + b - a, b
        elif b > end:
            tot, end = tot + b - end, b
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("trace", nargs="?")
    ap.add_argument("steps", nargs="?", default="auto")
    ap.add_argument("families", nargs="*")
    ap.add_argument("--parts", type=int, default=2, help="forward parts per step (bench --streams)")
    ap.add_argument("--ms-per-step", type=float, default=None,
                    help="the bench line's ms_per_step: a family union above it is an error")
    ap.add_argument("--profiled-log", default=None, help="bench.py log of the profiled command")
    ap.add_argument("--live-log", default=None, help="bench.py log of the unprofiled (quoted) run")
    a = ap.parse_args()
    stats(a.stats)
    if not a.trace:
        return 0
    rows = [(family(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(a.trace))]
    markers = sum(1 for f, _, _ in rows if MARKER.match(f))
    if a.steps == "auto":
        if markers == 0 or markers % a.parts:
            print(f"cannot derive the step count: {markers} pack_g16 dispatches for {a.parts} parts per step")
            return 2
        steps = markers // a.parts
        how = f"{markers} pack_g16 dispatches / {a.parts} parts"
    else:
        steps = int(a.steps)
        how = "given"
        if markers and markers != steps * a.parts:
            print(f"warning: {steps} steps x {a.parts} parts != {markers} pack_g16 dispatches in the trace")
    print(f"steps in the trace: {steps} ({how})")
    fams = a.families or ["conv3x3_winoc_kernel"]
    bad = 0
    for fam_name in fams:
        spans = [(s, e) for f, s, e in rows if f == fam_name]
        if not spans:
            print(f"{fam_name}: no dispatches")
            continue
        tot = union_ns(spans)
        dur = sum(e - s for s, e in spans)
        per = tot / 1e6 / steps
        print(f"{fam_name}: {len(spans)} dispatches ({len(spans) / steps:.1f} per step), busy (union) "
              f"{per:.3f} ms per step, sum of durations {dur / 1e6 / steps:.3f} ms per step, "
              f"overlap {dur / max(tot, 1):.3f}")
        if a.ms_per_step is not None and per > a.ms_per_step:
            print(f"ERROR: {fam_name} union {per:.3f} ms per step > the bench's {a.ms_per_step:.3f} ms per step")
            bad += 1
    allspans = [(s, e) for _, s, e in rows]
    all_union = union_ns(allspans) / 1e6 / steps
    conv = [(s, e) for f, s, e in rows if f in fams]
    conv_overlap = sum(e - s for s, e in conv) / max(union_ns(conv), 1) if conv else float("nan")
    print(f"all kernels: busy (union) {all_union:.3f} ms per step; trace overlap of {','.join(fams)}: "
          f"{conv_overlap:.3f}")
    prof = bench_line(a.profiled_log) if a.profiled_log else None
    live = bench_line(a.live_log) if a.live_log else None
    if prof:
        print(f"profiled run: {prof.get('ms_per_step')} ms per step, launch_overlap "
              f"{prof.get('launch_overlap')} (trace: union {all_union:.3f} ms per step, overlap {conv_overlap:.3f})")
        if prof.get("ms_per_step") and all_union > 1.05 * prof["ms_per_step"]:
            print(f"ERROR: all-kernel union {all_union:.3f} ms per step > the profiled run's own "
                  f"{prof['ms_per_step']:.3f} ms per step: the step count or the trace is wrong")
            bad += 1
    if live:
        print(f"live (quoted) run: {live.get('ms_per_step')} ms per step, launch_overlap {live.get('launch_overlap')}")
        if prof and prof.get("ms_per_step") and live.get("ms_per_step") and \
                prof["ms_per_step"] > 1.15 * live["ms_per_step"]:
            print(f"WARNING: profile not of the benched regime: profiled {prof['ms_per_step']:.3f} vs live "
                  f"{live['ms_per_step']:.3f} ms per step -- per-kernel averages here do not describe the "
                  f"benched forward")
    return 2 if bad else 0


def bench_line(path):
    """The last bench.py JSON line of a log, with the roofline's launch_overlap lifted up."""
    line = None
    for ln in open(path, errors="replace"):
        ln = ln.strip()
        if ln.startswith("{") and '"ms_per_step"' in ln:
            line = ln
    if line is None:
        return None
    d = json.loads(line)
    rf = d.get("roofline") or {}
    d.setdefault("launch_overlap", rf.get("launch_overlap"))
    return d


if __name__ == "__main__":
    sys.exit(main())
