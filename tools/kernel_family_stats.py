#!/usr/bin/env python3
"""Aggregate a rocprofv3 --stats kernel_stats.csv by kernel family (template
instantiations of one kernel summed), to compare the conv family's average
launch duration with the one bench.py measures with HIP events.

  python tools/kernel_family_stats.py profiles/r01_v9/kernel_stats_split16.csv [kernel_trace.csv FORWARDS [FAMILY]]

With a kernel_trace.csv and the number of forward steps it holds (warm-up
included), also the conv family's busy time per step = the union of its
dispatch spans (the quantity bench.py's roofline divides by when the batch is
split over several streams).
"""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    m = re.search(r"rrin::(\w+?)(<|\()", name)
    return m.group(1) if m else name[:48]


def main(path):
    fam = defaultdict(lambda: [0, 0.0])
    for row in csv.DictReader(open(path)):
        f = fam[family(row["Name"])]
        f[0] += int(row["Calls"])
        f[1] += float(row["TotalDurationNs"])
    total = sum(v[1] for v in fam.values())
    print(f"{'family':32s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'share':>6s}")
    for k, (n, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:32s} {n:6d} {ns / 1e6:10.3f} {ns / 1e6 / n:9.4f} {100 * ns / total:5.1f}%")


def busy(trace, forwards, fam_name="conv3x3_h8_kernel"):
    spans = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in csv.DictReader(open(trace)) if family(r["Kernel_Name"]) == fam_name)
    tot, end = 0, None
    for a, b in spans:
        if end is None or a > end:
            tot, end = tot + b - a, b
        elif b > end:
            tot, end = tot + b - end, b
    dur = sum(b - a for a, b in spans)
    print(f"{fam_name}: {len(spans)} dispatches, busy (union) {tot / 1e6 / forwards:.3f} ms per step, "
          f"sum of durations {dur / 1e6 / forwards:.3f} ms per step, overlap {dur / max(tot, 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
    if len(sys.argv) > 3:
        busy(sys.argv[2], int(sys.argv[3]), *sys.argv[4:5])
