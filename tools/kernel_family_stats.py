#!/usr/bin/env python3
"""Aggregate a rocprofv3 --stats kernel_stats.csv by kernel family (template
instantiations of one kernel summed), to compare the conv family's average
launch duration with the one bench.py measures with HIP events.

  python tools/kernel_family_stats.py profiles/r01_v9/kernel_stats_split16.csv
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


if __name__ == "__main__":
    main(sys.argv[1])
