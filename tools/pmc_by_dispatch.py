#!/usr/bin/env python3
"""Split the HBM traffic of a rocprofv3 --pmc run by dispatch shape: (kernel, template
arguments, grid size, workgroup size) -> dispatches, bytes per dispatch, bytes per step.

  python tools/pmc_by_dispatch.py --fetch DIR1 --write DIR2 --steps S [--top 40]

Bytes are priced as tools/pmc_summary.py does (MI355X_MICROARCH.md §HBM): hbm = 2 x FETCH_SIZE
+ WRITE_SIZE (KiB).  The two passes are separate runs of the same program; dispatches are paired
by Dispatch_Id (the launch sequence is deterministic), and a shape's rows are summed.
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def rows(dirname, counter):
    out = {}
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                out[int(r["Dispatch_Id"])] = r
    return out


def short(name):
    m = re.search(r"rrin::(\w+?)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"rrin::(\w+?)\(", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    fe, wr = rows(a.fetch, "FETCH_SIZE"), rows(a.write, "WRITE_SIZE")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for did, r in fe.items():
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        w = wr.get(did)
        agg[key][0] += 1
        agg[key][1] += 2.0 * float(r["Counter_Value"]) * 1024.0
        agg[key][2] += (float(w["Counter_Value"]) * 1024.0) if w is not None else 0.0
    tot = sum(v[1] + v[2] for v in agg.values())
    print(f"total {tot / a.steps / 1e9:.3f} GB/step over {a.steps} steps")
    print(f"{'kernel<template>':58s} {'grid':>8s} {'wg':>4s} {'n/step':>6s} {'rd MB/d':>8s} {'wr MB/d':>8s} {'GB/step':>8s}")
    for key, (n, rd, wb) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:a.top]:
        print(f"{key[0][:58]:58s} {key[1]:8d} {key[2]:4d} {n / a.steps:6.1f} {rd / n / 1e6:8.2f} {wb / n / 1e6:8.2f} "
              f"{(rd + wb) / a.steps / 1e9:8.3f}")


if __name__ == "__main__":
    main()
