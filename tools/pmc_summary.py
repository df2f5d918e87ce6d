#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs (FETCH_SIZE / WRITE_SIZE passes) per kernel.

HBM bytes are priced as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports ½ of the bytes of a wide
coalesced streaming read, so the read side is doubled; WRITE_SIZE is taken as is.

  python tools/pmc_summary.py --fetch DIR1 --write DIR2 --steps S --out traffic.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import sys
import os
import re
from collections import defaultdict


def load(dirname, counter):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: [0.0, 0])
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            per[name][0] += float(row["Counter_Value"])
            per[name][1] += 1
    return per


def family(name):
    m = re.search(r"rrin::(\w+?)(<|\()", name)
    return m.group(1) if m else name[:40]


def build_id():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rrin_amd._lib import build_id as bid
    return bid()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--steps", type=int, required=True, help="Net.forward calls in the profiled run")
    ap.add_argument("--out", default=None)
    ap.add_argument("--table", default=None,
                    help="merge the conv family's per-launch bytes into this table (read by bench.py)")
    ap.add_argument("--precision", default="fp32_split16")
    ap.add_argument("--config", default="1280x720x4", help="WxHxB of the profiled bench run")
    ap.add_argument("--family", default=None,
                    help="conv kernel family, comma-separated kernels summed (default by precision)")
    ap.add_argument("--key", default=None, help="table key prefix (default: --precision)")
    ap.add_argument("--build", default=None,
                    help="build id of the profiled library (default: the in-tree librrin_hip.so; set it when "
                         "re-deriving an entry from counter files of an earlier build)")
    a = ap.parse_args()
    fetch = load(a.fetch, "FETCH_SIZE")
    write = load(a.write, "WRITE_SIZE")
    fam = defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0, "dispatches": 0})
    for k, (v, n) in fetch.items():
        f = fam[family(k)]
        f["fetch_kib"] += v
        f["dispatches"] += n
    for k, (v, n) in write.items():
        fam[family(k)]["write_kib"] += v
    res = {}
    for k, f in fam.items():
        hbm = (2.0 * f["fetch_kib"] + f["write_kib"]) * 1024.0
        res[k] = {"hbm_bytes_per_step": hbm / a.steps, "dispatches_per_step": f["dispatches"] / a.steps,
                  "hbm_bytes_per_dispatch": hbm / max(f["dispatches"], 1),
                  "fetch_kib_raw": f["fetch_kib"], "write_kib_raw": f["write_kib"]}
        print(f"{k:28s} {res[k]['hbm_bytes_per_step'] / 1e9:9.3f} GB/step "
              f"{res[k]['dispatches_per_step']:6.1f} dispatches/step")
    if a.out:
        json.dump({"correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE = 1/2 of wide reads)",
                   "steps": a.steps, "kernels": res}, open(a.out, "w"), indent=1)
    if a.table:
        # the conv family = every body-conv kernel (bench.py's roofline covers all 77 body
        # convs of a forward part): exact fp32 runs the Winograd tiles (kinds 3/4:
        # conv3x3_winoq_kernel, 6/7: conv3x3_winoc_kernel, 14: conv3x3_winoc42_kernel) and the direct-form first conv
        # (fp16: the fused level-0 UNetConvBlock kernel runs 2 body convs per launch -- omitting it
        # dropped a third of the C3 conv bytes from the round-5 line)
        fam_name = a.family or {"fp32_planar": "conv3x3_mfma_kernel",
                                "fp32": "conv3x3_winoq_kernel,conv3x3_winoc_kernel,conv3x3_winoc42_kernel,conv3x3_h8_kernel",
                                "fp16": "conv3x3_h8_kernel,conv3x3_winoh_kernel,conv_block0_h8_kernel"}.get(
            a.precision, "conv3x3_h8_kernel")
        names = [n for n in fam_name.split(",") if n in res]
        if not names:
            sys.exit(f"no kernel of family {fam_name} in the counter files")
        hbm_step = sum(res[n]["hbm_bytes_per_step"] for n in names)
        launches = sum(res[n]["dispatches_per_step"] for n in names)
        tab = json.load(open(a.table)) if os.path.exists(a.table) else {}
        tab[f"{a.key or a.precision}@{a.config}"] = {
            "kernel_family": ",".join(names), "hbm_bytes_per_launch": hbm_step / max(launches, 1e-9),
            "hbm_bytes_per_step": hbm_step, "launches_per_step": launches,
            "per_kernel": {n: {"hbm_bytes_per_step": res[n]["hbm_bytes_per_step"],
                               "launches_per_step": res[n]["dispatches_per_step"]} for n in names},
            "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB, separate --pmc passes",
            "source": os.path.basename(os.path.normpath(a.fetch)) + " + " + os.path.basename(os.path.normpath(a.write)),
            # the library the profiled runs loaded (bench.py reports this entry only for that build)
            "build": a.build or build_id()}
        json.dump(tab, open(a.table, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
