#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel family: every counter's
per-dispatch average, plus derived rates when their inputs are present.

  python tools/pmc_counters.py DIR [DIR ...] [--family conv3x3_wino_kernel] [--mfma-cycles 64]

Derived (MI355X_MICROARCH.md, rocprofv3 PMC rows):
  eff_clock_ghz  = GRBM_GUI_ACTIVE / 8 (XCDs) / dispatch duration
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / 8)
                   (SIMDs = 1024: 256 CUs x 4)
  waves_per_simd = SQ_WAVE_CYCLES (quad-cycles) x 4 / (SIMDs x GRBM_GUI_ACTIVE / 8)
  wait_any / wait_inst_any / active_inst_any = shares of SQ_WAVE_CYCLES
  lds_conflict   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (when both present)
  hbm_bytes      = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950 FETCH_SIZE
                   is half of a wide streaming read)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

SIMDS = 1024


def family(name):
    m = re.search(r"rrin::(\w+?)(<|\()", name)
    return m.group(1) if m else name[:48]


def load(dirs, fam_filter=None):
    """{family: {"n": dispatches, "dur_ns": sum, counter: sum}} (per dispatch, summed)."""
    per = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                fam = family(row["Kernel_Name"])
                if fam_filter and fam != fam_filter:
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                p = per[fam]
                if key not in seen[fam]:
                    seen[fam].add(key)
                    p["n"] += 1
                    try:
                        p["dur_ns"] += int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                    except (KeyError, ValueError):
                        pass
                p[row["Counter_Name"]] += float(row["Counter_Value"])
    return per


def derive(p, mfma_cycles=None):
    n = max(p["n"], 1)
    out = {"dispatches": int(p["n"]), "avg_dur_us": p["dur_ns"] / n / 1e3}
    grbm = p.get("GRBM_GUI_ACTIVE")
    if grbm:
        cyc = grbm / 8.0
        if p["dur_ns"]:
            out["eff_clock_ghz"] = cyc / p["dur_ns"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in p:
            out["mfma_busy"] = p["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
        if "SQ_WAVE_CYCLES" in p:
            out["waves_per_simd"] = p["SQ_WAVE_CYCLES"] * 4 / (SIMDS * cyc)
    wc = p.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in p:
                out[c.lower()[3:] + "_share"] = p[c] / wc
    if "SQ_LDS_BANK_CONFLICT" in p and p.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict"] = p["SQ_LDS_BANK_CONFLICT"] / p["SQ_LDS_IDX_ACTIVE"]
    if "FETCH_SIZE" in p or "WRITE_SIZE" in p:
        out["hbm_bytes_per_dispatch"] = (2 * p.get("FETCH_SIZE", 0.0) + p.get("WRITE_SIZE", 0.0)) * 1024 / n
    if mfma_cycles and "SQ_VALU_MFMA_BUSY_CYCLES" in p:
        out["mfma_insts_per_dispatch"] = p["SQ_VALU_MFMA_BUSY_CYCLES"] / mfma_cycles / n
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--family", default=None)
    ap.add_argument("--mfma-cycles", type=float, default=None,
                    help="busy cycles per MFMA (64: v_mfma_f32_32x32x2_f32) to count MFMAs per dispatch")
    a = ap.parse_args()
    per = load(a.dirs, a.family)
    for fam, p in sorted(per.items(), key=lambda kv: -kv[1]["dur_ns"]):
        n = max(p["n"], 1)
        d = derive(p, a.mfma_cycles)
        print(f"== {fam}  dispatches {d['dispatches']}  avg {d['avg_dur_us']:.1f} us")
        for k, v in d.items():
            if k not in ("dispatches", "avg_dur_us"):
                print(f"   {k:28s} {v:.4g}")
        for k, v in sorted(p.items()):
            if k not in ("n", "dur_ns"):
                print(f"   avg {k:24s} {v / n:.6g}")


if __name__ == "__main__":
    main()
