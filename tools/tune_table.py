#!/usr/bin/env python3
"""Turn a `conv_lab.py tune` JSON into a tile table for engine.H8_TUNED and compare it
with the table in use: per conv shape (cin, rows, level; the epilogue variants of one
shape summed, weighted by how often the Net runs them) the fastest config, and the
schedule time of the current vs the new choice.

  python3 tools/tune_table.py gpurun_out/r04t/tune_fp16_1280x736x2.json --precision fp16

(Round 4 rewrite of the round-1 tool: same per-key choice -- the config with the least
schedule-weighted time over the key's epilogue variants -- plus the comparison.)
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("json")
    ap.add_argument("precision_pos", nargs="?", default=None, help="the precision, positionally (older usage)")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--height", type=int, default=736)
    ap.add_argument("--width", type=int, default=1280)
    a = ap.parse_args()
    if a.precision_pos:
        a.precision = a.precision_pos
    from rrin_amd import _lib, engine
    from tools.conv_lab import schedule
    prec = _lib.PRECISIONS[a.precision]
    cur = engine.H8_TUNED[prec]
    rows = json.load(open(a.json))
    t = {}
    for r in rows:
        kout = 4 * r["cout"] if r["epi"] == 4 else r["cout"]
        lvl = r["level"] + 1 if r["epi"] == 4 else r["level"]  # sub-pixel: the low-res grid
        t[(r["cin"], kout, lvl, r["epi"], r["cfg"])] = r["ms"]
    # how often each (shape, epi) runs per forward
    count = collections.Counter()
    for e in schedule(a.height, a.width, True):
        if e[5] < 0:
            continue
        cin, cout, L, src, epi = e[2], e[3], e[4], e[5], e[6]
        kout = 4 * cout if epi == 4 else cout
        lvl = L + 1 if epi == 4 else L
        count[(cin, kout, lvl, epi)] += 1
    shapes = collections.defaultdict(list)
    for (cin, kout, lvl, epi), c in count.items():
        shapes[(cin, kout, lvl)].append((epi, c))
    new, tot_cur, tot_new = {}, 0.0, 0.0
    for key in sorted(shapes):
        cfgs = {k[4] for k in t if k[:3] == key}
        def cost(cfg):
            s = 0.0
            for epi, c in shapes[key]:
                ms = t.get(key + (epi, cfg))
                if ms is None:
                    return None
                s += c * ms
            return s
        costs = {c: cost(c) for c in cfgs if cost(c) is not None}
        if not costs:
            continue
        best = min(costs, key=costs.get)
        c0 = cur.get(key)
        cc = costs.get(c0)
        new[key] = best
        tot_new += costs[best]
        tot_cur += cc if cc is not None else costs[best]
        flag = "" if best == c0 else f"  <- was cfg {c0} ({cc:.3f} ms)" if cc is not None else f"  <- was cfg {c0}"
        print(f"{key}: cfg {best} {costs[best]:.3f} ms{flag}")
    print(f"schedule sum: current {tot_cur:.3f} ms, new {tot_new:.3f} ms")
    print("table:", "{" + ", ".join(f"{k}: {v}" for k, v in sorted(new.items())) + "}")


if __name__ == "__main__":
    main()
