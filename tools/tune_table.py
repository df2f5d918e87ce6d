"""Derive the H8 tile-config table (engine.H8_TUNED keys: (cin, cout rows, grid
level)) from a `conv_lab.py tune` sweep: per key the config with the least
summed time over the schedule's convs of that key (only configs valid for every
epilogue mode of the key).

  python tools/tune_table.py gpurun_out/tune_split.json [fp32_split16]"""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import _lib  # noqa: E402
from rrin_amd.engine import H8_TUNED  # noqa: E402
from tools.conv_lab import schedule  # noqa: E402


def main(path, precision="fp32_split16"):
    r = json.load(open(path))
    cnt = collections.Counter((e[2], e[3], e[4], e[6]) for e in schedule(720, 1280, True) if e[5] >= 0)
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    variants = collections.defaultdict(set)
    have = collections.defaultdict(lambda: collections.defaultdict(set))
    ncfg = _lib.lib().rrin_conv_h8_cfg_count()
    for e in r:
        if e["cfg"] >= ncfg:  # a config of an older build, not in this library
            continue
        k = (e["cin"], 4 * e["cout"], e["level"] + 1) if e["epi"] == 4 else (e["cin"], e["cout"], e["level"])
        by[k][e["cfg"]] += e["ms"] * cnt[(e["cin"], e["cout"], e["level"], e["epi"])]
        variants[k].add(e["epi"])
        have[k][e["cfg"]].add(e["epi"])
    cur = H8_TUNED[_lib.PRECISIONS[precision]]
    new, tc, tn = {}, 0.0, 0.0
    for k, v in sorted(by.items()):
        ok = {c: t for c, t in v.items() if have[k][c] == variants[k]}
        b = min(ok, key=ok.get)
        c = cur.get(k)
        print(k, "cur", c, f"{ok.get(c, float('nan')):.3f}", "best", b, f"{ok[b]:.3f}")
        tc += ok.get(c, 0.0)
        tn += ok[b]
        new[k] = b
    print(f"sum over the schedule: current {tc:.3f} ms, best {tn:.3f} ms")
    print(json.dumps({str(k).replace(" ", ""): v for k, v in new.items() if cur.get(k) != v}))
    print("full table:", {k: new[k] for k in sorted(new)})


if __name__ == "__main__":
    main(*sys.argv[1:])
