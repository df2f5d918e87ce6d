"""Kind-14 time per step by epilogue and grid size (= grid level) from a rocprofv3 kernel trace.

    python3 tools/kind14_by_grid.py <run_kernel_trace.csv> <steps in the trace>

Sums of launch durations (the two streams overlap, so they add to more than the step)."""
import collections
import csv
import sys


def main(path, steps):
    agg = collections.defaultdict(lambda: [0, 0.0])
    total = 0.0
    for r in csv.DictReader(open(path)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        total += d
        name = r["Kernel_Name"]
        if "conv3x3_winoc42_kernel" in name:
            targs = [t.strip() for t in name.split("<")[1].split(">")[0].split(",")]
            persist = len(targs) > 2 and targs[2] == "true"
            key = (int(targs[0]), int(targs[1]) * (-1 if persist else 1),
                   int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
            agg[key][0] += 1
            agg[key][1] += d
    k14 = sum(v[1] for v in agg.values())
    print(f"all kernels {total / steps:.3f} ms/step (sum of durations), kind 14 {k14 / steps:.3f}")
    print("epi  PCW (-8: persistent)  workgroups  launches/step  ms/step  share of kind 14  avg us")
    for (epi, pcw, wg), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{epi:3d} {pcw:4d}                  {wg:11d} {n / steps:14.1f} {ms / steps:8.3f} {ms / k14:17.3f} {1000 * ms / n:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
