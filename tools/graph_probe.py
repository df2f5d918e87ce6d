"""Probe: does replaying a captured HIP graph of Net.forward beat enqueuing the
same ~96 launches per step?  Small, launch-gap-heavy workloads (C2 640x368 x1,
720p x1).  Static inputs/outputs (graph-captured pointers), no profiler events.

  python tools/graph_probe.py [--precision fp32_split16] [--steps 50]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import Net  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402


def timed(fn, steps, dev):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32_split16")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).eval()
    net.precision = args.precision
    eng = net.engine()
    for (b, h, w) in [(1, 368, 640), (1, 720, 1280), (4, 720, 1280)]:
        i0, i1 = synthetic_batch(b, h, w)
        i0, i1 = i0.to(dev), i1.to(dev)
        with torch.no_grad():
            ref = eng.forward(i0, i1, 0.5)
            for _ in range(3):
                eng.forward(i0, i1, 0.5)
            direct = timed(lambda: eng.forward(i0, i1, 0.5), args.steps, dev)
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):
                    eng.forward(i0, i1, 0.5)
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = eng.forward(i0, i1, 0.5)
            g.replay()
            torch.cuda.synchronize(dev)
            same = torch.equal(out, ref)
            graph = timed(g.replay, args.steps, dev)
        print(f"{w}x{h} x{b} {args.precision}: direct {direct:.3f} ms/step ({b / direct * 1e3:.1f} pairs/s), "
              f"graph replay {graph:.3f} ms/step ({b / graph * 1e3:.1f} pairs/s), bitwise equal {same}",
              flush=True)
        del g


if __name__ == "__main__":
    main()
