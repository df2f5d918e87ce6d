"""Phase-offset probe of the 2-stream batch split: the two parts run free
(no join per step) with the side stream started `offset` ms late
(torch.cuda._sleep), so their layer sequences are shifted against each other.
Prints pairs/s per offset (interleaved rounds).  Lab only: outputs are not used."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import Net  # noqa: E402
from rrin_amd.engine import t_coefficients  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).eval()
    net.precision = "fp32_split16"
    eng = net.engine()
    B, H, W, S = 4, 720, 1280, 20
    i0, i1 = synthetic_batch(B, H, W)
    i0, i1 = i0.to(dev), i1.to(dev)
    out = torch.empty_like(i0)
    coef = t_coefficients(0.5, B).to(dev)
    parts = [(0, 2), (2, 4)]
    wss = [eng.workspace(2, H, W, j) for j in range(2)]
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    # cycles per ms of the spin kernel (measured)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    torch.cuda._sleep(10_000_000)
    t1.record()
    torch.cuda.synchronize()
    cyc_per_ms = 10_000_000 / t0.elapsed_time(t1)

    def run(offset_ms, S=40, a=10, b=30):
        """Steady-state rate: each stream's forwards a..b timed by its own events
        (both streams are busy over that window for offsets <= ~a forwards)."""
        torch.cuda.synchronize()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            if offset_ms > 0:
                torch.cuda._sleep(int(offset_ms * cyc_per_ms))
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(S + 1)] for _ in range(2)]
        with torch.no_grad():
            for k in range(S):
                for j, (lo, hi) in enumerate(parts):
                    st = main_s if j == 0 else side
                    ev[j][k].record(st)
                    eng._forward_part(i0[lo:hi], i1[lo:hi], out[lo:hi], coef[lo:hi], j, wss[j], st, None, False)
        torch.cuda.synchronize()
        return sum(2 * (b - a) / (ev[j][a].elapsed_time(ev[j][b]) * 1e-3) for j in range(2))

    run(0)
    offsets = [0.0, 2.5, 5.0, 7.5, 10.0]
    res = {o: [] for o in offsets}
    for _ in range(3):
        for o in offsets:
            res[o].append(run(o))
    for o in offsets:
        v = sorted(res[o])
        print(f"offset {o:5.1f} ms: {v[1]:.1f} pairs/s  (runs {', '.join(f'{x:.1f}' for x in res[o])})", flush=True)


if __name__ == "__main__":
    main()
