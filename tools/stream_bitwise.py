#!/usr/bin/env python3
"""Round-5 probe: is a forward bitwise the same on one stream and on two (its two parts' kernels
share CUs)?  Runs the Net at --height x --width x --batch in --precision with engine knobs, R
rounds of (1-stream, 2-stream) forwards, and reports how many 2-stream outputs differ from the
1-stream one, the max abs difference and whether the fp16 range flag fired.

  python tools/stream_bitwise.py --precision fp16 --wino-f16-levels 3,4
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import Net, engine  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="fp16")
ap.add_argument("--height", type=int, default=736)
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--wino-f16-levels", default=None)
ap.add_argument("--no-wino", action="store_true")
a = ap.parse_args()
if a.wino_f16_levels is not None:
    engine.WINO_F16_LEVELS = tuple(int(v) for v in a.wino_f16_levels.split(","))
if a.no_wino:
    engine.WINO = engine.WINO_F16 = False
dev = torch.device("cuda:0")
net = Net()
net.load_state_dict(keyed_state_dict(net.state_dict()), strict=True)
net = net.to(dev).eval()
net.precision = a.precision
eng = net.engine()
i0, i1 = synthetic_batch(a.batch, a.height, a.width, first_index=0)
i0, i1 = i0.to(dev), i1.to(dev)
bad, worst, flag = 0, 0.0, None
with torch.no_grad():
    ref = eng.forward(i0, i1, 0.5, streams=1)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        o1 = eng.forward(i0, i1, 0.5, streams=1)
        o2 = eng.forward(i0, i1, 0.5, streams=2)
        torch.cuda.synchronize()
        for o in (o1, o2):
            if not torch.equal(o, ref):
                bad += 1
                worst = max(worst, float((o - ref).abs().nan_to_num(1e30).max()))
    try:
        eng.check_range()
    except RuntimeError as e:
        flag = str(e)[:60]
print(f"differ {bad}/{2 * a.rounds} forwards from the first 1-stream one, max abs {worst:.3e}, range flag: {flag}")
sys.exit(1 if bad or flag else 0)
