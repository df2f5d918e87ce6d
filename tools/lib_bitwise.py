#!/usr/bin/env python3
"""Are two builds of librrin_hip.so bitwise the same on the Net?  Run once per build (the library
is loaded once per process; RRIN_LIB_AB selects an A/B build) with the same arguments:

  RRIN_LIB_AB=ab/librrin_hip_old.so python tools/lib_bitwise.py --save gpurun_out/a.pt
  python tools/lib_bitwise.py --compare gpurun_out/a.pt

Every precision's forward of --batch pairs at --height x --width (stress weights, t = 0.5 and a
per-pair t) is saved / compared with torch.equal; exit 1 on any difference."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import Net, _lib  # noqa: E402
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--save")
ap.add_argument("--compare")
ap.add_argument("--height", type=int, default=736)
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--precisions", default="fp16,fp32_split16,fp32")
a = ap.parse_args()
dev = torch.device("cuda:0")
net = Net()
net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True), strict=True)
net = net.to(dev).eval()
i0, i1 = synthetic_batch(a.batch, a.height, a.width, first_index=17)
i0, i1 = i0.to(dev), i1.to(dev)
res = {}
with torch.no_grad():
    for p in a.precisions.split(","):
        net.precision = p
        for t in (0.5, torch.linspace(0.1, 0.9, a.batch)):
            key = f"{p}@{'vec' if isinstance(t, torch.Tensor) else t}"
            res[key] = net(i0, i1, t).cpu()
        net.check_range()
print(f"library {_lib.LIB_PATH} build {_lib.build_id()}")
if a.save:
    torch.save(res, a.save)
    print(f"saved {len(res)} outputs")
if a.compare:
    ref = torch.load(a.compare, weights_only=True)
    bad = [k for k in res if not torch.equal(res[k], ref[k])]
    for k in res:
        print(f"{k:22s} {'bitwise equal' if k not in bad else 'DIFFERS max %.3e' % (res[k] - ref[k]).abs().max()}")
    sys.exit(1 if bad else 0)
