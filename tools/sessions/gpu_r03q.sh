#!/bin/bash
# F(4x4) v2 (4-phase raw layout): parity, cfg 20 vs 22 timing, ablations
set -u
O=gpurun_out/r03q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread -k "wino or golden or pool or subpixel or rep or tail" > $O/h8.log 2>&1; echo "h8 rc=$?"; tail -2 $O/h8.log
S=32:32:0:1,64:32:0:1,128:64:1:1,256:128:2:1,256:256:3:1
timeout -k 10 300 python tools/conv_lab.py cfgab --cfgs 20,22 --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5 > $O/ab_c1.log 2>&1; echo rc=$?; grep -v amdgpu.ids $O/ab_c1.log
for abl in 0 3 4 8 12; do
  timeout -k 10 60 python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 30 --shape 256 128 2 1 22 --sched $abl 2>&1 | grep -v amdgpu.ids | sed "s/^/abl$abl /" | tee -a $O/abl.log
done
exit 0
