#!/bin/bash
# cfg 20 vs 22 (F(4x4)) on the Net's conv shapes at 1280x720 x 2
set -u
O=gpurun_out/r03o; mkdir -p $O; export TMPDIR=/tmp
S=32:32:0:1,32:32:0:2,64:32:0:1,16:32:0:1,64:128:0:4,32:64:1:1,64:64:1:2,128:64:1:1,128:256:1:4,64:128:2:1,128:128:2:2,256:128:2:1,256:512:2:4,128:256:3:1,256:256:3:1
timeout -k 10 300 python tools/conv_lab.py cfgab --cfgs 20,22 --precision fp32 --height 720 --width 1280 --batch 2 --shapes $S --rounds 5 > $O/ab_c1.log 2>&1
echo rc=$?; grep -v amdgpu.ids $O/ab_c1.log
