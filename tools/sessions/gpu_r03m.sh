#!/bin/bash
# 3-stage DMA ring (cfg 20) vs 2 stages on the few-tile deep convs of 640x368 x 1
set -u
O=gpurun_out/r03m; mkdir -p $O; export TMPDIR=/tmp
S=64:128:2:1:20,128:128:2:2:20,256:128:2:1:20,256:512:2:4:20,128:256:3:1:20,256:256:3:1:20,256:256:3:2:20,512:256:3:1:20,512:1024:3:4:20,256:512:4:1:20,512:512:4:1:20
timeout -k 10 300 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_s3.so --precision fp32 --height 368 --width 640 --batch 1 --shapes $S --rounds 7 > $O/ab_s3_c2.log 2>&1; echo rc=$?
cat $O/ab_s3_c2.log | grep -v amdgpu.ids
