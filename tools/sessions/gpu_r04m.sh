#!/bin/bash
# Round 4 session m: phase stamps of the kind-3 tile on the level-0 32-channel convs
# (ab/librrin_hip_qclk.so): where a workgroup's life goes (chunk-0 wait, main loop,
# epilogue + stores) and how the launch's workgroups start.
set -u
O=${O:-gpurun_out/r04m}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/clock_probe.py --kernel winoq --cfg 20 --batch 2 --shapes 64:32:0:1,32:32:0:1,32:32:0:2,16:32:0:1,256:256:3:1 > $O/qclk_720.log 2>&1; echo "rc=$?"
timeout -k 10 200 python3 -u tools/clock_probe.py --kernel winoq --cfg 20 --batch 1 --height 368 --width 640 --seconds 2 --shapes 64:32:0:1,32:32:0:1,16:32:0:1 > $O/qclk_c2.log 2>&1; echo "rc=$?"
cat $O/qclk_720.log $O/qclk_c2.log | grep -v amdgpu.ids
