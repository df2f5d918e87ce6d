#!/bin/bash
# Round 3: the 64-channel Winograd tile (cfg 19) vs cfg 18 -- record-conv parity
# (test_gpu_h8 runs every Winograd config), then cfg A/B (bitwise + timing),
# then the training tests.
set -u
O=gpurun_out/r03e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread > $O/tests_h8.log 2>&1
rc=$?; echo "h8 rc=$rc"; tail -3 $O/tests_h8.log
[ $rc -ne 0 ] && grep -E "^FAILED|Error" $O/tests_h8.log | head -5
timeout -k 10 300 python -u tools/conv_lab.py cfgab --cfgs 18,19 --batch 2 --reps 10 --rounds 5 --shapes 256:256:3:1,128:64:1:1,128:128:2:2,512:512:4:1,256:512:4:1,512:1024:4:4,128:256:2:4,64:128:1:4,32:64:1:1,64:64:1:3 > $O/cfgab.log 2>&1
echo "cfgab rc=$?"; grep -v amdgpu.ids $O/cfgab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q --timeout 180 --timeout-method thread > $O/train.log 2>&1
echo "train rc=$?"; tail -3 $O/train.log
