#!/bin/bash
# Round 3: 4-waves-per-SIMD Winograd tile (cfg 20) vs cfg 18 / cfg 19
set -u
O=gpurun_out/r03f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread > $O/tests_h8.log 2>&1
rc=$?; echo "h8 rc=$rc"; tail -2 $O/tests_h8.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/tests_h8.log | head -5; exit 1; }
SH=256:256:3:1,64:32:0:1,32:32:0:1,128:64:1:1,512:512:4:1,32:32:0:2,128:128:2:2,512:1024:4:4,128:256:2:4,64:128:1:4,32:64:1:1,512:256:3:0,16:32:0:1
timeout -k 10 300 python -u tools/conv_lab.py cfgab --cfgs 18,20 --batch 2 --reps 10 --rounds 5 --shapes $SH > $O/cfgab_18_20.log 2>&1
echo "cfgab 18/20 rc=$?"; grep -v amdgpu.ids $O/cfgab_18_20.log
timeout -k 10 300 python -u tools/conv_lab.py cfgab --cfgs 18,19 --batch 2 --reps 10 --rounds 5 --shapes 512:256:3:0,512:256:3:1,256:256:3:2,256:128:2:1 > $O/cfgab_18_19.log 2>&1
echo "cfgab 18/19 rc=$?"; grep -v amdgpu.ids $O/cfgab_18_19.log
