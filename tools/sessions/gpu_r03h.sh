#!/bin/bash
# Round 3: cfg 20 with a 3-stage LDS ring vs 2 stages (ab/librrin_hip_q2.so), then
# the default bench on the cfg 20 engine, GPU net tests
set -u
O=gpurun_out/r03h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread > $O/tests_h8.log 2>&1
rc=$?; echo "h8 rc=$rc"; tail -2 $O/tests_h8.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/tests_h8.log | head -5; exit 1; }
SH=256:256:3:1:20,64:32:0:1:20,32:32:0:1:20,128:64:1:1:20,512:512:4:1:20,32:32:0:2:20,128:128:2:2:20,512:1024:4:4:20,512:256:3:0:20,16:32:0:1:20
timeout -k 10 300 python -u tools/conv_lab.py abconv --lib ab/librrin_hip_q2.so --lib-b rrin_amd/librrin_hip.so --batch 2 --reps 10 --rounds 5 --shapes $SH > $O/ab_stages.log 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids $O/ab_stages.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests_net.log 2>&1
rc=$?; echo "net rc=$rc"; tail -2 $O/tests_net.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/tests_net.log | head -5; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
echo "bench rc=$?"; tail -1 $O/bench.log | cut -c1-300
