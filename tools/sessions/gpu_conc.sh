#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_net.py -x -v -k "concurrency or streams or side_stream" --timeout 200 --timeout-method thread > gpurun_out/conc.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/conc.log | tail -12; [ $rc -ne 0 ] && exit $rc
# sensitivity: the same concurrency test against the old (packed-FP32) build, in a copy of the tree
rm -rf /tmp/pkrepo && cp -r . /tmp/pkrepo && cp rrin_amd/librrin_hip_pk.so /tmp/pkrepo/rrin_amd/librrin_hip.so
(cd /tmp/pkrepo && timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py -v --timeout 200 --timeout-method thread > /tmp/pk.log 2>&1); echo "old build rc=$?"; grep -E "PASS|FAIL|differ" /tmp/pk.log | tail -6
exit 0
