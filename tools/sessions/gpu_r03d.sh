#!/bin/bash
# Round 3: training-path kernels (tests/test_gpu_train.py) and the documented ABI stub
set -u
O=gpurun_out/r03d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_abi_stub.py -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1
echo "rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -40
