#!/bin/bash
# Round 5: the Winograd conv concurrency test, default build and the BPC=1 builds
set -u
O=${O:-gpurun_out/r05k}; mkdir -p $O; export TMPDIR=/tmp
T="python -u -m pytest tests/test_gpu_winoh.py -q --timeout 200 --timeout-method thread -k side_stream"
timeout -k 10 300 $T > $O/conc_default.log 2>&1; echo "default rc=$?"; tail -3 $O/conc_default.log
RRIN_LIB_AB=ab/librrin_hip_hbpc1.so timeout -k 10 300 $T > $O/conc_hbpc1.log 2>&1; echo "hbpc1 rc=$?"; tail -3 $O/conc_hbpc1.log
RRIN_LIB_AB=ab/librrin_hip_bpc1.so timeout -k 10 300 $T > $O/conc_bpc1.log 2>&1; echo "bpc1 rc=$?"; tail -3 $O/conc_bpc1.log
