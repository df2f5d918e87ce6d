#!/bin/bash
# Round 5: the persistent-tile tests with one workgroup per CU (ab/ BPC=1 builds, more tiles per
# workgroup) and the C3 forward with fp16 kind 10 at levels 3-4 (default build and BPC=1) with
# parity against the CPU oracle.
set -u
O=${O:-gpurun_out/r05i}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1) $(grep -o '"max_abs": [0-9.e-]*' $O/$name.log | head -1)"
  grep -E "passed|failed|Error" $O/$name.log | tail -2
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run t_default 300 python -u -m pytest tests/test_gpu_winoh.py -x -q --timeout 120 --timeout-method thread
RRIN_LIB_AB=ab/librrin_hip_hbpc1.so run t_hbpc1 300 python -u -m pytest tests/test_gpu_winoh.py -x -q --timeout 120 --timeout-method thread -k "not fp32"
RRIN_LIB_AB=ab/librrin_hip_bpc1.so run t_bpc1 300 python -u -m pytest tests/test_gpu_winoh.py -x -q --timeout 120 --timeout-method thread -k fp32
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 10 --warmup 3 --no-alt --cpu-pairs 1"
run c3_k10 300 $C3 --wino-f16-kind 10 --wino-f16-levels 3,4
RRIN_LIB_AB=ab/librrin_hip_hbpc1.so run c3_k10_b1 300 $C3 --wino-f16-kind 10 --wino-f16-levels 3,4
