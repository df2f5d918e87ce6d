#!/bin/bash
# Round 5: fused level-0 block without the B-operand mask and the conv-a range check: tests,
# isolated timing, C3 A/B in the two-stream forward.
set -u
O=${O:-gpurun_out/r05p}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_block0.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/block0_lab.py > $O/lab.log 2>&1; echo "lab rc=$?"; grep cin $O/lab.log
RRIN_LIB_AB=ab/librrin_hip_a63.so timeout -k 10 120 python -u tools/block0_lab.py > $O/lab_a63.log 2>&1; echo "lab a63 rc=$?"; grep cin $O/lab_a63.log
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c3_f1 200 $C3 --fuse-l0 1
run c3_f0 200 $C3 --fuse-l0 0
run c3_f1b 200 $C3 --fuse-l0 1
run c3_f0b 200 $C3 --fuse-l0 0
