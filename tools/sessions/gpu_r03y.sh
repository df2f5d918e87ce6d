#!/bin/bash
# fp16 C3 (1280x736 x 4, 2 streams): current H8_TUNED[fp16] vs the table from the 1280x736 x 2 sweep, interleaved
set -u
O=gpurun_out/r03y; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
NEW='{(6,32,0):9,(9,32,0):9,(10,32,0):9,(16,32,0):13,(64,64,1):10,(64,128,1):11,(64,128,2):10,(128,64,1):11,(128,256,3):11,(256,128,2):10,(256,256,3):11,(256,512,3):10,(512,256,3):10}'
B='import sys, rrin_amd.engine as E; E.H8_TUNED[E._lib.PREC_F16].update(eval(sys.argv[1])); sys.argv = ["bench.py"] + sys.argv[2:]; import bench; bench.main()'
ARGS="--precision fp16 --height 736 --width 1280 --cpu-baseline off --no-alt"
for r in 1 2 3; do
  run old_$r 200 python bench.py $ARGS
  run new_$r 200 python -c "$B" "$NEW" $ARGS
done
run par_new 300 python -c "import sys, rrin_amd.engine as E; E.H8_TUNED[E._lib.PREC_F16].update(eval(sys.argv[1])); import pytest; sys.exit(pytest.main(['-x','-q','tests/test_gpu_configs.py','-k','c3 or fp16','--timeout','200']))" "$NEW"
