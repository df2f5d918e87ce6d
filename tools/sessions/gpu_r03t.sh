#!/bin/bash
# split-K parity + the GPU suite's Net / h8 files; C2 with the small-class split table
set -u
O=gpurun_out/r03t; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run split 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread
run net 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_h8.py tests/test_wino.py -x -q --timeout 120 --timeout-method thread
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c2 120 python bench.py $C2
run c2_none 120 python bench.py $C2 --wino-split none
run c2b 120 python bench.py $C2
