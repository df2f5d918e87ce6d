#!/bin/bash
# Winograd split-K: parity, then C2 / 720p x1 / default forward with level splits
set -u
O=gpurun_out/r03s; mkdir -p $O; export TMPDIR=/tmp
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
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c2_k3 120 python bench.py $C2
run c2_s4 120 python bench.py $C2 --wino-split 4:4
run c2_s34 120 python bench.py $C2 --wino-split 3:2,4:4
run c2_s234 120 python bench.py $C2 --wino-split 2:2,3:4,4:8
run c2_s2348 120 python bench.py $C2 --wino-split 2:2,3:2,4:8
run m_k3 120 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-alt
run m_s34 120 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-alt --wino-split 3:2,4:4
run c1_s4 120 python bench.py --cpu-baseline off --no-alt --wino-split 4:2
