#!/bin/bash
# profiler with one event record per launch (start shared with the previous launch's end)
set -u
O=gpurun_out/r03aa; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_concurrency.py -x -q --timeout 200 --timeout-method thread
run c1 200 python bench.py --cpu-baseline off --no-alt
run c2 200 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt
run m 200 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-alt
