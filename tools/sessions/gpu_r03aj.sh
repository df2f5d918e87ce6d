#!/bin/bash
# edge fix cross split gated to grids <= 256 workgroups in the Net: tests, C2, default bench x2
set -u
O=gpurun_out/r03aj; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "rc $rc in $name; stopping"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_net.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread
run c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt
run bench1 300 python bench.py --cpu-baseline off --no-alt
run bench2 300 python bench.py --cpu-baseline off --no-alt
