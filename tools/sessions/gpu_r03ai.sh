#!/bin/bash
# edge fix cross-workgroup K split (fp32 runs of 64 channels, ticketed run-order sum)
set -u
O=gpurun_out/r03ai; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "rc $rc in $name; stopping"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_gpu_h8.py tests/test_subpixel.py tests/test_gpu_ringfold.py tests/test_gpu_net.py tests/test_gpu_split.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread
run trace 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-prof --no-alt
run c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt
run bench 300 python bench.py --cpu-baseline off --no-alt
