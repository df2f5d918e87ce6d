#!/bin/bash
# fp32 records: GPU tests, bench, breakdown + tile sweep at the 2-pair part size
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x
run bench32r 300 python bench.py --steps 10 --warmup 3 --precision fp32 --cpu-baseline off --no-alt
run brk32r 300 python tools/conv_lab.py breakdown --precision fp32 --batch 2 --out gpurun_out/brk32r.json
run tune32r 600 python tools/conv_lab.py tune --precision fp32 --batch 2 --out gpurun_out/tune32r.json
