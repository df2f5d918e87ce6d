#!/bin/bash
# fp32: streams 1 vs 2 (interleaved), RCCL world-1 trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | python3 -c "import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'] if d.get('roofline') else None)
except Exception as e: print('no json', e)"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
for r in 1 2; do
  run s1_$r 300 python bench.py --steps 10 --warmup 3 --streams 1 --cpu-baseline off --no-alt
  run s2_$r 300 python bench.py --steps 10 --warmup 3 --streams 2 --cpu-baseline off --no-alt
  run s3_$r 300 python bench.py --steps 10 --warmup 3 --streams 4 --cpu-baseline off --no-alt
done
run b8s2 300 python bench.py --steps 10 --warmup 3 --batch 8 --streams 2 --cpu-baseline off --no-alt
run nccl_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nccl_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --dist-init --dist-backend nccl --cpu-baseline off --no-alt --no-prof
