#!/bin/bash
# streams 1 (xlarge table, one 3.7 Mpx part) vs 2 (large table); 4K lines with the xxlarge tables
set -u
mkdir -p gpurun_out
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
  run x_s1_$r 300 python bench.py --steps 10 --warmup 3 --streams 1 --cpu-baseline off --no-alt
  run x_s2_$r 300 python bench.py --steps 10 --warmup 3 --streams 2 --cpu-baseline off --no-alt
done
run x_b8s2 300 python bench.py --steps 10 --warmup 3 --batch 8 --streams 2 --cpu-baseline off --no-alt
run x_4k_fp32 300 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --steps 3 --warmup 1 --cpu-baseline off --no-alt
run x_4k_fp16 300 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --steps 5 --warmup 2 --precision fp16 --cpu-baseline off --no-alt
run x_c3_fp16 300 python bench.py --height 736 --width 1280 --batch 4 --steps 10 --warmup 3 --precision fp16 --cpu-baseline off --no-alt
