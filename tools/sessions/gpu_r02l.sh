#!/bin/bash
# tile table A/B at the 2-stream default: large (2-pair sweep) vs xlarge (4-pair) vs xxlarge (4K)
set -u
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/$name.log | python3 -c "import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['unprofiled']['value'])
except Exception as e: print('no json', e)")"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in 1 2; do
  run t_large_$r 300 $B
  run t_xlarge_$r 300 $B --size-class xlarge
  run t_xxlarge_$r 300 $B --size-class xxlarge
done
