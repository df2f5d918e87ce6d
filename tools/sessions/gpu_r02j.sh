#!/bin/bash
# world-1 RCCL all-gather cost: interleaved A/B of --dist-init nccl vs no gather
set -u
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/$name.log | python3 -c "import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('unprofiled'), d.get('gather_check'))
except Exception as e: print('no json', e)")"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
for r in 1 2; do
  run g0_$r 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt
  run g1_$r 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt --dist-init --dist-backend nccl
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/nccl_trace -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline off --no-alt --no-prof --dist-init --dist-backend nccl > gpurun_out/nccl_trace.log 2>&1
echo "trace rc=$?"
