#!/bin/bash
# HW-queue mapping of the two forward streams with RCCL in the process
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
  run q_dist_base_$r 300 $B --dist-init --dist-backend nccl
  run q_dist_hw8_$r 300 $B --dist-init --dist-backend nccl --hw-queues 8
  run q_dist_prio_$r 300 $B --dist-init --dist-backend nccl --side-priority -1
  run q_nodist_$r 300 $B
  run q_nodist_hw8_$r 300 $B --hw-queues 8
done
