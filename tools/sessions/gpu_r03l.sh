#!/bin/bash
# per-shape TH-4 table (engine.WINO_TH4): default bench and C2 with / without
set -u
O=gpurun_out/r03l; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run c1_th4 300 python bench.py --cpu-baseline off
run c1_no 300 python bench.py --cpu-baseline off --no-wino-th4
run c1_th4b 300 python bench.py --cpu-baseline off
run c2_th4 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off
run c2_no 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-wino-th4
run m_th4 300 python bench.py --batch 1 --streams 1 --cpu-baseline off
run m_no 300 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-wino-th4
exit 0
