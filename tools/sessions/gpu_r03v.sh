#!/bin/bash
# sub-pixel ring fold (sc1 hand-offs): parity (conv level, Net level), then fold on / off A/B
set -u
O=gpurun_out/r03v; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run fold 300 python -u -m pytest tests/test_gpu_ringfold.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread
run net 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread
run c1 200 python bench.py --cpu-baseline off --no-alt
run c1_nf 200 python bench.py --cpu-baseline off --no-alt --no-ring-fold
run c1b 200 python bench.py --cpu-baseline off --no-alt
run c1_nfb 200 python bench.py --cpu-baseline off --no-alt --no-ring-fold
run m 200 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-alt
run m_nf 200 python bench.py --batch 1 --streams 1 --cpu-baseline off --no-alt --no-ring-fold
C2="--height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
run c2 200 python bench.py $C2
run c2_nf 200 python bench.py $C2 --no-ring-fold
