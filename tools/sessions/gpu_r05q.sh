#!/bin/bash
# Round 5: fused level-0 blocks, modes 0 / 1 (down_path[0]) / 2 (+ last up block): tests incl. the
# fp16 Net configs (the default now fuses), C3 and C5 A/B.
set -u
O=${O:-gpurun_out/r05q}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_block0.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run c3_f1$r 200 $C3 --fuse-l0 1
  run c3_f2$r 200 $C3 --fuse-l0 2
  run c3_f0$r 200 $C3 --fuse-l0 0
done
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt"
run c5_f1 300 $C5 --fuse-l0 1
run c5_f0 300 $C5 --fuse-l0 0
run c5_f2 300 $C5 --fuse-l0 2
