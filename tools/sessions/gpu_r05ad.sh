#!/bin/bash
# Round 5: ring fix-up from scratch on a side stream beside the sub-pixel conv (RRIN_RING_MODE 1,
# the new default) -- targeted GPU tests, then interleaved A/B against the correction after the
# conv (mode 0) and the from-scratch fix after the conv (mode 2): C2, headline, C3
set -u
O=${O:-gpurun_out/r05ad}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_net.py tests/test_gpu_ringfold.py tests/test_gpu_configs.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"subpixel_ring_fix_ms_per_step": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  for m in 0 1 2; do RRIN_RING_MODE=$m run c2_m$m$r 200 $C2; done
  for m in 0 1; do RRIN_RING_MODE=$m run hl_m$m$r 200 $B; done
  for m in 0 1; do RRIN_RING_MODE=$m run c3_m$m$r 200 $C3; done
done
