#!/bin/bash
# Round 5: kind 13 (fp16 Winograd, two patch tiles per workgroup, U shared through LDS): bitwise
# tests against kind 6, per-conv A/B at the C3 part size (direct tiles 10 / 11, kind 6 = cfg 23,
# kind 13 = cfg 30), then the C3 forward with kind 13 at levels 3-4 / 2-4 vs the default.
set -u
O=${O:-gpurun_out/r05v}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_winoh.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
SH=32:64:1:1,64:64:1:2,64:64:1:3,128:64:1:1,64:128:2:1,128:128:2:2,128:128:2:3,256:128:2:1,128:256:3:1,256:256:3:1,256:256:3:3,512:256:3:0,256:512:4:1,512:512:4:1,64:128:0:4,128:256:1:4,256:512:2:4
timeout -k 10 400 python -u tools/conv_lab.py cfgab --precision fp16 --height 736 --width 1280 --batch 2 --cfgs 10,11,23,30 --shapes $SH --rounds 5 --reps 3 > $O/cfgab.log 2>&1; echo "cfgab rc=$?"
grep -v amdgpu $O/cfgab.log | cut -c1-170
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run c3_def$r 200 $C3
  run c3_k13l34$r 200 $C3 --wino-f16-kind 13 --wino-f16-levels 3,4
  run c3_k13l234$r 200 $C3 --wino-f16-kind 13 --wino-f16-levels 2,3,4
done
