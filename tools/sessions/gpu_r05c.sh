#!/bin/bash
# Round 5: fp16 Winograd kinds 6 / 9 and their persistent forms 10 / 11 against the direct-form
# tiles, per conv at the C3 part size; the fp16 Winograd tests and record-conv GPU tests; the
# training tests and line.
set -u
O=${O:-gpurun_out/r05c}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -4 | cut -c1-600
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run winohtests 300 python -u -m pytest tests/test_gpu_winoh.py -x -v --timeout 120 --timeout-method thread
run h8tests 400 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
SH=32:64:1:1,64:64:1:2,64:64:1:3,128:64:1:1,64:128:2:1,128:128:2:2,128:128:2:3,256:128:2:1,128:256:3:1,256:256:3:1,256:256:3:3,512:256:3:0,256:512:4:1,512:512:4:1,64:128:0:4,128:256:1:4,256:512:2:4
run cfgab 400 python -u tools/conv_lab.py cfgab --precision fp16 --height 736 --width 1280 --batch 2 --cfgs 10,11,23,26,27,28 --shapes $SH --rounds 5 --reps 5
run traintests 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread
run bench_train 300 python bench.py --train --steps 5 --warmup 2
SH32=32:64:1:1,64:64:1:2,64:64:1:3,128:64:1:1,64:128:2:1,128:128:2:2,256:128:2:1,128:256:3:1,256:256:3:1,512:512:4:1,64:128:0:4,128:256:1:4,256:512:2:4
run cfgab32 400 python -u tools/conv_lab.py cfgab --precision fp32 --height 720 --width 1280 --batch 2 --cfgs 23,29 --shapes $SH32 --rounds 5 --reps 3
