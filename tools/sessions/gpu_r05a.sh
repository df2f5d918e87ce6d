#!/bin/bash
# Round 5, first fp16 Winograd run: the record-conv GPU tests (every config incl. the fp16
# kind-6 tile against float64), per-conv A/B of the fp16 Winograd tile (cfg 23) against the
# direct-form tiles at the C3 part size (1280x736 x 2), C3 bench Winograd vs direct.
set -u
O=${O:-gpurun_out/r05a}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -4 | cut -c1-600
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run h8tests 400 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
SH=32:64:1:1,64:64:1:2,64:64:1:3,128:64:1:1,64:128:2:1,128:128:2:2,128:128:2:3,256:128:2:1,128:256:3:1,256:256:3:1,256:256:3:3,512:256:3:0,256:512:4:1,512:512:4:1,64:128:0:4,128:256:1:4,256:512:2:4
run cfgab 300 python -u tools/conv_lab.py cfgab --precision fp16 --height 736 --width 1280 --batch 2 --cfgs 10,11,4,23 --shapes $SH --rounds 5 --reps 5
run c3_wino 200 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --no-alt
run c3_direct 200 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --no-alt --cpu-baseline off --no-wino
