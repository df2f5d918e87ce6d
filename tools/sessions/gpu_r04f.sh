#!/bin/bash
# Round 4 session f: BASELINE C2 (640x368 x 1) -- per-conv tile kinds and split-K at
# the C2 grid (conv_lab cfgab: kinds 3 / 4 / 6, splits of kinds 3 / 4), then whole C2
# forwards under the candidate policies.
set -u
O=${O:-gpurun_out/r04f}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -40 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run clock 300 python3 -u tools/clock_probe.py --shapes 256:256:3:1,128:64:1:1,512:512:4:1,128:128:2:2,512:256:3:0,256:128:2:1,64:64:1:3,32:64:1:1 --batch 2
run clock_c2 200 python3 -u tools/clock_probe.py --shapes 256:256:3:1,128:64:1:1,64:64:1:3,256:128:2:1 --batch 1 --height 368 --width 640 --seconds 2
SH=32:64:1:1,64:64:1:2,128:64:1:1,64:64:1:3,64:128:1:4,64:128:2:1,128:128:2:2,256:128:2:1,128:128:2:3,128:256:2:4
SH=$SH,128:256:3:1,256:256:3:1,256:256:3:2,512:256:3:0,256:256:3:3,256:512:3:4,256:512:4:1,512:512:4:1,512:1024:4:4
run c2_kinds 400 python3 -u tools/conv_lab.py cfgab --cfgs 20,21,23,20s2,21s2,21s4 --height 368 --width 640 --batch 1 --shapes $SH --rounds 7 --reps 10
run c2_l0 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,21,24 --height 368 --width 640 --batch 1 --shapes 16:32:0:1,32:32:0:2,64:32:0:1,32:32:0:1,64:128:0:4 --rounds 7 --reps 10
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run c2_default_$r 200 $C2
  run c2_k3_$r 200 $C2 --wino-kind 3
  run c2_k3_split_$r 200 $C2 --wino-kind 3 --wino-split 3:2,4:4
done
for f in $O/c2_default_* $O/c2_k3_*; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
run bench_default 300 python bench.py --steps 20 --warmup 5
exit 0
