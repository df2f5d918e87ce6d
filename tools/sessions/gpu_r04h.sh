#!/bin/bash
# Round 4 session h: epilogue bias loaded right after the main loop (kinds 3 and 6),
# geometry split-K, the INTEGRATION stub with caller scratch -- GPU suite, per-conv A/B
# against the previous build (ab/librrin_hip_prev.so), default bench and C2.
set -u
O=${O:-gpurun_out/r04h}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -25 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
S6=256:256:3:1:23,128:64:1:1:23,512:512:4:1:23,128:128:2:2:23,512:256:3:0:23,256:128:2:1:23,64:64:1:3:23,32:64:1:1:23
S3=64:32:0:1:20,32:32:0:1:20,32:32:0:2:20,16:32:0:1:20
run ab_bias 400 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_prev.so --batch 2 --shapes $S6,$S3
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
run bench_a 200 $B && run c2_a 200 $C2 && run bench_b 200 $B && run c2_b 200 $C2
for f in bench_a bench_b c2_a c2_b; do python3 -c "
import json,sys; l=[x for x in open('$O/$f.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
