#!/bin/bash
# Round 4 session l: C2 (640x368 x 1) tile / split choices for the convs the trace ranks
# highest: the 256 -> 4 x 128 sub-pixel up conv on the 46 x 80 grid (kind 4, 65 us),
# the split deep convs, the level-0 32-channel convs; the kind-3 tile with a 3-stage
# raw ring + 2-stage U ring (ab/librrin_hip_qs3.so, RRIN_WINOQ_STAGES=3).
set -u
O=${O:-gpurun_out/r04l}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -25 | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
L="--height 368 --width 640 --batch 1 --rounds 9 --reps 10"
run sub 200 python3 -u tools/conv_lab.py cfgab --cfgs 21,23,20,21s2,21s4,20s2,20s4 $L --shapes 256:512:2:4,128:256:1:4
run deep 300 python3 -u tools/conv_lab.py cfgab --cfgs 21,23,21s2,21s4,21s8 $L --shapes 256:256:3:1,256:256:3:3,512:256:3:1,512:256:3:0,512:512:4:1,256:512:4:1
run l0 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,24,23 $L --shapes 64:32:0:1,32:32:0:1,32:32:0:2,16:32:0:1,10:32:0:1
S3=64:32:0:1:20,32:32:0:1:20,32:32:0:2:20,16:32:0:1:20
run ab_s3_720 200 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_qs3.so --batch 2 --shapes $S3
run ab_s3_c2 200 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_qs3.so --batch 1 --height 368 --width 640 --shapes $S3
cp rrin_amd/librrin_hip.so $O/prod.so.bak
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  cp $O/prod.so.bak rrin_amd/librrin_hip.so && run bench_prod_$r 200 $B
  cp ab/librrin_hip_qs3.so rrin_amd/librrin_hip.so && run bench_s3_$r 200 $B
done
cp $O/prod.so.bak rrin_amd/librrin_hip.so && rm -f $O/prod.so.bak
for f in $O/bench_*; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
