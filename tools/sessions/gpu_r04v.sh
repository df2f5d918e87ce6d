#!/bin/bash
# Round 4 session v: the C5 per-GPU share (3840x2176 x 1) on build 41c687a5, fp16 and
# exact fp32, after the fp16 epilogue change.
set -u
O=${O:-gpurun_out/r04v}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -2 | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run c5_fp16 300 python3 bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off
run c5_fp32 300 python3 bench.py --height 2176 --width 3840 --batch 1 --steps 5 --warmup 2 --cpu-baseline off
for f in $O/c5_*; do python3 -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], d.get('parity'))"; done
exit 0
