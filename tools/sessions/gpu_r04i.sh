#!/bin/bash
# Round 4 session i: stream count of the headline forward with the register-U default
# (4 pairs on 2 / 3 / 4 streams), interleaved on one box.
set -u
O=${O:-gpurun_out/r04i}; mkdir -p $O; export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  for s in 2 3 4; do
    timeout -k 10 200 $B --streams $s > $O/s${s}_$r.log 2>&1 || exit $?
  done
  timeout -k 10 200 $B --split 1,3 > $O/s13_$r.log 2>&1 || exit $?
done
for f in $O/s*.log; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
