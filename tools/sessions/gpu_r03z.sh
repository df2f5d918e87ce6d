#!/bin/bash
# first convs (cin 6/9/10/16 -> 32 at full resolution): Winograd cfg 20 vs the direct-form cfgs 9, 13, 15
set -u
O=gpurun_out/r03z; mkdir -p $O; export TMPDIR=/tmp
for c in 13 9 15; do
  timeout -k 10 200 python tools/conv_lab.py cfgab --cfgs 20,$c --precision fp32 --height 720 --width 1280 --batch 2 --shapes 6:32:0:1,9:32:0:1,10:32:0:1,16:32:0:1 --rounds 7 > $O/ab_$c.log 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_lab.py cfgab --cfgs 20,$c --precision fp32 --height 368 --width 640 --batch 1 --shapes 6:32:0:1,9:32:0:1,10:32:0:1,16:32:0:1 --rounds 7 > $O/ab_c2_$c.log 2>&1 || exit 1
done
grep -h 'cfg' $O/ab_*.log
