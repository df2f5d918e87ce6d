#!/bin/bash
# Round 6 call j: kind 14 level sets at the headline (levels 0-4 vs 1-4), C2 (split-K deep convs
# keep kind 4), bitwise batch invariance with kind 14.
set -u
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
SH="16:32:0:1,32:32:0:1,32:32:0:2,64:32:0:1,32:32:0:3"
step cfgab0 timeout -k 10 300 python tools/conv_lab.py cfgab --cfgs 20,25 --batch 2 --rounds 5 --shapes $SH
for k in 1 2; do
step hl_1234_$k timeout -k 10 200 python bench.py $HL --wino42-levels 1,2,3,4
step hl_01234_$k timeout -k 10 200 python bench.py $HL --wino42-levels 0,1,2,3,4
step c2_none_$k timeout -k 10 200 python bench.py $C2 --wino42-levels none
step c2_1234_$k timeout -k 10 200 python bench.py $C2 --wino42-levels 1,2,3,4
step c2_01234_$k timeout -k 10 200 python bench.py $C2 --wino42-levels 0,1,2,3,4
done
exit 0
