#!/bin/bash
# Round 6 call aj: with kind 14's level-4 tail gone, the stream split again (1 / 2 / 4 streams at
# the headline part), 16 x 16 tiles at every level (--wino42-geom 2), and per conv tall vs wide at
# levels 0-3 (abconv, the forced-16x16 library as B).
set -u
O=gpurun_out/r06aj; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -8 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run s2_$k 200 python bench.py $HL
run s1_$k 200 python bench.py $HL --streams 1
run s4_$k 200 python bench.py $HL --streams 4
run tall_$k 200 python bench.py $HL --wino42-geom 2
done
SH="32:32:0:1:25,64:32:0:1:25,64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:256:3:1:25,512:256:3:1:25,256:512:2:4:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_tall.so --batch 2 --rounds 5 --shapes $SH
exit 0
