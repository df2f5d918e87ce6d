#!/bin/bash
# Round 6 call f: the ring fix-up's cost bound at the headline (exact fp32, 2 streams) and at C2.
set -u
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
H="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
step hl_new1 timeout -k 10 200 python bench.py $H
step hl_noring1 env RRIN_LIB_AB=ab/librrin_hip_noring.so timeout -k 10 200 python bench.py $H
step hl_new2 timeout -k 10 200 python bench.py $H
step hl_noring2 env RRIN_LIB_AB=ab/librrin_hip_noring.so timeout -k 10 200 python bench.py $H
C2="--height 368 --width 640 --batch 1 --steps 100 --warmup 10 --cpu-baseline off --no-alt"
step c2_new1 timeout -k 10 200 python bench.py $C2
step c2_noring1 env RRIN_LIB_AB=ab/librrin_hip_noring.so timeout -k 10 200 python bench.py $C2
exit 0
