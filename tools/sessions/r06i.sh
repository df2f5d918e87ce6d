#!/bin/bash
# Round 6 call i: the Winograd F(4,3) x F(2,3) register-U tile (kind 14, conv_winoc42.hip):
# kernel sweeps vs float64, per-conv time vs kind 6 at the headline part size, whole-forward A/B.
set -u
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_h8 timeout -k 10 400 python -u -m pytest tests/test_gpu_h8.py -m gpu -x -q --timeout 120 --timeout-method thread
SH="64:64:1:1,128:64:1:1,128:128:2:1,256:128:2:1,256:256:3:1,512:256:3:1,512:512:4:1,1024:512:4:1,64:64:1:2,128:128:2:2,256:256:3:2,128:256:1:4,256:512:2:4,512:1024:3:4"
step cfgab timeout -k 10 400 python tools/conv_lab.py cfgab --cfgs 23,25 --batch 2 --rounds 5 --shapes $SH
step cfgab_agpr env RRIN_LIB_AB=ab/librrin_hip_w42agpr.so timeout -k 10 400 python tools/conv_lab.py cfgab --cfgs 23,25 --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
step hl_none timeout -k 10 200 python bench.py $HL --wino42-levels none
step hl_1234 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-pairs 1 --no-alt --wino42-levels 1,2,3,4
step hl_23 timeout -k 10 200 python bench.py $HL --wino42-levels 2,3
step hl_123 timeout -k 10 200 python bench.py $HL --wino42-levels 1,2,3
step hl_1234_agpr env RRIN_LIB_AB=ab/librrin_hip_w42agpr.so timeout -k 10 200 python bench.py $HL --wino42-levels 1,2,3,4
step hl_none2 timeout -k 10 200 python bench.py $HL --wino42-levels none
exit 0
