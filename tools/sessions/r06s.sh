#!/bin/bash
# Round 6 call s: kind 14's A^T_y exchange with three reads per record (24 instead of 32 per lane)
# vs the previous build; the headline on 1 stream vs 2.
set -u
O=gpurun_out/r06s; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run t42 300 python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q --timeout 120 --timeout-method thread
SH="32:32:0:1:25,64:64:1:1:25,128:64:1:1:25,256:256:3:1:25,64:64:1:2:25"
run abconv 300 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_prev.so --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_new$k 200 python bench.py $HL
run hl_prev$k 200 env RRIN_LIB_AB=ab/librrin_hip_prev.so python bench.py $HL
run hl_s1_$k 200 python bench.py $HL --streams 1
done
exit 0
