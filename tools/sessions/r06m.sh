#!/bin/bash
# Round 6 call m: kind-14 schedule variants (RRIN_WINO42_SCHED 1: point 5 interleaved with the next
# chunk's transform; 2: also the points 3-5 transform deferred beside point 0): correctness with
# each library, per-conv A/B (abconv, bitwise vs the default), whole-forward A/B.
set -u
O=gpurun_out/r06m; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -2 | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
for v in 1 2; do
run t_s$v 200 env RRIN_LIB_AB=ab/librrin_hip_w42s$v.so python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q --timeout 120 --timeout-method thread
done
SH="64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:128:2:1:25,256:256:3:1:25,512:256:3:1:25,512:512:4:1:25,1024:512:4:1:25,256:512:2:4:25,64:32:0:1:25"
run abconv 400 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_w42s1.so,ab/librrin_hip_w42s2.so --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_def$k 200 python bench.py $HL
run hl_s1_$k 200 env RRIN_LIB_AB=ab/librrin_hip_w42s1.so python bench.py $HL
run hl_s2_$k 200 env RRIN_LIB_AB=ab/librrin_hip_w42s2.so python bench.py $HL
done
exit 0
