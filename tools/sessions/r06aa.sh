#!/bin/bash
# Round 6 call aa: C3 stream count on the last build (2 / 3 / 4 streams).
set -u
O=gpurun_out/r06aa; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run c3_s4_$k 200 python bench.py $C3 --streams 4
run c3_s2_$k 200 python bench.py $C3 --streams 2
run c3_s3_$k 200 python bench.py $C3 --streams 3 --split 1,1,2
done
exit 0
