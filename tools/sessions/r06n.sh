#!/bin/bash
# Round 6 call n: with kind 14, the headline's stream count (2 / 3 / 4) and HIP-graph replay;
# C3 / C5 fp16 on this build.
set -u
O=gpurun_out/r06n; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-260; [ $rc -eq 0 ] || exit $rc; }
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_s2_$k 200 python bench.py $HL --streams 2
run hl_s3_$k 200 python bench.py $HL --streams 3 --split 1,1,2
run hl_s4_$k 200 python bench.py $HL --streams 4
run hl_graph_$k 200 python bench.py $HL --graph
done
run c3 300 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt
run c5 300 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt
exit 0
