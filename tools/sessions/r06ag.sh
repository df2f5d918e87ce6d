#!/bin/bash
# Round 6 call ag: C2 with the coalesced kind-14 epilogue -- geometry split-K (kind 4 on the
# few-tile deep convs, default) vs kind 14 everywhere (--wino-split none).
set -u
O=gpurun_out/r06ag; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
C2="--height 368 --width 640 --batch 1 --steps 60 --warmup 10 --cpu-baseline off --no-alt"
for k in 1 2; do
run def_$k 200 python bench.py $C2
run nosplit_$k 200 python bench.py $C2 --wino-split none
run gdef_$k 200 python bench.py $C2 --graph
run gnosplit_$k 200 python bench.py $C2 --graph --wino-split none
done
exit 0
