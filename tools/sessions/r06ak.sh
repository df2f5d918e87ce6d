#!/bin/bash
# Round 6 call ak: the headline-size batch bitwise test (level-4 geometry follows the batch), and
# the 16 x 16 level-4 tiles for a one-stream two-pair caller (auto vs forced 32 x 8, interleaved).
set -u
O=gpurun_out/r06ak; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -4 | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
run tnet 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -q -k "bitwise_1280x720" --timeout 200 --timeout-method thread
B="--batch 2 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run b2s1_auto$k 200 python bench.py $B
run b2s1_wide$k 200 python bench.py $B --wino42-geom 1
done
exit 0
