#!/bin/bash
# Round 6 call c: HIP-graph replay (RRINEngine.graph): its GPU tests, then C2 and the headline
# with --graph against eager, interleaved.
set -u
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_graph timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_net.py -m gpu -x -q --timeout 120 --timeout-method thread
C2="--height 368 --width 640 --batch 1 --steps 100 --warmup 10 --cpu-baseline off --no-alt"
step c2_eager1 timeout -k 10 200 python bench.py $C2
step c2_graph1 timeout -k 10 200 python bench.py $C2 --graph
step c2_eager2 timeout -k 10 200 python bench.py $C2
step c2_graph2 timeout -k 10 200 python bench.py $C2 --graph
H="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
step hl_eager1 timeout -k 10 200 python bench.py $H
step hl_graph1 timeout -k 10 200 python bench.py $H --graph
step hl_eager2 timeout -k 10 200 python bench.py $H
step hl_graph2 timeout -k 10 200 python bench.py $H --graph
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
step c3_eager1 timeout -k 10 200 python bench.py $C3
step c3_graph1 timeout -k 10 200 python bench.py $C3 --graph
step c2_graph_full timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --steps 100 --warmup 10 --graph
exit 0
