#!/bin/bash
# A/B: 720p x4 (2 streams, 2-pair parts = 1.84 Mpx) with the large tile table (default)
# vs the medium one (engine.MEDIUM_PX raised above the part size), interleaved.
set -u
mkdir -p gpurun_out
ARGS="--steps 10 --warmup 3 --cpu-baseline off --no-alt"
M='import sys; from rrin_amd import engine; engine.MEDIUM_PX = 2_000_000; sys.argv = ["bench.py"] + sys.argv[1:]; import bench; bench.main()'
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/cls_large_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -c "$M" $ARGS > gpurun_out/cls_medium_$r.log 2>&1 || exit 1
done
for f in gpurun_out/cls_*.log; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f'.split('/')[-1], d['value'], d['unprofiled']['value'])"; done
