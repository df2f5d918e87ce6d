#!/bin/bash
# BASELINE config lines with the current build: fp16 1280x736x4 (C3), 4K fp16 /
# split16 (C5 per-GPU share), and a 2-rank rehearsal of the distributed bench on
# one GPU (gloo transport; the driver's N>1 runs use RCCL).
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --precision fp16 --height 736 --batch 4 --cpu-baseline off --no-alt > gpurun_out/bench_fp16_736x4.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --precision fp16 --height 2176 --width 3840 --batch 1 --streams 1 --cpu-baseline off --no-alt > gpurun_out/bench_4k_fp16.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --height 2176 --width 3840 --batch 2 --cpu-baseline off --no-alt > gpurun_out/bench_4k_split16.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --batch 2 --dist-backend gloo > gpurun_out/mgpu.log 2>&1 || exit 1
for f in bench_fp16_736x4 bench_4k_fp16 bench_4k_split16 mgpu; do echo "== $f"; grep '"metric"' gpurun_out/$f.log | cut -c1-400; done
