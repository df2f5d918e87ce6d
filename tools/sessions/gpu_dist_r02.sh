#!/bin/bash
# Launcher rehearsal: bench.py under torch.distributed.run exactly as the driver's
# scaling run starts it (1 rank on the box's one GPU, RCCL), and --dist-init at
# world size 1 (all-gather + gather check through RCCL); then the C2 line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/torchrun_n1.log 2>&1
rc=$?; echo "torchrun n1 rc=$rc"; grep -o '"value": [0-9.]*\|"gather_check": [^,]*,[^,]*' gpurun_out/torchrun_n1.log | head -3
if [ $rc -ne 0 ]; then tail -20 gpurun_out/torchrun_n1.log; exit $rc; fi
timeout -k 10 300 python bench.py --dist-init --no-alt --cpu-baseline off > gpurun_out/dist_init.log 2>&1
rc=$?; echo "dist-init rc=$rc"; grep -o '"value": [0-9.]*\|"gather_check": {[^}]*}' gpurun_out/dist_init.log | head -3
if [ $rc -ne 0 ]; then tail -20 gpurun_out/dist_init.log; exit $rc; fi
timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --no-alt > gpurun_out/c2.log 2>&1
rc=$?; echo "c2 rc=$rc"; grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"direct_equivalent_tflops": [0-9.]*' gpurun_out/c2.log | head -4
exit $rc
