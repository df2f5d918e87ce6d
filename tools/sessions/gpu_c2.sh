set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_640x368x1.log 2>&1 && tail -1 gpurun_out/bench_c2_640x368x1.log && \
timeout -k 10 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 --precision fp32 --cpu-baseline off --no-alt > gpurun_out/bench_c2_640x368x1_fp32.log 2>&1 && tail -1 gpurun_out/bench_c2_640x368x1_fp32.log && \
timeout -k 10 300 python bench.py --batch 1 --streams 1 --steps 20 --warmup 5 --cpu-baseline off --no-alt > gpurun_out/bench_1280x720x1.log 2>&1 && tail -1 gpurun_out/bench_1280x720x1.log && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 10 --warmup 3 --cpu-baseline off --no-alt > gpurun_out/prof_c2.log 2>&1
