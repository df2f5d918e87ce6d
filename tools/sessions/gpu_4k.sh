set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --height 2176 --width 3840 --batch 1 --cpu-pairs 1 --no-alt > gpurun_out/bench_4k_split16.log 2>&1; echo "4k split16 rc=$?"
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --height 2176 --width 3840 --batch 1 --precision fp16 --cpu-baseline off --no-alt > gpurun_out/bench_4k_fp16.log 2>&1; echo "4k fp16 rc=$?"
