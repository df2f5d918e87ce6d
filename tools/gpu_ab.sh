mkdir -p gpurun_out
N='{}'
T='{"(32,32,0)": 8, "(32,64,1)": 10, "(64,32,0)": 15, "(128,256,2)": 13, "(256,128,2)": 10}'
for i in 1 2; do
timeout -k 10 300 python tools/bench_ab.py "$N" -- --steps 10 --warmup 3 --cpu-baseline off --no-alt > gpurun_out/ab_base_$i.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ab.py "$T" -- --steps 10 --warmup 3 --cpu-baseline off --no-alt > gpurun_out/ab_new_$i.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ab.py "$N" -- --steps 10 --warmup 3 --cpu-baseline off --no-alt --no-prof > gpurun_out/ab_base_noprof_$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_*.log; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"conv_ms_per_step": [0-9.]*' $f); done
