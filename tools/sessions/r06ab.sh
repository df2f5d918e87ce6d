#!/bin/bash
# Round 6 call ab: after the 2-stream fp16 default -- GPU suite, fp16 stream bitwise, C3 PMC traffic
# (key fp16@1280x736x4s2) for this build, C3 with parity, C5.
set -u
O=gpurun_out/r06ab; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bitwise_fp16 240 python tools/stream_bitwise.py --precision fp16 --height 736 --width 1280 --batch 4 --rounds 4
C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o run -- $C3P
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o run -- $C3P
python3 tools/pmc_summary.py --fetch $O/c3_fetch --write $O/c3_write --steps 3 --out $O/traffic_c3.json \
  --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 > $O/pmc_summary_c3.txt 2>&1; tail -2 $O/pmc_summary_c3.txt
cp profiles/pmc_traffic.json $O/pmc_traffic.json
run bench_c3 400 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5
run bench_c5 400 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-pairs 1
run bench 400 python bench.py
exit 0
