#!/bin/bash
# Round 3: fp16 BASELINE configs C3 (1280x736 x4, 2 streams) and the C5 per-GPU
# share (3840x2176 x1): per-layer breakdown, PMC HBM traffic (separate FETCH /
# WRITE passes -> profiles/pmc_traffic.json), bench lines.
set -u
O=gpurun_out/r03g; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-400
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run bd_c3 240 python3 tools/conv_lab.py breakdown --precision fp16 --batch 2 --height 736 --width 1280 --reps 5
C3="python3 bench.py --precision fp16 --height 736 --width 1280 --batch 4 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
C5="python3 bench.py --precision fp16 --height 2176 --width 3840 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc_fetch_c3 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c3 -o run -- $C3
run pmc_write_c3 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c3 -o run -- $C3
run pmc_fetch_c5 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c5 -o run -- $C5
run pmc_write_c5 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c5 -o run -- $C5
cp profiles/pmc_traffic.json $O/pmc_traffic_before.json
python3 tools/pmc_summary.py --fetch $O/pmc_fetch_c3 --write $O/pmc_write_c3 --steps 3 --out $O/traffic_c3.json --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 > $O/pmc_summary_c3.txt 2>&1
python3 tools/pmc_summary.py --fetch $O/pmc_fetch_c5 --write $O/pmc_write_c5 --steps 3 --out $O/traffic_c5.json --table profiles/pmc_traffic.json --precision fp16 --config 3840x2176x1 > $O/pmc_summary_c5.txt 2>&1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
cat $O/pmc_summary_c3.txt $O/pmc_summary_c5.txt
run bench_c3 300 python3 bench.py --precision fp16 --height 736 --width 1280 --batch 4 --steps 10 --warmup 3 --cpu-baseline off
run bench_c5 300 python3 bench.py --precision fp16 --height 2176 --width 3840 --batch 1 --streams 1 --steps 5 --warmup 2 --cpu-baseline off
exit 0
