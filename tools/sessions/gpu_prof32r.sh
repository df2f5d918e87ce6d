#!/bin/bash
# headline (exact fp32 records, 1280x720 x4, 2 streams): rocprofv3 kernel stats,
# PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes), default bench line
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run prof32r 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32r -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
run pmc_fetch_fp32 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_fp32 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision fp32
run pmc_write_fp32 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_fp32 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision fp32
python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_fp32 --write gpurun_out/pmc_write_fp32 --steps 3 --out gpurun_out/traffic_fp32.json --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 > gpurun_out/pmc_summary_fp32.log 2>&1; cat gpurun_out/pmc_summary_fp32.log
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
run bench_default 600 python bench.py --steps 20 --warmup 5
