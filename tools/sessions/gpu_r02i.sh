#!/bin/bash
# H8 head whole-record stores: GPU tests of the record paths, head PMC traffic (split16 default config)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
run pmc_fetch_s16 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_s16 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision fp32_split16
run pmc_write_s16 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_s16 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision fp32_split16
python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_s16 --write gpurun_out/pmc_write_s16 --steps 3 --out gpurun_out/traffic_s16.json --precision fp32_split16 > gpurun_out/pmc_summary_s16.log 2>&1; cat gpurun_out/pmc_summary_s16.log
run bench_s16 300 python bench.py --steps 10 --warmup 3 --precision fp32_split16 --cpu-baseline off --no-alt
