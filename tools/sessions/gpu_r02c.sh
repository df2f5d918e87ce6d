#!/bin/bash
# fp32 records, tuned table: GPU tests, bench, breakdown, ablations, clock/MFMA-busy counters
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run bench32r 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off
run brk32r 300 python tools/conv_lab.py breakdown --precision fp32 --batch 2 --out gpurun_out/brk32r.json
run abl32r 400 python tools/conv_lab.py ablate --precision fp32 --batch 2 --reps 5 --out gpurun_out/abl32r.json
for spec in "128 64 1 1 4 0 0" "128 64 1 1 4 11 0" "128 128 2 1 5 0 0" "128 128 2 1 5 11 0" "256 256 3 1 3 0 0"; do
  set -- $spec
  tag=clk32r_$1_$2_$3_$5_x$6
  run $tag 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/$tag -o run -- python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 40 --shape $1 $2 $3 $4 $5 --sched $6 --persist $7
done
