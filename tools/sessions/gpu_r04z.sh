#!/bin/bash
# Round 4 final validation of the committed build: GPU suite, smoke, default bench
# (headline), C2, C3 fp16, training line, rocprofv3 kernel stats of the default bench,
# PMC HBM traffic (separate FETCH / WRITE passes -> profiles/pmc_traffic.json keyed by
# the build) and SQ counters of the conv kernels (one summary per pass).
set -u
O=${O:-gpurun_out/r04z}; mkdir -p $O; export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,c2,c3,train,prof,pmc,sq}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -3 | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *tests* ]] && run tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 400 python bench.py && run bench_2 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt
[[ $STEPS == *c2* ]] && run bench_c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5
[[ $STEPS == *c3* ]] && run bench_c3 300 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off
[[ $STEPS == *train* ]] && run bench_train 300 python bench.py --train --steps 5 --warmup 2
B5="python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt"
[[ $STEPS == *prof* ]] && run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $B5 \
  && { KS=$(ls $O/prof/*/*kernel_stats.csv $O/prof/*kernel_stats.csv 2>/dev/null | head -1 || true)
       KT=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1 || true)
       python3 tools/kernel_family_stats.py $KS $KT 7 conv3x3_winoc_kernel > $O/kernel_family.txt 2>&1; head -12 $O/kernel_family.txt; }
B2="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
if [[ $STEPS == *pmc* ]]; then
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B2
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B2
  python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp32.json \
    --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 > $O/pmc_summary_fp32.txt 2>&1
  cat $O/pmc_summary_fp32.txt; cp profiles/pmc_traffic.json $O/pmc_traffic.json
fi
if [[ $STEPS == *sq* ]]; then
  run pmc_sq1 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq1 -o run -- $B2
  run pmc_sq2 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d $O/pmc_sq2 -o run -- $B2
  for f in conv3x3_winoc_kernel conv3x3_winoq_kernel; do
    for d in pmc_sq1 pmc_sq2; do
      python3 tools/pmc_counters.py $O/$d --family $f --mfma-cycles 64 > $O/sum_${d}_$f.txt 2>&1
    done
  done
  cat $O/sum_pmc_sq1_*.txt | cut -c1-200
fi
exit 0
