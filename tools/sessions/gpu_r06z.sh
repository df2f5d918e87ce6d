#!/bin/bash
# Round 6 final validation of the committed build.  Part A (STEPS=tests,smoke): GPU suite, smoke.
# Part B (STEPS=pmc,bench,c2,c3,train,prof,sq): PMC HBM traffic first (separate FETCH / WRITE
# passes -> profiles/pmc_traffic.json keyed by the build, so the bench lines after it carry
# `traffic`), the default bench (headline, CPU baseline + parity), C2, C3 fp16 with parity, the
# training line, rocprofv3 kernel stats of the headline and C3 (family unions checked against
# the profiled run's own ms_per_step) and SQ counters of the conv kernels.
set -u
O=${O:-gpurun_out/r06z}; mkdir -p $O; export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -2 | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
msps() { python3 -c "import json,sys; l=[x for x in open('$1') if x.startswith('{')][-1]; print(json.loads(l)['ms_per_step'])"; }
[[ $STEPS == *tests* ]] && run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [[ $STEPS == *pmc* ]]; then
  B2="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B2
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B2
  python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp32.json \
    --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 > $O/pmc_summary_fp32.txt 2>&1; tail -2 $O/pmc_summary_fp32.txt
  C2P="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o run -- $C2P
  run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o run -- $C2P
  python3 tools/pmc_summary.py --fetch $O/c2_fetch --write $O/c2_write --steps 3 --out $O/traffic_c2.json \
    --table profiles/pmc_traffic.json --precision fp32 --config 640x368x1 > $O/pmc_summary_c2.txt 2>&1; tail -2 $O/pmc_summary_c2.txt
  C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o run -- $C3P
  run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o run -- $C3P
  python3 tools/pmc_summary.py --fetch $O/c3_fetch --write $O/c3_write --steps 3 --out $O/traffic_c3.json \
    --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 > $O/pmc_summary_c3.txt 2>&1; tail -2 $O/pmc_summary_c3.txt
  cp profiles/pmc_traffic.json $O/pmc_traffic.json
fi
[[ $STEPS == *bench* ]] && run bench 400 python bench.py && run bench_2 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt
[[ $STEPS == *c2* ]] && run bench_c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5 && run bench_c2_graph 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 60 --warmup 10 --graph --cpu-baseline off --no-alt
[[ $STEPS == *c3* ]] && run bench_c3 400 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5
[[ $STEPS == *c5* ]] && run bench_c5 400 python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-pairs 1
[[ $STEPS == *train* ]] && run bench_train 300 python bench.py --train --steps 5 --warmup 2
if [[ $STEPS == *prof* ]]; then
  run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
  python3 tools/kernel_family_stats.py $O/prof/run_kernel_stats.csv $O/prof/run_kernel_trace.csv auto conv3x3_winoc42_kernel conv3x3_winoq_kernel --ms-per-step $(msps $O/prof.log) > $O/kernel_family.txt 2>&1; echo "family rc=$?"; tail -4 $O/kernel_family.txt
  run prof_c3 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 5 --warmup 2 --cpu-baseline off --no-alt
  python3 tools/kernel_family_stats.py $O/prof_c3/run_kernel_stats.csv $O/prof_c3/run_kernel_trace.csv auto conv3x3_h8_kernel conv_block0_h8_kernel conv3x3_winoh_kernel --parts 2 --ms-per-step $(msps $O/prof_c3.log) > $O/kernel_family_c3.txt 2>&1; echo "family c3 rc=$?"; tail -5 $O/kernel_family_c3.txt
fi
if [[ $STEPS == *sq* ]]; then
  B2="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  SQ2="SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA"
  run pmc_sq1 240 rocprofv3 --pmc $SQ1 --output-format csv -d $O/pmc_sq1 -o run -- $B2
  run pmc_sq2 240 rocprofv3 --pmc $SQ2 --output-format csv -d $O/pmc_sq2 -o run -- $B2
  run c3_sq1 240 rocprofv3 --pmc $SQ1 --output-format csv -d $O/c3_sq1 -o run -- $C3P
  run c3_sq2 240 rocprofv3 --pmc $SQ2 --output-format csv -d $O/c3_sq2 -o run -- $C3P
  for d in pmc_sq1 pmc_sq2; do
    for f in conv3x3_winoc42_kernel conv3x3_winoq_kernel; do
      python3 tools/pmc_counters.py $O/$d --family $f --mfma-cycles 64 > $O/sum_${d}_$f.txt 2>&1
    done
  done
  for d in c3_sq1 c3_sq2; do
    for f in conv3x3_h8_kernel conv_block0_h8_kernel conv3x3_winoh_kernel; do
      python3 tools/pmc_counters.py $O/$d --family $f --mfma-cycles 32 > $O/sum_${d}_$f.txt 2>&1
    done
  done
  head -8 $O/sum_c3_sq1_conv_block0_h8_kernel.txt
fi
exit 0
