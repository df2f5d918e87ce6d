#!/bin/bash
# Round 4 session w: SQ counters and rocprofv3 kernel stats of the fp16 record conv at C3
# on build 41c687a5 (after the epilogue change), beside round 4's earlier
# profiles/r04/sum_pmc_sq*_fp16_c3.txt of the build before it.
set -u
O=${O:-gpurun_out/r04w}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc16_sq1 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc16_sq1 -o run -- $B
run pmc16_sq2 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d $O/pmc16_sq2 -o run -- $B
for d in pmc16_sq1 pmc16_sq2; do
  python3 tools/pmc_counters.py $O/$d --family conv3x3_h8_kernel --mfma-cycles 32 > $O/sum_$d.txt 2>&1
done
B5="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 5 --warmup 2 --cpu-baseline off --no-alt"
run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $B5 \
  && { KS=$(ls $O/prof/*/*kernel_stats.csv $O/prof/*kernel_stats.csv 2>/dev/null | head -1 || true)
       KT=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1 || true)
       cp "$KS" $O/kernel_stats_c3.csv
       python3 tools/kernel_family_stats.py $KS $KT 7 conv3x3_h8_kernel > $O/kernel_family_c3.txt 2>&1; head -12 $O/kernel_family_c3.txt; }
cat $O/sum_pmc16_sq1.txt $O/sum_pmc16_sq2.txt
exit 0
