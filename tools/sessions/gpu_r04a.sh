#!/bin/bash
# Round 4 session a: the MFMA co-issue probe (tools/coissue_probe.*) and the SQ
# counters of the fp16 conv (conv3x3_h8_kernel) at the BASELINE C3 size.
set -u
O=${O:-gpurun_out/r04a}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run probe 180 python3 -u tools/coissue_probe.py
B="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc16_sq1 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc16_sq1 -o run -- $B
run pmc16_sq2 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d $O/pmc16_sq2 -o run -- $B
for d in pmc16_sq1 pmc16_sq2; do
  python3 tools/pmc_counters.py $O/$d --family conv3x3_h8_kernel --mfma-cycles 32 > $O/sum_$d.txt 2>&1
done
cat $O/probe.log $O/sum_pmc16_sq1.txt $O/sum_pmc16_sq2.txt
exit 0
