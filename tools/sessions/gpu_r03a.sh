#!/bin/bash
# Round 3, first call: counters of the round-2 Winograd conv (conv3x3_wino_kernel)
# at the headline config (1280x720 x4, 2 streams) and on single conv shapes,
# the HBM traffic passes, the kernel-trace summary and the default bench line.
set -u
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1; echo "list rc=$?"
run pmc_sq1 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq1 -o run -- $B
run pmc_sq2 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- $B
run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B
run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B
for shp in "256 256 3 1 18" "64 32 0 1 18" "32 32 0 1 18" "128 64 1 1 18"; do
  tag=$(echo $shp | tr ' ' '_')
  run sq_$tag 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/sq_$tag -o run -- python3 tools/conv_lab.py single --precision fp32 --batch 2 --reps 20 --shape $shp
done
run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
for d in pmc_sq1 pmc_sq2 pmc_fetch pmc_write; do
  python3 tools/pmc_counters.py $O/$d --family conv3x3_wino_kernel --mfma-cycles 64 > $O/sum_$d.txt 2>&1
done
for shp in 256_256_3_1_18 64_32_0_1_18 32_32_0_1_18 128_64_1_1_18; do
  python3 tools/pmc_counters.py $O/sq_$shp --family conv3x3_wino_kernel --mfma-cycles 64 > $O/sum_sq_$shp.txt 2>&1
done
run bench 400 python3 bench.py
exit 0
