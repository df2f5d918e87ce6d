#!/bin/bash
# Round 6 call l: profiles of the kind-14 build -- PMC HBM traffic (separate FETCH / WRITE passes
# -> profiles/pmc_traffic.json for this build: headline and C2), rocprofv3 kernel stats of the
# headline, SQ counters of conv3x3_winoc42_kernel / conv3x3_winoq_kernel.
set -u
O=gpurun_out/r06l; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -2 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
msps() { python3 -c "import json,sys; l=[x for x in open('$1') if x.startswith('{')][-1]; print(json.loads(l)['ms_per_step'])"; }
run pytest_w42 300 python -u -m pytest tests/test_gpu_wino42.py -m gpu -x -q --timeout 120 --timeout-method thread
B2="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B2
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B2
python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp32.json \
  --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 > $O/pmc_summary_fp32.txt 2>&1; tail -3 $O/pmc_summary_fp32.txt
C2P="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o run -- $C2P
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o run -- $C2P
python3 tools/pmc_summary.py --fetch $O/c2_fetch --write $O/c2_write --steps 3 --out $O/traffic_c2.json \
  --table profiles/pmc_traffic.json --precision fp32 --config 640x368x1 > $O/pmc_summary_c2.txt 2>&1; tail -3 $O/pmc_summary_c2.txt
cp profiles/pmc_traffic.json $O/pmc_traffic.json
run bench 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt
run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
python3 tools/kernel_family_stats.py $O/prof/run_kernel_stats.csv $O/prof/run_kernel_trace.csv auto conv3x3_winoc42_kernel conv3x3_winoq_kernel --ms-per-step $(msps $O/prof.log) > $O/kernel_family.txt 2>&1; echo "family rc=$?"; tail -5 $O/kernel_family.txt
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA"
run pmc_sq1 240 rocprofv3 --pmc $SQ1 --output-format csv -d $O/pmc_sq1 -o run -- $B2
run pmc_sq2 240 rocprofv3 --pmc $SQ2 --output-format csv -d $O/pmc_sq2 -o run -- $B2
for d in pmc_sq1 pmc_sq2; do
  for f in conv3x3_winoc42_kernel conv3x3_winoq_kernel; do
    python3 tools/pmc_counters.py $O/$d --family $f --mfma-cycles 64 > $O/sum_${d}_$f.txt 2>&1
  done
done
head -20 $O/sum_pmc_sq1_conv3x3_winoc42_kernel.txt
# A/B: conv_winoc42.hip under the max-ilp machine scheduler (ab/librrin_hip_w42ilp.so)
SH="64:64:1:1,128:64:1:1,128:128:2:1,256:128:2:1,256:256:3:1,512:256:3:1,512:512:4:1,1024:512:4:1,256:512:2:4,64:32:0:1"
run cfg_ilp 300 env RRIN_LIB_AB=ab/librrin_hip_w42ilp.so python tools/conv_lab.py cfgab --cfgs 25,23 --batch 2 --rounds 5 --shapes $SH
run cfg_def 300 python tools/conv_lab.py cfgab --cfgs 25,23 --batch 2 --rounds 5 --shapes $SH
HL="--steps 20 --warmup 5 --cpu-baseline off --no-alt"
for k in 1 2; do
run hl_def$k 200 python bench.py $HL
run hl_ilp$k 200 env RRIN_LIB_AB=ab/librrin_hip_w42ilp.so python bench.py $HL
done
exit 0
