#!/bin/bash
# Round 3 final validation (session 2): GPU suite, smoke, default bench, C2, 2-rank gloo rehearsal of
# the N>1 bench (bitwise gather check, parity + CPU baseline at N>1), kernel-trace
# stats and PMC counters (SQ, FETCH, WRITE) of the default forward.
set -u
O=${O:-gpurun_out/r03final}; mkdir -p $O; export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,c2,gloo,prof,pmc}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *tests* ]] && run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 400 python bench.py
[[ $STEPS == *c2* ]] && run bench_c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5
[[ $STEPS == *gloo* ]] && run gloo2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-alt
[[ $STEPS == *prof* ]] && run prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
if [[ $STEPS == *pmc* ]]; then
  run pmc_sq1 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq1 -o run -- $B
  run pmc_sq2 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- $B
  run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B
  run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B
  for d in pmc_sq1 pmc_sq2 pmc_fetch pmc_write; do
    python3 tools/pmc_counters.py $O/$d --family conv3x3_winoq_kernel --mfma-cycles 64 > $O/sum_$d.txt 2>&1
  done
  python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp32.json --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 --family conv3x3_winoq_kernel > $O/pmc_summary_fp32.txt 2>&1
  C2="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
  run pmc_fetch_c2 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c2 -o run -- $C2
  run pmc_write_c2 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c2 -o run -- $C2
  python3 tools/pmc_summary.py --fetch $O/pmc_fetch_c2 --write $O/pmc_write_c2 --steps 3 --out $O/traffic_fp32_c2.json --table profiles/pmc_traffic.json --precision fp32 --config 640x368x1 --family conv3x3_winoq_kernel > $O/pmc_summary_fp32_c2.txt 2>&1
  cp profiles/pmc_traffic.json $O/pmc_traffic.json
  cat $O/pmc_summary_fp32.txt $O/pmc_summary_fp32_c2.txt
fi
exit 0
