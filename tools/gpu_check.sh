#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel stats.
# Each GPU step has its own time limit; stop at the first crash/timeout
# (exit codes 124/134/137/139 or >128), continue past plain test failures (1).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench,prof}
[[ $STEPS == *tests* ]] && run tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
[[ $STEPS == *bsplit* ]] && run bench_split 600 python bench.py --steps 5 --warmup 2 --precision fp32_split16
[[ $STEPS == *bf16* ]] && run bench_fp16 600 python bench.py --steps 5 --warmup 2 --precision fp16 --cpu-baseline off
[[ $STEPS == *mgpu* ]] && run mgpu 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --batch 2 --dist-backend gloo
[[ $STEPS == *breakdown* ]] && run breakdown 300 python tools/conv_lab.py breakdown --out gpurun_out/breakdown.json
[[ $STEPS == *probe* ]] && run probe 300 python tools/precision_probe.py
[[ $STEPS == *tune* ]] && run tune 600 python tools/conv_lab.py tune --out gpurun_out/tune.json
[[ $STEPS == *tsplit* ]] && run tune_split 600 python tools/conv_lab.py tune --precision fp32_split16 --out gpurun_out/tune_split.json
[[ $STEPS == *tfp16* ]] && run tune_fp16 600 python tools/conv_lab.py tune --precision fp16 --out gpurun_out/tune_fp16.json
[[ $STEPS == *dsplit* ]] && run breakdown_split 300 python tools/conv_lab.py breakdown --precision fp32_split16 --out gpurun_out/breakdown_split.json
[[ $STEPS == *dfirst* ]] && run breakdown_first1 300 python tools/conv_lab.py breakdown --precision fp32_split16 --first-cfg 1
[[ $STEPS == *prof* ]] && run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --no-alt
if [[ $STEPS == *sqc* ]]; then
  for shp in "512 256 3 1 0" "32 32 0 1 1" "128 128 2 1 0"; do
    tag=$(echo $shp | tr ' ' '_')
    run sq_$tag 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_$tag -o run -- python3 tools/conv_lab.py single --precision ${SQPREC:-fp32_split16} --reps 20 --shape $shp
  done
fi
if [[ $STEPS == *pmc* ]]; then
  for prec in ${PMCPREC:-fp32_split16 fp32 fp16}; do
    run pmc_fetch_$prec 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$prec -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision $prec
    run pmc_write_$prec 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$prec -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt --precision $prec
    python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_$prec --write gpurun_out/pmc_write_$prec --steps 3 --out gpurun_out/traffic_$prec.json --table gpurun_out/pmc_traffic.json --precision $prec --config ${PMCCFG:-1280x720x4s2} > gpurun_out/pmc_summary_$prec.log 2>&1; cat gpurun_out/pmc_summary_$prec.log
  done
fi
exit 0
