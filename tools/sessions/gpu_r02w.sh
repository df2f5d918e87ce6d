#!/bin/bash
# Winograd exact-fp32 default: full GPU suite, smoke, default bench, direct-form A/B bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench,direct}
[[ $STEPS == *tests* ]] && run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
[[ $STEPS == *direct* ]] && run bench_direct 600 python bench.py --no-wino --no-alt --cpu-baseline off
[[ $STEPS == *c2* ]] && run bench_c2 600 python bench.py --height 368 --width 640 --batch 1 --no-alt --cpu-baseline off
[[ $STEPS == *x1* ]] && run bench_x1 600 python bench.py --batch 1 --no-alt --cpu-baseline off
[[ $STEPS == *prof* ]] && run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --no-alt
exit 0
