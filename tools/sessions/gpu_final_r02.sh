#!/bin/bash
# Round-2 final build: stream-count A/B of the Winograd default, then the GPU
# suite, smoke, default bench and the rocprofv3 kernel summary of the default.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-streams,tests,smoke,bench,prof}
if [[ $STEPS == *streams* ]]; then
  for rep in 1 2; do
    for s in 2 3 4 1; do
      timeout -k 10 300 python bench.py --streams $s --no-alt --cpu-baseline off > gpurun_out/st.log 2>&1
      rc=$?
      echo "r$rep streams $s: $(grep -o '"value": [0-9.]*' gpurun_out/st.log | head -1) $(grep -o '"frac": [0-9.]*' gpurun_out/st.log | head -1)"
      if [ $rc -ne 0 ]; then tail -5 gpurun_out/st.log; exit $rc; fi
    done
  done
fi
[[ $STEPS == *tests* ]] && run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
[[ $STEPS == *prof* ]] && run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-alt
exit 0
