#!/bin/bash
# Round 4 session b: ABI 12 (caller-provided split scratch), split-K off by default,
# autograd stream per device, warp-backward fixed-point headroom -- GPU suite, smoke,
# default bench, C2, and the new training bench line (bench.py --train).
set -u
O=${O:-gpurun_out/r04b}; mkdir -p $O; export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,c2,train}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *tests* ]] && run tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 400 python bench.py
[[ $STEPS == *c2* ]] && run bench_c2 300 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5
[[ $STEPS == *train* ]] && run bench_train 300 python bench.py --train --steps 5 --warmup 2
exit 0
