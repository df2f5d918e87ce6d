#!/bin/bash
# Round 3: Winograd conv rework -- record-conv parity, then A/B of the conv kernel
# (ab/librrin_hip_prev.so = round-2 build vs the in-tree library, bitwise compare),
# then the default bench.  STEPS selects parts (tests,ab,bench,net).
set -u
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab,bench}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
SH=${SHAPES:-256:256:3:1:18,64:32:0:1:18,32:32:0:1:18,128:64:1:1:18,512:512:4:1:18,32:32:0:2:18,128:128:2:2:18,16:32:0:1:18,512:1024:4:4:18,128:256:2:4:18}
[[ $STEPS == *tests* ]] && run tests_h8 600 python -u -m pytest tests/test_gpu_h8.py -x -q --timeout 120 --timeout-method thread
[[ $STEPS == *net* ]] && run tests_net 600 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *ab* ]] && run ab 300 python -u tools/conv_lab.py abconv --lib ab/librrin_hip_prev.so --lib-b rrin_amd/librrin_hip.so --batch 2 --reps 10 --rounds 5 --shapes $SH
[[ $STEPS == *bench* ]] && run bench 400 python bench.py --cpu-baseline off --no-alt
exit 0
