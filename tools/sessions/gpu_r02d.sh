#!/bin/bash
# new parity tests (taps, C3, C5, wide range) then the whole GPU suite
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -6 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests_new 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 240 --timeout-method thread
run tests_all 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
