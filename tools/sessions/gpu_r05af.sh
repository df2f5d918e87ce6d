#!/bin/bash
# Round 5: fp16 record conv epilogue through buffer stores (a.buf_store) -- record-conv and fused
# block suites (bitwise), then C3 / C5 interleaved against RRIN_NO_BUF_STORE=1 (the old stores)
set -u
O=${O:-gpurun_out/r05af}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h8.py tests/test_gpu_block0.py tests/test_gpu_net.py tests/test_gpu_configs.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 6 --warmup 2 --cpu-baseline off --no-alt"
for r in a b c; do
  run c3_buf$r 200 $C3
  RRIN_NO_BUF_STORE=1 run c3_old$r 200 $C3
done
for r in a b; do
  run c5_buf$r 200 $C5
  RRIN_NO_BUF_STORE=1 run c5_old$r 200 $C5
done
