#!/bin/bash
# Round 5: fp16 head conv on the matrix cores (head_conv_mfma): fp16 Net / config / kernel tests,
# then C3 / C5 A/B against the VALU head (ab/librrin_hip_old.so), same box, interleaved.
set -u
O=${O:-gpurun_out/r05t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_kernels.py tests/test_gpu_abi_stub.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"max_abs[a-z_]*": [0-9.e-]*\|"psnr[a-z_]*": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C5="python bench.py --height 2176 --width 3840 --batch 1 --precision fp16 --steps 10 --warmup 3 --cpu-baseline off --no-alt"
for r in a b; do
  run c3_new$r 200 $C3
  RRIN_LIB_AB=ab/librrin_hip_old.so run c3_old$r 200 $C3
done
run c5_new 300 $C5
RRIN_LIB_AB=ab/librrin_hip_old.so run c5_old 300 $C5
run c3_parity 400 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 5 --warmup 2 --no-alt
