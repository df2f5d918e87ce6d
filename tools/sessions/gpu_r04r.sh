#!/bin/bash
# Round 4 session r: the level-0 Winograd tile (kind 3, conv3x3_winoq_kernel) with a
# compiler-visible vmcnt(0) after its main loop (RRIN_WINOQ_EPIWAIT=1, product) vs the
# build without it (ab/librrin_hip_epw0.so: the compiler drains vmcnt at the first
# exchange barrier, which waits out the epilogue's bias loads).  Per conv (bitwise
# compare), the default bench and C2, A/B/A/B on one box.
set -u
O=${O:-gpurun_out/r04r}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -16 | cut -c1-240
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 900 python3 -u -m pytest tests/test_gpu_h8.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread
SH=64:32:0:1:20,32:32:0:1:20,32:32:0:2:20,16:32:0:1:20,512:512:4:1:21,256:512:4:1:21,256:256:3:1:20
run abconv 400 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_epw0.so --batch 2 --shapes $SH --check
run abconv_c2 300 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_epw0.so --batch 1 --height 368 --width 640 --shapes $SH --check
B="python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
cp rrin_amd/librrin_hip.so $O/../lib_product.so
for r in a b; do
  cp $O/../lib_product.so rrin_amd/librrin_hip.so && run b_new_$r 300 $B && run c2_new_$r 200 $C2
  cp ab/librrin_hip_epw0.so rrin_amd/librrin_hip.so && run b_old_$r 300 $B && run c2_old_$r 200 $C2
done
cp $O/../lib_product.so rrin_amd/librrin_hip.so; rm -f $O/../lib_product.so
for f in $O/b_* $O/c2_*; do python3 -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
