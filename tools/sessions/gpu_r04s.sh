#!/bin/bash
# Round 4 session s: the three-stage input ring of the record conv (conv3x3_h8_kernel,
# RRIN_H8_NS3=1: WRES tiles where it keeps the blocks per CU -- cfg 9 at cin <= 32, the
# fp16 level-0 convs) vs the two-stage loop (ab/librrin_hip_ns0.so).  Per conv (bitwise
# compare) and the C3 line, A/B/A/B on one box.
set -u
O=${O:-gpurun_out/r04s}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -12 | cut -c1-240
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 900 python3 -u -m pytest tests/test_gpu_h8.py tests/test_gpu_configs.py tests/test_gpu_net.py -x -q --timeout 300 --timeout-method thread
SH=32:32:0:2:9,32:32:0:1:9,16:32:0:1:9,64:32:0:1:9,64:64:1:2:9
run abconv 300 python3 -u tools/conv_lab.py abconv --precision fp16 --lib-b ab/librrin_hip_ns0.so --batch 2 --height 736 --width 1280 --shapes $SH --check
run abconv_c5 300 python3 -u tools/conv_lab.py abconv --precision fp16 --lib-b ab/librrin_hip_ns0.so --batch 1 --height 2176 --width 3840 --shapes $SH --check
C3="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
cp rrin_amd/librrin_hip.so $O/../lib_product.so
for r in a b; do
  cp $O/../lib_product.so rrin_amd/librrin_hip.so && run c3_ns3_$r 300 $C3
  cp ab/librrin_hip_ns0.so rrin_amd/librrin_hip.so && run c3_ns2_$r 300 $C3
done
cp $O/../lib_product.so rrin_amd/librrin_hip.so; rm -f $O/../lib_product.so
for f in $O/c3_*; do python3 -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
