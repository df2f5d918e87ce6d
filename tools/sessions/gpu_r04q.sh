#!/bin/bash
# Round 4 session q: epilogue bias of the record conv kernel (conv3x3_h8_kernel, the fp16
# path's conv): RRIN_H8_BIAS -1 (product: mode per tile shape, one compiler-visible
# wait) vs 0 (each epilogue piece loads its bias and waits out the tile's earlier stores)
# vs 2 everywhere.  Per conv (bitwise compare) and the C3 line, A/B/A/B.
set -u
O=${O:-gpurun_out/r04q}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -20 | cut -c1-260
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 900 python3 -u -m pytest tests/test_gpu_h8.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
SH=32:32:0:2:9,32:32:0:1:9,64:32:0:1:9,64:64:1:2:9,64:64:1:3:9,32:64:1:1:10,128:128:2:2:11,256:128:2:1:11,128:64:1:1:0,256:256:3:1:10,512:512:4:1:4,512:256:3:1:5,256:512:2:4:11,64:128:0:4:10
run abconv 400 python3 -u tools/conv_lab.py abconv --precision fp16 --lib-b ab/librrin_hip_bias0.so,ab/librrin_hip_bias2.so \
  --batch 2 --height 736 --width 1280 --shapes $SH --check
C3="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
cp rrin_amd/librrin_hip.so $O/../lib_product.so
for r in a b; do
  cp $O/../lib_product.so rrin_amd/librrin_hip.so && run c3_auto_$r 300 $C3
  cp ab/librrin_hip_bias0.so rrin_amd/librrin_hip.so && run c3_bias0_$r 300 $C3
done
cp $O/../lib_product.so rrin_amd/librrin_hip.so; rm -f $O/../lib_product.so
for f in $O/c3_*; do python3 -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
