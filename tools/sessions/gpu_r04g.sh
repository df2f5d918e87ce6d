#!/bin/bash
# Round 4 session g: split-K by per-image geometry (engine.geom_split) -- the split /
# batch-invariance tests, C2 with and without it; ablations of the register-U tile
# (ab/librrin_hip_abl*.so: 1 no U loads, 2 no raw DMA, 3 no loads, 4 no transform,
# 8 no stores, 16 no window reads, 31 all of them).
set -u
O=${O:-gpurun_out/r04g}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -30 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_net.py tests/test_gpu_abi_stub.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run c2_geo_$r 200 $C2
  run c2_nosplit_$r 200 $C2 --wino-split none
done
for f in $O/c2_*; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'], d['parity']['max_abs'] if d.get('parity') else None)"; done
L=ab/librrin_hip_abl1.so,ab/librrin_hip_abl2.so,ab/librrin_hip_abl3.so,ab/librrin_hip_abl4.so,ab/librrin_hip_abl8.so,ab/librrin_hip_abl16.so,ab/librrin_hip_abl31.so
run ablate 400 python3 -u tools/conv_lab.py abconv --lib-b $L --batch 2 --shapes 256:256:3:1:23,128:64:1:1:23,64:64:1:3:23,512:256:3:0:23,32:64:1:1:23
exit 0
