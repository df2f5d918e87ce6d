#!/bin/bash
# Round 4 session d: the scratch-allocation race fix (INTEGRATION stub test), MFMA
# accumulators in AGPRs (A/B libraries ab/librrin_hip_cagpr.so: kinds 6/7,
# ab/librrin_hip_qagpr.so: kind 3), and the whole forward with kind 6 on cout % 64 == 0.
set -u
O=${O:-gpurun_out/r04d}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -30 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run stub 300 python3 -u -m pytest tests/test_gpu_abi_stub.py tests/test_gpu_net.py -x -q --timeout 300 --timeout-method thread -k "stub or batch_size or streams_split or batch_equals"
S23=256:256:3:1:23,128:64:1:1:23,512:512:4:1:23,128:128:2:2:23,512:1024:4:4:23,512:256:3:0:23,256:128:2:1:23,64:64:1:3:23
S20=256:256:3:1:20,64:32:0:1:20,32:32:0:1:20,32:32:0:2:20,16:32:0:1:20,512:256:3:0:20
S24=64:32:0:1:24,32:32:0:1:24,32:32:0:2:24
run ab_agpr 400 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_cagpr.so,ab/librrin_hip_qagpr.so --batch 2 --shapes $S23,$S20,$S24
B="python3 bench.py --steps 20 --warmup 5 --no-alt --cpu-baseline off"
run bench_k3a 200 $B
run bench_k6a 200 $B --wino-kind 0
run bench_k3b 200 $B
run bench_k6b 200 $B --wino-kind 0
for f in bench_k3a bench_k6a bench_k3b bench_k6b; do python3 -c "
import json,sys; l=[x for x in open('$O/$f.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
exit 0
