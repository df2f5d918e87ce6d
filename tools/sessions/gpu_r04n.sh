#!/bin/bash
# Round 4 session n: the persistent register-U tile (kind 8 = config 25, conv_winop.hip)
# for the 32-channel convs -- Winograd sweeps (kind 8 included), per-conv A/B against
# kind 3 (bitwise), whole forward with --wino-kind32 8.
set -u
O=${O:-gpurun_out/r04n}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -12 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_gpu_h8.py tests/test_wino.py -x -q --timeout 300 --timeout-method thread
S=64:32:0:1,32:32:0:1,32:32:0:2,16:32:0:1,10:32:0:1
run ab_720 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,25 --batch 2 --shapes $S --rounds 7 --reps 5
run ab_c2 200 python3 -u tools/conv_lab.py cfgab --cfgs 20,25 --batch 1 --height 368 --width 640 --shapes $S --rounds 9 --reps 10
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 40 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run bench_k3_$r 200 $B && run bench_k8_$r 200 $B --wino-kind32 8
  run c2_k3_$r 200 $C2 && run c2_k8_$r 200 $C2 --wino-kind32 8
done
for f in $O/bench_* $O/c2_*; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'], (d.get('parity') or {}).get('max_abs'))"; done
exit 0
