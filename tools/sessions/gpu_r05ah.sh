#!/bin/bash
# Round 5: compiler scheduling strategy A/B on the exact-fp32 Winograd tiles (headline):
# ab/librrin_hip_{ilp6,mc6,ilp3}.so = conv_winoc.hip (kind 6) built with -amdgpu-sched-strategy
# max-ilp / max-memory-clause, conv_wino.hip (kinds 3/4) with max-ilp; interleaved x3, one box
set -u
O=${O:-gpurun_out/r05ah}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b c; do
  run base$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_ilp6.so run ilp6$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_mc6.so run mc6$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_ilp3.so run ilp3$r 200 $B
done
