#!/bin/bash
# Round 5: headline with the persistent exact-fp32 kind 12 at one workgroup per CU (the other
# slot left to the other stream) vs kind 6 (default) and kind 12 at two per CU; same box.
set -u
O=${O:-gpurun_out/r05s}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  run k6$r 200 $B
  RRIN_LIB_AB=ab/librrin_hip_wcp1.so run k12bpc1$r 200 $B --wino-persistent 1
  run k12bpc2$r 200 $B --wino-persistent 1
done
