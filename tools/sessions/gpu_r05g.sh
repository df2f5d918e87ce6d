#!/bin/bash
# Round 5: C2 (640x368 x 1, exact fp32) with the co-block group order in kinds 3/4 vs without
# (RRIN_WINOQ_UGROUP_KB=0 build in ab/); per-dispatch HBM traffic of both.
set -u
O=${O:-gpurun_out/r05g}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C2="python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
run c2_g1 200 $C2
RRIN_LIB_AB=ab/librrin_hip_noqg.so run c2_n1 200 $C2
run c2_g2 200 $C2
RRIN_LIB_AB=ab/librrin_hip_noqg.so run c2_n2 200 $C2
B2="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
for v in g n; do
  if [ $v = n ]; then export RRIN_LIB_AB=ab/librrin_hip_noqg.so; fi
  run pmc_fetch_$v 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$v -o run -- $B2
  run pmc_write_$v 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$v -o run -- $B2
  python3 tools/pmc_by_dispatch.py --fetch $O/pmc_fetch_$v --write $O/pmc_write_$v --steps 3 --top 30 > $O/by_dispatch_$v.txt
  head -12 $O/by_dispatch_$v.txt
done
