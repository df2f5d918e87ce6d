#!/bin/bash
# Round 5: headline (exact fp32 1280x720 x 4) on 4 streams (one pair each, size class medium) vs
# the default 2, and 2 streams with the medium / xlarge tables forced; interleaved x3, one box
set -u
O=${O:-gpurun_out/r05ag}; mkdir -p $O; export TMPDIR=/tmp
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
  run s2$r 200 $B
  run s4$r 200 $B --streams 4
  run s2med$r 200 $B --size-class medium
  run s2xl$r 200 $B --size-class xlarge
done
