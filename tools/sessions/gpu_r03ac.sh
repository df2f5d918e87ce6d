#!/bin/bash
# fp16 C3 PMC traffic with the round-3 fp16 table; C3 bench; 4K per-GPU shares (fp16, exact fp32)
set -u
O=gpurun_out/r03ac; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C3="python3 bench.py --precision fp16 --height 736 --width 1280 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $C3
run pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $C3
python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp16_c3.json --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 --family conv3x3_h8_kernel > $O/pmc_summary_fp16_c3.txt 2>&1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
run c3 200 python bench.py --precision fp16 --height 736 --width 1280
run c5_fp16 300 python bench.py --precision fp16 --height 2176 --width 3840 --batch 1 --streams 1 --steps 5 --warmup 2 --cpu-baseline off
run c5_fp32 300 python bench.py --height 2176 --width 3840 --batch 1 --streams 1 --steps 5 --warmup 2 --cpu-baseline off --no-alt
