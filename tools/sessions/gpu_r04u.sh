#!/bin/bash
# Round 4 session u: the re-swept fp16 tile table (engine.H8_TUNED[F16], r4) vs round 3's
# (bench.py --fp16-table r3) on the C3 line, A/B/A/B on one box; then PMC traffic of C3
# with the new table (the build is unchanged: the table is host-side).
set -u
O=${O:-gpurun_out/r04u}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -3 | cut -c1-240
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
C3="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b c; do
  run c3_r4_$r 300 $C3 && run c3_r3_$r 300 $C3 --fp16-table r3
done
for f in $O/c3_*; do python3 -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o run -- $C3P
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o run -- $C3P
python3 tools/pmc_summary.py --fetch $O/c3_fetch --write $O/c3_write --steps 3 --out $O/traffic_c3.json \
  --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 > $O/pmc_summary_c3.txt 2>&1; tail -3 $O/pmc_summary_c3.txt
cp profiles/pmc_traffic.json $O/pmc_traffic.json
exit 0
