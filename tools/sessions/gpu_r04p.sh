#!/bin/bash
# Round 4 session p: PMC traffic of BASELINE C2 (fp32 640x368 x 1) and C3 (fp16 1280x736
# x 4) for the current build (profiles/pmc_traffic.json entries read by bench.py), and the
# C3 forward on 1 / 2 / 3 / 4 streams.
set -u
O=${O:-gpurun_out/r04p}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -2 | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
C2="python3 bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
C3="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o run -- $C2
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o run -- $C2
python3 tools/pmc_summary.py --fetch $O/c2_fetch --write $O/c2_write --steps 3 --out $O/traffic_c2.json \
  --table profiles/pmc_traffic.json --precision fp32 --config 640x368x1 > $O/pmc_summary_c2.txt 2>&1; cat $O/pmc_summary_c2.txt
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o run -- $C3
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o run -- $C3
python3 tools/pmc_summary.py --fetch $O/c3_fetch --write $O/c3_write --steps 3 --out $O/traffic_c3.json \
  --table profiles/pmc_traffic.json --precision fp16 --config 1280x736x4s2 > $O/pmc_summary_c3.txt 2>&1; cat $O/pmc_summary_c3.txt
cp profiles/pmc_traffic.json $O/pmc_traffic.json
B="python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  for s in 2 1 3 4; do run c3_s${s}_$r 200 $B --streams $s; done
done
run c2_line 200 python bench.py --height 368 --width 640 --batch 1 --streams 1 --steps 20 --warmup 5
run c3_line 200 python bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 20 --warmup 5 --cpu-baseline off
for f in $O/c3_s*.log $O/c2_line.log $O/c3_line.log; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), r.get('traffic_per_step_gb'), r.get('algorithmic_bytes_per_step_gb'))"; done
exit 0
