#!/bin/bash
# Round 4 session j: register-U workgroup order in co-block groups whose U fits L2
# (launch_winoc: RRIN_WINOC_UGROUP_KB 2048 = product; ab/..._nogrp.so: one group;
# ab/..._grp4m.so: 4 MB groups) -- Winograd sweeps, per-conv A/B, whole-forward A/B
# (library swapped in place on the box), PMC traffic of the product order; the kind-3
# tile with register U (ab/librrin_hip_qru.so, RRIN_WINOQ_RU=1).
set -u
O=${O:-gpurun_out/r04j}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -25 | cut -c1-330
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_gpu_h8.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread -k "wino or split"
SH=256:512:2:4:23,512:512:4:1:23,256:512:4:1:23,512:256:3:0:23,256:256:3:1:23,128:256:3:1:23,256:128:2:1:23,128:128:2:2:23
run ab_order 400 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_nogrp.so,ab/librrin_hip_grp4m.so --batch 2 --shapes $SH
S3=64:32:0:1:20,32:32:0:1:20,32:32:0:2:20,16:32:0:1:20,256:256:3:1:20,512:512:4:1:21
run ab_qru 300 python3 -u tools/conv_lab.py abconv --lib-b ab/librrin_hip_qru.so --batch 2 --shapes $S3
cp rrin_amd/librrin_hip.so $O/prod.so.bak
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-alt"
for r in a b; do
  cp $O/prod.so.bak rrin_amd/librrin_hip.so && run bench_grp_$r 200 $B
  cp ab/librrin_hip_nogrp.so rrin_amd/librrin_hip.so && run bench_nogrp_$r 200 $B
  cp ab/librrin_hip_qru.so rrin_amd/librrin_hip.so && run bench_qru_$r 200 $B
done
cp $O/prod.so.bak rrin_amd/librrin_hip.so && rm -f $O/prod.so.bak
for f in $O/bench_*; do python3 -c "
import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$(basename $f)', d['value'], d['ms_per_step'], r['frac'], r['conv_busy_ms_per_step'], d['unprofiled']['value'])"; done
B2="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B2
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B2
python3 tools/pmc_summary.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 3 --out $O/traffic_fp32.json \
  --table profiles/pmc_traffic.json --precision fp32 --config 1280x720x4s2 > $O/pmc_summary_fp32.txt 2>&1
cat $O/pmc_summary_fp32.txt; cp profiles/pmc_traffic.json $O/pmc_traffic.json
exit 0
