#!/bin/bash
# Round 4 session c: co-issue probe 2 (instruction prices beside the f32 MFMA), the
# INTEGRATION stub debug, the register-U Winograd kinds 6/7 (configs 23/24): GPU conv
# suite, then bitwise + timing against config 20 on the Net's conv shapes at 720p x 2.
set -u
O=${O:-gpurun_out/r04c}; mkdir -p $O; export TMPDIR=/tmp
STEPS=${STEPS:-probe,dbg,h8,ab,train}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc in $name; stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *probe* ]] && run probe2 240 python3 -u tools/coissue_probe2.py
[[ $STEPS == *dbg* ]] && run dbg 150 python3 tools/dbg_stub.py
[[ $STEPS == *h8* ]] && run h8 900 python3 -u -m pytest tests/test_gpu_h8.py -x -q --timeout 300 --timeout-method thread
S64=256:256:3:1,128:64:1:1,512:512:4:1,128:128:2:2,512:1024:4:4,128:256:2:4,64:128:1:4,32:64:1:1,512:256:3:0,256:128:2:1,64:64:1:3
S32=64:32:0:1,32:32:0:1,32:32:0:2,16:32:0:1,64:32:0:4
if [[ $STEPS == *ab* ]]; then
  run ab_20_23 300 python3 -u tools/conv_lab.py cfgab --cfgs 20,23 --batch 2 --shapes $S64
  run ab_20_24 300 python3 -u tools/conv_lab.py cfgab --cfgs 20,24 --batch 2 --shapes $S64,$S32
fi
if [[ $STEPS == *train* ]]; then
  run train_tests 600 python3 -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread
  run bench_train 300 python3 bench.py --train --steps 5 --warmup 2
  run prof_train 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python3 bench.py --train --steps 3 --warmup 1
  python3 tools/kernel_family_stats.py $(ls $O/prof_train/*/*kernel_stats.csv $O/prof_train/*kernel_stats.csv 2>/dev/null | head -1) > $O/kernel_family_train.txt 2>&1; head -20 $O/kernel_family_train.txt
fi
cat $O/probe2.log 2>/dev/null | tail -50
exit 0
