#!/bin/bash
# Round 5: 1-stream vs 2-stream bitwise probe of the C3 forward for the fp16 Winograd kinds
set -u
O=${O:-gpurun_out/r05l}; mkdir -p $O; export TMPDIR=/tmp
P="python -u tools/stream_bitwise.py --precision fp16"
for cfg in "direct|--no-wino" "k6_l34|--wino-f16-kind 6 --wino-f16-levels 3,4" "k10_l34|--wino-f16-kind 10 --wino-f16-levels 3,4"; do
  n=${cfg%%|*}; f=${cfg#*|}
  timeout -k 10 200 $P $f > $O/$n.log 2>&1; echo "$n rc=$? $(tail -1 $O/$n.log)"
done
export RRIN_LIB_AB=ab/librrin_hip_hbpc1.so
timeout -k 10 200 $P --wino-f16-kind 10 --wino-f16-levels 3,4 > $O/k10_bpc1.log 2>&1; echo "k10_bpc1 rc=$? $(tail -1 $O/k10_bpc1.log)"
timeout -k 10 200 $P --wino-f16-kind 6 --wino-f16-levels 3,4 > $O/k6_bpc1lib.log 2>&1; echo "k6_bpc1lib rc=$? $(tail -1 $O/k6_bpc1lib.log)"
export RRIN_LIB_AB=ab/librrin_hip_bpc1.so
timeout -k 10 200 python -u tools/stream_bitwise.py --precision fp32 --height 720 --wino-persistent 1 > $O/k12_bpc1.log 2>&1; echo "k12_bpc1 rc=$? $(tail -1 $O/k12_bpc1.log)"
