#!/bin/bash
# Round 5: ablations of the fp16 Winograd tile (conv_winoh.hip, RRIN_WINOH_ABL builds in ab/):
# 1 no U loads, 2 no raw DMA, 4 no transform VALU, 8 no epilogue stores, 16 no window reads,
# 31 all of them; per conv at the C3 part size (1280x736 x 2), interleaved with the product build.
set -u
O=${O:-gpurun_out/r05b}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_lab.py abconv --precision fp16 --height 736 --width 1280 --batch 2 \
  --lib-b ab/librrin_hip_wh1.so,ab/librrin_hip_wh2.so,ab/librrin_hip_wh4.so,ab/librrin_hip_wh8.so,ab/librrin_hip_wh16.so,ab/librrin_hip_wh31.so \
  --shapes 256:256:3:1:23,512:512:4:1:23,128:64:1:1:23,64:64:1:3:23,256:128:2:1:23 --rounds 5 --reps 5 > $O/abl.log 2>&1
echo rc=$?; grep -v amdgpu.ids $O/abl.log
