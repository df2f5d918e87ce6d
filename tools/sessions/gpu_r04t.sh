#!/bin/bash
# Round 4 session t: re-sweep of the fp16 record-conv tile table at the C3 part size
# (1280x736 x 2) after the epilogue change.
set -u
O=${O:-gpurun_out/r04t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/conv_lab.py tune --precision fp16 --batch 2 --height 736 --width 1280 --reps 7 \
  --out $O/tune_fp16_1280x736x2.json > $O/tune_fp16_1280x736x2.txt 2>&1
rc=$?; echo "tune rc=$rc"; grep -v amdgpu $O/tune_fp16_1280x736x2.txt | cut -c1-60
exit $rc
