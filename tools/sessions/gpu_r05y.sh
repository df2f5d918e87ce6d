#!/bin/bash
# Round 5: fp16 record-conv tile table swept at the 4-stream C3 part size (1280x736 x 1, the
# "medium" class the fp16 parts fall in since engine.default_streams runs one pair per stream)
set -u
O=${O:-gpurun_out/r05y}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python3 -u tools/conv_lab.py tune --precision fp16 --batch 1 --height 736 --width 1280 --reps 7 \
  --out $O/tune_fp16_1280x736x1.json > $O/tune_fp16_1280x736x1.txt 2>&1
rc=$?; echo "tune rc=$rc"; grep -v amdgpu $O/tune_fp16_1280x736x1.txt | cut -c1-70 | tail -28
exit $rc
