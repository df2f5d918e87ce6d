#!/bin/bash
# Round 5: correctness of the max-ILP build of conv_winoc.hip (its counted vmcnt waits assume the
# load issue order): GPU suite, smoke, the default bench (720p parity of pair 0 vs the oracle),
# and repeat-determinism of the exact-fp32 forward on one vs two streams (tools/stream_bitwise.py)
set -u
O=${O:-gpurun_out/r05aj}; mkdir -p $O
O=$O STEPS=tests,smoke,bench bash tools/sessions/gpu_r05z.sh || exit $?
timeout -k 10 300 python3 tools/stream_bitwise.py --precision fp32 --height 720 --width 1280 --batch 4 --rounds 8 \
  > $O/stream_bitwise.log 2>&1; echo "stream_bitwise rc=$?"; tail -4 $O/stream_bitwise.log
