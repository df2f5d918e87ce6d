#!/bin/bash
# Round 5: Winograd source-view check (whole 2-group chunks) -- GPU suite + smoke, then the
# fp16 tile sweep at the 4-stream part size that faulted before the check (r05y).
set -u
O=${O:-gpurun_out/r05aa}; mkdir -p $O
O=$O STEPS=tests,smoke bash tools/sessions/gpu_r05z.sh || exit $?
grep -q "passed" $O/tests.log && ! grep -q "failed\|error" <(tail -1 $O/tests.log) || { echo "suite not green"; exit 1; }
O=$O bash tools/sessions/gpu_r05y.sh
