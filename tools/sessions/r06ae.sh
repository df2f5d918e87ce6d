#!/bin/bash
# Round 6 call ae: ablation bounds of kind 14 (outputs wrong by design), per conv at the headline
# part size: B no per-chunk s_barrier, C no U reloads, D no window reads / transforms, E no raw
# LDS-DMA after the prologue, F no epilogue stores.
set -u
O=gpurun_out/r06ae; mkdir -p $O; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$O/$name.log" | tail -12 | cut -c1-220; [ $rc -eq 0 ] || exit $rc; }
SH="32:32:0:1:25,64:32:0:1:25,64:64:1:1:25,128:64:1:1:25,128:128:2:1:25,256:256:3:1:25,512:256:3:1:25,512:512:4:1:25,256:512:2:4:25"
run abconv 600 python tools/conv_lab.py abconv --lib-b ab/librrin_hip_nobar.so,ab/librrin_hip_noU.so,ab/librrin_hip_noT.so,ab/librrin_hip_noD.so,ab/librrin_hip_noS.so --batch 2 --rounds 5 --shapes $SH
exit 0
