#!/bin/bash
# Round 5: fused level-0 block in isolation at the C3 part size: product (persistent, 2 per CU),
# one tile per workgroup, 1 per CU, and ablations (ab/librrin_hip_a*.so, RRIN_B0_ABL bits).
set -u
O=${O:-gpurun_out/r05o}; mkdir -p $O; export TMPDIR=/tmp
for v in prod bpc0 bpc1 a1 a2 a4 a8 a16 a32 a63; do
  if [ $v = prod ]; then unset RRIN_LIB_AB; else export RRIN_LIB_AB=ab/librrin_hip_$v.so; fi
  timeout -k 10 120 python -u tools/block0_lab.py > $O/$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep cin $O/$v.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
