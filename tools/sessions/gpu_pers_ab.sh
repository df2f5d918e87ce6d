#!/bin/bash
# Persistent Winograd grid A/B (make pers-variants / librrin_hip_pers<k>[b1].so): the
# product library (never persistent) and the variants named in $VARIANTS (pers<k>:
# persistent from k tiles per block slot, 2 blocks per CU; pers<k>b1: 1 block per CU,
# so the other stream's launch holds the CU's second slot), swapped in for
# librrin_hip.so in turn; default bench and 720p x 1, interleaved.
set -u
mkdir -p gpurun_out/pers
VARIANTS=${VARIANTS:-pers3 pers8}
cp rrin_amd/librrin_hip.so gpurun_out/pers/product.so
for v in $VARIANTS; do cp rrin_amd/librrin_hip_$v.so gpurun_out/pers/$v.so; done
for rep in 1 2; do
  for v in $VARIANTS product; do
    cp gpurun_out/pers/$v.so rrin_amd/librrin_hip.so
    for cfg in "--batch 4" "--batch 1"; do
      timeout -k 10 300 python bench.py $cfg --no-alt --cpu-baseline off > gpurun_out/pers/b.log 2>&1
      rc=$?
      echo "r$rep $v $cfg: $(grep -o '"value": [0-9.]*' gpurun_out/pers/b.log | head -1) $(grep -o '"frac": [0-9.]*' gpurun_out/pers/b.log | head -1)"
      if [ $rc -ne 0 ]; then tail -5 gpurun_out/pers/b.log; cp gpurun_out/pers/product.so rrin_amd/librrin_hip.so; exit $rc; fi
    done
  done
done
cp gpurun_out/pers/product.so rrin_amd/librrin_hip.so
rm -f gpurun_out/pers/*.so
exit 0
