#!/bin/bash
# Round 6 call e: the fp16 range flag accumulated per lane (one store per workgroup) on top of the
# whole-record epilogues: bitwise vs the r06b build, GPU suite, C3 A/B vs the r06d build, then the
# C3 SQ counters (block0 bank conflicts, record-conv MFMA busy) in two passes.
set -u
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step save_old env RRIN_LIB_AB=ab/librrin_hip_r06b.so timeout -k 10 300 python tools/lib_bitwise.py --save /tmp/old.pt
step cmp_new timeout -k 10 300 python tools/lib_bitwise.py --compare /tmp/old.pt
step pytest_gpu timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
step c3_new1 timeout -k 10 200 python bench.py $C3
step c3_r06d1 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
step c3_new2 timeout -k 10 200 python bench.py $C3
step c3_r06d2 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
step c3_new3 timeout -k 10 200 python bench.py $C3
step c3_r06d3 env RRIN_LIB_AB=ab/librrin_hip_r06d.so timeout -k 10 200 python bench.py $C3
# upper bound of the ring fix-up's cost: the same build without the fix-up launches (ring pixels wrong)
step c3_noring1 env RRIN_LIB_AB=ab/librrin_hip_noring.so timeout -k 10 200 python bench.py $C3
step c3_new4 timeout -k 10 200 python bench.py $C3
step c3_noring2 env RRIN_LIB_AB=ab/librrin_hip_noring.so timeout -k 10 200 python bench.py $C3
C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
step sq1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/sq1 -o run -- $C3P
step sq2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- $C3P
exit 0
