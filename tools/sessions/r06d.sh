#!/bin/bash
# Round 6 call d: whole-record fp16 epilogues (conv3x3_h8_kernel epi_pair, conv_block0 via
# v_permlane32_swap): bitwise against the r06b build (ab/librrin_hip_r06b.so), the GPU suite, the
# C3 A/B interleaved, then the block0 SQ counters (bank conflicts) of the new build.
set -u
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1; shift; "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step save_old env RRIN_LIB_AB=ab/librrin_hip_r06b.so timeout -k 10 300 python tools/lib_bitwise.py --save $O/old.pt
step cmp_new timeout -k 10 300 python tools/lib_bitwise.py --compare $O/old.pt
step pytest_gpu timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
C3="--height 736 --width 1280 --batch 4 --precision fp16 --steps 30 --warmup 5 --cpu-baseline off --no-alt"
step c3_new1 timeout -k 10 200 python bench.py $C3
step c3_old1 env RRIN_LIB_AB=ab/librrin_hip_r06b.so timeout -k 10 200 python bench.py $C3
step c3_new2 timeout -k 10 200 python bench.py $C3
step c3_old2 env RRIN_LIB_AB=ab/librrin_hip_r06b.so timeout -k 10 200 python bench.py $C3
step c3_new3 timeout -k 10 200 python bench.py $C3
step c3_old3 env RRIN_LIB_AB=ab/librrin_hip_r06b.so timeout -k 10 200 python bench.py $C3
C3P="python3 bench.py --height 736 --width 1280 --batch 4 --precision fp16 --steps 2 --warmup 1 --cpu-baseline off --no-prof --no-alt"
step sq_block0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/sq_new -o run -- $C3P
exit 0
