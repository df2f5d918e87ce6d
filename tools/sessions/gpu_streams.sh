#!/bin/bash
# throughput with the batch split over 1 / 2 / 4 HIP streams (no per-launch events), then the
# default profiled bench line at 2 streams
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q -k "streams or golden" --timeout 120 --timeout-method thread > gpurun_out/tests_streams.log 2>&1; rc=$?; tail -1 gpurun_out/tests_streams.log; [ $rc -ne 0 ] && exit $rc
for s in 1 2 4 1 2 4; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-prof --no-alt --cpu-baseline off --streams $s > gpurun_out/streams_$s.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/streams_$s.log').read().strip().splitlines()[-1]); print('streams $s', d['value'], d['ms_per_step'])"
done
for b in 8; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-prof --no-alt --cpu-baseline off --streams 2 --batch $b > gpurun_out/streams_b$b.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/streams_b$b.log').read().strip().splitlines()[-1]); print('batch $b streams 2', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-alt --cpu-baseline off --streams 2 > gpurun_out/streams_prof.log 2>&1; echo "prof rc=$?"
exit 0
