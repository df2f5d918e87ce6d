#!/bin/bash
# Submit one gpurun call; re-submit ONLY when gpurun reports an infrastructure
# transient (box not prepared: nothing ran, nothing charged).  Any result from a
# command that actually ran (pass or fail) is returned as is.
# usage: tools/gpu.sh TIMEOUT 'command'   (log in /tmp/gpu_last.log)
t=$1; shift
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpu_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpu_last.log; then
    echo "[gpu.sh] transient (attempt $attempt), waiting"; sleep 45; continue
  fi
  break
done
tail -3 /tmp/gpu_last.log
exit $rc
