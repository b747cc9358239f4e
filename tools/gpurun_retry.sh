#!/bin/bash
# Run one gpurun call; if the infrastructure reports a transient failure before anything ran
# (status=transient, nothing charged), wait and submit again, up to 5 times.  A call that ran is
# never repeated, whatever its exit code.
#   tools/gpurun_retry.sh <timeout-seconds> '<command>'
t=$1; shift
for attempt in 1 2 3 4 5; do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.log && grep -q "run 0.0s" /tmp/gpurun_last.log; then
    echo "[retry] transient infrastructure failure (attempt $attempt), waiting"; sleep 60; continue
  fi
  if [ $rc -eq 3 ]; then echo "[retry] no box free (attempt $attempt)"; sleep 90; continue; fi
  break
done
grep -v "amdgpu.ids" /tmp/gpurun_last.log | grep -v "^W2026\|^E2026" | tail -40
exit $rc
