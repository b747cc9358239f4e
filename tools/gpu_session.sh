#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time limit.  A step that
# faults, aborts, segfaults or times out (exit >= 124) ends the session; plain test failures
# (exit 1) do not.  Usage: tools/gpu_session.sh "<label>:<seconds>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$label] (${secs}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$label.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: step $label ended with rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
