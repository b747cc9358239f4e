#!/bin/bash
# round 5: the default bench line, then the same command under rocprofv3 --kernel-trace --stats
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && timeout -k 10 900 python -u bench.py > gpurun_out/bench_r05.json 2> gpurun_out/bench_r05.err || { echo "bench failed rc=$?"; exit 1; }
echo bench_done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05 -o run -- python -u $R/bench.py > $R/gpurun_out/bench_r05_prof.json 2> $R/gpurun_out/bench_r05_prof.err || { echo "prof failed rc=$?"; exit 1; }
echo prof_done
