#!/bin/bash
# round 5: the GPU suite, the default bench line, and the same command under rocprofv3 --stats
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; exit 1; }
echo tests_done
bash tools/r05_bench.sh || exit 1
