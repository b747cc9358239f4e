#!/bin/bash
# round 5: the GPU suite, the default bench line, the same command under rocprofv3 --stats, and
# the final tree kernel's counters (CF, C6)
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; exit 1; }
echo tests_done
bash tools/r05_bench.sh || exit 1
cd $R && bash tools/r05_pmc3.sh > gpurun_out/pmc3.log 2>&1 || { echo "pmc failed"; exit 1; }
echo all_done
