set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r04_suite.log 2>&1; rc=$?; echo suite_rc=$rc; tail -5 gpurun_out/r04_suite.log; exit $rc
