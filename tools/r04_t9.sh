set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_control.py tests/test_gpu_neigh_paths.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t9_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t9_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh 3 new=product old=build/var/wg0.so | tee gpurun_out/r04_t9_ab.txt
