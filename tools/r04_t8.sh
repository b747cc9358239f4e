set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reload.py tests/test_gpu_worker_loop.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t8_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t8_tests.log
[ $rc -ge 124 ] && exit $rc
bash tools/ab_bench.sh 3 wave=product old=build/var/wg0.so | tee gpurun_out/r04_t8_ab.txt
