set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_control.py tests/test_gpu_queue.py tests/test_gpu_worker_loop.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t20_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t20_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/r04_t19.sh && bash tools/ab_bench.sh 1 new=product seq=build/var/seq.so prev=build/var/prev.so | tee gpurun_out/r04_t20_ab.txt
