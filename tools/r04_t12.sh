set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_reload.py tests/test_gpu_split.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t12_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t12_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh 2 new=product prev=build/var/new.so | tee gpurun_out/r04_t12_ab.txt
