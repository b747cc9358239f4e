set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_mapped.py tests/test_gpu_lookback.py tests/test_gpu_batches.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t16_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t16_tests.log
[ $rc -ne 0 ] && exit $rc
UPE_GPU_LIB_DIAG=build/var/stamps.so timeout -k 10 120 python tools/stamps.py 1048576 emit B > gpurun_out/r04_stamps_B_dyn.txt 2>&1 || exit 1
bash tools/ab_bench.sh 2 dyn2=product dyn0=build/var/dyn0.so dyn1=build/var/dyn1.so dyn3=build/var/dyn3.so | tee gpurun_out/r04_t16_ab.txt
