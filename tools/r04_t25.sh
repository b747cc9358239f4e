set -o pipefail
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookback.py tests/test_gpu_reload.py tests/test_gpu_control.py tests/test_gpu_queue.py tests/test_gpu_worker_loop.py tests/test_gpu_batches.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t25_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t25_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/r04_t25_cprobe.jsonl; : > $out
for lib in product build/var/v11.so; do
  for s in packed agree c6; do
    if [ $lib = product ]; then timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t25.err || exit 1
    else UPE_GPU_LIB_DIAG=$lib timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t25.err || exit 1; fi
  done
done
cat $out
bash tools/ab_bench.sh 1 new=product v11=build/var/v11.so | tee gpurun_out/r04_t25_ab.txt
