set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_control.py tests/test_gpu_queue.py tests/test_gpu_worker_loop.py tests/test_gpu_dropin.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t18_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t18_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/r04_t18_cprobe.jsonl; : > $out
for lib in product build/var/prev.so; do
  for s in c6 packed; do
    if [ $lib = product ]; then timeout -k 10 180 python tools/c_probe.py $s 100 >> $out 2>> gpurun_out/r04_t18.err || exit 1
    else UPE_GPU_LIB_DIAG=$lib timeout -k 10 180 python tools/c_probe.py $s 100 >> $out 2>> gpurun_out/r04_t18.err || exit 1; fi
  done
done
cat $out
bash tools/ab_bench.sh 2 fam=product prev=build/var/prev.so | tee gpurun_out/r04_t18_ab.txt
