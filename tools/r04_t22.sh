set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_control.py tests/test_gpu_queue.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t22_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r04_t22_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/r04_t22_cprobe.jsonl; : > $out
for rep in 1 2; do
for lib in product build/var/famoff.so; do
  for s in packed c6; do
    if [ $lib = product ]; then timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t22.err || exit 1
    else UPE_GPU_LIB_DIAG=$lib timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t22.err || exit 1; fi
  done
done
done
cat $out
