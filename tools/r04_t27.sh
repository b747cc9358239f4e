set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "flavours or ipv6_forwarding or golden" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t27_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/r04_t27_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/r04_t27_cprobe.jsonl; : > $out
for rep in 1 2; do for lib in product build/var/v12.so; do for s in c6 packed; do
  if [ $lib = product ]; then timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t27.err || exit 1
  else UPE_GPU_LIB_DIAG=$lib timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t27.err || exit 1; fi
done; done; done
cat $out
