set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04_t19_cprobe.jsonl; : > $out
for rep in 1 2; do
for lib in product build/var/seq.so build/var/prev.so; do
  for s in packed c6; do
    if [ $lib = product ]; then timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t19.err || exit 1
    else UPE_GPU_LIB_DIAG=$lib timeout -k 10 180 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t19.err || exit 1; fi
  done
done
done
cat $out
