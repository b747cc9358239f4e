set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04_t13_cprobe.jsonl
: > $out
for s in packed split agree agree_split; do
  timeout -k 10 120 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t13.err || exit 1
done
for a in a1 a2 a16; do
  for s in packed agree; do
    UPE_GPU_LIB_DIAG=build/var/$a.so timeout -k 10 120 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t13.err || exit 1
  done
done
cat $out
bash tools/pmc_c.sh packed fetch write sq sq2 clk && bash tools/pmc_c.sh split fetch write sq sq2 clk && bash tools/pmc_c.sh agree fetch write sq sq2 clk && echo cpmc_done && \
PMC_STEPS=10 bash tools/pmc_run.sh D emit sq clk fetch write && echo dpmc_done
