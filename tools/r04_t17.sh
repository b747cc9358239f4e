set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r04_t17_suite.log 2>&1; rc=$?; echo suite_rc=$rc; tail -3 gpurun_out/r04_t17_suite.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh 1 newC=product | tee gpurun_out/r04_t17_ab.txt || exit 1
PMC_STEPS=20 bash tools/pmc_run.sh C emit fetch write || exit 1
out=gpurun_out/r04_t17_cprobe.jsonl; : > $out
for s in packed agree; do timeout -k 10 120 python tools/c_probe.py $s 200 >> $out 2>> gpurun_out/r04_t17.err || exit 1; done
cat $out
bash tools/pmc_c.sh packed fetch write sq sq2 clk && echo cpmc_done
