set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r04_final_suite.log 2>&1; rc=$?; echo suite_rc=$rc; tail -3 gpurun_out/r04_final_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err; rc=$?; echo bench_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_final_prof -o b --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/r04_final_prof_bench.json 2> gpurun_out/r04_final_prof_bench.err; rc=$?; echo prof_rc=$rc; exit $rc
