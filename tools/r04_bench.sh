set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err; rc=$?; echo bench_rc=$rc; tail -c 600 gpurun_out/r04_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof -o b --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/r04_prof_bench.json 2> gpurun_out/r04_prof_bench.err; rc=$?; echo prof_rc=$rc; exit $rc
