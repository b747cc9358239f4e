set -o pipefail
export TMPDIR=/tmp
D="python bench.py --config D --steps 40 --warmup 5 --no-cpu-baseline --host-reps 0 --no-other-mode --no-hbm-probe"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_worker_loop.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t3_dropin.log 2>&1; echo dropin_rc=$?
timeout -k 10 240 $D > gpurun_out/r04_t3_D_base.json 2> gpurun_out/r04_t3_D_base.err || exit 1
UPE_GPU_WIN6=1 timeout -k 10 240 $D > gpurun_out/r04_t3_D_win6.json 2>> gpurun_out/r04_t3_D_base.err || exit 1
UPE_GPU_LIB_DIAG=build/var/a16.so timeout -k 10 240 $D > gpurun_out/r04_t3_D_a16.json 2>> gpurun_out/r04_t3_D_base.err || exit 1
C="python bench.py --config C --steps 100 --warmup 10 --no-cpu-baseline --host-reps 0 --no-other-mode --no-hbm-probe --mode inplace"
timeout -k 10 200 $C > gpurun_out/r04_t3_C_inpl.json 2>> gpurun_out/r04_t3_D_base.err || exit 1
UPE_GPU_WIN6=1 timeout -k 10 200 $C > gpurun_out/r04_t3_C_inpl_win6.json 2>> gpurun_out/r04_t3_D_base.err || exit 1
echo done
