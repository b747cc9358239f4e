bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --config B --no-cpu-baseline" \
 "benchC:300:python bench.py --config C --no-cpu-baseline" \
 "stamps1M:200:UPE_GPU_LIB_DIAG=$PWD/build/diag/libupe_gpu_stamps.so python tools/stamps.py 1048576" \
 "sweep:400:bash tools/size_sweep.sh"
