bash tools/gpu_session.sh \
 "ctrl:300:python -u -m pytest tests/test_gpu_control.py -x -v --timeout 240 --timeout-method thread" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "C:100:python bench.py --config C --no-cpu-baseline" \
 "Ctss:100:UPE_GPU_TSS=1 python bench.py --config C --no-cpu-baseline"
