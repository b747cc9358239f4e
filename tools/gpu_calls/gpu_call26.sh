bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "var:400:bash tools/variants_run.sh dyn0=UPE_GPU_LIB_DIAG=$PWD/build/var/dyn0.so" \
 "benchC:200:python bench.py --config C --no-cpu-baseline" \
 "benchC0:200:UPE_GPU_LIB_DIAG=$PWD/build/var/dyn0.so python bench.py --config C --no-cpu-baseline" \
 "benchD:200:python bench.py --config D --no-cpu-baseline"
