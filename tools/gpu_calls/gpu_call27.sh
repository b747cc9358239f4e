bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "var:400:bash tools/variants_run.sh g4=UPE_GPU_BLOCKS_PER_CU=4 g3=UPE_GPU_BLOCKS_PER_CU=3" \
 "benchC4:200:UPE_GPU_BLOCKS_PER_CU=4 python bench.py --config C --no-cpu-baseline" \
 "benchC:200:python bench.py --config C --no-cpu-baseline" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --steps 20 --warmup 2"
