bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Ctss:100:UPE_GPU_TSS=1 python bench.py --config C --no-cpu-baseline --no-hbm-probe"
