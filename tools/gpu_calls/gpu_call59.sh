bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3"
