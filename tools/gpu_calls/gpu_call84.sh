bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchB:300:python bench.py"
