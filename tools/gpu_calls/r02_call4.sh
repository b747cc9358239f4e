# round 2, session 3: check HEAD as restored (GPU tests, smoke, config B bench line)
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchB:400:python bench.py > gpurun_out/benchB.json"
