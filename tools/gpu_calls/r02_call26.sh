# round 2: records host round trip with the apply two chunks behind (H2D never waits for the
# host threads): parity of both modes, B and C rates with 8 / 16 threads and 512k chunks
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix --steps 20 --warmup 5 --host-reps 10"
bash tools/gpu_session.sh \
 "hostt:600:python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "B8:200:python bench.py $O --host-threads 8" \
 "B16:200:python bench.py $O --host-threads 16" \
 "B8c:200:python bench.py $O --host-threads 8 --host-chunk 524288" \
 "B8s:200:python bench.py $O --host-threads 8 --host-chunk 131072" \
 "C8:200:python bench.py --config C $O --host-threads 8" \
 "D8:300:python bench.py --config D --max-copies 4 $O --host-threads 8"
