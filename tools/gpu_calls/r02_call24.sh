# round 2: host round trip with records instead of the copied-back header span
# (upe_gpu_process_host_emit): parity (both modes), then B and C rates with 4 / 8 / 16 threads
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix --steps 20 --warmup 5 --host-reps 10"
bash tools/gpu_session.sh \
 "hostt:600:python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "B8:200:python bench.py $O --host-threads 8" \
 "B4:200:python bench.py $O --host-threads 4" \
 "B16:200:python bench.py $O --host-threads 16" \
 "C8:200:python bench.py --config C $O --host-threads 8" \
 "B8c:200:python bench.py $O --host-threads 8 --host-chunk 524288"
