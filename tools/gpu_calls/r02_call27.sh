# round 2: host round trip of 4M-packet config-B calls (steady state of the chunk pipeline),
# both modes, 256k and 512k chunks
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --steps 10 --warmup 2 --max-copies 8 --host-reps 5 --packets 4194304"
bash tools/gpu_session.sh \
 "B4M256:300:python bench.py $O --host-threads 8" \
 "B4M512:300:python bench.py $O --host-threads 8 --host-chunk 524288" \
 "B4M128:300:python bench.py $O --host-threads 8 --host-chunk 131072"
