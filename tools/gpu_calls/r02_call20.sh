# round 2: config B batch-size sweep on the mid-chunk prefetch kernel (one launch per batch;
# --packets disables the IMIX leg), emit mode
O="--no-cpu-baseline --no-hbm-probe --no-other-mode"
bash tools/gpu_session.sh \
 "n64k:120:python bench.py --packets 65536 $O" \
 "n256k:120:python bench.py --packets 262144 $O" \
 "n1M:120:python bench.py --packets 1048576 $O" \
 "n4M:120:python bench.py --packets 4194304 --max-copies 64 $O" \
 "n16M:200:python bench.py --packets 16777216 --max-copies 16 --steps 60 --warmup 5 $O" \
 "n64M:200:python bench.py --packets 67108864 --max-copies 4 --steps 20 --warmup 3 $O"
