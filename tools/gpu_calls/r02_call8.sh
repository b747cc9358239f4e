# round 2: does the number of distinct batch copies the bench cycles through (its HBM working
# set) change the config-B step time?  8 / 16 / 32 copies (512 MB - 2 GB, 2-8x the Infinity
# Cache) against the default (one copy per step, 14 GB)
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
bash tools/gpu_session.sh \
 "c220:120:python bench.py $O" \
 "c8:120:python bench.py --max-copies 8 $O" \
 "c16:120:python bench.py --max-copies 16 $O" \
 "c32:120:python bench.py --max-copies 32 $O" \
 "c220b:120:python bench.py $O" \
 "c8b:120:python bench.py --max-copies 8 $O" \
 "c16b:120:python bench.py --max-copies 16 $O" \
 "C32:120:python bench.py --config C $O" \
 "C8:120:python bench.py --config C --max-copies 8 $O" \
 "C220:120:python bench.py --config C $O --max-copies 160"
