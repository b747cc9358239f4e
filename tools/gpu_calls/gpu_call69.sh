bash tools/gpu_session.sh \
 "w2:200:python bench.py --workers-per-gpu 2 --no-cpu-baseline --no-hbm-probe" \
 "w3:200:python bench.py --workers-per-gpu 3 --no-cpu-baseline --no-hbm-probe" \
 "w4:200:python bench.py --workers-per-gpu 4 --no-cpu-baseline --no-hbm-probe" \
 "Cw2:200:python bench.py --config C --workers-per-gpu 2 --no-cpu-baseline --no-hbm-probe"
