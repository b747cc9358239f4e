# round 2: config C with line-aligned frames (every header window inside one 128-byte line)
# against the packed layout; parity of the aligned layout
O="--config C --no-cpu-baseline --no-hbm-probe --no-other-mode"
bash tools/gpu_session.sh \
 "Cp:150:python bench.py $O" \
 "Cl:150:UPE_SYNTH_LAYOUT=line python bench.py $O" \
 "Cpb:150:python bench.py $O" \
 "Clb:150:UPE_SYNTH_LAYOUT=line python bench.py $O" \
 "Cli:150:UPE_SYNTH_LAYOUT=line python bench.py $O --mode inplace" \
 "Cpi:150:python bench.py $O --mode inplace" \
 "alt:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k line_aligned"
