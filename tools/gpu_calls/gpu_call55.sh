bash tools/gpu_session.sh \
 "tssT:300:python -u -m pytest tests/test_gpu_parity.py -x -q -k 'config_d or digest or kinds or tuple' --timeout 200 --timeout-method thread" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Ctss:100:UPE_GPU_TSS=1 python bench.py --config C --no-cpu-baseline --no-hbm-probe"
