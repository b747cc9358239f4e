bash tools/gpu_session.sh \
 "profC:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C"
