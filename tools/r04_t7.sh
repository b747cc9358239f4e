set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_reload.py tests/test_gpu_worker_loop.py tests/test_gpu_dropin.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t7_tests.log 2>&1; echo tests_rc=$?
bash tools/r04_t6.sh
