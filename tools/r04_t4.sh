set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t4_dropin.log 2>&1; echo dropin_rc=$?
timeout -k 10 300 python -u -m pytest tests/test_gpu_reload.py tests/test_gpu_worker_loop.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stream or rule_reload" > gpurun_out/r04_t4_tests.log 2>&1; echo tests_rc=$?
