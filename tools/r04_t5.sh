set -o pipefail
timeout -k 10 120 python -u tools/r04_debug_reload.py > gpurun_out/r04_t5_debug.log 2>&1; echo dbg_rc=$?
