set -o pipefail
export TMPDIR=/tmp
UPE_GPU_LIB_DIAG=build/var/stamps.so timeout -k 10 120 python tools/stamps.py 1048576 emit B > gpurun_out/r04_stamps_B.txt 2>&1 || exit 1
UPE_GPU_LIB_DIAG=build/var/stamps.so timeout -k 10 120 python tools/stamps.py 1048576 emit C > gpurun_out/r04_stamps_C.txt 2>&1 || exit 1
tail -25 gpurun_out/r04_stamps_B.txt
