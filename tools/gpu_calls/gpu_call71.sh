V=$PWD/build/var
bash tools/gpu_session.sh \
 "stamps:200:UPE_GPU_LIB_DIAG=$V/stamps.so python tools/stamps.py 1048576"
