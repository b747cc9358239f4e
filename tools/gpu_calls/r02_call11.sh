# round 2: config B with the ARP index read from memory instead of staged in LDS (prologue
# without the 16 KB staging; every lookup a memory round trip)
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bnoarp:120:UPE_GPU_LIB_DIAG=$V/noarp.so python bench.py $O" \
 "B0b:120:python bench.py $O" \
 "Bnoarpb:120:UPE_GPU_LIB_DIAG=$V/noarp.so python bench.py $O"
