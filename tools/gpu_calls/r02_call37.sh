# round 2: diagnostic — the look-back code compiled out (SGPR spills 70 -> 58; config B has no
# look-back candidates, so its results are unaffected) against the product build
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bnolb:120:UPE_GPU_LIB_DIAG=$V/nolb.so python bench.py $O" \
 "B0b:120:python bench.py $O" \
 "Bnolbb:120:UPE_GPU_LIB_DIAG=$V/nolb.so python bench.py $O"
