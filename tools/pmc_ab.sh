#!/bin/bash
# HBM traffic per classify launch for library variants (A/B of a layout or load change):
#   tools/pmc_ab.sh <config> label=[lib.so] ...      (empty lib = the product build)
# One rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE cannot share one), kernel trace only;
# summary by tools/pmc_ab_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; shift
export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%=*}; lib=${spec#*=}
  [ "$lib" = "$spec" ] && lib=""
  envs=""; [ -n "$lib" ] && envs="UPE_GPU_LIB_DIAG=$lib"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 env $envs rocprofv3 --pmc $c -d gpurun_out/pmcab/$cfg/$label/$c -o p --output-format csv \
      -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-hbm-probe --host-reps 0 \
         --config $cfg --no-other-mode --no-imix > gpurun_out/pmcab_${cfg}_${label}_$c.log 2>&1 \
      || echo "pass $label $c failed rc=$?"
  done
done
python tools/pmc_ab_summary.py $cfg $([ "$cfg" = D ] && echo 16777216)
