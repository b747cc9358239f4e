#!/bin/bash
# round 5: HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the tree legs (CF, C6) and config D's
# frame / table split (tools/d_probe.py full | small)
set -e
PMC_STEPS=10 PMC_LABEL=CF bash tools/pmc_run.sh C emit fetch write
PMC_STEPS=10 PMC_LABEL=C6 bash tools/pmc_run.sh C6 emit fetch write
for v in full small; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -d gpurun_out/pmc_Dsplit/$v/$c -o p --output-format csv -- python tools/d_probe.py $v --steps 6 > gpurun_out/pmc_Dsplit_${v}_$c.log 2>&1 || { echo "pass $v $c failed"; exit 1; }
  done
done
timeout -k 10 200 python tools/d_probe.py full > gpurun_out/d_probe.log 2>&1
timeout -k 10 200 python tools/d_probe.py small >> gpurun_out/d_probe.log 2>&1
echo pmc2_done
