#!/bin/bash
# round 5: SQ counters of config D's classify, full table and frames only (tools/d_probe.py)
set -e
for v in full small; do
  for g in sq sq2 clk; do
    case $g in
      sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" ;;
      sq2) ctr="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" ;;
      clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    esac
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d gpurun_out/pmc_Dsq/$v/$g -o p --output-format csv -- python tools/d_probe.py $v --steps 4 > gpurun_out/pmc_Dsq_${v}_$g.log 2>&1 || { echo "pass $v $g failed"; exit 1; }
  done
done
echo pmcD_done
