#!/bin/bash
# PMC passes over a bench config (each counter group in its own rocprofv3 run, kernel trace only,
# as the MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   tools/pmc_run.sh [config] [groups...]   groups: fetch write sq clk
set -e
cfg=${1:-B}; shift || true
groups=${*:-fetch write sq clk}
steps="--steps 20 --warmup 2 --no-cpu-baseline --config $cfg"
for g in $groups; do
  case $g in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" ;;
    sq2) ctr="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM" ;;
    clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  esac
  rocprofv3 --pmc $ctr -d gpurun_out/pmc_$cfg/$g -o p --output-format csv -- python bench.py $steps > gpurun_out/pmc_${cfg}_$g.log 2>&1
done
