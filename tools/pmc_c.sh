#!/bin/bash
# PMC passes over tools/c_probe.py settings (config C): traffic (FETCH_SIZE, WRITE_SIZE) and SQ
# groups, each counter group in its own rocprofv3 run (kernel trace only).
#   tools/pmc_c.sh <setting> [groups...]   -> gpurun_out/pmc_C<setting>_emit/<group>/
set -e
setting=${1:-packed}; shift || true
groups=${*:-fetch write sq sq2 sq3 clk}
for g in $groups; do
  case $g in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" ;;
    sq2) ctr="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" ;;
    sq3) ctr="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM" ;;
    clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  esac
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmc_C${setting}_emit/$g -o p --output-format csv -- python tools/c_probe.py $setting 40 > gpurun_out/pmc_C${setting}_$g.log 2>&1 || { echo "pass $g failed rc=$?"; exit 1; }
done
