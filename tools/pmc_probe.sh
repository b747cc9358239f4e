#!/bin/bash
# PMC passes over one tools/tree_probe.py case (kernel trace only, one counter group per run).
#   tools/pmc_probe.sh <label> <case:flavour> [groups...]  -> gpurun_out/pmc_probe/<label>/<group>/
# then: python tools/pmc_table.py <out.json> <label>=gpurun_out/pmc_probe/<label> ...
set -e
label=$1; case_=$2; shift 2
groups=${*:-sq sq2 sq3 clk}
for g in $groups; do
  case $g in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" ;;
    sq2) ctr="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" ;;
    sq3) ctr="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM" ;;
    clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  esac
  mkdir -p gpurun_out/pmc_probe/$label
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_probe/$label/$g -o p --output-format csv -- python tools/tree_probe.py --steps 12 --out gpurun_out/pmc_probe/$label/probe.jsonl $case_ > gpurun_out/pmc_probe/$label/$g.log 2>&1 || { echo "pass $label $g failed rc=$?"; exit 1; }
done
