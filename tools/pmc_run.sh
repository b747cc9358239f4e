#!/bin/bash
# PMC passes over a bench config (each counter group in its own rocprofv3 run, kernel trace only,
# as the MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   tools/pmc_run.sh [config] [mode] [groups...]   mode: emit | inplace
#   groups: fetch write sq sq2 clk ta tcp
set -e
cfg=${1:-B}; shift || true
mode=${1:-emit}; shift || true
groups=${*:-fetch write sq clk}
lab=${PMC_LABEL:-$cfg}   # the output name (gpurun_out/pmc_<label>_<mode>/, tools/pmc_traffic.py <label>)
steps="--steps ${PMC_STEPS:-20} --warmup 2 --no-cpu-baseline --no-hbm-probe --host-reps 0 --config $cfg --mode $mode --no-other-mode --no-imix --ring 0 --config-d-steps 0"
for g in $groups; do
  case $g in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" ;;
    sq2) ctr="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" ;;
    sq3) ctr="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM" ;;
    clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    ta) ctr="TA_BUSY_avr TA_TA_BUSY_sum" ;;
    tcp) ctr="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" ;;
    tcc) ctr="TCC_HIT_sum TCC_MISS_sum" ;;
    rdreq) ctr="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" ;;
    dram) ctr="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum" ;;
  esac
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${lab}_$mode/$g -o p --output-format csv -- python bench.py $steps > gpurun_out/pmc_${lab}_${mode}_$g.log 2>&1 || { echo "pass $g failed rc=$?"; exit 1; }
done
