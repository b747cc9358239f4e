#!/bin/bash
# Round-6 PMC passes over bench.py legs, one counter group per rocprofv3 run (kernel trace only,
# as MI355X_MICROARCH.md prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).  Each pass
# directory also records when it ran and the sha256 of the libupe_gpu.so it profiled, so that
# tools/pmc_r06.py can tie every counter to the build bench.py loads.
#   tools/pmc_refresh.sh <label> <config> <mode> [groups...]
#     label: output name (B, CF, C6, C3, D); config: bench.py --config; mode: emit | inplace
#     groups: fetch write sq sq2 clk (default: fetch write sq clk)
# -> gpurun_out/pmc_r06/<label>_<mode>/<group>/p_counter_collection.csv + stamp.txt
set -e
label=$1; cfg=$2; mode=$3; shift 3
groups=${*:-fetch write sq clk}
steps="--steps ${PMC_STEPS:-20} --warmup 2 --no-cpu-baseline --no-hbm-probe --host-reps 0 --config $cfg --mode $mode --no-other-mode --no-imix --ring 0 --config-d-steps 0 --strong 0"
if [ "$cfg" = D ]; then steps="$steps --max-copies 8"; fi
lib_sha=$(sha256sum upe_amd/libupe_gpu.so | cut -c1-16)
for g in $groups; do
  case $g in
    fetch) ctr="FETCH_SIZE" ;;
    write) ctr="WRITE_SIZE" ;;
    sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" ;;
    sq2) ctr="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" ;;
    clk) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    *) echo "unknown group $g"; exit 2 ;;
  esac
  out=gpurun_out/pmc_r06/${label}_$mode/$g
  mkdir -p $out
  echo "label=$label config=$cfg mode=$mode group=$g counters=\"$ctr\" lib_sha16=$lib_sha utc=$(date -u +%Y-%m-%dT%H:%M:%SZ)" > $out/stamp.txt
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $out -o p --output-format csv -- python bench.py $steps > $out/bench.log 2>&1 || { echo "pass $label $mode $g failed rc=$?"; exit 1; }
  echo "pass $label $mode $g ok"
done
