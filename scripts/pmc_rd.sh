#!/bin/bash
# Read-path PMC passes: bash scripts/pmc_rd.sh <outdir> <kernel-regex> -- <python args...>
OUT=$1; RE=$2; shift 2; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" \
         "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS" \
         "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- python3 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; }
done
