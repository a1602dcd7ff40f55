#!/bin/bash
# Write-path PMC passes: bash scripts/pmc_wr.sh <outdir> <kernel-regex> -- <python args...>
OUT=$1; RE=$2; shift 2; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for P in "SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_BUSY_avr" \
         "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TD_TC_STALL_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- python3 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; }
done
