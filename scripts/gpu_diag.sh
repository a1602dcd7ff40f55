#!/bin/bash
# Diagnostics round trip: forward ablations, store-bandwidth microbenchmark, PMC HBM traffic.
set -o pipefail
TAG=${1:-diag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 ./scripts/micro/store_bw > $O/store_bw.log 2>&1 || { echo "store_bw failed"; exit 1; }
cat $O/store_bw.log
for V in base nostore noupdate nothing storeonly skeleton; do
  if [ "$V" = base ]; then L=""; else L=scripts/_abl/$V/libcustma_hip.so; fi
  CUSTMA_LIB=$L timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c3_win --ops fwd --reps 5 > $O/kb_$V.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_$V.log; exit 1; }
  echo "== $V"; grep cfg $O/kb_$V.log
done
for NW in 2 3 4; do
  CUSTMA_SWEEP_NW=$NW timeout -k 10 300 python scripts/kbench.py --cfg c3_win --ops fwd --reps 5 > $O/kb_nw$NW.log 2>&1 || { echo "kbench nw failed"; exit 1; }
  echo "== NW=$NW"; grep cfg $O/kb_nw$NW.log
done
timeout -k 10 900 python scripts/pmc_traffic.py $O/pmc full > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log | cut -c1-400
