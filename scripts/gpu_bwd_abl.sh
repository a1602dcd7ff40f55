#!/bin/bash
# Backward ablations: kbench bwd time + FETCH_SIZE per variant (GPU box; diagnostic only).
set -o pipefail
TAG=${1:-babl}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=scripts/_abl/$V/libcustma_hip.so; fi
  CUSTMA_LIB=$L timeout -k 10 200 python scripts/kbench.py --cfg c2_full --ops bwd --reps 5 > $O/kb_$V.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_$V.log; exit 1; }
  echo "== $V"; grep cfg $O/kb_$V.log
  CUSTMA_LIB=$L timeout -k 10 300 python scripts/pmc_run.py $O/pmc_$V k_bwd_sweep "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" -- python3 scripts/kbench.py --cfg c2_full --ops bwd --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
