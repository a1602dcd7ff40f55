#!/bin/bash
# Backward ablation round trip: parity subset on the default build, then kbench per variant.
set -o pipefail
TAG=${1:-abl}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "backward or autograd or band" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=scripts/_abl/$V/libcustma_hip.so; fi
  CUSTMA_LIB=$L timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c3_win --ops bwd --reps 5 > $O/kb_$V.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_$V.log; exit 1; }
  echo "== $V"; cat $O/kb_$V.log | grep cfg
done
