#!/bin/bash
# GPU parity tests, then backward timings for the default build and ablation builds.
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for A in base "$@"; do
  LIBV=""; [ "$A" != "base" ] && LIBV="CUSTMA_LIB=$PWD/scripts/_abl/$A/libcustma_hip.so"
  env $LIBV timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops bwd --reps 5 > $O/kb_$A.log 2>&1 || { echo "kbench $A failed"; tail -5 $O/kb_$A.log; exit 1; }
  echo "== $A"; grep cfg $O/kb_$A.log
done
