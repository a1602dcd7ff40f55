#!/bin/bash
# Forward variants: GPU parity tests, then kbench fwd for the base build and each ablation build named.
set -o pipefail
TAG=${1:-fv}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=scripts/_abl/$V/libcustma_hip.so; fi
  CUSTMA_LIB=$L timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops fwd,disp --reps 5 > $O/kb_$V.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_$V.log; exit 1; }
  echo "== $V"; grep cfg $O/kb_$V.log
done
