#!/bin/bash
# Backward bring-up: GPU parity tests, then kbench bwd for env variants.
set -o pipefail
TAG=${1:-bw}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in NONE=1 "$@"; do
  env $V timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops bwd --reps 5 > $O/kb.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb.log; exit 1; }
  echo "== $V"; grep cfg $O/kb.log
done
