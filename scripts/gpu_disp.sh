#!/bin/bash
# GPU parity tests, then disparity timings (tile kernel vs the LDS-form partials).
set -o pipefail
TAG=$1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --cfg c2_win,c3_win --ops disp --reps 5 > $O/kb.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb.log; exit 1; }
echo "== tile"; grep cfg $O/kb.log
CUSTMA_FWD_TILE=0 timeout -k 10 300 python scripts/kbench.py --cfg c2_win,c3_win --ops disp --reps 5 > $O/kb0.log 2>&1 || { echo "kbench0 failed"; tail -5 $O/kb0.log; exit 1; }
echo "== lds-form"; grep cfg $O/kb0.log
