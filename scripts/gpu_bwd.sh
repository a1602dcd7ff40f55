#!/bin/bash
# Backward bring-up: parity tests then kernel timings.
set -o pipefail
TAG=${1:-bwd}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "backward or autograd or band" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops fwd,bwd --reps 5 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
