#!/bin/bash
# Forward bring-up: full GPU parity tests, then kbench fwd with env variants ("name=ENV=VAL ...").
set -o pipefail
TAG=${1:-fwd}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops fwd --reps 5 > $O/kb_base.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb_base.log; exit 1; }
echo "== base"; grep cfg $O/kb_base.log
for V in "$@"; do
  env $V timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops fwd --reps 5 > $O/kb_v.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_v.log; exit 1; }
  echo "== $V"; grep cfg $O/kb_v.log
done
