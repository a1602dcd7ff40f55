#!/bin/bash
# Forward: GPU parity tests, then kbench fwd for the default build and ablation builds.
# Usage (via gpurun): bash scripts/gpu_fwdabl.sh <tag> [cfgs] [abl ...]
set -o pipefail
TAG=${1:-fwdabl}; CFG=${2:-c2_full,c3_win}; shift; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --cfg $CFG --ops fwd --reps 5 > $O/kb_base.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb_base.log; exit 1; }
echo "== base"; grep cfg $O/kb_base.log
for A in "$@"; do
  CUSTMA_LIB=$PWD/scripts/_abl/$A/libcustma_hip.so timeout -k 10 300 python scripts/kbench.py --cfg $CFG --ops fwd --reps 5 > $O/kb_$A.log 2>&1 || { echo "kbench $A failed"; tail -5 $O/kb_$A.log; exit 1; }
  echo "== $A"; grep cfg $O/kb_$A.log
done
