#!/bin/bash
# Round 5: localise the window k = 4 backward failure (scripts/diag_bwd.py, every BWD_CASES entry),
# then the whole GPU suite without -x so that every test is reached.
# Usage: bash scripts/gpu_r05a.sh <tag>
set -o pipefail
TAG=${1:-r05a}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u scripts/diag_bwd.py --all > $O/diag_bwd.log 2>&1
rc=$?
grep -B1 -A2 FAIL $O/diag_bwd.log | head -80
echo "diag rc=$rc"
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -40
exit $rc
