#!/bin/bash
# GPU tests + per-kernel A/B (rocprofv3 kernel trace) of the working tree against a HEAD build.
# Usage: bash scripts/gpu_r03c.sh <tag> <cfgs> <ops> [pytest -k expr]
set -o pipefail
TAG=$1; CFG=$2; OPS=$3; KX=${4:-}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$KX" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$KX" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
bash scripts/gpu_kprof.sh $TAG $CFG $OPS "new:base:" "head:head:" "new2:base:" "head2:head:"
