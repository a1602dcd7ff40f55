#!/bin/bash
# GPU test subset (or the whole suite): bash scripts/gpu_tests.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-tests}
K=${2:-}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
fi
tail -3 $O/gpu_tests.log
