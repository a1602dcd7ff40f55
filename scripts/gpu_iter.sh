#!/bin/bash
# parity subset then interleaved A/B: bash scripts/gpu_iter.sh <tag> "<pytest -k expr>" <cfg> <ops> <rounds> <spec>...
set -o pipefail
TAG=$1; TK=$2; shift 2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$TK" > gpurun_out/$TAG/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$TAG/test.log; exit 1; }
tail -1 gpurun_out/$TAG/test.log
bash scripts/gpu_ab.sh $TAG "$@"
