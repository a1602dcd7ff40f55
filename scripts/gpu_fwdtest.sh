#!/bin/bash
# GPU parity tests, then the forward timing matrix (scripts/gpu_fwdmatrix.sh arguments).
set -o pipefail
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash scripts/gpu_fwdmatrix.sh "$@"
