#!/bin/bash
# Round 5 (f): which stage of the window k = 4 backward reads state a previous kernel left behind.
set -o pipefail
TAG=${1:-r05f}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
timeout -k 10 300 python -u scripts/diag_pollute.py > $O/diag_pollute.log 2>&1
rc=$?; echo "diag_pollute rc=$rc"; cat $O/diag_pollute.log | cut -c1-600
