#!/bin/bash
# Round 5 (e): the window k = 4 backward failure -- workspace-fill dependence (scripts/diag_ws.py, per
# region), the same case after other ops, the parity file alone, then the whole suite.
set -o pipefail
TAG=${1:-r05e}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u scripts/diag_ws.py > $O/diag_ws.log 2>&1
rc=$?; echo "diag_ws rc=$rc"; grep -v "amdgpu.ids" $O/diag_ws.log | grep -E "depends on fill \[.*True|e-0[1-4]|after|recompute, only|pixels" | head -60; fatal $rc diag_ws
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "^FAILED|passed|failed" $O/parity.log | tail -12; fatal $rc parity
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^FAILED|passed|failed" $O/gpu_tests.log | tail -12; fatal $rc suite
