#!/bin/bash
# Round 5 (s): the exact forward with batched patch-row loads: the suite, then exact-forward timings (vs
# r05d: C3 window k = 19 / 25 / 31 8.51 / 15.0 / 23.3 ms) with a kernel trace.
set -o pipefail
TAG=${1:-r05s}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win_k19,c3_win_k25,c3_win_k31,c3_full_k19 --ops fwd --reps 5 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep cfg $O/kbench.log; fatal $rc kbench
