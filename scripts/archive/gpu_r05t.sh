#!/bin/bash
# Round 5 (t): the backward combine with batched tile and output loads: the suite, then backward timings
# with a kernel trace (vs r05o: combine3 C3 0.0754, C5 0.562 ms).
set -o pipefail
TAG=${1:-r05t}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win,c5_win,c2_full --ops bwd --reps 5 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep cfg $O/kbench.log; fatal $rc kbench
