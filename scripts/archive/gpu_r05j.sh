#!/bin/bash
# Round 5 (j): sweep_fwd.hip (full-layout forward / disparity loader) under vmcnt_check: the suite, the
# full-layout kbench (vs r05i: C2 1.224 / C3 9.89 ms kernel) and the bench line.
set -o pipefail
TAG=${1:-r05j}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 python3 scripts/kbench.py --cfg c2_full,c3_full,c3_win --ops fwd,disp --reps 5 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep cfg $O/kbench.log; fatal $rc kbench
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
