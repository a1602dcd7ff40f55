#!/bin/bash
# Round 5 (q): the per-slot gather (more than 8 slots: full layouts) in batches of 8 unconditional loads: the
# suite, then backward timings with a kernel trace (vs r05o: C2 full gather 0.187 ms).
set -o pipefail
TAG=${1:-r05q}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c2_full,c3_full,c3_win --ops bwd --reps 5 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep cfg $O/kbench.log; fatal $rc kbench
