#!/bin/bash
# Round 5: localise the window k = 4 backward failure (scripts/diag_bwd.py, every BWD_CASES entry),
# the whole GPU suite without -x (every test reached), the split-forward A/B, a kernel trace of the
# C3 / C5 ops and the contract bench line.  A test failure does not stop the measurements; a crash,
# abort or time limit (rc 124 / 134 / 137 / 139) ends the script.
# Usage: bash scripts/gpu_r05a.sh <tag> [--no-bench]
set -o pipefail
TAG=${1:-r05a}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u scripts/diag_bwd.py --all > $O/diag_bwd.log 2>&1
rc=$?; echo "diag rc=$rc"; fatal $rc diag
grep -B1 -A2 FAIL $O/diag_bwd.log | head -60
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -40
timeout -k 10 300 python -u scripts/ab_split.py 4 > $O/ab_split.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $O/ab_split.log | tail -4; fatal $rc ab_split
[ "$2" = "--no-bench" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win,c5_win --ops fwd,bwd,disp --reps 5 > $O/kbench.log 2>&1
rc=$?; echo "trace rc=$rc"; fatal $rc trace
grep cfg $O/kbench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" $O/kernel_stats.csv
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cat $O/bench.json
