#!/bin/bash
# Round 5 (b): the suite at the new defaults, the forward A/B/C/D (fused sc1 / fused acquire / split /
# single), kernel sizes >= 18 (exact forward, even-k sliding backward and disparity) and the bench line.
# A test failure does not stop the measurements; a crash, abort or time limit ends the script.
# Usage: bash scripts/gpu_r05b.sh <tag>
set -o pipefail
TAG=${1:-r05b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 python -u scripts/ab_split.py 4 > $O/ab_split.log 2>&1
rc=$?; echo "ab rc=$rc"; grep cfg $O/ab_split.log; fatal $rc ab_split
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win_k19,c3_win_k25,c3_win_k31,c3_full_k19,c3_win_k18,c3_win_k22,c3_win_k30 --ops fwd,bwd,disp --reps 3 > $O/kbench_bigk.log 2>&1
rc=$?; echo "bigk rc=$rc"; grep cfg $O/kbench_bigk.log; fatal $rc bigk
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cat $O/bench.json
