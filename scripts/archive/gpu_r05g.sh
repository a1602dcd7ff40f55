#!/bin/bash
# Round 5 (g): the in-flight-register fix (backward prologue, build-time vmcnt_check.py) -- the window
# k = 4 backward after other kernels, the suite, the forward A/B (single-stream times vs r05d) and the
# bench line.  Usage: bash scripts/gpu_r05g.sh <tag>
set -o pipefail
TAG=${1:-r05g}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u scripts/diag_pollute.py > $O/diag_pollute.log 2>&1
rc=$?; echo "diag_pollute rc=$rc"; grep -v amdgpu.ids $O/diag_pollute.log | cut -c1-300; fatal $rc diag_pollute
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 python -u scripts/ab_split.py 3 > $O/ab_split.log 2>&1
rc=$?; echo "ab rc=$rc"; grep cfg $O/ab_split.log | cut -c1-400; fatal $rc ab_split
timeout -k 10 300 python3 scripts/kbench.py --cfg c3_win,c5_win --ops disp,bwd --reps 3 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep cfg $O/kbench.log | cut -c1-300; fatal $rc kbench
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-600 $O/bench.json
