#!/bin/bash
# Round 6 (e): the suite with the soft-argmax two-pass scans and the full-layout 16-byte stores; same-box A/B
# of those stores against the dword build (scripts/_abl/sweep_dword); disparity / soft timings.
set -o pipefail
TAG=${1:-r06e}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 400 bash scripts/gpu_ab.sh $TAG c2_full,c3_full fwd 3 "x4:base:" "dword:sweep_dword:"
rc=$?; echo "ab x4 rc=$rc"; fatal $rc ab_x4
timeout -k 10 300 python3 scripts/kbench.py --cfg c3_win,c5_win,c2_full --ops fwd,disp,soft --reps 10 > $O/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; fatal $rc kbench
cat $O/kbench.log
