#!/bin/bash
# Round 6 (g): the suite with the tail-balanced grids (tile forward band height, backward column segments) and
# the med3 plain scans; same-box A/B of the tail balancing (scripts/_abl/no_tail) at configs[3], configs[2]'s
# window, and one rank's band of configs[4] at N = 2 / 4 / 8.
set -o pipefail
TAG=${1:-r06g}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c3_win,c2_win fwd,bwd,disp,soft 2 "tail:base:" "notail:no_tail:"
rc=$?; echo "ab tail c3/c2 rc=$rc"; fatal $rc ab_tail1
timeout -k 10 500 bash scripts/gpu_ab.sh ${TAG}b c5_r8,c5_r4,c5_r2 fwd,bwd 2 "tail:base:" "notail:no_tail:"
rc=$?; echo "ab tail c5 bands rc=$rc"; fatal $rc ab_tail2
