#!/bin/bash
# Round 6 (d): the full-layout store pattern (micro) and the sweep's store policy A/B (nt vs default);
# 32-row bands for the window tile kernel (A/B).
set -o pipefail
TAG=${1:-r06d}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 ./scripts/micro/store_full > $O/store_full.txt 2>&1
rc=$?; echo "store_full rc=$rc"; fatal $rc store_full
cat $O/store_full.txt
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c2_full,c3_full fwd 3 "nt:base:" "plain:sweep_plain:"
rc=$?; echo "ab policy rc=$rc"; fatal $rc ab_policy
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c3_win,c5_win fwd,disp 2 "th64:base:" "th32:th32:"
rc=$?; echo "ab th rc=$rc"; fatal $rc ab_th
