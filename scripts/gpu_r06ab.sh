#!/bin/bash
# Round 6 (ab): window tile forward / disparity with 128-row bands (scripts/_abl/wth128, CUSTMA_WAVE_TH=128) against
# the main library's 64: interleaved A/B at C5 and C3, forward and disparity.
set -o pipefail
TAG=${1:-r06ab}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 700 bash scripts/gpu_ab.sh $TAG c5_win,c3_win,c5_r8 fwd,disp 3 "base:base:" "wth128:wth128:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
