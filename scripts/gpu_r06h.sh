#!/bin/bash
# Round 6 (h): the C5 store pattern (micro); the backward's tail-balanced segments on realistic rank bands
# (A/B against scripts/_abl/no_tail); the suite; the bench line.
set -o pipefail
TAG=${1:-r06h}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 ./scripts/micro/store_shape c5 > $O/store_shape_c5.txt 2>&1
rc=$?; echo "store_shape c5 rc=$rc"; fatal $rc store_c5
cat $O/store_shape_c5.txt
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c5_r8,c5_r4,c5_r2,c2_win,c2_full bwd 2 "tail:base:" "notail:no_tail:"
rc=$?; echo "ab tail rc=$rc"; fatal $rc ab_tail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
