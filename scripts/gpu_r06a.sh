#!/bin/bash
# Round 6 (a): the round's starting library (split / fused forwards removed) -- suite, kernel baselines,
# the backward's no-volume knock-out, the persistent store pattern, and the bench line.
set -o pipefail
TAG=${1:-r06a}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 ./scripts/micro/store_shape > $O/store_shape.txt 2>&1
rc=$?; echo "store_shape rc=$rc"; fatal $rc store_shape
tail -4 $O/store_shape.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
for c in "c3_win fwd,bwd,disp,soft" "c5_win fwd,bwd,disp" "c2_full fwd,bwd,disp"; do
  set -- $c
  timeout -k 10 400 bash scripts/prof_kernels.sh $TAG/$1 $1 $2 > $O/prof_$1.txt 2>&1
  rc=$?; echo "prof $1 rc=$rc"; fatal $rc prof_$1
  cat $O/$1/prof.log | grep '^{'
  head -12 $O/prof_$1.txt
done
timeout -k 10 400 bash scripts/gpu_ko.sh $TAG/ko c5_win ko_novol
rc=$?; echo "ko rc=$rc"; fatal $rc ko
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
