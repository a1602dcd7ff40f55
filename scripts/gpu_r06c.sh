#!/bin/bash
# Round 6 (c): the suite at kFastVolumeMaxK = 11; the full-layout store pattern (micro) and the sweep's store
# policy A/B; 32-row bands for the window tile kernel (A/B); a 2-rank gloo rehearsal of bench.py's N > 1 path
# on one GPU; the bench line.
set -o pipefail
TAG=${1:-r06c}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 ./scripts/micro/store_full > $O/store_full.txt 2>&1
rc=$?; echo "store_full rc=$rc"; fatal $rc store_full
cat $O/store_full.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 900 bash scripts/gpu_ab.sh $TAG c2_full,c3_full fwd 3 "nt:base:" "plain:sweep_plain:"
rc=$?; echo "ab policy rc=$rc"; fatal $rc ab_policy
timeout -k 10 900 bash scripts/gpu_ab.sh $TAG c3_win,c5_win fwd,disp 2 "th64:base:" "th32:th32:"
rc=$?; echo "ab th rc=$rc"; fatal $rc ab_th
timeout -k 10 600 python3 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err
rc=$?; echo "gloo rehearsal rc=$rc"; fatal $rc gloo
cut -c1-600 $O/bench_n2_gloo.json
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
