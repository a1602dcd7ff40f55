#!/bin/bash
# Round 6 (f): the med3 plain-scan A/B; kernel traces of the north-star forward (C3) and of the bench workload (C5), smoke, the bench line.
set -o pipefail
TAG=${1:-r06f}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
# the plain argmax scans with v_med3 / v_max (scripts/_abl/scan_med3): disparity tests, then a same-box A/B
CUSTMA_LIB=$PWD/scripts/_abl/scan_med3/libcustma_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "disparity or tile_variants or config3 or sliding" > $O/gpu_tests_med3.log 2>&1
rc=$?; echo "med3 subset rc=$rc"; fatal $rc med3_subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_med3.log | tail -20
timeout -k 10 400 bash scripts/gpu_ab.sh $TAG c3_win,c5_win,c2_full disp 2 "scan:base:" "med3:scan_med3:"
rc=$?; echo "ab med3 rc=$rc"; fatal $rc ab_med3
timeout -k 10 300 bash scripts/prof_kernels.sh $TAG/c3 c3_win fwd,bwd,disp,soft > $O/prof_c3.txt 2>&1
rc=$?; echo "prof c3 rc=$rc"; fatal $rc prof_c3
head -14 $O/prof_c3.txt
timeout -k 10 300 bash scripts/prof_kernels.sh $TAG/c2 c2_full fwd,bwd,disp,soft > $O/prof_c2.txt 2>&1
rc=$?; echo "prof c2 rc=$rc"; fatal $rc prof_c2
head -10 $O/prof_c2.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
