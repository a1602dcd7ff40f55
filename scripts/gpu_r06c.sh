#!/bin/bash
# Round 6 (c): the suite at kFastVolumeMaxK = 11; the two-pass disparity scan (scripts/_abl/scan2: its parity
# subset and a same-box A/B); a 2-rank gloo rehearsal of bench.py's N > 1 path on one GPU.
set -o pipefail
TAG=${1:-r06c}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/scan2/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
CUSTMA_LIB=$PWD/scripts/_abl/scan2/libcustma_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fast_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "disparity or soft or tile_variants or config3 or sliding or config0" > $O/gpu_tests_scan2.log 2>&1
rc=$?; echo "scan2 subset rc=$rc"; fatal $rc scan2_subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_scan2.log | tail -20
timeout -k 10 400 bash scripts/gpu_ab.sh $TAG c3_win,c5_win,c2_full disp,soft 2 "scan1:base:" "scan2:scan2:"
rc=$?; echo "ab scan rc=$rc"; fatal $rc ab_scan
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err
rc=$?; echo "gloo rehearsal rc=$rc"; fatal $rc gloo
cut -c1-700 $O/bench_n2_gloo.json
