#!/bin/bash
# Round 6 (j): band height of the full-layout sweep (k_sweep_fwd): 64 (base) vs 96 vs 128 rows, volume and
# disparity at C2 full and C3 full, interleaved on one box; parity subset on the 128-row build.
set -o pipefail
TAG=${1:-r06j}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
timeout -k 10 600 bash scripts/gpu_ab.sh $TAG c2_full,c3_full fwd,disp 3 "base:base:" "th96:sweep_th96:" "th128:sweep_th128:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
CUSTMA_LIB=$PWD/scripts/_abl/sweep_th128/libcustma_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "full or config2 or config3" > $O/gpu_tests_th128.log 2>&1
rc=$?; echo "th128 subset rc=$rc"; fatal $rc th128
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_th128.log | tail -8
