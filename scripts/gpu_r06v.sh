#!/bin/bash
# Round 6 (v): k_bwd_rem_rows row bands halved until the grid has CUSTMA_REM_WAVES waves (2048 / 4096 / 8192;
# the main library: fixed 64-row bands): backward parity subset on the 4096 build, interleaved A/B, traces.
set -o pipefail
TAG=${1:-r06v}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/rw4096/libcustma_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_rowband_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "backward or grad or config or autograd or after_a_large or rowband or determin or rem" > $O/gpu_tests_rw4096.log 2>&1
rc=$?; echo "rw4096 subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_rw4096.log | tail -12
timeout -k 10 600 bash scripts/gpu_ab.sh $TAG c2_win,c3_win,c5_r8,c5_win bwd 2 "base:base:" "rw2048:rw2048:" "rw4096:rw4096:" "rw8192:rw8192:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base rw4096; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  for c in c3_win c2_win; do
    CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_${v}_$c $c bwd > $O/prof_${c}_bwd_$v.txt 2>&1
    rc=$?; echo "prof $v $c rc=$rc"; fatal $rc prof_$v
    grep -E "rem_rows|coop" $O/prof_${c}_bwd_$v.txt | cut -c1-110
  done
done
