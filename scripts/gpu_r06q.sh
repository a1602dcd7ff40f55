#!/bin/bash
# Round 6 (q): disparity merge tile height (CUSTMA_MTY: 4 rows = base, 8, 16 -- fewer projector-strip rows
# staged per pixel): disparity parity subset on each variant, interleaved A/B, kernel traces.
set -o pipefail
TAG=${1:-r06q}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for v in mty8 mty16; do
  CUSTMA_LIB=$PWD/scripts/_abl/$v/libcustma_hip.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "disparity or soft or config" > $O/gpu_tests_$v.log 2>&1
  rc=$?; echo "$v subset rc=$rc"; fatal $rc subset_$v
  grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_$v.log | tail -6
done
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c3_win,c5_win,c2_win disp,soft 3 "base:base:" "mty8:mty8:" "mty16:mty16:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base mty8 mty16; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$v c5_win disp > $O/prof_c5_disp_$v.txt 2>&1
  rc=$?; echo "prof $v rc=$rc"; fatal $rc prof_$v
  grep -E "merge" $O/prof_c5_disp_$v.txt | cut -c1-110
done
