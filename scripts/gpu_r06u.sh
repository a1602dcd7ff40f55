#!/bin/bash
# Round 6 (u): k_bwd_cover with one wave per (class, column) and a ballot prefix (scripts/_abl/cover) against the
# main library: the backward parity subset on the variant, interleaved backward A/B, kernel traces (C2 full).
set -o pipefail
TAG=${1:-r06u}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/cover/libcustma_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_rowband_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "backward or grad or config or autograd or after_a_large or rowband or determin" > $O/gpu_tests_cover.log 2>&1
rc=$?; echo "cover subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_cover.log | tail -12
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c2_full,c2_win,c3_win,c5_r8 bwd 3 "base:base:" "cover:cover:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base cover; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$v c2_full bwd > $O/prof_c2_full_bwd_$v.txt 2>&1
  rc=$?; echo "prof $v rc=$rc"; fatal $rc prof_$v
  grep -E "cover|gather|coop" $O/prof_c2_full_bwd_$v.txt | cut -c1-110
done
