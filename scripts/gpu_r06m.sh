#!/bin/bash
# Round 6 (m): k_bwd_coop at three workgroups per CU (CUSTMA_BWD_OCC3: 6-step flushes, single-buffered A rows, no camera LDS block) (scripts/_abl/occ3) against the main library:
# (The variant was a working-tree change, measured and reverted: DESIGN.md §6 round-6 table describes it.)
# backward parity subset on the variant, interleaved backward A/B (C5, C3, configs[2] window), kernel traces.
set -o pipefail
TAG=${1:-r06m}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/occ3/libcustma_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread -k "backward or grad or config or autograd or after_a_large" > $O/gpu_tests_occ3.log 2>&1
rc=$?; echo "occ3 subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_occ3.log | tail -12
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c5_win,c3_win,c2_win,c5_r8 bwd 3 "base:base:" "occ3:occ3:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base occ3; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$v c5_win bwd > $O/prof_c5_bwd_$v.txt 2>&1
  rc=$?; echo "prof $v rc=$rc"; fatal $rc prof_$v
  head -8 $O/prof_c5_bwd_$v.txt | cut -c1-120
done
