#!/bin/bash
# Round 6 (l): k_bwd_rem_rows with a 4-deep load ring (scripts/_abl/remring) against the main library:
# (Run as r06o: the first run, r06l, compared two builds that both held the change -- build_variant relinked the main library then.)
# backward parity subset on the variant, interleaved backward A/B (C5, C3, configs[2] window), kernel traces.
set -o pipefail
TAG=${1:-r06l}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/remring/libcustma_hip.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread -k "backward or grad or config or autograd or after_a_large" > $O/gpu_tests_remring.log 2>&1
rc=$?; echo "remring subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_remring.log | tail -12
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c5_win,c3_win,c2_win bwd 3 "base:base:" "remring:remring:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base remring; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$v c5_win bwd > $O/prof_c5_bwd_$v.txt 2>&1
  rc=$?; echo "prof $v rc=$rc"; fatal $rc prof_$v
  head -8 $O/prof_c5_bwd_$v.txt | cut -c1-120
done
