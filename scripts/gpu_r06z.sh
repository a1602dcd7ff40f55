#!/bin/bash
# Round 6 (z): fewer, wider backward column segments when the grid fills the chip with a partial last round
# (The variant was a working-tree change, measured and reverted: DESIGN.md §6 round-6 table describes it.)
# (scripts/_abl/segcap; Geo::seg_min < 0): backward parity subset on the variant (with the rank-band test),
# interleaved A/B on the rank bands and full images.
set -o pipefail
TAG=${1:-r06z}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/segcap/libcustma_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_rowband_gpu.py -m gpu -q --timeout 240 --timeout-method thread -k "backward or grad or config2 or config3 or rank_band or autograd or rowband or determin" > $O/gpu_tests_segcap.log 2>&1
rc=$?; echo "segcap subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_segcap.log | tail -12
timeout -k 10 700 bash scripts/gpu_ab.sh $TAG c5_r8,c5_r4,c5_r2,c3_win,c2_full,c2_win bwd 2 "base:base:" "segcap:segcap:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
timeout -k 10 300 bash scripts/gpu_ab.sh ${TAG}b c5_win bwd 2 "base:base:" "segcap:segcap:"
rc=$?; echo "ab c5 rc=$rc"; fatal $rc ab_c5
