#!/bin/bash
# Round 6 (x): the LDS-tiled disparity merge for full layouts too (4-row tiles, whole-row projector strips; scripts/_abl/mfull)
# (The variant was a working-tree change, measured and reverted: DESIGN.md §6 round-6 table describes it.)
# against the main library: disparity parity subset on the variant, interleaved A/B, kernel traces.
set -o pipefail
TAG=${1:-r06x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/*/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
CUSTMA_LIB=$PWD/scripts/_abl/mfull/libcustma_hip.so timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "disparity or soft or argmax or config or select or rowband" > $O/gpu_tests_mfull.log 2>&1
rc=$?; echo "mfull subset rc=$rc"; fatal $rc subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_mfull.log | tail -12
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c2_full,c3_win disp,soft 3 "base:base:" "mfull:mfull:"
rc=$?; echo "ab rc=$rc"; fatal $rc ab
for v in base mfull; do
  L=$PWD/scripts/_abl/$v/libcustma_hip.so; [ $v = base ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  for c in c2_full; do
    CUSTMA_LIB=$L timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_${v}_$c $c disp > $O/prof_${c}_disp_$v.txt 2>&1
    rc=$?; echo "prof $v $c rc=$rc"; fatal $rc prof_$v
    grep -E "recheck|merge|k_fwd_tile|k_sweep|k_stats" $O/prof_${c}_disp_$v.txt | cut -c1-110
  done
done
