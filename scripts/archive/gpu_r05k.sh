#!/bin/bash
# Round 5 (k): knock-out timing of the fused disparity's post-barrier scan (wrong results: timing only),
# k = 11 unit rebuilt with -DCUSTMA_KO_AMX_SCAN into custereomatching_amd/_abl/ko, alternating processes.
set -o pipefail
TAG=${1:-r05k}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for r in 1 2; do
  for v in base ko; do
    if [ $v = ko ]; then export CUSTMA_LIB=$PWD/custereomatching_amd/_abl/ko/libcustma_hip.so; else unset CUSTMA_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$r -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win,c5_win --ops disp --reps 5 > $O/kb_${v}_$r.log 2>&1
    rc=$?; echo "$v $r rc=$rc $(grep cfg $O/kb_${v}_$r.log | tr '\n' ' ' | cut -c1-300)"; fatal $rc kb_$v
    grep -h "k_fwd_tile\|merge\|recheck\|k_stats" $O/prof_${v}_$r/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
  done
done
