#!/bin/bash
# Round 5 (h): forward A/B on one box -- the three-phase sweep (HEAD) against the previous single-loop
# sweep (k = 11 unit rebuilt from 90993cb into custereomatching_amd/_abl/oldsw), alternating processes.
set -o pipefail
TAG=${1:-r05h}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export CUSTMA_LIB=$PWD/custereomatching_amd/_abl/oldsw/libcustma_hip.so; else unset CUSTMA_LIB; fi
    timeout -k 10 200 python3 scripts/kbench.py --cfg c3_win,c5_win --ops fwd,disp --reps 5 > $O/kb_${v}_$r.log 2>&1
    rc=$?; echo "$v $r rc=$rc $(grep cfg $O/kb_${v}_$r.log | tr '\n' ' ' | cut -c1-400)"; fatal $rc kb_$v
  done
done
