#!/bin/bash
# Round 5 (x): volume argmax, the batched loads for rows longer than 512 only -- A/B against the previous
# HEAD~ linked into custereomatching_amd/_abl/oldsel), alternating processes, then the suite.
set -o pipefail
TAG=${1:-r05x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for r in 1; do
  for v in new old; do
    if [ $v = old ]; then export CUSTMA_LIB=$PWD/custereomatching_amd/_abl/oldsel/libcustma_hip.so; else unset CUSTMA_LIB; fi
    timeout -k 10 200 python3 scripts/ab_argmax.py > $O/am_${v}_$r.log 2>&1
    rc=$?; echo "$v $r rc=$rc $(grep cfg $O/am_${v}_$r.log | tr '\n' ' ')"; fatal $rc am_$v
  done
done
unset CUSTMA_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
