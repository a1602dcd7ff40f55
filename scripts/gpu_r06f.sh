#!/bin/bash
# Round 6 (f): kernel traces of the north-star forward (C3) and of the bench workload (C5), smoke, the bench line.
set -o pipefail
TAG=${1:-r06f}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 bash scripts/prof_kernels.sh $TAG/c3 c3_win fwd,bwd,disp,soft > $O/prof_c3.txt 2>&1
rc=$?; echo "prof c3 rc=$rc"; fatal $rc prof_c3
head -14 $O/prof_c3.txt
timeout -k 10 300 bash scripts/prof_kernels.sh $TAG/c2 c2_full fwd,bwd,disp,soft > $O/prof_c2.txt 2>&1
rc=$?; echo "prof c2 rc=$rc"; fatal $rc prof_c2
head -10 $O/prof_c2.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-400 $O/bench.json
