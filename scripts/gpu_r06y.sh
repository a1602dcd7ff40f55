#!/bin/bash
# Round 6 (y): kernel traces of the N = 8 per-rank band (c5_r8: 512 rows of BASELINE configs[4] + halos), forward
# and backward, against the whole image (c5_win) -- what the strong-scaling efficiency loses per rank.
set -o pipefail
TAG=${1:-r06y}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for c in c5_r8 c5_r4; do
  timeout -k 10 200 python3 scripts/kbench.py --cfg $c --ops fwd,bwd --reps 10 > $O/kbench_$c.log 2>&1
  rc=$?; echo "kbench $c rc=$rc"; fatal $rc kbench_$c
  grep cfg $O/kbench_$c.log
  timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$c $c fwd,bwd > $O/prof_$c.txt 2>&1
  rc=$?; echo "prof $c rc=$rc"; fatal $rc prof_$c
  head -16 $O/prof_$c.txt | cut -c1-130
done
