#!/bin/bash
# Forward timing matrix on one box: each argument "name:abl:ENV=VAL,ENV=VAL" (abl = ablation build
# under scripts/_abl or "base"), kbench fwd over CFG.  Usage: bash scripts/gpu_fwdmatrix.sh <tag> <cfgs> <spec...>
set -o pipefail
TAG=$1; CFG=$2; shift; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for S in "$@"; do
  IFS=: read NAME ABL ENVS <<< "$S"
  LIBV=""; [ "$ABL" != "base" ] && LIBV="CUSTMA_LIB=$PWD/scripts/_abl/$ABL/libcustma_hip.so"
  env $LIBV ${ENVS//,/ } timeout -k 10 300 python scripts/kbench.py --cfg $CFG --ops fwd --reps 10 > $O/kb_$NAME.log 2>&1 || { echo "kbench $NAME failed"; tail -5 $O/kb_$NAME.log; exit 1; }
  echo "== $NAME"; grep cfg $O/kb_$NAME.log
done
