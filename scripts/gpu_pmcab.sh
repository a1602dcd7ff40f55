#!/bin/bash
# FETCH / WRITE per launch of one kernel, per library variant (separate rocprofv3 --pmc passes).
# Usage: [PASSES="FETCH_SIZE;WRITE_SIZE;..."] bash scripts/gpu_pmcab.sh <tag> <kernel-regex> <cfg> <op> "<name>:<variant|base>:<ENV=V,...>" ...
set -o pipefail
TAG=$1; KR=$2; CFG=$3; OP=$4; shift 4
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for spec in "$@"; do
  IFS=: read -r NAME V ENVS <<< "$spec"
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  EV=$(echo "$ENVS" | tr ',' ' ')
  IFS=';' read -ra PA <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum}"
  env CUSTMA_LIB=$L $EV timeout -k 10 600 python3 scripts/pmc_run.py $O/$NAME "$KR" "${PA[@]}" -- python3 scripts/kbench.py --cfg $CFG --ops $OP --reps 2 > $O/$NAME.log 2>&1 || { echo "$NAME failed"; tail -20 $O/$NAME.log; exit 1; }
  echo "== $NAME"; cat $O/$NAME.log | grep -v '^{'
done
