#!/bin/bash
# Interleaved A/B timing of library variants / env settings on one box (box-to-box spread is ~5 %).
# Usage: bash scripts/gpu_ab.sh <tag> <cfg> <ops> <rounds> "<name>:<lib-variant or base>:<ENV=V,...>" ...
set -o pipefail
TAG=$1; CFG=$2; OPS=$3; ROUNDS=$4; shift 4
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    IFS=: read -r NAME V ENVS <<< "$spec"
    L=$PWD/scripts/_abl/$V/libcustma_hip.so
    [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
    EV=$(echo "$ENVS" | tr ',' ' ')
    env CUSTMA_LIB=$L $EV timeout -k 10 200 python scripts/kbench.py --cfg $CFG --ops $OPS --reps 10 > $O/ab_${NAME}_$r.log 2>&1 || { echo "$NAME failed"; tail -5 $O/ab_${NAME}_$r.log; exit 1; }
    echo "$r $NAME $(grep cfg $O/ab_${NAME}_$r.log | tr '\n' ' ')"
  done
done
