#!/bin/bash
# Parity subset per library variant, then interleaved A/B timing.
# Usage: bash scripts/gpu_abt.sh <tag> "<pytest -k expr>" <cfg> <ops> <rounds> "<name>:<variant|base>:<ENV=V,...>" ...
set -o pipefail
TAG=$1; TK=$2; CFG=$3; OPS=$4; ROUNDS=$5; shift 5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for spec in "$@"; do
  IFS=: read -r NAME V ENVS <<< "$spec"
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  EV=$(echo "$ENVS" | tr ',' ' ')
  env CUSTMA_LIB=$L $EV timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$TK" > $O/test_$NAME.log 2>&1 || { echo "tests $NAME failed"; tail -30 $O/test_$NAME.log; exit 1; }
  echo "tests $NAME: $(tail -1 $O/test_$NAME.log)"
done
bash scripts/gpu_ab.sh $TAG $CFG $OPS $ROUNDS "$@"
