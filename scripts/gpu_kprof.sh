#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of kbench ops, per library variant, one box.
# Usage: bash scripts/gpu_kprof.sh <tag> <cfgs> <ops> "<name>:<variant|base>:<ENV=V,...>" ...
set -o pipefail
TAG=$1; CFG=$2; OPS=$3; shift 3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for spec in "$@"; do
  IFS=: read -r NAME V ENVS <<< "$spec"
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  EV=$(echo "$ENVS" | tr ',' ' ')
  for c in ${CFG//,/ }; do
    env CUSTMA_LIB=$L $EV timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${NAME}_$c -o run --output-format csv -- python3 scripts/kbench.py --cfg $c --ops $OPS --reps 4 > $O/${NAME}_$c.log 2>&1 || { echo "$NAME $c failed"; tail -5 $O/${NAME}_$c.log; exit 1; }
    f=$(find $O/${NAME}_$c -name "*kernel_trace.csv" | head -1)
    python3 scripts/ktrace_summary.py "$f" "$NAME $c"
  done
done
