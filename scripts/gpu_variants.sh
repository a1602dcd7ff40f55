#!/bin/bash
# Compare library variants (scripts/_abl/<name>): parity subset, per-op times, PMC traffic of a kernel.
# Usage: bash scripts/gpu_variants.sh <tag> <kernel-regex> <cfgs> <ops> <test -k expr> <variant>...
set -o pipefail
TAG=$1; KRX=$2; CFGS=$3; OPS=$4; TK=$5; shift 5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for V in "$@"; do
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  [ "$V" = "base" ] && L=$PWD/custereomatching_amd/_lib/libcustma_hip.so
  echo "== $V"
  CUSTMA_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$TK" > $O/test_$V.log 2>&1 || { echo "tests $V failed"; tail -30 $O/test_$V.log; exit 1; }
  tail -1 $O/test_$V.log
  CUSTMA_LIB=$L timeout -k 10 300 python scripts/kbench.py --cfg $CFGS --ops $OPS --reps 5 > $O/kb_$V.log 2>&1 || { echo "kbench $V failed"; tail -5 $O/kb_$V.log; exit 1; }
  grep cfg $O/kb_$V.log
  CUSTMA_LIB=$L timeout -k 10 400 python scripts/pmc_run.py $O/pmc_$V "$KRX" "FETCH_SIZE" "WRITE_SIZE" -- python3 scripts/kbench.py --cfg $CFGS --ops $OPS --reps 1 > $O/pmc_$V.log 2>&1 || { echo "pmc $V failed"; tail -10 $O/pmc_$V.log; exit 1; }
  grep -v amdgpu.ids $O/pmc_$V.log
done
