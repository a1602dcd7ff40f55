#!/bin/bash
# Whole GPU suite, then per-kernel durations (rocprofv3 kernel trace) and FETCH / WRITE of one kernel.
# Usage: bash scripts/gpu_check.sh <tag> <cfgs> <ops> [kernel-regex for the PMC passes]
set -o pipefail
TAG=$1; CFG=$2; OPS=$3; KR=${4:-}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in ${CFG//,/ }; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_$c -o run --output-format csv -- python3 scripts/kbench.py --cfg $c --ops $OPS --reps 4 > $O/kt_$c.log 2>&1 || { echo "kprof $c failed"; tail -5 $O/kt_$c.log; exit 1; }
  grep '^{' $O/kt_$c.log
  f=$(find $O/kt_$c -name "*kernel_trace.csv" | head -1)
  python3 scripts/ktrace_summary.py "$f" "$c"
done
if [ -n "$KR" ]; then
  c=${CFG%%,*}
  timeout -k 10 600 python3 scripts/pmc_run.py $O/pmc "$KR" "FETCH_SIZE" "WRITE_SIZE" -- python3 scripts/kbench.py --cfg $c --ops $OPS --reps 2 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
  grep -v '^{' $O/pmc.log
fi
