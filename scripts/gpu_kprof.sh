#!/bin/bash
# Backward-subset GPU tests, then a rocprofv3 kernel-trace summary of kbench ops.
# Usage: bash scripts/gpu_kprof.sh <tag> <cfgs> <ops> [pytest -k expr]
set -o pipefail
TAG=$1; CFGS=$2; OPS=$3; TK=${4:-backward}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TK" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg $CFGS --ops $OPS --reps 5 > $O/kbench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/kbench.log; exit 1; }
grep cfg $O/kbench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]; i = n.find("k_"); n = n[i:i + 70] if i >= 0 else n[:70]
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {n}")
PY
