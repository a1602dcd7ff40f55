#!/bin/bash
# full GPU suite, per-op timings, rocprof kernel stats of the c5 fwd+bwd ops
set -o pipefail
TAG=${1:-r03b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python scripts/kbench.py --cfg c5_win,c3_win,c2_full --ops fwd,bwd --reps 5 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c5_win,c3_win --ops fwd,bwd --reps 3 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv,glob
for f in glob.glob("gpurun_out/*/prof/**/*kernel_stats.csv", recursive=True):
    if "/r03b/" not in f and "/$TAG/" not in f: pass
import sys, os
tag=os.environ.get("TAG","")
PY
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']; i=n.find('k_'); n=n[i:i+44] if i>=0 else n[:44]
    print(f\"{n:46s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}\")
"
