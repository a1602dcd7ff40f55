#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "backward or config or autograd or rowband" > $O/test.log 2>&1 || { echo "tests failed"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python scripts/kbench.py --cfg c5_win,c3_win,c2_full --ops fwd,bwd --reps 5 > $O/kb.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb.log; exit 1; }
grep cfg $O/kb.log
CUSTMA_BWD_NOREM=1 timeout -k 10 300 python scripts/kbench.py --cfg c5_win,c3_win --ops bwd --reps 5 > $O/kb_norem.log 2>&1 || { echo "kbench norem failed"; tail -5 $O/kb_norem.log; exit 1; }
grep cfg $O/kb_norem.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c5_win --ops bwd --reps 3 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
