#!/bin/bash
# Round 4 (late): validate and time the statistics micro-tiles, STATS_MSB and the split forward --
# full GPU suite, a rocprofv3 kernel trace of the C3 / C5 forward, backward and disparity, and the
# contract bench line (north star + configs[2] included).
# Usage: bash scripts/gpu_r04c.sh <tag>
set -o pipefail
TAG=${1:-r04c}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
bash scripts/gpu_tests.sh $TAG || exit 1
echo "== trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win,c5_win --ops fwd,bwd,disp --reps 5 > $O/kbench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/kbench.log; exit 1; }
grep cfg $O/kbench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]; i = n.find("k_"); n = n[i:i + 70] if i >= 0 else n[:70]
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {n}")
PY
echo "== bench"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
