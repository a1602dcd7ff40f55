#!/bin/bash
# Round-trip: GPU tests, PMC traffic, contract bench, rocprofv3 kernel stats of the bench.
set -o pipefail
TAG=${1:-full}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python scripts/pmc_traffic.py $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log | cut -c1-300
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
