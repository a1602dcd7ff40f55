#!/bin/bash
# Round check at HEAD: whole GPU suite, smoke(), the contract bench line, a 2-rank gloo rehearsal of
# the launcher path and a rocprofv3 --kernel-trace --stats summary of the bench workload.
# Usage: bash scripts/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_c5.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > $O/bench_c5_n2_gloo_rehearsal.json 2> $O/bench_n2.err || { echo "bench n2 failed"; tail -30 $O/bench_n2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-config2 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/bench_c5_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]; i = n.find("k_"); n = n[i:i + 60] if i >= 0 else n[:60]
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {n}")
PY
