#!/bin/bash
# Bench round trip: bash scripts/gpu_bench.sh <tag>
#   row-band GPU test, contract bench (default workload), a 2-rank gloo rehearsal of the
#   launcher path, and a rocprofv3 kernel-trace summary of the bench workload.
set -o pipefail
TAG=${1:-bench}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/rowband.log 2>&1 || { echo "rowband test failed"; tail -30 $O/rowband.log; exit 1; }
tail -2 $O/rowband.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > $O/bench_n2_gloo.json 2> $O/bench_n2.err || { echo "bench n2 failed"; tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_n2_gloo.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-config2 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:110]}")
PY
