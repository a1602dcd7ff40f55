#!/bin/bash
# One GPU-box round trip: parity tests, per-op kernel timings, contract bench, rocprof stats.
# Usage (via gpurun): bash scripts/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --cfg c2_full,c2_win,c3_win --ops fwd,bwd,disp --reps 5 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
