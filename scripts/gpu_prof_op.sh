#!/bin/bash
# rocprofv3 kernel stats of one kbench op.  Usage: bash scripts/gpu_prof_op.sh <tag> <cfg> <ops>
set -o pipefail
TAG=$1; CFG=${2:-c3_win}; OPS=${3:-fwd}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg $CFG --ops $OPS --reps 5 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | cut -c1-160
