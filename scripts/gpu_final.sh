#!/bin/bash
# Round-end GPU check: parity tests, smoke(), per-op timings, contract bench, rocprof stats,
# PMC traffic of the bench's sweeps.  Usage (via gpurun): bash scripts/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_check.sh $TAG > $O/check.txt 2>&1 || { echo "check failed"; tail -30 $O/check.txt; exit 1; }
tail -3 $O/pytest.log | tail -1
timeout -k 10 600 python3 scripts/pmc_traffic.py $O/pmc full > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -10 $O/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win --ops fwd,bwd,disp --reps 5 > $O/prof_c3.log 2>&1 || { echo "rocprof c3 failed"; tail -10 $O/prof_c3.log; exit 1; }
echo done
