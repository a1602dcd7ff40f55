#!/bin/bash
# Clock-ramp probe, kbench op lines (steady-state clocks) for the forward / disparity ops, and the bench line.
set -o pipefail
TAG=${1:-r03e}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python scripts/throttle_probe.py > $O/throttle_probe.log 2>&1 || { echo "probe failed"; tail -20 $O/throttle_probe.log; exit 1; }
grep -E "burst|after" $O/throttle_probe.log
timeout -k 10 400 python scripts/kbench.py --cfg c3_win,c2_full,c2_win --ops fwd,disp,soft --reps 20 > $O/kbench_fwd_disp.jsonl 2> $O/kbench.err || { echo "kbench failed"; tail -20 $O/kbench.err; exit 1; }
cat $O/kbench_fwd_disp.jsonl
timeout -k 10 500 python bench.py > $O/bench_c5.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench_c5.json
