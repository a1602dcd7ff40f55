#!/bin/bash
# Round 5 (v): HEAD record after the load-batching changes -- smoke, the bench line (with its PMC passes and CPU baseline),
# the bench workload and of the C3 north star / disparity / backward.
set -o pipefail
TAG=${1:-r05v}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-300 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 5 --no-pmc --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err
rc=$?; echo "traced bench rc=$rc"; fatal $rc traced_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win --ops fwd,disp,bwd --reps 10 > $O/kbench_c3.log 2>&1
rc=$?; echo "c3 trace rc=$rc"; grep cfg $O/kbench_c3.log; fatal $rc c3_trace
