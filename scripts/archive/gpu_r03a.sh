#!/bin/bash
# round-3 first check: new parity tests, the whole GPU suite, contract bench
set -o pipefail
TAG=${1:-r03a}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_configs.py -m gpu -x -v --timeout 240 --timeout-method thread -k "graph or config4" > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $O/new_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/new_tests.log | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
