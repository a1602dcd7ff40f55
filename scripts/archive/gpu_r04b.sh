#!/bin/bash
# Round 4: whole GPU suite after the row-band / statistics-rows / pruning changes, smoke, and a
# 2-rank gloo rehearsal of the N > 1 bench path (per-rank timing fields).
set -o pipefail
TAG=${1:-r04b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > $O/bench_c5_n2_gloo_rehearsal.json 2> $O/bench_n2.err || { echo "bench n2 failed"; tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_c5_n2_gloo_rehearsal.json
