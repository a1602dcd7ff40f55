#!/bin/bash
# Round 6 (ad): the contract bench three times on one box (same-box run-to-run spread, against the box-to-box
# spread of r06/r, r06/w, r06/ac).
set -o pipefail
TAG=${1:-r06ad}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err
  rc=$?; echo "bench $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d = json.load(open('$O/bench_$i.json')); r = d['roofline']; print(d['ms_per_step'], d['value'], r['avg_launch_ms'], d['north_star']['op_ms'])"
done
