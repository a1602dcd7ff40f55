#!/bin/bash
# Round 6 (s): the contract bench line with the SURVEY-nominal north-star fields.
set -o pipefail
TAG=${1:-r06s}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
python3 -c "import json; d = json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['north_star']))"
