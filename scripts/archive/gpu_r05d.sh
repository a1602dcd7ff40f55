#!/bin/bash
# Round 5 (d): gpu_r05b.sh (suite, forward forms, k >= 18, bench line) then gpu_r05c.sh (backward A/B, SQ
# counters, traced bench) in one call.  Usage: bash scripts/gpu_r05d.sh <tag>
set -o pipefail
TAG=${1:-r05d}
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r05b.sh $TAG || { rc=$?; echo "r05b part rc=$rc"; exit $rc; }
bash scripts/gpu_r05c.sh $TAG
