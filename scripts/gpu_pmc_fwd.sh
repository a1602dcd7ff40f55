#!/bin/bash
# PMC passes over the forward sweep on one kbench config: bash scripts/gpu_pmc_fwd.sh <tag> <cfg> [regex]
set -o pipefail
TAG=$1; CFG=${2:-c3_win}; RE=${3:-k_sweep_fwd}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
bash scripts/pmc.sh $O "$RE" -- scripts/kbench.py --cfg $CFG --ops fwd --reps 2 || exit 1
python3 scripts/pmc_summary.py $O "$RE"
