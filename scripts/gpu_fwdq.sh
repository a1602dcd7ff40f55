#!/bin/bash
# forward iteration: parity subset, per-op times, SQ counters of the tile kernel.  bash scripts/gpu_fwdq.sh <tag>
set -o pipefail
TAG=$1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "forward or disparity or config3 or config4 or soft" > $O/test.log 2>&1 || { echo "tests failed"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python scripts/kbench.py --cfg c3_win,c5_win,c2_win --ops fwd,disp --reps 10 > $O/kb.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb.log; exit 1; }
grep cfg $O/kb.log
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
timeout -k 10 300 python scripts/pmc_run.py $O/sq_fwd k_fwd_tile "$P1" "$P2" -- python3 scripts/kbench.py --cfg c3_win --ops fwd --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
