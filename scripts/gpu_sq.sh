#!/bin/bash
# SQ / LDS counters of the forward tile kernel (C3 window) and the backward sweep (C5 window),
# plus the verify driver test.  bash scripts/gpu_sq.sh <tag>
set -o pipefail
TAG=$1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_examples.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/examples.log 2>&1 || { echo "examples failed"; tail -30 $O/examples.log; exit 1; }
tail -1 $O/examples.log
timeout -k 10 200 python examples/verify.py > $O/verify_default.log 2>&1 || { echo "verify default failed"; tail -20 $O/verify_default.log; exit 1; }
grep -v "tensor\|device\|\[" $O/verify_default.log | head -20
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
echo "== fwd tile C3"
timeout -k 10 400 python scripts/pmc_run.py $O/sq_fwd k_fwd_tile "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c3_win --ops fwd --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
echo "== bwd coop C5"
timeout -k 10 400 python scripts/pmc_run.py $O/sq_bwd k_bwd_coop "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c5_win --ops bwd --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
