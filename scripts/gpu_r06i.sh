#!/bin/bash
# Round 6 (i): SQ counters of the tile forward at C3 and C5 (does C5 wait on its stores?); the double-buffered
# full-layout disparity tiles and the chip-filling-only backward segments (scripts/_abl/dbuf): parity subset and
# A/B against the main library.
set -o pipefail
TAG=${1:-r06i}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so scripts/_abl/dbuf/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
for c in c3_win c5_win; do
  echo "== fwd tile $c"
  timeout -k 10 300 python scripts/pmc_run.py $O/sq_$c 'k_fwd_tile<11, __half, true, 0, true>' "$P1" "$P2" -- python3 scripts/kbench.py --cfg $c --ops fwd --reps 2 > $O/sq_$c.txt 2>&1
  rc=$?; echo "sq $c rc=$rc"; fatal $rc sq_$c
  grep -v amdgpu.ids $O/sq_$c.txt | tail -20
done
CUSTMA_LIB=$PWD/scripts/_abl/dbuf/libcustma_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread -k "disparity or soft or backward or config2 or sliding or workspace or graph" > $O/gpu_tests_dbuf.log 2>&1
rc=$?; echo "dbuf subset rc=$rc"; fatal $rc dbuf_subset
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_dbuf.log | tail -20
timeout -k 10 500 bash scripts/gpu_ab.sh $TAG c2_full,c3_full disp,soft 2 "base:base:" "dbuf:dbuf:"
rc=$?; echo "ab dbuf disp rc=$rc"; fatal $rc ab_dbuf1
timeout -k 10 300 bash scripts/gpu_ab.sh ${TAG}b c2_win,c5_r8 bwd 2 "base:base:" "dbuf:dbuf:"
rc=$?; echo "ab dbuf bwd rc=$rc"; fatal $rc ab_dbuf2
