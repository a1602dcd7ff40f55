#!/bin/bash
# Round 4, first GPU pass: store-shape micro, SQ counters of k_bwd_coop at C5 (HEAD), backward
# load-depth variants (parity subset + interleaved timing), C3-only forward kernel trace.
# Usage: bash scripts/gpu_r04a.sh <tag>
set -o pipefail
TAG=${1:-r04a}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
echo "== store shapes"
timeout -k 10 180 ./scripts/micro/store_shape > $O/store_shape.txt 2>&1 || { echo "store micro failed"; tail -20 $O/store_shape.txt; exit 1; }
cat $O/store_shape.txt
echo "== C3 forward kernel trace"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c3fwd -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win --ops fwd --reps 30 > $O/c3fwd.log 2>&1 || { echo "c3 trace failed"; tail -20 $O/c3fwd.log; exit 1; }
grep cfg $O/c3fwd.log
f=$(find $O/c3fwd -name "*kernel_stats.csv" | head -1); cp "$f" $O/c3_fwd_kernel_stats.csv; cut -d, -f1-8 $O/c3_fwd_kernel_stats.csv | cut -c1-160
for V in bdp2 bdp2f12; do
  L=$PWD/scripts/_abl/$V/libcustma_hip.so
  CUSTMA_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "backward" > $O/test_$V.log 2>&1 || { echo "tests $V failed"; tail -30 $O/test_$V.log; exit 1; }
  echo "$V: $(tail -1 $O/test_$V.log)"
done
echo "== A/B c5 backward"
bash scripts/gpu_ab.sh $TAG c5_win bwd 2 "base:base:" "bdp2:bdp2:" "bdp2f12:bdp2f12:" || exit 1
echo "== SQ k_bwd_coop C5"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
timeout -k 10 500 python scripts/pmc_run.py $O/sq_bwd k_bwd_coop "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c5_win --ops bwd --reps 1 > $O/sq_bwd.txt 2>&1 || { echo "sq failed"; tail -20 $O/sq_bwd.txt; exit 1; }
grep -v amdgpu.ids $O/sq_bwd.txt
