#!/bin/bash
# Round 6 (k): the library with the 128-row full-layout volume bands and the chip-filling-only backward
# segments: whole GPU suite, smoke, the contract bench line, kbench + kernel traces (C3 window, C5, C2 full),
# and SQ counters of the statistics pass (C3 / C5) to see what bounds it.
set -o pipefail
TAG=${1:-r06k}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; fatal $rc suite
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; fatal $rc smoke
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
cut -c1-300 $O/bench.json
for c in c3_win c2_full; do
  timeout -k 10 200 python3 scripts/kbench.py --cfg $c --ops fwd,bwd,disp,soft --reps 10 > $O/kbench_$c.log 2>&1
  rc=$?; echo "kbench $c rc=$rc"; fatal $rc kbench_$c
  grep cfg $O/kbench_$c.log
  timeout -k 10 320 bash scripts/prof_kernels.sh $TAG/p_$c $c fwd,bwd,disp > $O/prof_$c.txt 2>&1
  rc=$?; echo "prof $c rc=$rc"; fatal $rc prof_$c
  cp $(find $O/p_$c/prof -name "*kernel_stats.csv" | head -1) $O/${c}_kernel_stats.csv
  head -14 $O/prof_$c.txt | cut -c1-140
done
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
for c in c3_win c5_win; do
  timeout -k 10 300 python scripts/pmc_run.py $O/sq_stats_$c 'k_stats<__half, 11, 3>' "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg $c --ops fwd --reps 2 > $O/sq_stats_$c.txt 2>&1
  rc=$?; echo "sq stats $c rc=$rc"; fatal $rc sq_$c
  grep -v amdgpu.ids $O/sq_stats_$c.txt | tail -21
done
