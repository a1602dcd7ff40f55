#!/bin/bash
# Round 5 (c): backward A/B (batched-load gather), SQ counters of the statistics pass, the forward tile
# sweep (C3) and the backward sweep (C5), and a kernel trace of the contract bench workload itself.
# Usage: bash scripts/gpu_r05c.sh <tag>
set -o pipefail
TAG=${1:-r05c}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
md5sum custereomatching_amd/_lib/libcustma_hip.so
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u scripts/ab_bwd.py 4 > $O/ab_bwd.log 2>&1
rc=$?; echo "ab_bwd rc=$rc"; grep cfg $O/ab_bwd.log; fatal $rc ab_bwd
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
echo "== stats + fwd tile C3"
timeout -k 10 400 python scripts/pmc_run.py $O/sq_stats k_stats "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c3_win --ops fwd --reps 2 > $O/sq_stats.log 2>&1
rc=$?; grep -v amdgpu.ids $O/sq_stats.log | tail -25; fatal $rc sq_stats
timeout -k 10 400 python scripts/pmc_run.py $O/sq_fwd k_fwd_tile "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c3_win --ops fwd --reps 2 > $O/sq_fwd.log 2>&1
rc=$?; grep -v amdgpu.ids $O/sq_fwd.log | tail -25; fatal $rc sq_fwd
echo "== bwd coop C5"
timeout -k 10 400 python scripts/pmc_run.py $O/sq_bwd k_bwd_coop "$P1" "$P2" "$P3" -- python3 scripts/kbench.py --cfg c5_win --ops bwd --reps 1 > $O/sq_bwd.log 2>&1
rc=$?; grep -v amdgpu.ids $O/sq_bwd.log | tail -25; fatal $rc sq_bwd
echo "== bench kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 5 --no-pmc --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err
rc=$?; echo "traced bench rc=$rc"; fatal $rc traced_bench
cat $O/bench_traced.json | cut -c1-400
