cd $GRAFT_REPO_ROOT
export CUSTMA_SWEEP_NW=3
CUSTMA_LIB=scripts/_abl/skeleton/libcustma_hip.so bash scripts/pmc_rd.sh gpurun_out/rd_skel k_sweep_fwd -- scripts/kbench.py --cfg c2_full --ops fwd --reps 3
python scripts/pmc_summary.py gpurun_out/rd_skel
