#!/bin/bash
# k_bwd_coop at C2 full: kernel time (rocprofv3) and PMC traffic for block orders 1 and 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for ORD in 1 2; do
  CUSTMA_BWD_ORDER=$ORD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_o$ORD -o run --output-format csv -- python3 scripts/kbench.py --cfg c2_full --ops bwd --reps 5 > $O/prof_o$ORD.log 2>&1 || { echo "rocprof o$ORD failed"; tail -20 $O/prof_o$ORD.log; exit 1; }
  python3 - "$O/prof_o$ORD" $ORD <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_bwd_coop" in r["Name"]:
        print(f"order {sys.argv[2]}: k_bwd_coop {float(r['AverageNs'])/1e3:.1f} us x{r['Calls']}")
PY
  CUSTMA_BWD_ORDER=$ORD timeout -k 10 300 python scripts/pmc_run.py $O/pmc_o$ORD k_bwd_coop "FETCH_SIZE" "WRITE_SIZE" -- python3 scripts/kbench.py --cfg c2_full --ops bwd --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
