#!/bin/bash
# Round 4: statistics kernel micro-tiles -- full GPU suite, interleaved A/B against the previous
# statistics kernel (C3 forward, C5 backward), the C3 window forward at D = 255 (no remainder
# diagonal), and a kernel trace of the new statistics passes.
# Usage: bash scripts/gpu_r04c.sh <tag>
set -o pipefail
TAG=${1:-r04c}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
bash scripts/gpu_tests.sh $TAG || exit 1
echo "== A/B c3 fwd"
bash scripts/gpu_ab.sh $TAG c3_win,c3_win_d255 fwd 3 "new:base:" "nosplit:base:CUSTMA_FWD_SPLIT=0" "old:oldstats:" || exit 1
echo "== A/B c5 bwd"
bash scripts/gpu_ab.sh $TAG c5_win fwd,bwd 2 "new:base:" "nosplit:base:CUSTMA_FWD_SPLIT=0" "old:oldstats:" || exit 1
echo "== trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c3_win,c5_win --ops fwd,bwd,disp --reps 5 > $O/kbench.log 2>&1 || { echo "rocprof failed"; tail -20 $O/kbench.log; exit 1; }
grep cfg $O/kbench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]; i = n.find("k_"); n = n[i:i + 70] if i >= 0 else n[:70]
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {n}")
PY
echo "== occupancy probe (sweep launches with 2 KB more LDS: tile forward 2 WG/CU, backward sweep 1 WG/CU)"
bash scripts/gpu_ab.sh $TAG c5_win fwd,bwd 1 "base:base:" "occ:occ:" || exit 1
echo "== backward sweep stamps (diagnostic build: shares only)"
for C in c5_win c3_win; do
  CUSTMA_LIB=$PWD/scripts/_abl/stamps/libcustma_hip.so timeout -k 10 200 python scripts/kbench.py --cfg $C --ops bwd --reps 2 > $O/stamps_$C.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_$C.log; exit 1; }
  echo "$C $(grep STAMPS $O/stamps_$C.log | tail -1)"
done
