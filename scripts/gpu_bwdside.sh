#!/bin/bash
# Backward side-kernel round trip: backward parity tests, interleaved A/B of library variants at C5 / C2,
# and a rocprofv3 kernel trace of the C5 window backward.  Usage: bash scripts/gpu_bwdside.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
bash scripts/gpu_tests.sh $TAG -k "backward or bwd or grad or config or rowband or verify" || exit 1
SPECS=()
for V in "$@"; do SPECS+=("$V:$V:"); done
bash scripts/gpu_ab.sh $TAG/c5 c5_win bwd 2 "${SPECS[@]}" || exit 1
bash scripts/gpu_ab.sh $TAG/c2 c2_full bwd 2 "${SPECS[@]}" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/kbench.py --cfg c5_win --ops bwd --reps 5 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -10 $O/prof.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:110]}")
PY
