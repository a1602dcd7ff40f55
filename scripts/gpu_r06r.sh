#!/bin/bash
# Round 6 (r): the library at HEAD -- whole GPU suite, smoke, the contract bench line, a rocprofv3 kernel-trace
# summary of the same bench command, kbench on C3 window / C5 / C2 full, and a 2-rank gloo rehearsal.
set -o pipefail
TAG=${1:-r06r}
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
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pmc > $O/bench_traced.json 2> $O/prof.log
rc=$?; echo "traced bench rc=$rc"; fatal $rc traced
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/bench_c5_traced_kernel_stats.csv
python3 - $O/bench_c5_traced_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    n = r["Name"]; i = n.find("k_"); n = n[i:i + 60] if i >= 0 else n[:60]
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {n}")
PY
for c in c3_win c5_win c2_full; do
  timeout -k 10 300 python3 scripts/kbench.py --cfg $c --ops fwd,bwd,disp,soft --reps 10 > $O/kbench_$c.log 2>&1
  rc=$?; echo "kbench $c rc=$rc"; fatal $rc kbench_$c
  grep cfg $O/kbench_$c.log
done
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > $O/bench_n2_gloo.json 2> $O/bench_n2.err
rc=$?; echo "gloo rehearsal rc=$rc"; fatal $rc gloo
cut -c1-200 $O/bench_n2_gloo.json
