"""Summarise rocprofv3 PMC passes (scripts/pmc.sh output): mean per dispatch per counter."""
import collections, csv, glob, sys
out = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(list); dur = []
for f in sorted(glob.glob(f"{out}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat and pat not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
