"""Median duration per kernel name from a rocprofv3 kernel_trace.csv (benchmarking helper)."""
import collections
import csv
import statistics
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    i = n.find("k_")
    n = n[i:n.find("(", i)] if i >= 0 else n[:40]
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tag = sys.argv[2] if len(sys.argv) > 2 else ""
for n, v in sorted(d.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    if n.startswith("void at::"):
        continue
    print(f"{tag:16s} {n:44s} n={len(v):3d} median_us={statistics.median(v):9.1f} min_us={min(v):9.1f}")
