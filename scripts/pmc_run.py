"""Run rocprofv3 PMC passes (one process per pass, never combined with tracing) and print the
mean per dispatch of every counter for kernels matching a regex (GPU box; diagnostic only).

Usage: python scripts/pmc_run.py <outdir> <kernel-regex> "<counters pass 1>" ["<pass 2>" ...] -- <cmd...>
"""
import collections
import csv
import glob
import os
import re
import subprocess
import sys


def main():
    out, rex = sys.argv[1], sys.argv[2]
    rest = sys.argv[3:]
    cut = rest.index("--")
    passes, cmd = rest[:cut], rest[cut + 1:]
    env = dict(os.environ, TMPDIR="/tmp")
    vals = collections.defaultdict(list)
    for i, p in enumerate(passes):
        d = os.path.join(out, f"pass{i}")
        r = subprocess.run(["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *p.split(), "-d", d, "-o", "run",
                            "--output-format", "csv", "--"] + cmd, env=env, capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stdout[-1500:], r.stderr[-1500:])
            raise SystemExit(f"pass {i} ({p}) failed")
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if re.search(rex, row["Kernel_Name"]):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in vals.items():
        print(f"{k:32s} n={len(v):3d} mean={sum(v) / len(v):.5g}")


if __name__ == "__main__":
    main()
