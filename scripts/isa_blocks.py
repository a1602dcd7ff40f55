#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing.
Usage: python scripts/isa_blocks.py file.s kernel-substring [--loops]"""
import re
import sys

t = open(sys.argv[1]).read().splitlines()
sub = sys.argv[2]
loops = "--loops" in sys.argv
i = next(i for i, l in enumerate(t) if re.match(r"^_Z\w*" + re.escape(sub) + r"\w*:", l))
j = next(k for k in range(i, len(t)) if ".Lfunc_end" in t[k])
blocks, cur = [], None
for l in t[i:j]:
    if re.match(r"^\.?\w+:", l):
        cur = [l.split(":")[0], "Loop" in l, []]
        blocks.append(cur)
        continue
    s = l.strip()
    if cur and s and not s.startswith((".", ";")):
        cur[2].append(s)
tot = {}
for lab, inloop, ins in blocks:
    if loops and not inloop:
        continue
    c = lambda p: sum(1 for s in ins if s.startswith(p))
    row = dict(n=len(ins), v=c("v_"), rl=c("v_readlane"), wl=c("v_writelane"), nop=c("s_nop"), ds=c("ds_"),
               buf=c("buffer_"), s=sum(1 for s in ins if s.startswith("s_")),
               dpp=sum(1 for s in ins if "_dpp" in s), trans=sum(1 for s in ins if s.startswith(("v_rsq", "v_rcp", "v_exp", "v_sqrt"))))
    for k, v in row.items():
        tot[k] = tot.get(k, 0) + v
    print(f"{lab:12s} " + " ".join(f"{k}={v:4d}" for k, v in row.items()))
print("total       " + " ".join(f"{k}={v:4d}" for k, v in tot.items()))
