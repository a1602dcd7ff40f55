#!/usr/bin/env python3
"""Per-kernel register use and instruction mix from a hipcc `--cuda-device-only -S` listing.

Usage: python scripts/isa_stats.py file.s [name-substring]
Prints, per kernel: VGPRs, SGPRs, spills, and counts of VALU / readlane / writelane / DPP /
s_nop / LDS / VMEM instructions in the kernel body (a static count, not per-iteration).
"""
import re
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().splitlines()
    bodies, cur = {}, None
    for ln in text:
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", ln)
        if m:
            cur = m.group(1)
            bodies[cur] = []
            continue
        if cur and re.match(r"^\s+\.end_amdhsa_kernel|^\s*\.Lfunc_end", ln):
            cur = None
        if cur:
            bodies[cur].append(ln.strip())
    meta = {}
    blocks = re.split(r"\n  - ", "\n".join(text[next((i for i, l in enumerate(text) if "amdhsa.kernels:" in l), 0):]))
    for blk in blocks:
        sym = re.search(r"\.symbol:\s+(\S+)\.kd", blk)
        if not sym:
            continue
        get = lambda f: (re.search(r"\." + f + r":\s+(\d+)", blk) or [None, "?"])[1]
        meta[sym.group(1)] = (get("sgpr_count"), get("sgpr_spill_count"), get("vgpr_count"), get("vgpr_spill_count"))
    cats = {
        "valu": lambda s: s.startswith("v_"),
        "readlane": lambda s: s.startswith("v_readlane") or s.startswith("v_readfirstlane"),
        "writelane": lambda s: s.startswith("v_writelane"),
        "dpp": lambda s: s.startswith("v_") and ("row_" in s or "quad_perm" in s or "wave_" in s),
        "s_nop": lambda s: s.startswith("s_nop"),
        "lds": lambda s: s.startswith("ds_"),
        "vmem": lambda s: s.startswith("buffer_") or s.startswith("global_"),
        "salu": lambda s: s.startswith("s_") and not s.startswith("s_nop") and not s.startswith("s_waitcnt"),
    }
    for k, body in bodies.items():
        if filt not in k:
            continue
        ins = [b for b in body if b and not b.startswith((";", ".")) and not b.endswith(":")]
        c = {n: sum(1 for s in ins if f(s)) for n, f in cats.items()}
        sg, ss, vg, vs = meta.get(k, ("?", "?", "?", "?"))
        print(f"{k[:90]}\n  vgpr {vg} sgpr {sg} (spill v{vs} s{ss})  total {len(ins)}  " +
              " ".join(f"{n}={v}" for n, v in c.items()))


if __name__ == "__main__":
    main()
