#!/usr/bin/env python3
"""Load-completion check of a gfx950 .s listing: no instruction touches a VGPR that an
outstanding vector-memory load still has to write.

The hand-pipelined kernels issue their loads as inline asm and wait for them with hand-counted
`s_waitcnt vmcnt(N)`.  The compiler takes an asm load's destination as written when the asm
issues, so it may read it (a register copy at a loop back-edge, a value moved into another
register) or reuse it before the load has landed; gfx9 has no scoreboard for VMEM destinations,
so such a read sees the register's OLD contents -- whatever the previous wave on that SIMD left
there for the first load of a wave.  That is a timing- and history-dependent wrong answer, not
a fault, so it is checked here on the emitted code.

Model (per program point, a fixpoint over the control-flow graph; joins keep the younger age):
  every VMEM instruction (buffer_ / global_ / flat_ / scratch_) ages every outstanding load by
  one; a load's destination registers become outstanding with age 0; `s_waitcnt vmcnt(N)`
  retires the loads with age >= N (the counter retires in issue order); any other mention of an
  outstanding register by an instruction (read or write) is a hit.

Usage: python custereomatching_amd/vmcnt_check.py file.s [kernel-substring ...]
Exit status 1 when any kernel has a hit.
"""
from __future__ import annotations

import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from hazard_check import blocks_of, kernels, regs_of, split_operands  # noqa: E402

VMEM = ("buffer_", "global_", "flat_", "scratch_")
CAP = 64


def vm_dest(ins):
    """VGPRs a VMEM instruction writes when it completes (loads, returning atomics)."""
    op = ins.op
    if not op.startswith(VMEM) or not ins.fields:
        return []
    if "_load" in op:
        if re.search(r"\blds\b", ins.args):  # LDS DMA: no VGPR destination
            return []
        return [r for r in regs_of(ins.fields[0]) if r[0] == "v"]
    if "_atomic" in op and re.search(r"\b(glc|sc0)\b", ins.args):
        return [r for r in regs_of(ins.fields[0]) if r[0] == "v"]
    return []


def vmcnt_of(ins):
    if ins.op != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", ins.args)
    return int(m.group(1)) if m else None


# v_mad_u64_u32 / v_mad_i64_i32 is also the compiler's 32-bit multiply-add: the addend's high register
# is then an undefined operand -- any register, possibly one with a load in flight -- and only the
# result's low half is used.  The inline-asm loads here all fill 16/32-bit values or doubles of their
# own, never the high half of a 64-bit integer, so such an addend-high read is exempt (the addend's
# low register is still checked).
MAD64 = ("v_mad_u64_u32", "v_mad_i64_i32")


def exempt(ins, r):
    if not ins.op.startswith(MAD64) or len(ins.fields) < 5:
        return False
    c = sorted((x for x in regs_of(ins.fields[4]) if x[0] == "v"), key=lambda x: x[1])
    return len(c) == 2 and r == c[1]


def transfer(state, ins, hits=None):
    """state: {vgpr: (age, load instruction)}"""
    n = vmcnt_of(ins)
    if n is not None:
        return {r: v for r, v in state.items() if v[0] < n}
    if ins.op == "s_waitcnt":  # lgkmcnt / expcnt only
        return state
    dest = vm_dest(ins)
    # a load may name the destination of an earlier load still in flight: the loads return in issue
    # order, so the later one wins (its address operands are still checked)
    touched = [r for r in regs_of(",".join(ins.fields[1:]) if dest else ins.args) if r[0] == "v"]
    if hits is not None:
        for r in touched:
            if r in state and not exempt(ins, r):
                hits.append((r, state[r][1], ins))
    if ins.op.startswith(VMEM):
        state = {r: (min(a + 1, CAP), p) for r, (a, p) in state.items()}
        for r in dest:
            state[r] = (0, ins)
    return state


def merge(a, b):
    out = dict(a)
    for r, v in b.items():
        if r not in out or v[0] < out[r][0]:
            out[r] = v
    return out


# ---- branch facts: the compiler selects between two waits with a flag in an SGPR pair and two
# vcc branches (`s_mov_b64 s[8:9], -1` / `0`, `s_andn2_b64 vcc, exec, s[8:9]`,
# `s_cbranch_vccnz`), so a path-insensitive analysis would see a path through neither wait.
# States are kept apart by the SGPR constants and the vcc-zero flag they imply.
NOWRITE = ("s_cmp", "s_bitcmp", "s_waitcnt", "s_branch", "s_cbranch", "s_nop", "s_barrier", "s_setprio",
           "s_sleep", "s_endpgm", "s_dcache", "s_icache", "s_sendmsg", "s_trap", "s_setpc", "s_ttrace")


def written_sregs(ins):
    """SGPR / vcc / exec names an instruction may write (conservative)."""
    op = ins.op
    if op.startswith(NOWRITE) or not ins.fields:
        return set()
    out = set()
    if op.startswith("s_") or op.startswith(("v_cmp", "v_readfirstlane", "v_readlane")):
        out |= {str(r[1]) for r in regs_of(ins.fields[0]) if r[0] == "s"}
    if len(ins.fields) > 1 and ("_co_" in op or "div_scale" in op or "_e64" in op):
        out |= {str(r[1]) for r in regs_of(ins.fields[1]) if r[0] == "s"}
    if op.startswith("v_cmpx") or "saveexec" in op:
        out.add("exec")
    if op.startswith("v_cmp") and "_e32" in op:
        out.add("vcc")
    return out


def facts_transfer(facts, ins):
    f = dict(facts)
    w = written_sregs(ins)
    for r in w:
        f.pop(r, None)
    if "vcc" in w or "exec" in w:
        f.pop("vccz", None)
    op = ins.op
    # (only 64-bit lane masks set to all / none: other constants would split the states for nothing)
    if op == "s_mov_b64" and len(ins.fields) == 2 and ins.fields[1] in ("0", "-1"):
        v = int(ins.fields[1])
        for r in regs_of(ins.fields[0]):
            if r[0] == "s":
                f[str(r[1])] = v
    if op in ("s_andn2_b64", "s_and_b64") and len(ins.fields) == 3 and ins.fields[0] == "vcc" and \
            "exec" in ins.fields[1:] and (op == "s_and_b64" or ins.fields[1] == "exec"):
        other = ins.fields[2] if ins.fields[1] == "exec" else ins.fields[1]
        vals = [f.get(str(r[1])) for r in regs_of(other) if r[0] == "s"]
        if vals and all(v in (0, -1) for v in vals) and len(set(vals)) == 1:
            # exec & ~mask / exec & mask; exec is non-zero in any block that runs
            f["vccz"] = (vals[0] == -1) if op == "s_andn2_b64" else (vals[0] == 0)
    return frozenset(f.items())


def check_kernel(lines, a, b):
    blocks, _ = blocks_of(lines, a, b)
    if not blocks:
        return []
    labels = {bl["label"]: i for i, bl in enumerate(blocks)}

    def successors(bi, facts):
        last = blocks[bi]["ins"][-1] if blocks[bi]["ins"] else None
        fall = [bi + 1] if bi + 1 < len(blocks) else []
        if last is None:
            return fall
        if last.op == "s_branch":
            return [labels[last.fields[0]]] if last.fields[0] in labels else []
        if last.op in ("s_endpgm", "s_setpc_b64"):
            return []
        if last.op.startswith("s_cbranch"):
            tgt = [labels[last.fields[0]]] if last.fields[0] in labels else []
            vz = dict(facts).get("vccz")
            if last.op == "s_cbranch_vccz" and vz is not None:
                return tgt if vz else fall
            if last.op == "s_cbranch_vccnz" and vz is not None:
                return fall if vz else tgt
            return tgt + fall
        return fall

    entry = [dict() for _ in blocks]  # facts -> pending
    entry[0][frozenset()] = {}
    work = [0]

    def run(bi, facts, st, hits=None):
        for ins in blocks[bi]["ins"]:
            st = transfer(st, ins, hits)
            facts = facts_transfer(facts, ins)
        return facts, st

    while work:
        bi = work.pop()
        for facts, pend in list(entry[bi].items()):
            f2, st = run(bi, facts, dict(pend))
            for s in successors(bi, f2):
                e = entry[s]
                key = f2
                if key not in e and len(e) >= 64:  # too many distinct facts: collapse
                    key = frozenset()
                    allp = {}
                    for p in e.values():
                        allp = merge(allp, p)
                    e.clear()
                    e[key] = allp
                old = e.get(key)
                m = st if old is None else merge(old, st)
                if old is None or m != old:
                    e[key] = m
                    if s not in work:
                        work.append(s)
    hits = []
    for bi in range(len(blocks)):
        for facts, pend in entry[bi].items():
            run(bi, facts, dict(pend), hits)
    return hits


def main(argv):
    path, subs = argv[1], argv[2:]
    lines = open(path).read().split("\n")
    bad, per = 0, {}
    for name, (a, b) in kernels(lines, subs).items():
        seen = set()
        for r, prod, cons in check_kernel(lines, a, b):
            key = (prod.line, cons.line)
            if key in seen:
                continue
            seen.add(key)
            bad += 1
            if bad <= 40:
                print(f"{name[:70]} {r[0]}{r[1]}: L{prod.line}{' [asm]' if prod.asm else ''} {prod.text!r} -> "
                      f"L{cons.line}{' [asm]' if cons.asm else ''} {cons.text!r}")
        if seen:
            per[name] = len(seen)
    for name, c in per.items():
        print(f"  {c:5d}  {name}")
    print(f"vmcnt_check: {bad} read(s) of registers with a load in flight")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
