#!/usr/bin/env python3
"""Wait-state check of a gfx950 (gfx9-family) .s listing: every hazard pair below, over the
kernel's control-flow graph (a fixpoint of "wait states since the last VALU write" per
register at every block entry, so loop back-edges and branch joins are covered).

Rules (producer = a VALU instruction, consumer needs at least N wait states after it; one
issued instruction = 1 state, `s_nop n` = n + 1):
  R1  VALU writes SGPR  -> VMEM (buffer_* / global_*) reads it (descriptor, soffset)   5
  R2  VALU writes VGPR  -> DPP instruction reads it as src0                           2
  R3  VALU writes VGPR  -> v_permlane{16,32}_swap reads either operand                2
  R4  VALU writes SGPR  -> v_readlane / v_writelane uses it as lane select            4
  R5  VALU writes EXEC  -> DPP instruction                                            5
  R6  VALU writes VGPR  -> v_readlane / v_readfirstlane reads it (gfx950)             1

The compiler pads its own code; it does not look inside inline asm, so the rules that matter
are those whose producer or consumer sits between ;;#ASMSTART and ;;#ASMEND.  Every hit is
reported with the side(s) that are inline asm.  Exit status 1 when any hit has an asm side.

Usage: python custereomatching_amd/hazard_check.py file.s [kernel-substring ...]
"""
from __future__ import annotations

import re
import sys

NEED = {"R1": 5, "R2": 2, "R3": 2, "R4": 4, "R5": 5, "R6": 1}


def _range(tok):
    m = re.fullmatch(r"([sv])\[(\d+):(\d+)\]", tok)
    if m:
        return [(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.fullmatch(r"([sv])(\d+)", tok)
    if m:
        return [(m.group(1), int(m.group(2)))]
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return [("s", "vcc")]
    if tok in ("exec", "exec_lo", "exec_hi"):
        return [("s", "exec")]
    return []


def regs_of(field):
    out = []
    for tok in re.findall(r"[sv]\[\d+:\d+\]|\b[sv]\d+\b|\bvcc(?:_lo|_hi)?\b|\bexec(?:_lo|_hi)?\b", field):
        out += _range(tok)
    return out


def split_operands(args):
    # operands before the first modifier keyword (row_..., offset:, etc.)
    core = re.split(r"\s(?=[a-z_]+:|row_|wave_|quad_perm|offen|idxen|glc|slc|nt\b|sc0|sc1|bound_ctrl|op_sel|neg_)", args,
                    maxsplit=1)[0]
    return [f.strip() for f in core.split(",") if f.strip()]


class Ins:
    __slots__ = ("op", "args", "fields", "asm", "line", "text")

    def __init__(self, text, asm, line):
        parts = text.split(None, 1)
        self.op = parts[0]
        self.args = parts[1] if len(parts) > 1 else ""
        self.fields = split_operands(self.args)
        self.asm = asm
        self.line = line
        self.text = text

    def states(self):
        m = re.match(r"s_nop\s+(\d+)", self.text)
        return int(m.group(1)) + 1 if m else 1

    def is_valu(self):
        return self.op.startswith("v_") and self.op != "v_nop"

    def writes(self):
        if not self.is_valu() or not self.fields:
            return []
        w = regs_of(self.fields[0])
        if ("_co_" in self.op or "div_scale" in self.op) and len(self.fields) > 1 and not self.fields[1].startswith("v"):
            w += regs_of(self.fields[1])
        if self.op.startswith("v_cmpx"):
            w.append(("s", "exec"))
        return w

    def is_dpp(self):
        return "_dpp" in self.op or bool(re.search(r"\b(row_|wave_|quad_perm|row_newbcast)", self.args))


def kernels(lines, subs):
    out = {}
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\w+):", lines[i])
        if m and (not subs or any(s in m.group(1) for s in subs)):
            j = i + 1
            while j < len(lines) and ".Lfunc_end" not in lines[j]:
                j += 1
            out[m.group(1)] = (i, j)
            i = j
        i += 1
    return out


def blocks_of(lines, a, b):
    blocks, labels, cur, asm = [], {}, None, False
    for ln in range(a, b):
        raw = lines[ln]
        s = raw.strip()
        if "#ASMSTART" in s:
            asm = True
            continue
        if "#ASMEND" in s:
            asm = False
            continue
        m = re.match(r"^(\.?[\w$.]+):", raw)
        if m:
            cur = {"label": m.group(1), "ins": []}
            labels[m.group(1)] = len(blocks)
            blocks.append(cur)
            continue
        if re.match(r"^; %bb\.\d+:", s):  # a fall-through block without a label
            cur = None
            continue
        if not s or s.startswith((";", ".")):
            continue
        s = s.split(";")[0].strip()
        if not s:
            continue
        if cur is None:
            cur = {"label": f"<bb@{ln + 1}>", "ins": []}
            blocks.append(cur)
        cur["ins"].append(Ins(s, asm, ln + 1))
        if cur["ins"][-1].op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            cur = None  # a branch ends its block: what follows is the fall-through block
    succ = []
    for bi, bl in enumerate(blocks):
        nxt = []
        last = bl["ins"][-1] if bl["ins"] else None
        fall = True
        if last is not None:
            if last.op == "s_branch":
                nxt.append(labels.get(last.fields[0]))
                fall = False
            elif last.op.startswith("s_cbranch"):
                nxt.append(labels.get(last.fields[0]))
            elif last.op in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and bi + 1 < len(blocks):
            nxt.append(bi + 1)
        succ.append([n for n in nxt if n is not None])
    return blocks, succ


def transfer(state, ins, hits=None):
    """state: {reg: (wait states since the last VALU write, producing instruction)}."""
    def check(rule, regs):
        if hits is None:
            return
        for r in regs:
            if r in state and state[r][0] < NEED[rule]:
                prod = state[r][1]
                hits.append((rule, r, state[r][0], prod, ins))

    if ins.op.startswith(("buffer_", "global_")):
        check("R1", [r for r in regs_of(ins.args) if r[0] == "s"])
    if ins.is_dpp() and ins.op.startswith("v_") and len(ins.fields) > 1:
        check("R2", [r for r in regs_of(ins.fields[1]) if r[0] == "v"])
        check("R5", [("s", "exec")])
    if ins.op.startswith(("v_permlane16_swap", "v_permlane32_swap")):
        check("R3", [r for f in ins.fields[:2] for r in regs_of(f) if r[0] == "v"])
    if ins.op in ("v_readlane_b32", "v_writelane_b32") and len(ins.fields) > 2:
        check("R4", [r for r in regs_of(ins.fields[2]) if r[0] == "s"])
    if ins.op in ("v_readlane_b32", "v_readfirstlane_b32") and len(ins.fields) > 1:
        check("R6", [r for r in regs_of(ins.fields[1]) if r[0] == "v"])
    n = ins.states()
    new = {r: (ws + n, p) for r, (ws, p) in state.items() if ws + n < 5}
    for r in ins.writes():
        new[r] = (0, ins)
    return new


def merge(a, b):
    out = dict(a)
    for r, v in b.items():
        if r not in out or v[0] < out[r][0]:
            out[r] = v
    return out


def check_kernel(lines, a, b):
    blocks, succ = blocks_of(lines, a, b)
    entry = [None] * len(blocks)
    if not blocks:
        return []
    entry[0] = {}
    work = [0]
    while work:
        bi = work.pop()
        st = dict(entry[bi])
        for ins in blocks[bi]["ins"]:
            st = transfer(st, ins)
        for s in succ[bi]:
            m = st if entry[s] is None else merge(entry[s], st)
            if entry[s] is None or m != entry[s]:
                entry[s] = m
                work.append(s)
    hits = []
    for bi, bl in enumerate(blocks):
        if entry[bi] is None:
            continue
        st = dict(entry[bi])
        for ins in bl["ins"]:
            st = transfer(st, ins, hits)
    return hits


def main(argv):
    verbose = "-v" in argv
    argv = [a for a in argv if a != "-v"]
    path, subs = argv[1], argv[2:]
    lines = open(path).read().split("\n")
    bad = 0
    for name, (a, b) in kernels(lines, subs).items():
        hits = check_kernel(lines, a, b)
        asm_hits = [h for h in hits if h[3].asm or h[4].asm]
        seen = set()
        for rule, r, ws, prod, cons in asm_hits:
            key = (rule, prod.line, cons.line)
            if key in seen:
                continue
            seen.add(key)
            bad += 1
            if bad <= 30:
                print(f"{name[:60]} {rule} {r} after {ws} states: L{prod.line}{' [asm]' if prod.asm else ''} "
                      f"{prod.text!r} -> L{cons.line}{' [asm]' if cons.asm else ''} {cons.text!r}")
        comp = [h for h in hits if not (h[3].asm or h[4].asm)]
        if comp and verbose:
            print(f"{name[:60]}: {len(comp)} compiler-only pairs (compiler pads these itself or the rule is looser)")
    print(f"hazard_check: {bad} inline-asm hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
