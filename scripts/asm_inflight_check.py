"""Static check of hand-pipelined inline-asm loads in a gfx950 .s listing (diagnostic only).

The compiler believes an inline-asm load writes its destination when the asm issues; the
hardware writes it when the load returns.  This flags every instruction that reads or
writes a VGPR of a load that is still in flight, i.e. before the `s_waitcnt vmcnt(N)` that
retires it (vmcnt counts in issue order, loads and stores alike).  Straight-line scan of
the listing in layout order, with a fresh state at every loop header, so it is a screen,
not a proof.  Usage: python scripts/asm_inflight_check.py <file.s> <kernel-symbol-substring>
"""
import re
import sys


def regs(text):
    out = set()
    for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if c:
            out.add(int(c))
        else:
            out |= set(range(int(a), int(b) + 1))
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.split()[0].endswith(":"))
    inflight = []  # [regs, ...] oldest first, one entry per VMEM op (stores carry no registers)
    issues = []
    for i in range(start + 1, len(lines)):
        t = lines[i].strip()
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith(";") or t.startswith("."):
            continue
        parts = t.split(None, 1)
        op, args = parts[0], (parts[1] if len(parts) > 1 else "")
        m = re.match(r"s_waitcnt\b.*vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            inflight = inflight[len(inflight) - n:] if n < len(inflight) else inflight
            continue
        fields = [f.strip() for f in args.split(",")]
        first = regs(fields[0]) if fields else set()
        rest = regs(",".join(fields[1:]))
        pending = set().union(*inflight) if inflight else set()
        if op.startswith(("buffer_load", "global_load")):
            if rest & pending or first & pending:
                issues.append((i + 1, t, sorted((rest | first) & pending)))
            inflight.append(first)
            continue
        if op.startswith(("buffer_store", "global_store")):
            if (first | rest) & pending:
                issues.append((i + 1, t, sorted((first | rest) & pending)))
            inflight.append(set())
            continue
        used = first | rest
        if used & pending:
            issues.append((i + 1, t, sorted(used & pending)))
    print(f"{len(issues)} instructions touch a register of an in-flight load")
    for x in issues[:40]:
        print(x)

    # second screen: VALU writes an SGPR, a VMEM reads it within 5 wait states (gfx9 hazard;
    # the compiler does not pad inline asm for it)
    def sregs(text):
        out = set()
        for a, b, c in re.findall(r"s\[(\d+):(\d+)\]|\bs(\d+)\b", text):
            if c:
                out.add(int(c))
            else:
                out |= set(range(int(a), int(b) + 1))
        return out

    recent = []  # (wait states since, sgprs written)
    haz = []
    for i in range(start + 1, len(lines)):
        t = lines[i].strip()
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith(";") or t.startswith("."):
            continue
        parts = t.split(None, 1)
        op, args = parts[0], (parts[1] if len(parts) > 1 else "")
        if op.startswith(("buffer_", "global_")):
            used = sregs(args)
            for ws, regs_w in recent:
                if ws < 5 and used & regs_w:
                    haz.append((i + 1, t, sorted(used & regs_w), ws))
        n = 1
        m = re.match(r"s_nop\s+(\d+)", t)
        if m:
            n = int(m.group(1)) + 1
        recent = [(ws + n, r) for ws, r in recent if ws + n < 5]
        if op.startswith("v_"):
            dst = args.split(",")[0] if args else ""
            w = sregs(dst)
            if w:
                recent.append((0, w))
    print(f"{len(haz)} VMEM instructions read an SGPR written by VALU < 5 wait states earlier")
    for x in haz[:20]:
        print(x)


if __name__ == "__main__":
    main()
