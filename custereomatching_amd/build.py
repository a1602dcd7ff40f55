"""Build libcustma_hip.so for gfx950 with hipcc (in-tree, so it travels with
the repo snapshot to the GPU box).  Usage: python custereomatching_amd/build.py [--force]

Each .hip translation unit is compiled separately (parallel) and linked
into one shared library exporting the C ABI of include/custma.h.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libcustma_hip.so")
SOURCES = ["capi.hip", "stats.hip", "fwd_exact.hip", "sweep_fwd.hip", "sweep_wave.hip", "bwd_fused.hip", "bwd_generic.hip", "select.hip", "preprocess.hip"]
SWEEP_KS = tuple(range(1, 32))  # CUSTMA_SWEEP_KS in csrc/sweep.h
# translation units: (object name, source, defines).  sweep_wave.hip compiles once per kernel
# size (its instantiations dominate the build) plus once for the dispatch.
UNITS = [(os.path.splitext(src)[0], src, []) for src in SOURCES if src != "sweep_wave.hip"]
UNITS += [("sweep_wave_d", "sweep_wave.hip", ["-DCUSTMA_SW_DISPATCH"])]
UNITS += [(f"sweep_wave_k{k}", "sweep_wave.hip", [f"-DCUSTMA_SW_K={k}"]) for k in SWEEP_KS]
# translation units whose inline asm omits wait states where the listing shows none are needed
HAZARD_CHECKED = ("bwd_fused.hip", "sweep_wave.hip", "sweep_fwd.hip")
ARCH = os.environ.get("CUSTMA_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: fused multiply-adds only where written (__builtin_fmaf / fma);
# the exact path replays the reference's nvcc contraction explicitly.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-fno-gpu-rdc", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def _obj(unit, libdir=LIBDIR):
    return os.path.join(libdir, unit[0] + ".o")


def _deps():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))] + [
        os.path.join(HERE, "..", "include", "custma.h")]


def _compile(unit, extra=(), libdir=LIBDIR):
    name, src, defs = unit
    out = _obj(unit, libdir)
    cmd = [HIPCC, *CFLAGS, *defs, *extra, "-c", os.path.join(CSRC, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {name} ({src}):\n{r.stderr}")
    if src in HAZARD_CHECKED:
        _check_hazards(unit, extra, libdir)
    return out


def _check_hazards(unit, extra, libdir):
    """Inline asm that leaves out wait states (hazard_check.py) is only safe in the code the
    compiler actually emitted: check the device listing of the same compile."""
    name, src, defs = unit
    listing = os.path.join(libdir, name + ".s")
    cmd = [HIPCC, *CFLAGS, *defs, *extra, "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", listing]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc -S failed for {name} ({src}):\n{r.stderr}")
    r = subprocess.run([sys.executable, os.path.join(HERE, "hazard_check.py"), listing], capture_output=True, text=True)
    if r.returncode != 0:
        os.remove(_obj(unit, libdir))
        raise RuntimeError(f"wait-state hazards in {name} ({src}):\n{r.stdout}")
    # and no instruction touches a register whose (hand-waited) load is still in flight
    r = subprocess.run([sys.executable, os.path.join(HERE, "vmcnt_check.py"), listing], capture_output=True, text=True)
    if r.returncode != 0:
        os.remove(_obj(unit, libdir))
        raise RuntimeError(f"registers read with their load in flight in {name} ({src}):\n{r.stdout}")
    with open(listing) as f:
        scratch = scratch_lines(f.read())
    if scratch:
        os.remove(_obj(unit, libdir))
        raise RuntimeError(f"scratch use in {name} ({src}): {scratch[:4]}")
    os.remove(listing)


def scratch_lines(listing: str):
    """The `; ScratchSize: N` lines of a device listing with N != 0.  The hand-pipelined kernels
    must not spill VGPRs to scratch: the compiler takes an asm load's destination as written when
    the asm issues, so a spill could store it while the load is still in flight."""
    return [ln.strip() for ln in listing.splitlines()
            if ln.startswith("; ScratchSize:") and ln.split(":", 1)[1].strip() != "0"]


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [
        os.path.join(HERE, "..", "include", "custma.h")]


def _stale(unit, hdr_mtime):
    o = _obj(unit)
    if not os.path.exists(o):
        return True
    return os.path.getmtime(o) < max(hdr_mtime, os.path.getmtime(os.path.join(CSRC, unit[1])))


def build(force: bool = False, verbose: bool = False) -> str:
    """Incremental: a translation unit is recompiled when it or any header is newer than its object."""
    os.makedirs(LIBDIR, exist_ok=True)
    newest = max(os.path.getmtime(p) for p in _deps())
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        return LIB
    hdr = max(os.path.getmtime(p) for p in _headers())
    todo = [u for u in UNITS if force or _stale(u, hdr)]
    with cf.ThreadPoolExecutor(max_workers=max(1, min(len(todo), os.cpu_count() or 4))) as ex:
        list(ex.map(_compile, todo))
    objs = [_obj(u) for u in UNITS]
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


def build_variant(libdir: str, defines, only=None) -> str:
    """Ablation build (benchmarking only): the same library with extra -D switches into
    another directory; load it with CUSTMA_LIB=<path>.  `only`: the translation units the
    switches affect, by source file or unit name (the rest link from the main build's objects
    as they are).  The main library is never rebuilt here: an A/B's base is whatever was built
    last, so a working-tree change under test cannot leak into it."""
    os.makedirs(libdir, exist_ok=True)
    extra = [d if d.startswith("-") else f"-D{d}" for d in defines]  # "-f..." flags pass through
    todo = [u for u in UNITS if only is None or u[1] in only or u[0] in only]
    missing = [u[0] for u in UNITS if u not in todo and not os.path.exists(_obj(u))]
    if missing:
        raise RuntimeError(f"main-build objects missing for {missing}: run build() first")
    with cf.ThreadPoolExecutor(max_workers=max(1, min(len(todo), os.cpu_count() or 4))) as ex:
        done = dict(zip([u[0] for u in todo], ex.map(lambda u: _compile(u, extra, libdir), todo)))
    objs = [done.get(u[0], _obj(u)) for u in UNITS]
    lib = os.path.join(libdir, "libcustma_hip.so")
    r = subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", lib, *objs], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
