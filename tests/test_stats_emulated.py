"""The statistics kernel (custereomatching_amd/csrc/stats.hip) emulated on the CPU, every mode and
row range, against the oracle's per-pixel fp32 mean / centred squares (oracle/zncc_oracle.c
orc_stats, the reference's stereo_matching_kernel.cu:40-69 order) and numpy fp64 patch sums.

The kernel source is compiled for the host (clang++) with tests/emu/shim/common.h in place of
csrc/common.h: workgroups run in turn, their 256 threads as std::threads meeting at a std::barrier
for __syncthreads(), the dynamic LDS a per-workgroup buffer filled with garbage first.  This checks
the kernel's thread / LDS indexing and its arithmetic order without a GPU; the GPU suite
(test_gpu_parity.py) checks the same kernel compiled for gfx950 through the whole op."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.inputs import make_pair

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "custereomatching_amd", "csrc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
FULL, BOX, PREP, FWD, MSB = 0, 1, 2, 3, 4
ALL_ROWS, BAND_ROWS = 0, 1


def _decls():
    src = open(os.path.join(CSRC, "common.h")).read()
    out = []
    for pat in (r"struct Geo \{.*?\n\};", r"struct Stats \{.*?\n\};", r"enum StatsMode \{[^}]*\};",
                r"enum StatsRows \{[^}]*\};"):
        m = re.search(pat, src, re.S)
        assert m, pat
        out.append(m.group(0))
    return "\n".join(out)


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no host clang++ (ROCm LLVM) in this image")
    d = tmp_path_factory.mktemp("stats_emu")
    shim = open(os.path.join(HERE, "emu", "shim", "common.h")).read().replace("@EMU_DECLS@", _decls())
    (d / "common.h").write_text(shim)
    shutil.copy(os.path.join(HERE, "emu", "shim", "sweep.h"), d / "sweep.h")
    shutil.copy(os.path.join(CSRC, "stats_body.h"), d / "stats_body.h")
    shutil.copy(os.path.join(ROOT, "include", "custma.h"), d / "custma.h")
    src = open(os.path.join(CSRC, "stats.hip")).read()
    lds = re.search(r"extern __shared__[^;]*double lds_d\[\];", src)
    assert lds, "the kernel's dynamic LDS declaration"
    (d / "stats_emu.cpp").write_text(src.replace(lds.group(0), "double* lds_d = g_lds;"))
    shutil.copy(os.path.join(HERE, "emu", "stats_emu_main.cpp"), d / "main.cpp")
    exe = d / "stats_emu"
    r = subprocess.run([CLANG, "-std=c++20", "-O1", "-pthread", "-ffp-contract=off", "-I", str(d),
                        str(d / "stats_emu.cpp"), str(d / "main.cpp"), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return d, exe


def _run(emu, cam, proj, k, mode, rows=ALL_ROWS, band=None, shift=(0.25, -0.125)):
    d, exe = emu
    H, W = cam.shape
    h_lo, h_hi = band or (0, H)
    inp, out = d / "in.bin", d / "out.bin"
    with open(inp, "wb") as f:
        np.ascontiguousarray(cam, np.float32).tofile(f)
        np.ascontiguousarray(proj, np.float32).tofile(f)
        np.asarray(shift, np.float32).tofile(f)
    r = subprocess.run([str(exe), str(inp), str(out), str(H), str(W), str(k), str(mode), str(rows), str(h_lo),
                        str(h_hi)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr)
    n = H * W
    raw = open(out, "rb").read()
    off = 0

    def take(count, dt):
        nonlocal off
        a = np.frombuffer(raw, dt, count, off)
        off += count * np.dtype(dt).itemsize
        return a

    mean, sq = take(2 * n, np.float32).reshape(2, H, W), take(2 * n, np.float32).reshape(2, H, W)
    box, sqt = take(2 * n, np.float64).reshape(2, H, W), take(2 * n, np.float32).reshape(2, H, W)
    prep = take(6 * n, np.float32).reshape(2, 3, H, W)
    return mean, sq, box, sqt, prep


def _box_ref(img, k):
    """fp64 patch sums and sums of squares in the kernel's order: k-tap row sums (j ascending), then
    the k row sums down the column (i ascending); taps -k/2 .. k-1-k/2, zero outside the image."""
    H, W = img.shape
    r0 = k // 2
    pad = np.zeros((H + k, W + k), np.float64)
    pad[r0:r0 + H, r0:r0 + W] = img
    rs = np.zeros((H + k, W))
    rs2 = np.zeros((H + k, W))
    for j in range(k):
        v = pad[:, j:j + W]
        rs = rs + v
        rs2 = rs2 + v * v  # v * v is exact in fp64, so this is fma(v, v, b)
    b = np.zeros((H, W))
    b2 = np.zeros((H, W))
    for i in range(k):
        b = b + rs[i:i + H]
        b2 = b2 + rs2[i:i + H]
    c2 = b2 - b * b / float(k * k)
    return b, np.where(c2 > 0.0, c2, 0.0).astype(np.float32)


def _eq(a, b):
    return np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


CASES = [(70, 45, 11), (33, 70, 3), (20, 44, 4), (65, 33, 5), (9, 40, 7), (1, 31, 3), (40, 50, 16), (35, 70, 31),
         (30, 41, 33)]


@pytest.mark.parametrize("H,W,k", CASES, ids=[f"{h}x{w}_k{k}" for h, w, k in CASES])
@pytest.mark.parametrize("mode", [FULL, BOX, PREP, FWD, MSB], ids=["full", "box", "prep", "fwd", "msb"])
def test_stats_kernel_emulated(emu, H, W, k, mode):
    cam, proj = make_pair(H, W, 16, seed=H * 131 + W + k)
    shift = (0.25, -0.125)
    mean, sq, box, sqt, prep = _run(emu, cam, proj, k, mode, shift=shift)
    for z, img in enumerate((cam, proj)):
        m_ref, s_ref = O.stats(img, k, contract=1)
        b_ref, t_ref = _box_ref(img, k)
        chain = mode in (FULL, FWD, MSB)
        assert _eq(box[z], b_ref), ("box", z)
        assert _eq(sq[z], s_ref) if chain else np.isnan(sq[z]).all(), ("sq", z)
        assert _eq(mean[z], m_ref) if mode in (FULL, MSB) else np.isnan(mean[z]).all(), ("mean", z)
        assert _eq(sqt[z], t_ref) if mode in (FULL, BOX) else np.isnan(sqt[z]).all(), ("sqt", z)
        if mode == PREP:
            assert _eq(prep[z, 0], t_ref)
            assert _eq(prep[z, 1], (b_ref / float(k * k) - float(np.float32(shift[z]))).astype(np.float32))
            assert _eq(prep[z, 2], img.astype(np.float32))
        else:
            assert np.isnan(prep[z]).all()


@pytest.mark.parametrize("mode", [FWD, MSB])
def test_stats_kernel_emulated_band_rows(emu, mode):
    """STATS_BAND_ROWS: only the volume rows [h_lo, h_hi) are written (their patches still read the
    halo rows around them)."""
    H, W, k = 70, 45, 11
    cam, proj = make_pair(H, W, 16, seed=5)
    mean, sq, box, _, _ = _run(emu, cam, proj, k, mode, rows=BAND_ROWS, band=(9, 50))
    for z, img in enumerate((cam, proj)):
        m_ref, s_ref = O.stats(img, k, contract=1)
        b_ref, _ = _box_ref(img, k)
        assert _eq(sq[z, 9:50], s_ref[9:50]) and _eq(box[z, 9:50], b_ref[9:50])
        assert np.isnan(sq[z, :9]).all() and np.isnan(sq[z, 50:]).all() and np.isnan(box[z, :9]).all()
        if mode == MSB:
            assert _eq(mean[z, 9:50], m_ref[9:50])
