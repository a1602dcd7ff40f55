"""Pin the CPU oracle (oracle/zncc_oracle.c) against the reference.

Golden vectors (tests/golden/*.npz) were produced by the REFERENCE's own
torch path, examples/verify.py:81-133, in fp32 and fp64
(tests/golden/gen_golden.py).  The oracle restates the reference CUDA
arithmetic (stereo_matching_kernel.cu:39-71, :97-179); these tests show it
agrees with the reference's torch path to within the reference's own fp32
rounding, and that the exact-arithmetic flavours are internally consistent.
"""
import glob
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.inputs import make_pair

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SMALL = sorted(p for p in glob.glob(os.path.join(GOLD, "*.npz")) if not os.path.basename(p).startswith("verify_"))
VERIFY = sorted(glob.glob(os.path.join(GOLD, "verify_*.npz")))


def _load(p):
    z = np.load(p)
    return z, z["cam"], z["proj"], int(z["k"]), int(z["D"])


@pytest.mark.parametrize("path", SMALL, ids=os.path.basename)
def test_literal_equals_hoisted(path):
    """Per-voxel literal restatement == per-pixel-stats restatement, bitwise."""
    _, cam, proj, k, D = _load(path)
    for contract in (1, 0):
        a = O.forward(cam, proj, k, contract=contract)
        b = O.forward(cam, proj, k, contract=contract, literal=True)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("path", SMALL, ids=os.path.basename)
def test_forward_vs_reference_golden(path):
    z, cam, proj, k, D = _load(path)
    v = O.forward(cam, proj, k)
    bound = O.cost_error_bound(k)
    # vs fp64 truth of the reference torch path (eps is 1e-8f here, 1e-8 there: ~1e-9 relative)
    assert np.abs(v - z["vol64"]).max() <= bound
    # vs the reference torch path in fp32 (both carry fp32 rounding)
    assert np.abs(v - z["vol32"]).max() <= 2 * bound
    # the oracle's own fp64 restatement reproduces the reference fp64 truth
    assert np.abs(O.forward_f64(cam, proj, k) - z["vol64"]).max() < 1e-7


@pytest.mark.parametrize("path", SMALL, ids=os.path.basename)
def test_backward_vs_reference_golden(path):
    z, cam, proj, k, D = _load(path)
    H, W = cam.shape
    g = np.ones((H, W, W), np.float32)
    dc, dp = O.backward_f64(g, cam, proj, k)
    mg = max(1.0, np.abs(z["cg64"]).max())
    assert np.abs(dc - z["cg64"]).max() <= 1e-7 * mg
    mp = max(1.0, np.abs(z["pg64"]).max())
    assert np.abs(dp - z["pg64"]).max() <= 1e-7 * mp
    # fp32 reference arithmetic (what the CUDA kernel computes, minus atomics)
    fc, fp = O.backward(g, cam, proj, k)
    assert np.abs(fc - z["cg64"]).max() <= 3e-5 * mg
    assert np.abs(fp - z["pg64"]).max() <= 3e-5 * mp


@pytest.mark.parametrize("path", VERIFY, ids=os.path.basename)
def test_verify_config_golden(path):
    """BASELINE configs[0]: 128x256, D=32, window 5."""
    z, cam, proj, k, D = _load(path)
    v = O.forward(cam, proj, k)
    flat = v.reshape(-1)
    bound = O.cost_error_bound(k)
    assert np.abs(flat[z["sample_idx"]] - z["sample64"]).max() <= bound
    idx, best = O.argmax(v)
    assert np.abs(best - z["max64"]).max() <= bound
    # argmax bit-exact wherever the reference's top-2 gap exceeds the rounding band
    clear = z["gap64"] > 2 * bound
    assert clear.mean() > 0.5
    assert np.array_equal(idx[clear], z["argmax64"][clear].astype(np.int64))
    g = np.ones_like(v)
    dc, dp = O.backward_f64(g, cam, proj, k)
    mg = max(1.0, np.abs(z["cg64"]).max())
    assert np.abs(dc - z["cg64"]).max() <= 1e-7 * mg
    assert np.abs(dp - z["pg64"]).max() <= 1e-7 * max(1.0, np.abs(z["pg64"]).max())


def test_window_is_slice_of_full():
    z, cam, proj, k, _ = _load(os.path.join(GOLD, "tex_24x48_k5.npz"))
    D = 7
    full = O.forward(cam, proj, k)
    win = O.forward(cam, proj, k, layout=O.WINDOW, D=D)
    H, W = cam.shape
    for w in range(W - D):
        assert np.array_equal(win[:, w, :], full[:, w, w:w + D + 1])


def test_window_backward_matches_masked_full():
    z, cam, proj, k, _ = _load(os.path.join(GOLD, "tiny_16x24_k5.npz"))
    H, W = cam.shape
    D = 5
    rng = np.random.default_rng(3)
    gw = rng.standard_normal((H, W - D, D + 1)).astype(np.float32)
    gf = np.zeros((H, W, W), np.float32)
    for w in range(W - D):
        gf[:, w, w:w + D + 1] = gw[:, w, :]
    a = O.backward_f64(gw, cam, proj, k, layout=O.WINDOW, D=D)
    b = O.backward_f64(gf, cam, proj, k)
    for x, y in zip(a, b):
        assert np.abs(x - y).max() <= 1e-9 * max(1, np.abs(y).max())


def test_constant_and_zero_images():
    for v in (0.0, 0.5):
        a = np.full((9, 13), v, np.float32)
        out = O.forward(a, a, 3)
        # interior patches are flat: E = 0, X = Y = 0 -> eps / sqrt(eps)
        expect = np.float32(1e-8) / np.sqrt(np.float32(1e-8))
        inner = out[1:-1, 1:-1, 1:-1] if v else out
        assert np.abs(inner - expect).max() < 1e-9 + 1e-6 * abs(expect)


def test_argmax_first_index_on_ties():
    v = np.array([[1, 3, 3, 2], [0, 0, 0, 0]], np.float32)
    idx, best = O.argmax(v)
    assert idx.tolist() == [1, 0] and best.tolist() == [3, 0]


# ---- the timed CPU baseline (oracle/torch_ref.py) pinned to the reference's torch path ----

@pytest.mark.parametrize("name", ["tiny_16x24_k5", "tex_20x48_k9", "quant_24x48_k5", "tall_40x12_k11",
                                  "row_1x32_k5"])
@pytest.mark.parametrize("row_chunk", [None, 7])
def test_torch_ref_matches_reference_torch_goldens(name, row_chunk):
    """bench.py's cpu_baseline runs oracle/torch_ref.py: it must be the reference's
    examples/verify.py:81-133 computation (goldens made by importing it), whole and in
    haloed row bands (row_chunk)."""
    import torch

    from oracle import torch_ref as T

    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    cam, proj, k = torch.from_numpy(z["cam"]), torch.from_numpy(z["proj"]), int(z["k"])
    vol, gc, gp = T.forward_backward(cam, proj, k, row_chunk=row_chunk)
    if vol is None:
        vol = T.forward_only(cam, proj, k, row_chunk=row_chunk)
    assert np.abs(vol.numpy() - z["vol32"]).max() <= 2e-6
    for got, ref in ((gc, z["cg64"]), (gp, z["pg64"])):
        assert np.abs(got.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("k", [2, 4, 6])
def test_torch_ref_even_k_matches_c_oracle(k):
    """Even k (taps at -k/2 .. k/2-1, stereo_matching_kernel.cu:44,60): the torch
    restatement and the C oracle agree in fp64."""
    import torch

    from oracle import torch_ref as T

    cam, proj = make_pair(13, 17, 4, seed=k)
    v, gc, gp = T.forward_backward(torch.from_numpy(cam).double(), torch.from_numpy(proj).double(), k)
    rc, rp = O.backward_f64(np.ones((13, 17, 17), np.float32), cam, proj, k)
    assert np.abs(v.numpy() - O.forward_f64(cam, proj, k)).max() <= 1e-9
    assert np.abs(gc.numpy() - rc).max() <= 1e-9 * max(1.0, np.abs(rc).max())
    assert np.abs(gp.numpy() - rp).max() <= 1e-9 * max(1.0, np.abs(rp).max())


@pytest.mark.parametrize("k,D,row_chunk", [(5, 7, None), (11, 12, 5), (4, 3, 4)])
def test_torch_ref_window_layout_matches_c_oracle(k, D, row_chunk):
    """The window-layout CPU baseline (bench.py's c5 workload) against the C oracle."""
    import torch

    from oracle import torch_ref as T

    cam, proj = make_pair(16, 40, D, seed=k + D)
    g = np.random.default_rng(1).standard_normal((16, 40 - D, D + 1)).astype(np.float32)
    v, gc, gp = T.forward_backward(torch.from_numpy(cam).double(), torch.from_numpy(proj).double(), k,
                                   grad=torch.from_numpy(g).double(), layout="window", D=D, row_chunk=row_chunk)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
    if v is not None:
        assert np.abs(v.numpy() - O.forward_f64(cam, proj, k, layout=O.WINDOW, D=D)).max() <= 1e-9
    assert np.abs(gc.numpy() - rc).max() <= 1e-9 * max(1.0, np.abs(rc).max())
    assert np.abs(gp.numpy() - rp).max() <= 1e-9 * max(1.0, np.abs(rp).max())


def test_tile_backward_crop_is_exact():
    """tests/oracle_tiles.tile_backward (the C5 backward check's oracle) equals the whole-image
    fp64 oracle on the tile it returns, at both image edges and in the middle."""
    from tests.golden.inputs import make_pair
    from tests.oracle_tiles import tile_backward

    H, W, k, D = 20, 150, 5, 24
    cam, proj = make_pair(H, W, D, seed=9)
    g = np.random.default_rng(10).standard_normal((H, W - D, D + 1)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
    for h0, c0 in ((0, 0), (7, 30), (15, W - 100)):
        h1 = min(H, h0 + 4)
        tc, tp, (a, b), (c, d) = tile_backward(g, cam, proj, k, D, h0, h1, c0, 100)
        assert b > a and d > c
        np.testing.assert_allclose(tc, rc[h0:h1, a:b], rtol=0, atol=1e-9)
        np.testing.assert_allclose(tp, rp[h0:h1, c:d], rtol=0, atol=1e-9)
