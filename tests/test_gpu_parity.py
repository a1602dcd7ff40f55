"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bars (task contract / BASELINE north_star):
  * exact forward: bit-identical to the oracle's reference arithmetic
    (nvcc -fmad=true flavour of stereo_matching_kernel.cu:39-71);
  * fast forward: |cost - exact| <= min(1e-5, (k^2+6) 2^-24) (oracle.fast_tolerance:
    north_star's 1e-5, tighter where the worst-case bound is);
  * disparity (fused, certified) and volume argmax: bit-identical indices;
  * gradients (both images): |g - g_f64| <= 1e-5 * max(1, max|g_f64|).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.golden.inputs import make_pair

import custereomatching_amd as cm

pytestmark = pytest.mark.gpu

FULL, WIN = "full", "window"


def _dev(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(dtype)


def _layout_args(layout, D):
    return (O.FULL, 0) if layout == FULL else (O.WINDOW, D)


def gpu_forward(cam, proj, k, layout, D, precision, dev, dtype=torch.float32):
    out = cm.cost_volume_forward(_dev(cam, dev, dtype), _dev(proj, dev, dtype), D, k, layout, precision)
    torch.cuda.synchronize()
    return out.cpu().numpy()


CASES = [
    # H, W, k, D, kind
    (24, 48, 5, 16, "textured"),
    (20, 48, 9, 16, "textured"),
    (1, 32, 5, 8, "textured"),
    (40, 12, 11, 4, "textured"),
    (33, 70, 3, 20, "smooth"),
    (17, 40, 1, 10, "textured"),
    (30, 64, 15, 31, "quantized"),
    (24, 48, 7, 0, "textured"),
    (26, 40, 5, 39, "textured"),
    # k > 11: the volume is the exact kernel's (the fast volume stops at k = 11, capi.hip
    # kFastVolumeMaxK); the sliding instantiations up to k = 31 serve the disparity and backward
    (19, 37, 21, 9, "textured"),
    (22, 60, 31, 12, "textured"),
    (16, 40, 25, 9, "smooth"),
    (30, 70, 17, 31, "textured"),  # the largest sweep instantiation (16 + 2r = 32 columns)
    (20, 44, 4, 9, "textured"),   # even k: taps at -k/2 .. k/2-1 (reference .cu:44,60), sliding kernels
    (17, 33, 10, 6, "smooth"),
    (21, 50, 2, 11, "textured"),
    (26, 70, 16, 24, "quantized"),  # the largest even sliding instantiation (16 + 15 = 31 columns)
    (19, 45, 18, 9, "textured"),   # even k > 17: sliding kernels (round 5), the exact volume
    (19, 80, 34, 9, "textured"),   # even k beyond the sliding instantiations: exact kernel only
    (12, 70, 33, 20, "textured"),  # beyond the sliding instantiations: exact kernel only
    (24, 48, 5, 16, "constant"),
    (24, 48, 5, 16, "zeros"),
]
IDS = [f"{h}x{w}_k{k}_D{d}_{kind}" for h, w, k, d, kind in CASES]


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_exact_forward_bit_identical(gpu, case, layout):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=11, kind=kind)
    lay, Dl = _layout_args(layout, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    got = gpu_forward(cam, proj, k, layout, D, "exact", gpu)
    assert got.shape == ref.shape
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism}/{ref.size} voxels differ; max |d| {np.abs(got - ref).max()}"


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_fast_forward_within_bound(gpu, case, layout):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=12, kind=kind)
    lay, Dl = _layout_args(layout, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    got = gpu_forward(cam, proj, k, layout, D, "fast", gpu)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= O.fast_tolerance(k)
    truth = O.forward_f64(cam, proj, k, layout=lay, D=Dl)
    # vs the fp64 truth: the reference's own worst-case rounding (k > 17 runs the exact
    # reference arithmetic, whose k^2-long fp32 chain can exceed 1e-5 of the truth)
    assert np.abs(got - truth).max() <= O.cost_error_bound(k)


REM_CASES = [
    # window D = 64 n: D + 1 diagonals, the last one computed by the final chunk's waves
    (24, 100, 5, 64, torch.float32),
    (20, 200, 9, 128, torch.float32),
    (18, 300, 11, 256, torch.float16),
    (19, 90, 15, 64, torch.float32),
    (22, 150, 6, 64, torch.float32),    # even k
    (17, 300, 16, 256, torch.float16),
]


@pytest.mark.parametrize("case", REM_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}" for c in REM_CASES])
def test_fast_forward_window_remainder_diagonal(gpu, case):
    H, W, k, D, dt = case
    cam, proj = make_pair(H, W, D, seed=21)
    if dt == torch.float16:
        cam = cam.astype(np.float16).astype(np.float32)
        proj = proj.astype(np.float16).astype(np.float32)
    ref = O.forward(cam, proj, k, layout=O.WINDOW, D=D, contract=1)
    got = gpu_forward(cam, proj, k, WIN, D, "fast", gpu, dtype=dt)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= O.fast_tolerance(k)


@pytest.mark.parametrize("lds_form", ["0", "1"])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_fast_forward_both_kernel_forms(gpu, monkeypatch, lds_form, layout):
    # CUSTMA_FWD_LDS selects the forward kernel form (LDS-loader or wave-independent sweep)
    monkeypatch.setenv("CUSTMA_FWD_LDS", lds_form)
    H, W, k, D = 40, 150, 9, 64
    cam, proj = make_pair(H, W, D, seed=22)
    lay, Dl = _layout_args(layout, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    got = gpu_forward(cam, proj, k, layout, D, "fast", gpu)
    assert np.abs(got - ref).max() <= O.fast_tolerance(k)


@pytest.mark.parametrize("precision", ["exact", "fast"])
def test_fp16_inputs(gpu, precision):
    H, W, k, D = 32, 64, 9, 20
    cam, proj = make_pair(H, W, D, seed=5)
    ch = cam.astype(np.float16).astype(np.float32)
    ph = proj.astype(np.float16).astype(np.float32)
    for layout in (FULL, WIN):
        lay, Dl = _layout_args(layout, D)
        ref = O.forward(ch, ph, k, layout=lay, D=Dl)
        got = gpu_forward(cam, proj, k, layout, D, precision, gpu, dtype=torch.float16)
        if precision == "exact":
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        else:
            assert np.abs(got - ref).max() <= O.fast_tolerance(k)


def test_volume_argmax_bit_identical(gpu):
    rng = np.random.default_rng(0)
    vol = rng.integers(0, 7, size=(13, 29, 301)).astype(np.float32)  # many ties
    vol[3, 4, :] = -np.inf
    vol[5, 6, 17] = np.nan
    idx, best = cm.volume_argmax(_dev(vol, gpu))
    ridx = torch.from_numpy(vol).argmax(-1)
    assert np.array_equal(idx.cpu().numpy(), ridx.numpy())
    v2 = rng.standard_normal((7, 1000)).astype(np.float32)
    i2, b2 = cm.volume_argmax(_dev(v2, gpu))
    oi, ob = O.argmax(v2)
    assert np.array_equal(i2.cpu().numpy(), oi) and np.array_equal(b2.cpu().numpy(), ob)


DISP_CASES = [
    (48, 96, 5, 24, "textured"),
    (40, 80, 9, 30, "quantized"),
    (30, 64, 11, 16, "smooth"),
    (24, 48, 5, 16, "constant"),
    (24, 48, 5, 16, "zeros"),
    (20, 40, 19, 12, "textured"),  # odd k > 17 on the sliding kernels
    (20, 40, 33, 12, "textured"),  # no sweep instance: every pixel decided exactly
    (24, 64, 17, 20, "textured"),  # the largest sweep instance
    (20, 40, 4, 12, "textured"),   # even k (sliding kernels)
    (22, 70, 16, 20, "quantized"),
    (20, 40, 18, 12, "textured"),  # even k > 17 on the sliding kernels
    (20, 80, 34, 12, "textured"),  # even k beyond the sliding instantiations: decided exactly
]


@pytest.mark.parametrize("case", DISP_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_{c[4]}" for c in DISP_CASES])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_disparity_certified_bit_identical(gpu, case, layout):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, D, seed=21, kind=kind)
    lay, Dl = _layout_args(layout, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    ridx, rbest = O.argmax(ref)
    idx, best, nre = cm.stereo_disparity(_dev(cam, gpu), _dev(proj, gpu), D, k, layout, return_rechecked=True)
    idx, best = idx.cpu().numpy(), best.cpu().numpy()
    assert np.array_equal(idx, ridx), f"{np.count_nonzero(idx != ridx)} pixels differ"
    assert np.array_equal(best.view(np.uint32), rbest.view(np.uint32))
    if kind in ("constant", "zeros"):
        assert int(nre.item()) > 0  # ties everywhere: the exact re-decision ran


DISP_TILE_CASES = [
    # window layout, fused disparity through the tile kernel: 1, 2 (+remainder), 3 and 4 (+remainder)
    # diagonal chunks per workgroup
    (18, 150, 5, 90, "textured"),
    (24, 300, 9, 128, "quantized"),
    (20, 200, 7, 150, "smooth"),
    (20, 320, 11, 256, "textured"),
]


@pytest.mark.parametrize("case", DISP_TILE_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}" for c in DISP_TILE_CASES])
def test_disparity_window_tile(gpu, case):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, D, seed=23, kind=kind)
    ref = O.forward(cam, proj, k, layout=O.WINDOW, D=D, contract=1)
    ridx, rbest = O.argmax(ref)
    idx, best = cm.stereo_disparity(_dev(cam, gpu), _dev(proj, gpu), D, k, WIN)
    idx, best = idx.cpu().numpy(), best.cpu().numpy()
    assert np.array_equal(idx, ridx), f"{np.count_nonzero(idx != ridx)} pixels differ"
    assert np.array_equal(best.view(np.uint32), rbest.view(np.uint32))


def _rand_grad(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


BWD_CASES = [
    (16, 24, 5, 8, "textured"),
    (24, 48, 9, 16, "textured"),
    (20, 40, 7, 12, "smooth"),
    (24, 48, 5, 16, "quantized"),
    (1, 32, 5, 8, "textured"),
    (40, 12, 11, 4, "textured"),
    (22, 50, 15, 30, "textured"),
    (24, 48, 3, 0, "textured"),
    (24, 48, 5, 16, "constant"),
    # many steps per segment: several flush blocks of the backward's load pipeline
    (36, 200, 11, 60, "textured"),
    (34, 260, 9, 100, "smooth"),
    # window D = 64 n: the last diagonal goes through the remainder kernels (k_bwd_rem_*)
    (20, 100, 5, 64, "textured"),
    (18, 300, 11, 256, "smooth"),
    (16, 140, 15, 128, "quantized"),
    # k = 17: one workgroup per CU (92 KB of LDS)
    (26, 80, 17, 20, "textured"),
    (20, 140, 17, 64, "smooth"),
    # even k on the fused sweep: rows / columns y - k/2 + 1 .. y + k/2 of the gradient feed pixel y
    (18, 36, 4, 10, "textured"),
    (15, 30, 6, 8, "quantized"),
    (1, 20, 2, 5, "textured"),
    (24, 90, 16, 30, "smooth"),
    (22, 120, 8, 64, "textured"),  # even k with D = 64 n: the last diagonal as a fifth chunk of sweeps
    (30, 200, 10, 70, "textured"),
    # odd k > 17 on the fused sweep (up to 8 halo rows per wave, one workgroup per CU)
    (20, 44, 19, 9, "textured"),
    (16, 40, 25, 12, "smooth"),
    (20, 80, 31, 20, "textured"),
    (18, 100, 21, 64, "quantized"),  # with D = 64 n: the remainder kernel at k = 21
    # even k > 17 on the fused sweep (round 5)
    (17, 40, 18, 10, "textured"),
    (20, 64, 30, 12, "smooth"),
    # generic fp64 backward (no fused instantiation): k > 31
    (17, 80, 34, 10, "textured"),
    (16, 44, 33, 10, "smooth"),
]


@pytest.mark.parametrize("case", BWD_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}_{c[4]}" for c in BWD_CASES])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_backward_both_images(gpu, case, layout):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    lay, Dl = _layout_args(layout, D)
    shape = O.volume_shape(H, W, lay, Dl)
    g = _rand_grad(shape, 7)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
    gc, gp = cm.cost_volume_backward(_dev(g, gpu), _dev(cam, gpu), _dev(proj, gpu), k, layout, D,
                                     camera_grad=True, projector_grad=True)
    gc, gp = gc.cpu().numpy(), gp.cpu().numpy()
    tol_c = 1e-5 * max(1.0, np.abs(rc).max())
    tol_p = 1e-5 * max(1.0, np.abs(rp).max())
    assert np.abs(gc - rc).max() <= tol_c, np.abs(gc - rc).max() / max(1.0, np.abs(rc).max())
    assert np.abs(gp - rp).max() <= tol_p, np.abs(gp - rp).max() / max(1.0, np.abs(rp).max())


@pytest.mark.parametrize("case", [(18, 36, 4, 10, "textured"), (15, 30, 6, 8, "quantized"), (22, 120, 8, 64, "textured")],
                         ids=["18x36_k4", "15x30_k6", "22x120_k8_D64"])
def test_backward_even_k_window_repeated(gpu, case):
    """The round-4 suite failed once on the window k = 4 backward (camera gradient 2.1e-4 relative) and the
    failure did not reproduce at round-5 HEAD: the even-k window backward, recompute path, 20 times on the
    same inputs -- every call bit-identical and within the bar (an intermittent race would show here)."""
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    g = _rand_grad(O.volume_shape(H, W, O.WINDOW, D), 7)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
    c, p, gd = _dev(cam, gpu), _dev(proj, gpu), _dev(g, gpu)
    first = None
    for _ in range(20):
        gc, gp = cm.cost_volume_backward(gd, c, p, k, WIN, D, camera_grad=True, projector_grad=True)
        if first is None:
            first = (gc, gp)
            assert np.abs(gc.cpu().numpy() - rc).max() <= 1e-5 * max(1.0, np.abs(rc).max())
            assert np.abs(gp.cpu().numpy() - rp).max() <= 1e-5 * max(1.0, np.abs(rp).max())
        else:
            assert torch.equal(gc, first[0]) and torch.equal(gp, first[1])


_COLD = {}


def _cold_caches(gpu):
    """A large exact forward (256 x 2048 fp16, k = 19, D = 256: 0.47 GB written) between the calls: the next
    kernel starts with cold TLB and caches, and its waves inherit registers and LDS the exact kernel left --
    the state in which the round-4/5 window k = 4 backward read registers whose loads were still in flight
    (DESIGN.md §3.6)."""
    if "pair" not in _COLD:
        from bench import synth_pair
        _COLD["pair"] = synth_pair(256, 2048, 256, 5, str(gpu), torch.float16)
    c3, p3 = _COLD["pair"]
    v = cm.cost_volume_forward(c3, p3, 256, 19, WIN, "exact")
    torch.cuda.synchronize()
    del v


@pytest.mark.parametrize("k", [2, 3, 4, 5, 6, 11])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_ops_after_a_large_kernel(gpu, k, layout):
    """Every op right after a large kernel (cold caches, foreign register / LDS contents) equals the same op
    run warm, bit for bit: forward, backward with and without the volume, disparity."""
    H, W, D = 18, 36, 10
    cam, proj = make_pair(H, W, D, seed=31, kind="textured")
    lay, Dl = _layout_args(layout, D)
    g = _rand_grad(O.volume_shape(H, W, lay, Dl), 7)
    c, p, gd = _dev(cam, gpu), _dev(proj, gpu), _dev(g, gpu)
    def tensors(x):
        return [x] if torch.is_tensor(x) else [y for y in x if torch.is_tensor(y)]

    ops = {
        "forward": lambda: cm.cost_volume_forward(c, p, Dl, k, layout, "fast"),
        "backward(volume)": lambda: cm.cost_volume_backward(gd, c, p, k, layout, Dl, camera_grad=True,
                                                            projector_grad=True, cost_volume=warm_vol),
        "backward(recompute)": lambda: cm.cost_volume_backward(gd, c, p, k, layout, Dl, camera_grad=True,
                                                               projector_grad=True),
    }
    if layout == WIN:
        ops["disparity"] = lambda: cm.stereo_disparity(c, p, Dl, k, layout)
    warm_vol = cm.cost_volume_forward(c, p, Dl, k, layout, "fast")
    for name, op in ops.items():
        op()
        ref = [x.clone() for x in tensors(op())]
        _cold_caches(gpu)
        got = tensors(op())
        assert len(got) == len(ref) > 0
        for a, b in zip(got, ref):
            assert torch.equal(a, b), f"{name}: differs after a large kernel"


# every hand-counted store pattern of the window tile kernel (sweep_wave.hip wave_body's ST): one chunk
# (4 scan passes), one chunk + the remainder diagonal (REM), two chunks (2 passes), four chunks + REM
# (1 pass), fp32 (dword stores when the block base is unaligned) and fp16 (camera preload)
TILE_VARIANTS = [(64, torch.float32), (100, torch.float32), (256, torch.float32), (256, torch.float16),
                 (10, torch.float16)]


@pytest.mark.parametrize("D,dtype", TILE_VARIANTS, ids=[f"D{d}_{str(t)[6:]}" for d, t in TILE_VARIANTS])
@pytest.mark.parametrize("k", [5, 11])
def test_tile_variants_after_a_large_kernel(gpu, k, D, dtype):
    """The tile kernel's volume, argmax and soft-argmax variants right after a large kernel equal the same
    call run warm, bit for bit (each variant's vmcnt waits count its own stores)."""
    H, W = 18, D + 40
    cam, proj = make_pair(H, W, D, seed=31, kind="textured")
    c, p = _dev(cam, gpu).to(dtype), _dev(proj, gpu).to(dtype)
    ops = {
        "forward": lambda: [cm.cost_volume_forward(c, p, D, k, WIN, "fast")],
        "disparity": lambda: list(cm.stereo_disparity(c, p, D, k, WIN)),
        "soft": lambda: [x for x in cm.stereo_disparity_soft(c, p, D, k, WIN) if torch.is_tensor(x)],
    }
    for name, op in ops.items():
        op()
        ref = [x.clone() for x in op()]
        _cold_caches(gpu)
        got = op()
        assert len(got) == len(ref) > 0
        for a, b in zip(got, ref):
            assert torch.equal(a, b), f"{name}: differs after a large kernel"


@pytest.mark.parametrize("case", BWD_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}_{c[4]}" for c in BWD_CASES])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_backward_given_volume(gpu, case, layout):
    """The backward handed the forward's volume (the autograd path) against the fp64 oracle, and equal to
    the recompute path (cost_volume=None: the volume rebuilt in the workspace, as the forward builds it --
    the fast sweep up to k = 11, the exact kernel above) bit for bit."""
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    lay, Dl = _layout_args(layout, D)
    g = _rand_grad(O.volume_shape(H, W, lay, Dl), 7)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
    c, p, gd = _dev(cam, gpu), _dev(proj, gpu), _dev(g, gpu)
    vol = cm.cost_volume_forward(c, p, D, k, layout, "fast")
    gc, gp = cm.cost_volume_backward(gd, c, p, k, layout, D, camera_grad=True, projector_grad=True, cost_volume=vol)
    gc2, gp2 = cm.cost_volume_backward(gd, c, p, k, layout, D, camera_grad=True, projector_grad=True)
    gc, gp = gc.cpu().numpy(), gp.cpu().numpy()
    assert np.abs(gc - rc).max() <= 1e-5 * max(1.0, np.abs(rc).max())
    assert np.abs(gp - rp).max() <= 1e-5 * max(1.0, np.abs(rp).max())
    assert np.array_equal(gc, gc2.cpu().numpy()) and np.array_equal(gp, gp2.cpu().numpy())


@pytest.mark.parametrize("case", [(20, 44, 33, 9, "textured"), (18, 80, 34, 10, "smooth")], ids=["k33", "k34"])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_backward_generic_small_bands(gpu, case, layout, monkeypatch):
    """The generic fp64 backward's band loop (A / VA / BA recomputed per band of output rows, halo
    included) with 3-row bands gives the same gradients as the oracle."""
    monkeypatch.setenv("CUSTMA_GEN_BAND_ROWS", "3")
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=33, kind=kind)
    lay, Dl = _layout_args(layout, D)
    g = _rand_grad(O.volume_shape(H, W, lay, Dl), 8)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
    gc, gp = cm.cost_volume_backward(_dev(g, gpu), _dev(cam, gpu), _dev(proj, gpu), k, layout, D,
                                     camera_grad=True, projector_grad=True)
    assert np.abs(gc.cpu().numpy() - rc).max() <= 1e-5 * max(1.0, np.abs(rc).max())
    assert np.abs(gp.cpu().numpy() - rp).max() <= 1e-5 * max(1.0, np.abs(rp).max())


def test_backward_ones_matches_reference_golden(gpu):
    """g = ones, exactly what examples/verify.py:68,123 backpropagates."""
    import glob
    import os

    for p in sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*_k*.npz"))):
        z = np.load(p)
        if "vol32" not in z:
            continue
        cam, proj, k = z["cam"], z["proj"], int(z["k"])
        H, W = cam.shape
        g = torch.ones(H, W, W, device=gpu)
        gc, gp = cm.cost_volume_backward(g, _dev(cam, gpu), _dev(proj, gpu), k, camera_grad=True,
                                         projector_grad=True)
        mc = max(1.0, np.abs(z["cg64"]).max())
        mp = max(1.0, np.abs(z["pg64"]).max())
        assert np.abs(gc.cpu().numpy() - z["cg64"]).max() <= 1e-5 * mc, p
        assert np.abs(gp.cpu().numpy() - z["pg64"]).max() <= 1e-5 * mp, p


def test_backward_deterministic(gpu):
    cam, proj = make_pair(32, 64, 16, seed=2)
    g = _dev(_rand_grad((32, 64, 64), 3), gpu)
    a = cm.cost_volume_backward(g, _dev(cam, gpu), _dev(proj, gpu), 9, projector_grad=True)
    b = cm.cost_volume_backward(g, _dev(cam, gpu), _dev(proj, gpu), 9, projector_grad=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_autograd_drop_in(gpu):
    import custma

    cam, proj = make_pair(20, 40, 10, seed=4)
    c = _dev(cam, gpu).requires_grad_(True)
    p = _dev(proj, gpu)
    vol = custma.stereo_matching(c.contiguous(), p.contiguous(), 200, 5)  # verify.py:66 call shape
    assert vol.shape == (20, 40, 40) and vol.requires_grad
    vol.backward(torch.ones_like(vol))  # verify.py:68
    rc, _ = O.backward_f64(np.ones((20, 40, 40), np.float32), cam, proj, 5)
    assert np.abs(c.grad.cpu().numpy() - rc).max() <= 1e-5 * max(1, np.abs(rc).max())
    assert p.grad is None
    # superset: projector gradient on request, and .sum().backward() (stride-0 grad)
    c2 = _dev(cam, gpu).requires_grad_(True)
    p2 = _dev(proj, gpu).requires_grad_(True)
    custma.stereo_matching(c2, p2, 0, 5).sum().backward()
    _, rp = O.backward_f64(np.ones((20, 40, 40), np.float32), cam, proj, 5)
    assert np.abs(p2.grad.cpu().numpy() - rp).max() <= 1e-5 * max(1, np.abs(rp).max())
    # reference extension surface
    v = custma.src.stereo_matching_forward(c.detach(), p, 0, 5)
    gcam = custma.src.stereo_matching_backward(torch.ones_like(v), c.detach(), p, 5)
    assert torch.allclose(gcam, c.grad, rtol=0, atol=1e-6 * float(c.grad.abs().max()))


def test_errors_on_device(gpu):
    c = torch.rand(8, 16, device=gpu)
    with pytest.raises(RuntimeError, match="must be contiguous"):
        cm.stereo_matching(c.t(), c.t(), 0, 5)
    with pytest.raises(RuntimeError, match="expected scalar type Float but found Double"):
        cm.stereo_matching(c.double(), c.double(), 0, 5)
    with pytest.raises(ValueError, match="kernel_size"):
        cm.stereo_matching(c, c, 0, 0)
    with pytest.raises(ValueError, match="kernel_size"):
        cm.stereo_matching(c, c, 0, 65)
    with pytest.raises(ValueError):
        cm.stereo_matching(c, c, 16, 5, layout="window")
    e = torch.empty(0, 16, device=gpu)
    assert cm.stereo_matching(e, e, 0, 5).shape == (0, 16, 16)


# ---- larger sizes: property checks the oracle cannot afford whole ----

def _band_oracle_forward(cam, proj, k, h0, h1, layout, D):
    r = k // 2
    a0, a1 = max(0, h0 - r), min(cam.shape[0], h1 + r)
    lay, Dl = _layout_args(layout, D)
    v = O.forward(cam[a0:a1], proj[a0:a1], k, layout=lay, D=Dl)
    return v[h0 - a0:h1 - a0]


@pytest.mark.parametrize("layout,D", [(FULL, 0), (WIN, 128)])
def test_large_1024_rows_vs_oracle_bands(gpu, layout, D):
    H, W, k = 1024, 1024, 9
    cam, proj = make_pair(H, W, 128, seed=8)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    ex = cm.cost_volume_forward(c, p, D, k, layout, "exact")
    fa = cm.cost_volume_forward(c, p, D, k, layout, "fast")
    assert float((ex - fa).abs().max()) <= O.fast_tolerance(k)
    for h0 in (0, 511, 1016):
        ref = _band_oracle_forward(cam, proj, k, h0, h0 + 8, layout, D)
        got = ex[h0:h0 + 8].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    idx, best = cm.stereo_disparity(c, p, D, k, layout)
    vi, vb = cm.volume_argmax(ex)
    assert torch.equal(idx, vi)
    assert torch.equal(best, vb)


def test_large_backward_band_vs_oracle(gpu):
    H, W, k = 256, 512, 9
    r = k // 2
    cam, proj = make_pair(H, W, 64, seed=9)
    g = _rand_grad((H, W, W), 10)
    gc, gp = cm.cost_volume_backward(_dev(g, gpu), _dev(cam, gpu), _dev(proj, gpu), k, projector_grad=True)
    h0, h1 = 120, 126
    a0, a1 = h0 - 2 * r, h1 + 2 * r
    rc, rp = O.backward_f64(g[a0:a1], cam[a0:a1], proj[a0:a1], k)
    rc, rp = rc[h0 - a0:h1 - a0], rp[h0 - a0:h1 - a0]
    assert np.abs(gc[h0:h1].cpu().numpy() - rc).max() <= 1e-5 * max(1, np.abs(rc).max())
    assert np.abs(gp[h0:h1].cpu().numpy() - rp).max() <= 1e-5 * max(1, np.abs(rp).max())


@pytest.mark.parametrize("layout,D", [(FULL, 0), (WIN, 12)])
def test_band_api_matches_whole_image(gpu, layout, D):
    """custma_*_band: volume rows [b, e) of a haloed buffer equal the whole-image
    volume's rows; band gradients + halo partials add up to the whole-image gradient."""
    H, W, k = 40, 48, 7
    r = k // 2
    cam, proj = make_pair(H, W, 16, seed=44)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    full = cm.cost_volume_forward(c, p, D, k, layout, "exact")
    g = _dev(_rand_grad(tuple(full.shape), 45), gpu)
    rc, rp = cm.cost_volume_backward(g, c, p, k, layout, D, projector_grad=True)
    # two bands: rows [0, 17) and [17, 40), buffers with r halo rows
    acc_c = torch.zeros_like(rc)
    acc_p = torch.zeros_like(rp)
    for b, e in ((0, 17), (17, 40)):
        a0, a1 = max(0, b - r), min(H, e + r)
        vb = cm.cost_volume_forward(c[a0:a1].contiguous(), p[a0:a1].contiguous(), D, k, layout, "exact",
                                    rows=(b - a0, e - a0))
        assert torch.equal(vb, full[b:e])
        fb = cm.cost_volume_forward(c[a0:a1].contiguous(), p[a0:a1].contiguous(), D, k, layout, "fast",
                                    rows=(b - a0, e - a0))
        assert float((fb - full[b:e]).abs().max()) <= O.fast_tolerance(k)
        gc, gp = cm.cost_volume_backward(g[b:e].contiguous(), c[a0:a1].contiguous(), p[a0:a1].contiguous(), k,
                                         layout, D, projector_grad=True, rows=(b - a0, e - a0))
        acc_c[a0:a1] += gc
        acc_p[a0:a1] += gp
        ib, bb = cm.stereo_disparity(c[a0:a1].contiguous(), p[a0:a1].contiguous(), D, k, layout,
                                     rows=(b - a0, e - a0))
        vi, vb2 = cm.volume_argmax(full[b:e].contiguous())
        assert torch.equal(ib, vi) and torch.equal(bb, vb2)
    assert float((acc_c - rc).abs().max()) <= 1e-5 * max(1.0, float(rc.abs().max()))
    assert float((acc_p - rp).abs().max()) <= 1e-5 * max(1.0, float(rp.abs().max()))


@pytest.mark.parametrize("layout,D", [(FULL, 0), (WIN, 12)])
@pytest.mark.parametrize("k", [7, 6, 11])
def test_band_forward_reads_only_its_patch_rows(gpu, monkeypatch, layout, D, k):
    """Volume rows [b, e) of a band depend only on image rows [b - k/2, e + k-1-k/2) and on the
    statistics of rows [b, e): with every other image row NaN and the workspace filled with NaN,
    the band's forward (fast and exact) and disparity equal the whole-image results.  This is what
    lets the row-band forward compute its interior rows while the halo rows are still in flight."""
    import custereomatching_amd.stereo_matching_wrapper as smw
    import custereomatching_amd.disparity as disp

    H, W = 48, 64
    o, a = k // 2, k - 1 - k // 2
    cam, proj = make_pair(H, W, 16, seed=46)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    ref = {pr: cm.cost_volume_forward(c, p, D, k, layout, pr) for pr in ("fast", "exact")}
    ri, rb = cm.stereo_disparity(c, p, D, k, layout)
    nan_ws = lambda nb, dev: torch.full((max(nb, 1) // 4 + 1,), float("nan"), device=dev).view(torch.uint8)
    monkeypatch.setattr(smw, "_workspace", nan_ws)
    if hasattr(disp, "_workspace"):
        monkeypatch.setattr(disp, "_workspace", nan_ws)
    for b, e in ((0, 9), (13, 30), (40, 48)):
        cn, pn = c.clone(), p.clone()
        lo, hi = max(0, b - o), min(H, e + a)
        for x in (cn, pn):
            x[:lo] = float("nan")
            x[hi:] = float("nan")
        for pr in ("fast", "exact"):
            vb = cm.cost_volume_forward(cn, pn, D, k, layout, pr, rows=(b, e))
            assert torch.equal(vb, ref[pr][b:e]), (pr, b, e)
        ib, bb = cm.stereo_disparity(cn, pn, D, k, layout, rows=(b, e))
        assert torch.equal(ib, ri[b:e]) and torch.equal(bb, rb[b:e])


@pytest.mark.parametrize("layout,D", [(FULL, 0), (WIN, 20)])
def test_backward_given_volume_matches_recompute(gpu, layout, D):
    """The autograd op hands the forward's volume to the backward (V = g * cost / S); the
    recompute path (no volume, the reference's backward signature) must agree with it."""
    H, W, k = 37, 90, 11
    cam, proj = make_pair(H, W, max(D, 1), seed=61, kind="smooth")
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    vol = cm.cost_volume_forward(c, p, D, k, layout, "fast")
    g = _dev(_rand_grad(tuple(vol.shape), 62), gpu)
    a = cm.cost_volume_backward(g, c, p, k, layout, D, projector_grad=True, cost_volume=vol)
    b = cm.cost_volume_backward(g, c, p, k, layout, D, projector_grad=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    lay, Dl = _layout_args(layout, D)
    rc, rp = O.backward_f64(g.cpu().numpy(), cam, proj, k, layout=lay, D=Dl)
    assert np.abs(a[0].cpu().numpy() - rc).max() <= 1e-5 * max(1, np.abs(rc).max())
    assert np.abs(a[1].cpu().numpy() - rp).max() <= 1e-5 * max(1, np.abs(rp).max())


def test_backward_wide_full_layout_many_chunks(gpu):
    """Full layout with W = 300: 10 diagonal chunks of 64, several partial slots per column,
    and row groups that straddle the volume edge."""
    H, W, k = 45, 300, 9
    cam, proj = make_pair(H, W, 40, seed=71)
    g = _rand_grad((H, W, W), 72)
    rc, rp = O.backward_f64(g, cam, proj, k)
    gc, gp = cm.cost_volume_backward(_dev(g, gpu), _dev(cam, gpu), _dev(proj, gpu), k, projector_grad=True)
    assert np.abs(gc.cpu().numpy() - rc).max() <= 1e-5 * max(1, np.abs(rc).max())
    assert np.abs(gp.cpu().numpy() - rp).max() <= 1e-5 * max(1, np.abs(rp).max())


def _soft_argmax_ref(vol, beta):
    """examples/verify.py:31-39 restated in float64 on the oracle's exact volume."""
    x = torch.from_numpy(vol).double()
    p = torch.softmax(x * beta, dim=-1)
    return (p * torch.arange(x.shape[-1], dtype=torch.float64)).sum(-1).numpy(), p.numpy()


SOFT_CASES = [
    (24, 96, 5, 24, "full"), (24, 96, 9, 40, "window"), (20, 320, 11, 256, "window"),  # tile kernel
    (18, 200, 7, 150, "window"), (20, 40, 19, 12, "full"), (16, 48, 4, 10, "window"),  # exact-decided
    (24, 48, 5, 16, "full"),
]


@pytest.mark.parametrize("case", SOFT_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}_{c[4]}" for c in SOFT_CASES])
@pytest.mark.parametrize("kind", ["textured", "constant"])
def test_disparity_soft_argmax_and_mask(gpu, case, kind):
    """Fused soft-argmax (beta = 50) and max-cost mask (threshold 0.6), examples/verify.py:31-39, 72-74,
    without the volume.  Index / best / mask bit-identical to the exact volume's; soft within the
    first-order propagation of the fast path's cost error eps: |d soft| <= 2 beta eps E_w|s - soft|
    (+ fp32 rounding of the sums, 1e-5 relative)."""
    H, W, k, D, layout = case
    beta, thr = 50.0, 0.6
    cam, proj = make_pair(H, W, D, seed=81, kind=kind)
    lay, Dl = _layout_args(layout, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl)
    ridx, rbest = O.argmax(ref)
    rsoft, pw = _soft_argmax_ref(ref, beta)
    idx, best, soft, mask = cm.stereo_disparity_soft(_dev(cam, gpu), _dev(proj, gpu), D, k, layout, beta, thr)
    idx, best, soft, mask = (t.cpu().numpy() for t in (idx, best, soft, mask))
    assert np.array_equal(idx, ridx)
    assert np.array_equal(best.view(np.uint32), rbest.view(np.uint32))
    assert np.array_equal(mask, (rbest > thr).astype(np.float32))
    s = np.arange(ref.shape[-1], dtype=np.float64)
    spread = (pw * np.abs(s - rsoft[..., None])).sum(-1)
    tol = 2.0 * beta * O.fast_tolerance(k) * spread + 1e-5 * np.maximum(1.0, rsoft)
    err = np.abs(soft - rsoft)
    assert np.all(err <= tol), float((err / tol).max())
    # the caller pipeline (examples/test.py:78-86) from the fused pass
    dmap, dsoft, m2 = cm.disparity_maps(_dev(cam, gpu), _dev(proj, gpu), D, k, layout, beta, thr)
    w = np.arange(ref.shape[1], dtype=np.float32)
    want = ((-ridx if layout == "window" else w - ridx) * (rbest > thr)).astype(np.float32)
    assert np.array_equal(dmap.cpu().numpy(), want)


# ---- workspace contents: no op may read a workspace byte it did not write.  The round-4 and round-5 window
# k = 4 backward failures (camera gradient 2.1e-4 relative, the same value twice) came and went with the test
# order, i.e. with what the caching allocator's reused workspace held; here the C ABI is called directly with
# workspaces pre-filled with different byte patterns, and every output must equal the zero-filled run's ----

WS_CASES = [(18, 36, 4, 10, "textured"), (15, 30, 6, 8, "quantized"), (24, 48, 5, 16, "textured"),
            (22, 120, 8, 64, "textured"), (20, 100, 5, 64, "textured"), (17, 40, 18, 10, "textured")]


def _filled_ws(nbytes, fill, gpu):
    ws = torch.empty(nbytes + 256, dtype=torch.uint8, device=gpu)
    ws = ws[(-ws.data_ptr()) % 256:][:nbytes]
    if fill == "rand":
        ws.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=gpu,
                               generator=torch.Generator(device=gpu).manual_seed(5)))
    else:
        ws.fill_(fill)
    return ws


@pytest.mark.parametrize("case", WS_CASES, ids=[f"{c[0]}x{c[1]}_k{c[2]}_D{c[3]}" for c in WS_CASES])
@pytest.mark.parametrize("layout", [FULL, WIN])
def test_outputs_independent_of_workspace_contents(gpu, case, layout):
    from custereomatching_amd import _lib

    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    lay = _lib.LAYOUT_WINDOW if layout == WIN else _lib.LAYOUT_FULL
    Dl = D if layout == WIN else 0
    WO, DO = _lib.volume_dims(H, W, lay, Dl)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    gd = _dev(_rand_grad((H, WO, DO), 7), gpu)
    st = torch.cuda.current_stream(gpu).cuda_stream

    def fwd(fill):
        nb = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_FORWARD)
        ws, out = _filled_ws(nb, fill, gpu), torch.empty((H, WO, DO), device=gpu)
        _lib.check(_lib.lib.custma_forward_band(c.data_ptr(), p.data_ptr(), _lib.F32, H, W, k, lay, Dl, _lib.FAST, 0,
                                                H, out.data_ptr(), ws.data_ptr(), nb, st), "fwd")
        return out

    def bwd(fill, vol):
        nb = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_BACKWARD if vol is not None else _lib.OP_BACKWARD_RECOMPUTE)
        ws = _filled_ws(nb, fill, gpu)
        gc, gp = torch.empty((H, W), device=gpu), torch.empty((H, W), device=gpu)
        _lib.check(_lib.lib.custma_backward_band(gd.data_ptr(), vol.data_ptr() if vol is not None else None,
                                                 c.data_ptr(), p.data_ptr(), _lib.F32, H, W, k, lay, Dl, 0, H,
                                                 gc.data_ptr(), gp.data_ptr(), ws.data_ptr(), nb, st), "bwd")
        return gc, gp

    v0 = fwd(0)
    r_given, r_rec = bwd(0, v0), bwd(0, None)
    for fill in (0xFF, 0x7F, "rand"):
        assert torch.equal(fwd(fill), v0), ("forward", fill)
        for name, got, ref in (("given", bwd(fill, v0), r_given), ("recompute", bwd(fill, None), r_rec)):
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), (name, fill)
    assert torch.equal(r_given[0], r_rec[0]) and torch.equal(r_given[1], r_rec[1])
