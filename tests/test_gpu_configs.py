"""GPU parity at the BASELINE.json configs' own sizes (configs[0] .. configs[4]).

Small configs are checked whole against the reference-derived goldens or the
oracle; large ones through oracle row bands (output row h reads image rows
h-r .. h+r only, stereo_matching_kernel.cu:44,60, so an oracle run on a haloed
band is exact for the band's rows) plus size-independent properties on the
whole volume (fast vs exact within the 1e-5 contract, fused disparity ==
argmax of the exact volume).  Tolerances (north_star): costs within
min(1e-5, (k^2+6) 2^-24) (oracle.fast_tolerance), indices bit-exact, gradients
within 1e-5 * max(1, max|g_ref|) of the fp64 oracle.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.golden.inputs import make_pair
from tests.oracle_tiles import tile_backward as _tile_backward

import custereomatching_amd as cm

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _dev(x, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(dtype)


def _f16(x):
    return x.astype(np.float16).astype(np.float32)


def _rel(got, ref):
    return float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))


def _band_forward(cam, proj, k, h0, h1, layout, D):
    """Oracle (reference arithmetic) for volume rows [h0, h1) from a haloed band."""
    o, a = k // 2, k - 1 - k // 2
    a0, a1 = max(0, h0 - o), min(cam.shape[0], h1 + a)
    lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
    v = O.forward(cam[a0:a1], proj[a0:a1], k, layout=lay, D=Dl)
    return v[h0 - a0:h1 - a0]


def _band_backward(gband, cam, proj, k, h0, h1, layout, D):
    """fp64 oracle gradients for image rows [h0, h1): gband holds volume rows
    [h0 - 2r, h1 + 2r) (clipped); the band's own edge padding only reaches rows outside."""
    r = k // 2
    a0, a1 = max(0, h0 - 2 * r), min(cam.shape[0], h1 + 2 * r)
    lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
    rc, rp = O.backward_f64(gband, cam[a0:a1], proj[a0:a1], k, layout=lay, D=Dl)
    return rc[h0 - a0:h1 - a0], rp[h0 - a0:h1 - a0]


def _max_abs_diff_rows(x, y, chunk=64):
    m = 0.0
    for h in range(0, x.shape[0], chunk):
        m = max(m, float((x[h:h + chunk] - y[h:h + chunk]).abs().max()))
    return m


# ---------------- configs[0]: examples/verify.py, 128x256, D=32, window 5 ----------------

@pytest.mark.parametrize("kind", ["textured", "quantized"])
def test_config0_verify_goldens(gpu, kind):
    """The reference driver's sequence (verify.py:65-74) on the goldens made by the
    reference's own torch path (tests/golden/gen_golden.py)."""
    import custma

    z = np.load(os.path.join(GOLD, f"verify_{kind}_128x256_k5.npz"))
    cam, proj, k, D = z["cam"], z["proj"], int(z["k"]), int(z["D"])
    H, W = cam.shape
    tol = O.fast_tolerance(k)
    c = _dev(cam, gpu).requires_grad_(True)
    p = _dev(proj, gpu).requires_grad_(True)
    vol = custma.stereo_matching(c.contiguous(), p.contiguous(), D, k)  # verify.py:66
    vol.backward(torch.ones_like(vol))  # verify.py:68
    v = vol.detach()
    flat = v.reshape(-1)[torch.from_numpy(z["sample_idx"]).to(gpu)].cpu().numpy()
    assert np.abs(flat - z["sample64"]).max() <= tol
    mx, am = torch.max(v.reshape(H * W, -1), dim=-1)  # verify.py:72
    assert np.abs(mx.cpu().numpy().reshape(H, W) - z["max64"]).max() <= tol
    sure = z["gap64"] > 2 * tol  # outside the float tie band the index is the truth's
    assert np.array_equal(am.cpu().numpy().reshape(H, W)[sure], z["argmax64"][sure].astype(np.int64))
    assert _rel(c.grad.cpu().numpy(), z["cg64"]) <= 1e-5
    assert _rel(p.grad.cpu().numpy(), z["pg64"]) <= 1e-5
    # exact arithmetic: bit-identical to the oracle, and the fused disparity equals its argmax
    ex = cm.cost_volume_forward(c.detach(), p.detach(), D, k, "full", "exact")
    ref = O.forward(cam, proj, k)
    assert np.array_equal(ex.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    idx, best = cm.stereo_disparity(c.detach(), p.detach(), D, k)
    ridx, rbest = O.argmax(ref)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(best.cpu().numpy().view(np.uint32), rbest.view(np.uint32))
    assert np.array_equal(ridx[sure], z["argmax64"][sure].astype(np.int64))
    # mask (verify.py:73-74) from the fused path equals the one from the volume
    assert torch.equal(cm.confidence_mask(best, 0.6), cm.confidence_mask(mx.reshape(H, W), 0.6))


def test_config0_window_layout(gpu):
    H, W, k, D = 128, 256, 5, 32
    cam, proj = make_pair(H, W, D, seed=3)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    ref = O.forward(cam, proj, k, layout=O.WINDOW, D=D)
    ex = cm.cost_volume_forward(c, p, D, k, "window", "exact").cpu().numpy()
    fa = cm.cost_volume_forward(c, p, D, k, "window", "fast").cpu().numpy()
    assert np.array_equal(ex.view(np.uint32), ref.view(np.uint32))
    assert np.abs(fa - ref).max() <= O.fast_tolerance(k)
    g = np.random.default_rng(4).standard_normal(ref.shape).astype(np.float32)
    gc, gp = cm.cost_volume_backward(_dev(g, gpu), c, p, k, "window", D, projector_grad=True)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
    assert _rel(gc.cpu().numpy(), rc) <= 1e-5 and _rel(gp.cpu().numpy(), rp) <= 1e-5


# ---------------- configs[2]: 1024x1024 fp32, D=128, k=9, forward + backward (both images) ----------------

@pytest.mark.parametrize("layout,D", [("full", 0), ("window", 128)])
def test_config2_forward_backward_full_size(gpu, layout, D):
    H, W, k = 1024, 1024, 9
    r = k // 2
    cam, proj = make_pair(H, W, 128, seed=81)
    c = _dev(cam, gpu).requires_grad_(True)
    p = _dev(proj, gpu).requires_grad_(True)
    vol = cm.stereo_matching(c, p, D, k, layout)
    gen = torch.Generator(device=gpu).manual_seed(82)
    g = torch.randn(vol.shape, generator=gen, device=gpu)
    vol.backward(g)
    for h0 in (0, 509, 1018):
        h1 = min(H, h0 + 6)
        ref = _band_forward(cam, proj, k, h0, h1, layout, D)
        assert np.abs(vol[h0:h1].detach().cpu().numpy() - ref).max() <= O.fast_tolerance(k)
        a0, a1 = max(0, h0 - 2 * r), min(H, h1 + 2 * r)
        rc, rp = _band_backward(g[a0:a1].cpu().numpy(), cam, proj, k, h0, h1, layout, D)
        assert _rel(c.grad[h0:h1].cpu().numpy(), rc) <= 1e-5
        assert _rel(p.grad[h0:h1].cpu().numpy(), rp) <= 1e-5


# ---------------- k > 17 (generic fp64 backward) and even k (fused sweep) at a mid size ----------------

@pytest.mark.parametrize("layout,D,k", [("window", 64, 34), ("full", 0, 33), ("window", 64, 16), ("full", 0, 12),
                                        ("window", 128, 25), ("window", 64, 18)])
def test_generic_backward_mid_size(gpu, layout, D, k):
    """Mid-size problems: k = 33, 34 through the banded generic backward (grid-stride kernels, bounded
    workspace; the 512 x 512 full layout takes two bands of output rows at the default 2 GiB band
    budget), k = 12, 16, 18, 25 through the fused sweep; checked on haloed oracle bands."""
    H = W = 1024 if layout == "window" else 512
    o = k // 2
    cam, proj = make_pair(H, W, max(D, 1), seed=85)
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    vol = cm.cost_volume_forward(c, p, D, k, layout, "exact")
    gen = torch.Generator(device=gpu).manual_seed(86)
    g = torch.randn(vol.shape, generator=gen, device=gpu)
    gc, gp = cm.cost_volume_backward(g, c, p, k, layout, D, projector_grad=True, cost_volume=vol)
    for h0 in (0, H // 2 + 3, H - 3):
        h1 = min(H, h0 + 3)
        a0, a1 = max(0, h0 - 2 * o), min(H, h1 + 2 * o)
        rc, rp = _band_backward(g[a0:a1].cpu().numpy(), cam, proj, k, h0, h1, layout, D)
        assert _rel(gc[h0:h1].cpu().numpy(), rc) <= 1e-5
        assert _rel(gp[h0:h1].cpu().numpy(), rp) <= 1e-5


# ---------------- configs[3]: 2048x2048 fp16, D=256, k=11, window ----------------

def test_config3_window_fp16(gpu):
    H, W, k, D = 2048, 2048, 11, 256
    cam, proj = make_pair(H, W, D, seed=91)
    c, p = _dev(cam, gpu, torch.float16), _dev(proj, gpu, torch.float16)
    c32, p32 = _f16(cam), _f16(proj)
    ex = cm.cost_volume_forward(c, p, D, k, "window", "exact")
    for h0 in (0, 1021, 2040):
        ref = _band_forward(c32, p32, k, h0, h0 + 8, "window", D)
        assert np.array_equal(ex[h0:h0 + 8].cpu().numpy().view(np.uint32), ref.view(np.uint32))
    fa = cm.cost_volume_forward(c, p, D, k, "window", "fast")
    assert _max_abs_diff_rows(fa, ex) <= O.fast_tolerance(k)
    del fa
    idx, best = cm.stereo_disparity(c, p, D, k, "window")
    vi, vb = cm.volume_argmax(ex)
    assert torch.equal(idx, vi) and torch.equal(best, vb)
    # window backward at full size, checked on a band
    gen = torch.Generator(device=gpu).manual_seed(92)
    g = torch.randn(ex.shape, generator=gen, device=gpu)
    gc, gp = cm.cost_volume_backward(g, c, p, k, "window", D, projector_grad=True, cost_volume=ex)
    r = k // 2
    h0, h1 = 777, 783
    rc, rp = _band_backward(g[h0 - 2 * r:h1 + 2 * r].cpu().numpy(), c32, p32, k, h0, h1, "window", D)
    assert _rel(gc[h0:h1].cpu().numpy(), rc) <= 1e-5
    assert _rel(gp[h0:h1].cpu().numpy(), rp) <= 1e-5


# ---------------- configs[4] on one GPU: 4096x8192 fp16, D=256, k=11, window ----------------

def test_config4_window_fp16_one_gpu(gpu):
    H, W, k, D = 4096, 8192, 11, 256
    cam, proj = make_pair(H, W, D, seed=101)
    c, p = _dev(cam, gpu, torch.float16), _dev(proj, gpu, torch.float16)
    c32, p32 = _f16(cam), _f16(proj)
    fa = cm.cost_volume_forward(c, p, D, k, "window", "fast")  # 33.4 GB
    for h0 in (0, 2049, 4090):
        h1 = min(H, h0 + 6)
        ref = _band_forward(c32, p32, k, h0, h1, "window", D)
        assert np.abs(fa[h0:h1].cpu().numpy() - ref).max() <= O.fast_tolerance(k)
    # row bands of the whole image (the multi-GPU shards) equal the whole-image rows
    o = k // 2
    for b, e in ((0, 1024), (1024, 2048), (3072, 4096)):
        a0, a1 = max(0, b - o), min(H, e + o)
        vb = cm.cost_volume_forward(c[a0:a1].contiguous(), p[a0:a1].contiguous(), D, k, "window", "fast",
                                    rows=(b - a0, e - a0))
        assert torch.equal(vb, fa[b:e])
        del vb
    idx, best = cm.stereo_disparity(c[:512].contiguous(), p[:512].contiguous(), D, k, "window")
    ex = cm.cost_volume_forward(c[:512].contiguous(), p[:512].contiguous(), D, k, "window", "exact")
    vi, vb = cm.volume_argmax(ex)
    assert torch.equal(idx, vi) and torch.equal(best, vb)
    del ex, vi, vb
    # the bench's own step: backward of both images at 4096x8192 from the forward's 33.4 GB volume
    # (volume offsets past 2^32 bytes), checked on haloed oracle tiles (rows x columns)
    gen = torch.Generator(device=gpu).manual_seed(102)
    g = torch.randn(fa.shape, generator=gen, device=gpu)
    gc, gp = cm.cost_volume_backward(g, c, p, k, "window", D, projector_grad=True, cost_volume=fa)
    for h0 in (2049, 4090):
        for c0 in (0, W - 768):
            h1 = min(H, h0 + 6)
            rc, rp, (xc0, xc1), (xp0, xp1) = _tile_backward(g, c32, p32, k, D, h0, h1, c0, 768)
            assert _rel(gc[h0:h1, xc0:xc1].cpu().numpy(), rc) <= 1e-5, (h0, c0)
            assert _rel(gp[h0:h1, xp0:xp1].cpu().numpy(), rp) <= 1e-5, (h0, c0)
    assert torch.isfinite(gc).all() and torch.isfinite(gp).all()


def test_backward_rank_band_full_width(gpu):
    """The N = 8 rank band of configs[4] (512 rows + 2 x 5 halo rows of 4096 x 8192 fp16, D = 256, k = 11): a
    backward grid with a partial last round, where run_bwd may re-segment the columns (bwd_fused.hip
    tail_seg_min); checked on haloed oracle tiles at both ends of the row and in the middle."""
    H, W, k, D = 522, 8192, 11, 256
    cam, proj = make_pair(H, W, D, seed=111)
    c, p = _dev(cam, gpu, torch.float16), _dev(proj, gpu, torch.float16)
    c32, p32 = _f16(cam), _f16(proj)
    fa = cm.cost_volume_forward(c, p, D, k, "window", "fast")
    gen = torch.Generator(device=gpu).manual_seed(112)
    g = torch.randn(fa.shape, generator=gen, device=gpu)
    gc, gp = cm.cost_volume_backward(g, c, p, k, "window", D, projector_grad=True, cost_volume=fa)
    for h0 in (0, 258, 516):
        for c0 in (0, 3712, W - 768):
            h1 = min(H, h0 + 6)
            rc, rp, (xc0, xc1), (xp0, xp1) = _tile_backward(g, c32, p32, k, D, h0, h1, c0, 768)
            assert _rel(gc[h0:h1, xc0:xc1].cpu().numpy(), rc) <= 1e-5, (h0, c0)
            assert _rel(gp[h0:h1, xp0:xp1].cpu().numpy(), rp) <= 1e-5, (h0, c0)
    assert torch.isfinite(gc).all() and torch.isfinite(gp).all()



# ---------------- kernel sizes beyond the fused instantiations (generic paths) ----------------

@pytest.mark.parametrize("k", [33, 35, 34, 18, 20, 30])
def test_large_and_even_kernel_sizes_through_autograd(gpu, k):
    """k = 33, 34, 35 (above the sliding instantiations: exact forward + generic fp64 backward) and even
    k = 18, 20, 30 (the reference's kernel_size / 2 origin; sliding backward and disparity, exact
    volume) via the op."""
    H, W, D = 28, 60, 12
    cam, proj = make_pair(H, W, D, seed=200 + k)
    for layout in ("full", "window"):
        c = _dev(cam, gpu).requires_grad_(True)
        p = _dev(proj, gpu).requires_grad_(True)
        vol = cm.stereo_matching(c, p, D, k, layout)
        lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
        ref = O.forward(cam, proj, k, layout=lay, D=Dl)
        got = vol.detach().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))  # exact path for these k
        g = np.random.default_rng(k).standard_normal(ref.shape).astype(np.float32)
        vol.backward(_dev(g, gpu))
        rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
        assert _rel(c.grad.cpu().numpy(), rc) <= 1e-5
        assert _rel(p.grad.cpu().numpy(), rp) <= 1e-5
        idx, best = cm.stereo_disparity(c.detach(), p.detach(), D, k, layout)
        ridx, _ = O.argmax(ref)
        assert np.array_equal(idx.cpu().numpy(), ridx)


@pytest.mark.parametrize("layout", ["full", "window"])
def test_disparity_recheck_both_forms(gpu, layout):
    """k = 33 (no sliding instantiation: every pixel is re-decided with the exact arithmetic).  Full layout,
    W = 600: the projector strip k x (W + k - 1) floats exceeds 64 KiB, so the re-decision runs the global-
    load kernel (select.hip k_disp_recheck); window layout, D = 40: the LDS-tiled k_disp_recheck_lds.  Both
    bit-identical to the oracle's argmax and best."""
    H, W, D, k = 6, 600, 40, 33
    cam, proj = make_pair(H, W, D, seed=733, kind="quantized")
    c, p = _dev(cam, gpu), _dev(proj, gpu)
    lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl)
    idx, best, nre = cm.stereo_disparity(c, p, D, k, layout, return_rechecked=True)
    ridx, rbest = O.argmax(ref)
    assert int(nre.item()) == H * ref.shape[1]  # every pixel re-decided
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(best.cpu().numpy().view(np.uint32), np.asarray(rbest, np.float32).view(np.uint32))


@pytest.mark.parametrize("k", [2, 4, 8, 16, 19, 22, 25, 28, 31])
def test_sliding_kernel_sizes_through_autograd(gpu, k):
    """Even k (taps -k/2 .. k/2-1, stereo_matching_kernel.cu:44,60) and every k up to 31 on the sliding kernels:
    fast forward within the cost bound (k <= 11; larger k write the exact volume), fused backward of
    both images within 1e-5, certified disparity (sliding partials) bit-identical to the exact
    volume's argmax."""
    H, W, D = 30, 72, 14
    cam, proj = make_pair(H, W, D, seed=300 + k)
    for layout in ("full", "window"):
        c = _dev(cam, gpu).requires_grad_(True)
        p = _dev(proj, gpu).requires_grad_(True)
        vol = cm.stereo_matching(c, p, D, k, layout, "fast")
        lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
        ref = O.forward(cam, proj, k, layout=lay, D=Dl)
        if k <= 11:
            assert np.abs(vol.detach().cpu().numpy() - ref).max() <= O.fast_tolerance(k)
        else:  # k >= 12: the volume is the exact kernel's (capi.hip kFastVolumeMaxK)
            assert np.array_equal(vol.detach().cpu().numpy().view(np.uint32), ref.view(np.uint32))
        g = np.random.default_rng(k).standard_normal(ref.shape).astype(np.float32)
        vol.backward(_dev(g, gpu))
        rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
        assert _rel(c.grad.cpu().numpy(), rc) <= 1e-5
        assert _rel(p.grad.cpu().numpy(), rp) <= 1e-5
        idx, best = cm.stereo_disparity(c.detach(), p.detach(), D, k, layout)
        ridx, _ = O.argmax(ref)
        assert np.array_equal(idx.cpu().numpy(), ridx)


def test_autograd_volume_edited_in_place_recomputes(gpu):
    """The op keeps only a weak reference to its output: an in-place edit of the returned
    volume (legal with the reference, which saves only the inputs) makes the backward
    recompute the costs instead of reading the edited values."""
    H, W, k = 24, 48, 7
    cam, proj = make_pair(H, W, 12, seed=300)
    g = np.random.default_rng(301).standard_normal((H, W, W)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k)
    for mode in ("keep", "edit", "drop"):
        c = _dev(cam, gpu).requires_grad_(True)
        p = _dev(proj, gpu).requires_grad_(True)
        vol = cm.stereo_matching(c, p, 0, k)
        out = vol * 1.0
        if mode == "edit":
            vol.mul_(0.0)  # in-place edit after the forward
            out = vol + out
        elif mode == "drop":
            del vol
        out.backward(_dev(g, gpu))
        assert _rel(c.grad.cpu().numpy(), rc) <= 1e-5, mode
        assert _rel(p.grad.cpu().numpy(), rp) <= 1e-5, mode
