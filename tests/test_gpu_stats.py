"""The statistics kernel (csrc/stats.hip, compiled for gfx950) directly, through the diagnostics entry
point custma_patch_stats, in every mode and row range, against the oracle's fp32 mean / centred squares
(oracle/zncc_oracle.c orc_stats: the reference's stereo_matching_kernel.cu:40-69 order) and numpy fp64
patch sums in the kernel's order -- bit for bit.  The CPU emulation (test_stats_emulated.py) checks the
same source on the host; this checks what the GPU runs, so that a statistics fault shows here and not
only as a gradient or cost error further down."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.golden.inputs import make_pair
from tests.test_stats_emulated import _box_ref, _eq

from custereomatching_amd import _lib

pytestmark = pytest.mark.gpu

FULL, BOX, PREP, FWD, MSB = (_lib.STATS_FULL, _lib.STATS_BOX, _lib.STATS_BWD_PREP, _lib.STATS_FWD,
                             _lib.STATS_MSB)
CASES = [(70, 45, 11), (33, 70, 3), (18, 36, 4), (20, 44, 4), (65, 33, 5), (9, 40, 7), (1, 31, 3), (40, 50, 16),
         (35, 70, 31), (30, 41, 33), (17, 33, 10), (15, 30, 6), (1, 20, 2), (24, 90, 16), (22, 120, 8)]


def _stats_gpu(cam, proj, k, mode, band=None, shift=(0.25, -0.125), dtype=torch.float32):
    dev = torch.device("cuda:0")
    H, W = cam.shape
    b, e = band or (0, H)
    c = torch.from_numpy(cam).to(dev).to(dtype)
    p = torch.from_numpy(proj).to(dev).to(dtype)
    nan = float("nan")
    box = torch.full((2, H, W), nan, dtype=torch.float64, device=dev)
    mean = torch.full((2, H, W), nan, device=dev)
    sq, sqt = mean.clone(), mean.clone()
    sh = torch.tensor(shift, dtype=torch.float32, device=dev)
    prep = torch.full((2, 3, H, W), nan, device=dev)
    code = _lib.F16 if dtype == torch.float16 else _lib.F32
    _lib.check(_lib.lib.custma_patch_stats(c.data_ptr(), p.data_ptr(), code, H, W, k, mode, b, e, box.data_ptr(),
                                           mean.data_ptr(), sq.data_ptr(), sqt.data_ptr(), sh.data_ptr(),
                                           prep.data_ptr(), torch.cuda.current_stream(dev).cuda_stream),
               "patch_stats")
    torch.cuda.synchronize()
    return tuple(x.cpu().numpy() for x in (mean, sq, box, sqt, prep))


@pytest.mark.parametrize("H,W,k", CASES, ids=[f"{h}x{w}_k{k}" for h, w, k in CASES])
@pytest.mark.parametrize("mode", [FULL, BOX, PREP, FWD, MSB], ids=["full", "box", "prep", "fwd", "msb"])
def test_stats_kernel_gpu(gpu, H, W, k, mode):
    cam, proj = make_pair(H, W, 16, seed=H * 131 + W + k)
    shift = (0.25, -0.125)
    mean, sq, box, sqt, prep = _stats_gpu(cam, proj, k, mode, shift=shift)
    for z, img in enumerate((cam, proj)):
        m_ref, s_ref = O.stats(img, k, contract=1)
        b_ref, t_ref = _box_ref(img, k)
        chain = mode in (FULL, FWD, MSB)
        assert _eq(box[z], b_ref), ("box", z, np.abs(box[z] - b_ref).max())
        assert _eq(sq[z], s_ref) if chain else np.isnan(sq[z]).all(), ("sq", z)
        assert _eq(mean[z], m_ref) if mode in (FULL, MSB) else np.isnan(mean[z]).all(), ("mean", z)
        assert _eq(sqt[z], t_ref) if mode in (FULL, BOX) else np.isnan(sqt[z]).all(), ("sqt", z)
        if mode == PREP:
            assert _eq(prep[z, 0], t_ref), ("X", z)
            assert _eq(prep[z, 1], (b_ref / float(k * k) - float(np.float32(shift[z]))).astype(np.float32)), ("m'", z)
            assert _eq(prep[z, 2], img.astype(np.float32)), ("raw", z)
        else:
            assert np.isnan(prep[z]).all()


@pytest.mark.parametrize("mode", [FWD, MSB, FULL])
@pytest.mark.parametrize("k", [4, 11])
def test_stats_kernel_gpu_band_rows_fp16(gpu, mode, k):
    """fp16 images and a row band: only rows [9, 50) are written (their patches read the rows around)."""
    H, W = 70, 45
    cam, proj = make_pair(H, W, 16, seed=5)
    cam = cam.astype(np.float16).astype(np.float32)
    proj = proj.astype(np.float16).astype(np.float32)
    mean, sq, box, _, _ = _stats_gpu(cam, proj, k, mode, band=(9, 50), dtype=torch.float16)
    for z, img in enumerate((cam, proj)):
        m_ref, s_ref = O.stats(img, k, contract=1)
        b_ref, _ = _box_ref(img, k)
        assert _eq(sq[z, 9:50], s_ref[9:50]) and _eq(box[z, 9:50], b_ref[9:50])
        assert np.isnan(sq[z, :9]).all() and np.isnan(sq[z, 50:]).all() and np.isnan(box[z, :9]).all()
        if mode != FWD:
            assert _eq(mean[z, 9:50], m_ref[9:50])
