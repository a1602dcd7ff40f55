"""Per-pixel disparity selection -- the caller-side step of the reference
(examples/verify.py:31-39, 72-74; examples/test.py:78-86), made native.

* :func:`stereo_disparity` -- fused, certified argmax straight from the two
  images; the [H, W, W] volume is never written to HBM.  The index map is
  bit-identical to ``argmax`` of the exact (reference-arithmetic) volume:
  pixels whose fast top-2 gap is inside the fast path's error margin are
  re-decided with the exact arithmetic on the GPU.
* :func:`stereo_disparity_soft` -- the same fused pass also returning the
  soft-argmax (softmax(beta * cost) . index, verify.py:31-39) and the max-cost
  confidence mask (verify.py:72-74), still without the volume;
  :func:`disparity_maps` turns them into the caller's disparity maps
  (examples/test.py:78-86).
* :func:`volume_argmax` -- first-index argmax of a materialised volume
  (``torch.max(cost_volume.reshape(H*W, -1), -1)`` at verify.py:72).
* :func:`disparity_from_index`, :func:`confidence_mask`, :func:`soft_argmax`
  -- the reference's post-processing (test.py:82-86, verify.py:73-74,
  verify.py:31-39), as small torch expressions over the native results.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from .stereo_matching_wrapper import _LAYOUTS, _check_input, _check_pair, _rows, _stream_ptr, _workspace


def stereo_disparity(camera: torch.Tensor, projector: torch.Tensor, D: int, kernel_size: int,
                     layout: str = "full", return_rechecked: bool = False,
                     rows: Optional[Tuple[int, int]] = None):
    """(index [H, WO] int64, best cost [H, WO] fp32) without materialising the volume.
    ``rows=(b, e)``: only rows [b, e) of a haloed row band."""
    code = _check_pair(camera, projector, kernel_size)
    lay = _LAYOUTS[layout]
    H, W = camera.shape
    r0, r1 = _rows(H, rows)
    Dl = int(D) if lay == _lib.LAYOUT_WINDOW else 0
    WO, _ = _lib.volume_dims(H, W, lay, Dl)
    dev = camera.device
    idx = torch.empty((r1 - r0, WO), dtype=torch.int64, device=dev)
    best = torch.empty((r1 - r0, WO), dtype=torch.float32, device=dev)
    nre = torch.zeros(1, dtype=torch.int32, device=dev)
    if idx.numel():
        with torch.cuda.device(dev):
            nb = _lib.workspace_bytes(H, W, kernel_size, lay, Dl, _lib.OP_DISPARITY)
            ws = _workspace(nb, dev)
            _lib.check(_lib.lib.custma_disparity_band(camera.data_ptr(), projector.data_ptr(), code, H, W,
                                                      kernel_size, lay, Dl, r0, r1, idx.data_ptr(), best.data_ptr(),
                                                      nre.data_ptr(), ws.data_ptr(), ws.numel(), _stream_ptr(dev)),
                       "stereo_disparity")
    if return_rechecked:
        return idx, best, nre
    return idx, best


def stereo_disparity_soft(camera: torch.Tensor, projector: torch.Tensor, D: int, kernel_size: int,
                          layout: str = "full", beta: float = 50.0, threshold: float = 0.6,
                          rows: Optional[Tuple[int, int]] = None, return_rechecked: bool = False):
    """(index int64, best fp32, soft fp32, mask fp32), each [H, WO], from one fused pass
    (custma_disparity_soft_band): index / best as :func:`stereo_disparity`; soft =
    sum_s s * softmax(beta * cost)_s over the volume's last axis (verify.py:31-39, the
    defaults are its beta = 50 and threshold = 0.6, verify.py:12-13); mask = 1 where
    best > threshold else 0 (verify.py:72-74).  The volume is never materialised."""
    code = _check_pair(camera, projector, kernel_size)
    if not beta > 0:
        raise ValueError(f"beta must be > 0, got {beta}")
    lay = _LAYOUTS[layout]
    H, W = camera.shape
    r0, r1 = _rows(H, rows)
    Dl = int(D) if lay == _lib.LAYOUT_WINDOW else 0
    WO, _ = _lib.volume_dims(H, W, lay, Dl)
    dev = camera.device
    idx = torch.empty((r1 - r0, WO), dtype=torch.int64, device=dev)
    best = torch.empty((r1 - r0, WO), dtype=torch.float32, device=dev)
    soft = torch.empty((r1 - r0, WO), dtype=torch.float32, device=dev)
    mask = torch.empty((r1 - r0, WO), dtype=torch.float32, device=dev)
    nre = torch.zeros(1, dtype=torch.int32, device=dev)
    if idx.numel():
        with torch.cuda.device(dev):
            nb = _lib.workspace_bytes(H, W, kernel_size, lay, Dl, _lib.OP_DISPARITY)
            ws = _workspace(nb, dev)
            _lib.check(_lib.lib.custma_disparity_soft_band(
                camera.data_ptr(), projector.data_ptr(), code, H, W, kernel_size, lay, Dl, r0, r1, float(beta),
                float(threshold), idx.data_ptr(), best.data_ptr(), soft.data_ptr(), mask.data_ptr(), nre.data_ptr(),
                ws.data_ptr(), ws.numel(), _stream_ptr(dev)), "stereo_disparity_soft")
    if return_rechecked:
        return idx, best, soft, mask, nre
    return idx, best, soft, mask


def disparity_maps(camera: torch.Tensor, projector: torch.Tensor, D: int, kernel_size: int, layout: str = "full",
                   beta: float = 50.0, threshold: float = 0.6):
    """The reference caller's disparity pipeline (examples/test.py:71-86) from one fused pass:
    returns (disparity, disparity_softargmax, mask), both disparities multiplied by the mask
    (test.py:84, 86).  Full layout: template - argmax with template = camera column w
    (test.py:82-83); window layout: the index s is the offset d - w, so the disparity is -s."""
    idx, best, soft, mask = stereo_disparity_soft(camera, projector, D, kernel_size, layout, beta, threshold)
    if layout == "window":
        disp, disp_soft = -idx.to(torch.float32), -soft
    else:
        w = torch.arange(idx.shape[-1], device=idx.device, dtype=torch.float32)
        disp, disp_soft = w - idx.to(torch.float32), w - soft
    return disp * mask, disp_soft * mask, mask


def volume_argmax(cost_volume: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """First-index argmax over the last axis: (index int64, max value)."""
    _check_input(cost_volume, "cost_volume")
    if cost_volume.dtype != torch.float32:
        raise RuntimeError(f"expected scalar type Float but found {cost_volume.dtype}")
    n = cost_volume.shape[-1]
    lead = tuple(cost_volume.shape[:-1])
    rows = cost_volume.numel() // n if n else 0
    idx = torch.empty(lead, dtype=torch.int64, device=cost_volume.device)
    best = torch.empty(lead, dtype=torch.float32, device=cost_volume.device)
    if rows:
        with torch.cuda.device(cost_volume.device):
            _lib.check(_lib.lib.custma_argmax(cost_volume.data_ptr(), rows, n, idx.data_ptr(), best.data_ptr(),
                                              _stream_ptr(cost_volume.device)), "volume_argmax")
    return idx, best


def disparity_from_index(index: torch.Tensor, layout: str = "full") -> torch.Tensor:
    """Full layout: ``w - argmax`` (examples/test.py:80-83).  Window layout: the
    index is the offset s with d = w + s, so the disparity is ``-s``."""
    if layout == "window":
        return -index
    w = torch.arange(index.shape[-1], device=index.device, dtype=index.dtype)
    return w - index


def confidence_mask(best: torch.Tensor, threshold: float = 0.6) -> torch.Tensor:
    """1 where the best cost exceeds the threshold (examples/verify.py:73-74)."""
    return (best > threshold).to(best.dtype)


def soft_argmax(x: torch.Tensor, beta: float = 50.0) -> torch.Tensor:
    """softmax(beta * x) . index over the last axis (examples/verify.py:31-39)."""
    p = torch.softmax(x * beta, dim=-1)
    ar = torch.arange(x.shape[-1], device=x.device, dtype=p.dtype)
    return (p * ar).sum(-1)
