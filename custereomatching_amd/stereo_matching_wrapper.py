"""The ``stereo_matching`` autograd operator -- drop-in for
``custma.stereo_matching`` (reference: custma/stereo_matching_wrapper.py:7-35).

Same call, same meaning::

    cost_volume = stereo_matching(camera, projector, D, kernel_size)   # [H, W, W]
    cost_volume.backward(grad)                                         # camera.grad

``camera`` / ``projector``: [H, W] contiguous float32 (or float16, a
superset) tensors on the same ROCm device.  ``D`` is accepted and ignored by
the default ``layout="full"``, exactly like the reference
(stereo_matching_kernel.cu:14).  Supersets, all opt-in or harmless:

* ``layout="window"`` returns the reference's intended [H, W-D, D+1] volume,
  ``out[h, w, s] = full[h, w, w+s]``;
* ``precision``: ``"fast"`` (default; fp64 sliding sums, within
  (k^2+6)*2^-24 of the exact value) or ``"exact"`` (bit-identical to the
  reference arithmetic, nvcc -fmad=true).  The process default can be set
  with ``CUSTMA_PRECISION=exact``;
* the projector also gets a gradient when it requires one (the reference
  returns None, stereo_matching_wrapper.py:33);
* a non-contiguous incoming gradient is made contiguous (the reference
  raises, stereo_matching.cpp:52), so ``volume.sum().backward()`` works.

Errors mirror the reference's CHECK_INPUT messages
(custma/include/stereo_matching.hpp:20-29): ``"camera must be a CUDA
tensor"``, ``"camera must be contiguous"``; a wrong dtype raises ``"expected
scalar type Float but found ..."`` like ``data_ptr<float>()`` does.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional, Tuple

import torch

from . import _lib

_PRECISIONS = {"exact": _lib.EXACT, "fast": _lib.FAST}
_LAYOUTS = {"full": _lib.LAYOUT_FULL, "window": _lib.LAYOUT_WINDOW}


def default_precision() -> str:
    p = os.environ.get("CUSTMA_PRECISION", "fast")
    if p not in _PRECISIONS:
        raise ValueError(f"CUSTMA_PRECISION must be one of {sorted(_PRECISIONS)}, got {p!r}")
    return p


def _check_input(x: torch.Tensor, name: str) -> None:
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not x.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _dtype_code(x: torch.Tensor) -> int:
    if x.dtype == torch.float32:
        return _lib.F32
    if x.dtype == torch.float16:
        return _lib.F16
    name = str(x.dtype).replace("torch.", "").capitalize()
    name = {"Float64": "Double", "Bfloat16": "BFloat16", "Int64": "Long", "Int32": "Int"}.get(name, name)
    raise RuntimeError(f"expected scalar type Float but found {name}")


def _check_pair(camera: torch.Tensor, projector: torch.Tensor, kernel_size: int):
    _check_input(camera, "camera")
    _check_input(projector, "projector")
    if camera.dim() != 2:
        raise RuntimeError(f"camera must be a 2-D [H, W] tensor, got shape {tuple(camera.shape)}")
    if projector.shape != camera.shape:
        raise RuntimeError(f"projector shape {tuple(projector.shape)} != camera shape {tuple(camera.shape)}")
    if projector.dtype != camera.dtype:
        raise RuntimeError(f"projector dtype {projector.dtype} != camera dtype {camera.dtype}")
    if projector.device != camera.device:
        raise RuntimeError("camera and projector must be on the same device")
    code = _dtype_code(camera)
    if not isinstance(kernel_size, int) or isinstance(kernel_size, bool):
        raise TypeError("kernel_size must be an int")
    return code


def _stream_ptr(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _workspace(nbytes: int, dev: torch.device) -> torch.Tensor:
    return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)


def _rows(H: int, rows: Optional[Tuple[int, int]]) -> Tuple[int, int]:
    if rows is None:
        return 0, H
    r0, r1 = int(rows[0]), int(rows[1])
    if not 0 <= r0 <= r1 <= H:
        raise ValueError(f"rows {rows} must satisfy 0 <= begin <= end <= {H}")
    return r0, r1


def cost_volume_forward(camera: torch.Tensor, projector: torch.Tensor, D: int, kernel_size: int,
                        layout: str = "full", precision: Optional[str] = None,
                        rows: Optional[Tuple[int, int]] = None,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Forward volume without autograd (reference: stereo::stereo_matching_forward,
    custma/src/stereo_matching.cpp:16-42).  ``rows=(b, e)`` computes only volume
    rows [b, e) of a haloed row band (custma_forward_band).  ``out`` is an optional
    preallocated contiguous float32 volume on the images' device."""
    code = _check_pair(camera, projector, kernel_size)
    lay = _LAYOUTS[layout]
    prec = _PRECISIONS[precision or default_precision()]
    H, W = camera.shape
    r0, r1 = _rows(H, rows)
    D = int(D)
    Dl = D if lay == _lib.LAYOUT_WINDOW else 0
    WO, DO = _lib.volume_dims(H, W, lay, Dl)
    dev = camera.device
    if out is None:
        out = torch.empty((r1 - r0, WO, DO), dtype=torch.float32, device=dev)
    elif (tuple(out.shape) != (r1 - r0, WO, DO) or out.dtype != torch.float32 or out.device != dev
          or not out.is_contiguous()):
        raise ValueError(f"out must be a contiguous float32 tensor of shape {(r1 - r0, WO, DO)} on {dev}")
    if out.numel() == 0:
        return out
    with torch.cuda.device(dev):
        nb = _lib.workspace_bytes(H, W, kernel_size, lay, Dl, _lib.OP_FORWARD)
        ws = _workspace(nb, dev)
        _lib.check(_lib.lib.custma_forward_band(camera.data_ptr(), projector.data_ptr(), code, H, W, kernel_size,
                                                lay, Dl, prec, r0, r1, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                                _stream_ptr(dev)), "stereo_matching_forward")
    return out


def cost_volume_backward(cost_volume_grad: torch.Tensor, camera: torch.Tensor, projector: torch.Tensor,
                         kernel_size: int, layout: str = "full", D: int = 0, camera_grad: bool = True,
                         projector_grad: bool = False, rows: Optional[Tuple[int, int]] = None,
                         cost_volume: Optional[torch.Tensor] = None
                         ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Gradients of sum(grad * volume) (reference: stereo::stereo_matching_backward,
    custma/src/stereo_matching.cpp:45-73; camera only there).  ``cost_volume`` is the
    forward's output for these images (the autograd op passes the one it returned);
    without it the library recomputes it in its workspace.  With ``rows=(b, e)`` the
    grad covers volume rows [b, e) of a haloed band and the returned image gradients
    cover every buffer row (halo rows hold partial sums)."""
    _check_input(cost_volume_grad, "cost_volume_grad")
    code = _check_pair(camera, projector, kernel_size)
    lay = _LAYOUTS[layout]
    H, W = camera.shape
    r0, r1 = _rows(H, rows)
    Dl = int(D) if lay == _lib.LAYOUT_WINDOW else 0
    WO, DO = _lib.volume_dims(H, W, lay, Dl)
    vshape = (r1 - r0, WO, DO)
    if tuple(cost_volume_grad.shape) != vshape:
        raise RuntimeError(f"cost_volume_grad shape {tuple(cost_volume_grad.shape)} != volume shape {vshape}")
    if cost_volume_grad.dtype != torch.float32:
        raise RuntimeError(f"expected scalar type Float but found {cost_volume_grad.dtype}")
    if cost_volume is not None:
        _check_input(cost_volume, "cost_volume")
        if tuple(cost_volume.shape) != vshape or cost_volume.dtype != torch.float32:
            raise RuntimeError(f"cost_volume must be a float32 tensor of shape {vshape}")
    dev = camera.device
    gc = torch.empty((H, W), dtype=torch.float32, device=dev) if camera_grad else None
    gp = torch.empty((H, W), dtype=torch.float32, device=dev) if projector_grad else None
    if H * W == 0 or (gc is None and gp is None):
        return (gc.zero_() if gc is not None else None), (gp.zero_() if gp is not None else None)
    with torch.cuda.device(dev):
        op = _lib.OP_BACKWARD if cost_volume is not None else _lib.OP_BACKWARD_RECOMPUTE
        nb = _lib.workspace_bytes(H, W, kernel_size, lay, Dl, op)
        ws = _workspace(nb, dev)
        _lib.check(_lib.lib.custma_backward_band(cost_volume_grad.data_ptr(),
                                                 cost_volume.data_ptr() if cost_volume is not None else None,
                                                 camera.data_ptr(), projector.data_ptr(), code, H, W, kernel_size,
                                                 lay, Dl, r0, r1,
                                                 gc.data_ptr() if gc is not None else None,
                                                 gp.data_ptr() if gp is not None else None,
                                                 ws.data_ptr(), ws.numel(), _stream_ptr(dev)),
                   "stereo_matching_backward")
    return gc, gp


class _StereoMatching(torch.autograd.Function):
    """Reference: custma/stereo_matching_wrapper.py:7-33.

    Saves only the two images, as the reference does (:16).  The backward also
    needs the forward's costs (V = g * cost / S); it reads the returned volume
    when that tensor is still alive and unmodified (a weak reference plus its
    version counter -- no reference cycle, no extra lifetime).  Otherwise it
    recomputes the volume here, with ``cost_volume_forward`` and the precision
    the forward used, into a transient tensor of the volume's size (4 bytes per
    voxel, e.g. 33 GB at 4096 x 8192 with D = 256), and passes it to the
    library.  So an in-place edit of the returned volume, or dropping it before
    ``.backward()``, behaves as with the reference, at that peak-memory cost."""

    @staticmethod
    def forward(ctx, camera_image, projector_image, D, kernel_size, layout="full", precision=None):
        vol = cost_volume_forward(camera_image, projector_image, D, kernel_size, layout, precision)
        ctx.save_for_backward(camera_image, projector_image)
        ctx.vol_ref = weakref.ref(vol)
        ctx.vol_version = vol._version
        ctx.D = D
        ctx.kernel_size = kernel_size
        ctx.layout = layout
        ctx.precision = precision or default_precision()
        return vol

    @staticmethod
    def backward(ctx, cost_volume_grad):
        camera_image, projector_image = ctx.saved_tensors
        vol = ctx.vol_ref()
        if vol is not None and vol._version != ctx.vol_version:
            vol = None  # edited in place after the forward: recompute the costs
        if vol is not None:
            vol = vol.detach()
        else:
            # recompute with the forward's own arithmetic, so V = A * cost / S uses the costs the
            # caller saw (a transient volume-sized buffer during the backward, as the reference's
            # own backward recomputes its forward per voxel, stereo_matching_kernel.cu:97-128)
            vol = cost_volume_forward(camera_image, projector_image, ctx.D, ctx.kernel_size, ctx.layout,
                                      ctx.precision)
        want_c, want_p = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gc, gp = cost_volume_backward(cost_volume_grad.contiguous(), camera_image, projector_image,
                                      ctx.kernel_size, ctx.layout, ctx.D, camera_grad=want_c,
                                      projector_grad=want_p, cost_volume=vol)
        if gc is not None and camera_image.dtype != torch.float32:
            gc = gc.to(camera_image.dtype)
        if gp is not None and projector_image.dtype != torch.float32:
            gp = gp.to(projector_image.dtype)
        return gc, gp, None, None, None, None


def stereo_matching(camera: torch.Tensor, projector: torch.Tensor, D: int, kernel_size: int,
                    layout: str = "full", precision: Optional[str] = None) -> torch.Tensor:
    """custma.stereo_matching (reference: stereo_matching_wrapper.py:35)."""
    if layout not in _LAYOUTS:
        raise ValueError(f"layout must be one of {sorted(_LAYOUTS)}, got {layout!r}")
    if precision is not None and precision not in _PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}, got {precision!r}")
    return _StereoMatching.apply(camera, projector, D, kernel_size, layout, precision)
