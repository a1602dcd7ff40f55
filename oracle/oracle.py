"""ctypes/numpy front end of the C oracle -- TEST INFRASTRUCTURE ONLY.

Each function cites the reference lines it restates (via zncc_oracle.c):
  forward   custma/src/stereo_matching_kernel.cu:39-71
  backward  custma/src/stereo_matching_kernel.cu:97-179
  argmax    examples/verify.py:72, examples/test.py:78-83 (caller side)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liborc.so")
_lib = None

FULL, WINDOW = 0, 1


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "zncc_oracle.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "liborc.so"], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        i64 = ctypes.c_int64
        i64p = ctypes.POINTER(ctypes.c_int64)
        ci = ctypes.c_int
        L.orc_stats.argtypes = [fp, i64, i64, ci, ci, fp, fp]
        L.orc_forward_literal.argtypes = [fp, fp, i64, i64, ci, ci, ci, ci, fp]
        L.orc_forward.argtypes = [fp, fp, i64, i64, ci, ci, ci, ci, fp]
        L.orc_forward_f64.argtypes = [fp, fp, i64, i64, ci, ci, ci, dp]
        L.orc_backward.argtypes = [fp, fp, fp, i64, i64, ci, ci, ci, fp, fp]
        L.orc_backward_f64.argtypes = [fp, fp, fp, i64, i64, ci, ci, ci, dp, dp]
        L.orc_argmax.argtypes = [fp, i64, i64, i64p, fp]
        L.orc_volume_dims.argtypes = [i64, i64, ci, ci, i64p, i64p]
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a, t=ctypes.c_float):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _check(rc, what):
    if rc != 0:
        raise ValueError(f"oracle {what} failed with code {rc}")


def volume_shape(H, W, layout=FULL, D=0):
    if layout == FULL:
        return (H, W, W)
    return (H, W - D, D + 1)


def stats(img, k, contract=1):
    img = _f32(img)
    H, W = img.shape
    m = np.empty((H, W), np.float32)
    s = np.empty((H, W), np.float32)
    _check(lib().orc_stats(_p(img), H, W, k, contract, _p(m), _p(s)), "stats")
    return m, s


def forward(cam, proj, k, layout=FULL, D=0, contract=1, literal=False):
    """Reference forward arithmetic (stereo_matching_kernel.cu:39-71)."""
    cam, proj = _f32(cam), _f32(proj)
    H, W = cam.shape
    assert proj.shape == (H, W)
    out = np.empty(volume_shape(H, W, layout, D), np.float32)
    fn = lib().orc_forward_literal if literal else lib().orc_forward
    _check(fn(_p(cam), _p(proj), H, W, k, layout, D, contract, _p(out)), "forward")
    return out


def forward_f64(cam, proj, k, layout=FULL, D=0):
    cam, proj = _f32(cam), _f32(proj)
    H, W = cam.shape
    out = np.empty(volume_shape(H, W, layout, D), np.float64)
    _check(lib().orc_forward_f64(_p(cam), _p(proj), H, W, k, layout, D, _p(out, ctypes.c_double)),
           "forward_f64")
    return out


def backward(grad, cam, proj, k, layout=FULL, D=0):
    """Camera and projector gradients (stereo_matching_kernel.cu:97-179)."""
    cam, proj, grad = _f32(cam), _f32(proj), _f32(grad)
    H, W = cam.shape
    assert grad.shape == volume_shape(H, W, layout, D)
    dc = np.empty((H, W), np.float32)
    dp = np.empty((H, W), np.float32)
    _check(lib().orc_backward(_p(grad), _p(cam), _p(proj), H, W, k, layout, D, _p(dc), _p(dp)),
           "backward")
    return dc, dp


def backward_f64(grad, cam, proj, k, layout=FULL, D=0):
    """fp64 truth of the backward (same formula, all in double)."""
    cam, proj, grad = _f32(cam), _f32(proj), _f32(grad)
    H, W = cam.shape
    assert grad.shape == volume_shape(H, W, layout, D)
    dc = np.empty((H, W), np.float64)
    dp = np.empty((H, W), np.float64)
    dptr = ctypes.c_double
    _check(lib().orc_backward_f64(_p(grad), _p(cam), _p(proj), H, W, k, layout, D,
                                  _p(dc, dptr), _p(dp, dptr)), "backward_f64")
    return dc, dp


def argmax(vol):
    """First-index argmax over the last axis (torch.argmax semantics)."""
    vol = _f32(vol)
    n = vol.shape[-1]
    rows = vol.size // n
    idx = np.empty(rows, np.int64)
    best = np.empty(rows, np.float32)
    _check(lib().orc_argmax(_p(vol), rows, n, _p(idx, ctypes.c_int64), _p(best)), "argmax")
    return idx.reshape(vol.shape[:-1]), best.reshape(vol.shape[:-1])


def cost_error_bound(k: int) -> float:
    """Worst-case |cost_fast - cost_reference| for the fast path.

    The reference's fp32 fma chain of k*k centred products errs by at most
    (k^2 + 2) u * sum|x||y| / S <= (k^2 + 2) u; the fast path is fp64-exact in
    the numerator and shares S bit-for-bit, adding <= 4 u of final rounding.
    """
    u = 2.0 ** -24
    return (k * k + 6) * u


def fast_tolerance(k: int) -> float:
    """The gate every fast-path cost is held to: BASELINE north_star's 1e-5 on the
    float cost volume, or the tighter worst-case bound where that is below it
    (k <= 11)."""
    return min(1e-5, cost_error_bound(k))


def image_u8_to_unit(image, channel=0, dtype=np.float32):
    """The reference driver's preprocessing (examples/verify.py:138-142, 148):
    ``np.array(cv2.imread(...)) / 255`` (numpy float64 true division), then
    ``torch.tensor(..., dtype=float32)`` and the camera channel ``[:, :, 0]``."""
    img = np.asarray(image)
    if img.ndim == 3:
        img = img[:, :, channel]
    return (img / 255).astype(dtype)
