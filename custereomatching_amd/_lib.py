"""ctypes binding of libcustma_hip.so (C ABI: include/custma.h).

There is no CPU or eager fallback: if the HIP library is missing the import
fails loudly, and every op requires its tensors on a ROCm device.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- must load torch's libamdhip64 before ours (same soname)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CUSTMA_LIB selects another build of the same library (ablation builds, scripts/ablate.sh)
LIB_PATH = os.environ.get("CUSTMA_LIB") or os.path.join(_HERE, "_lib", "libcustma_hip.so")

F32, F16 = 0, 1
LAYOUT_FULL, LAYOUT_WINDOW = 0, 1
EXACT, FAST = 0, 1
OP_FORWARD, OP_BACKWARD, OP_DISPARITY, OP_BACKWARD_RECOMPUTE = 0, 1, 2, 3
E_ARG, E_NULL, E_WORKSPACE, E_LAUNCH, E_UNSUPPORTED = -1, -2, -3, -4, -5

EXPORTS = ("custma_abi_version", "custma_last_error", "custma_volume_dims", "custma_workspace_bytes",
           "custma_forward", "custma_backward", "custma_argmax", "custma_disparity", "custma_forward_band",
           "custma_backward_band", "custma_disparity_band", "custma_profile_enable", "custma_profile_mean_ms",
           "custma_image_u8_to_unit", "custma_disparity_soft_band", "custma_patch_stats")
STATS_FULL, STATS_BOX, STATS_BWD_PREP, STATS_FWD, STATS_MSB = 0, 1, 2, 3, 4


class CustmaError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"custereomatching_amd: HIP library not found at {LIB_PATH}; build it with "
            "`python custereomatching_amd/build.py` (hipcc, gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
    i64p = ctypes.POINTER(ctypes.c_int64)
    lib.custma_abi_version.restype = ctypes.c_int
    lib.custma_last_error.restype = ctypes.c_char_p
    lib.custma_volume_dims.argtypes = [i64, i64, i32, i32, i64p, i64p]
    lib.custma_workspace_bytes.argtypes = [i64, i64, i32, i32, i32, i32]
    lib.custma_workspace_bytes.restype = sz
    lib.custma_forward.argtypes = [vp, vp, i32, i64, i64, i32, i32, i32, i32, vp, vp, sz, vp]
    lib.custma_backward.argtypes = [vp, vp, vp, vp, i32, i64, i64, i32, i32, i32, vp, vp, vp, sz, vp]
    lib.custma_argmax.argtypes = [vp, i64, i64, vp, vp, vp]
    lib.custma_disparity.argtypes = [vp, vp, i32, i64, i64, i32, i32, i32, vp, vp, vp, vp, sz, vp]
    lib.custma_forward_band.argtypes = [vp, vp, i32, i64, i64, i32, i32, i32, i32, i64, i64, vp, vp, sz, vp]
    lib.custma_backward_band.argtypes = [vp, vp, vp, vp, i32, i64, i64, i32, i32, i32, i64, i64, vp, vp, vp, sz,
                                         vp]
    lib.custma_disparity_band.argtypes = [vp, vp, i32, i64, i64, i32, i32, i32, i64, i64, vp, vp, vp, vp, sz,
                                          vp]
    f32 = ctypes.c_float
    lib.custma_disparity_soft_band.argtypes = [vp, vp, i32, i64, i64, i32, i32, i32, i64, i64, f32, f32, vp, vp, vp,
                                               vp, vp, vp, sz, vp]
    lib.custma_profile_enable.argtypes = [i32]
    lib.custma_patch_stats.argtypes = [vp, vp, i32, i64, i64, i32, i32, i64, i64, vp, vp, vp, vp, vp, vp, vp]
    lib.custma_image_u8_to_unit.argtypes = [vp, i64, i64, i32, i32, i32, vp, vp]
    lib.custma_profile_mean_ms.argtypes = [i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32)]
    for name in ("custma_profile_enable", "custma_profile_mean_ms", "custma_forward", "custma_backward", "custma_argmax", "custma_disparity",
                 "custma_volume_dims", "custma_forward_band", "custma_backward_band", "custma_disparity_band",
                 "custma_image_u8_to_unit", "custma_disparity_soft_band", "custma_patch_stats"):
        getattr(lib, name).restype = ctypes.c_int
    return lib


lib = _load()


def check(rc: int, what: str) -> None:
    if rc == 0:
        return
    msg = lib.custma_last_error().decode(errors="replace")
    if rc in (E_ARG, E_UNSUPPORTED):
        raise ValueError(f"{what}: {msg}")
    raise CustmaError(f"{what}: {msg} (code {rc})")


def volume_dims(H: int, W: int, layout: int, D: int):
    wo, do = ctypes.c_int64(), ctypes.c_int64()
    check(lib.custma_volume_dims(H, W, layout, D, ctypes.byref(wo), ctypes.byref(do)), "volume_dims")
    return wo.value, do.value


def workspace_bytes(H, W, k, layout, D, op) -> int:
    return int(lib.custma_workspace_bytes(H, W, k, layout, D, op))


PROF_FWD, PROF_BWD = 0, 1


def profile_enable(on: bool) -> None:
    """HIP-event timing of the main kernel of each op (bench only; see include/custma.h)."""
    check(lib.custma_profile_enable(1 if on else 0), "profile_enable")


def profile_mean_ms(which: int):
    """(mean kernel ms, launches) since profile_enable(True); clears the collection."""
    ms, n = ctypes.c_float(), ctypes.c_int32()
    check(lib.custma_profile_mean_ms(which, ctypes.byref(ms), ctypes.byref(n)), "profile_mean_ms")
    return float(ms.value), int(n.value)
