"""Image preprocessing before the hot path -- the reference driver's
``np.array(cv2.imread(path)) / 255`` -> ``torch.tensor(..., dtype=float32).cuda()``
-> ``rgb[:, :, 0]`` (examples/verify.py:138-142, 148), as one device pass over the
8-bit image (custma_image_u8_to_unit, csrc/preprocess.hip).  PNG decoding stays
with the caller (cv2 / PIL); this takes the decoded uint8 array on the GPU.
"""
from __future__ import annotations

import torch

from . import _lib
from .stereo_matching_wrapper import _check_input, _stream_ptr

_DTYPES = {torch.float32: _lib.F32, torch.float16: _lib.F16}


def image_u8_to_unit(image: torch.Tensor, channel: int = 0, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """[H, W] or [H, W, C] uint8 (cv2 layout; channel 0 = blue for cv2's BGR) ->
    [H, W] ``image[..., channel] / 255`` in ``dtype`` (float32 or float16), rounded
    exactly as numpy's float64 division followed by the cast."""
    _check_input(image, "image")
    if image.dtype != torch.uint8:
        raise RuntimeError(f"expected scalar type Byte but found {image.dtype}")
    if dtype not in _DTYPES:
        raise RuntimeError(f"unsupported output dtype {dtype} (float32 or float16)")
    if image.dim() == 2:
        H, W = image.shape
        C = 1
    elif image.dim() == 3:
        H, W, C = image.shape
    else:
        raise RuntimeError(f"image must be [H, W] or [H, W, C] (got {tuple(image.shape)})")
    out = torch.empty((H, W), dtype=dtype, device=image.device)
    with torch.cuda.device(image.device):
        _lib.check(_lib.lib.custma_image_u8_to_unit(image.data_ptr(), H, W, C, channel, _DTYPES[dtype],
                                                    out.data_ptr(), _stream_ptr(image.device)),
                   "image_u8_to_unit")
    return out
