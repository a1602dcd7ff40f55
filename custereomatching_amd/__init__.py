"""custereomatching_amd -- MI355X (gfx950) native ZNCC stereo cost volume.

Drop-in for lzhnb/CuStereoMatching's ``custma`` package (also importable as
``custma``, see the alias package next to this one).  Hot path: the cost
volume forward, its backward into both images, and per-pixel disparity, as
hand-written HIP kernels behind the C ABI of include/custma.h.
"""
from .version import __version__
from .stereo_matching_wrapper import stereo_matching, cost_volume_forward, cost_volume_backward, default_precision
from .disparity import (stereo_disparity, stereo_disparity_soft, disparity_maps, volume_argmax, disparity_from_index,
                        confidence_mask, soft_argmax)
from .preprocess import image_u8_to_unit
from .utils import Timer, TimerError

__all__ = [k for k in globals().keys() if not k.startswith("_")]
