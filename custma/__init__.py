"""``custma`` -- import-compatible alias of :mod:`custereomatching_amd`.

Code written against lzhnb/CuStereoMatching (``import custma``;
``custma.stereo_matching``, ``custma.Timer``, ``custma.__version__``, and the
extension module ``custma.src``) runs unchanged (reference: custma/__init__.py:1-7).
"""
from custereomatching_amd import *  # noqa: F401,F403
from custereomatching_amd import __version__, stereo_matching, Timer  # noqa: F401
from . import src  # noqa: F401

__all__ = ["stereo_matching", "Timer", "__version__", "src"]
