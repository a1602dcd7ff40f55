"""``custma.stereo_matching_wrapper`` (reference module path,
custma/stereo_matching_wrapper.py) re-exporting the HIP-backed operator."""
from custereomatching_amd.stereo_matching_wrapper import _StereoMatching, stereo_matching  # noqa: F401
