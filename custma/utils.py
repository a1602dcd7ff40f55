"""``custma.utils`` (reference: custma/utils.py) -- Timer."""
from custereomatching_amd.utils import Timer, TimerError  # noqa: F401
