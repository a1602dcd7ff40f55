"""Volume argmax timing (HIP events) on the C3 window and C2 full volume shapes; the library is the
one CUSTMA_LIB selects (an A/B runs this twice).  Usage: python scripts/ab_argmax.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from bench import EventTimer  # noqa: E402
from kbench import warm  # noqa: E402

for name, shape in (("c3_win", (2048, 1792, 257)), ("c2_full", (1024, 1024, 1024))):
    vol = torch.empty(shape, device="cuda").uniform_(-1.0, 1.0)
    ref = vol.argmax(-1)
    warm(lambda: cm.volume_argmax(vol))
    et = EventTimer()
    out = None
    for _ in range(10):
        out = et.record(lambda: cm.volume_argmax(vol))
    assert torch.equal(out[0], ref), "argmax differs from torch"
    gb = vol.numel() * 4 / 1e9
    print(json.dumps({"cfg": name, "argmax_ms": round(et.mean_ms(), 4), "GBps": round(gb / et.mean_ms() * 1e3, 1)}),
          flush=True)
    del vol, ref, out
    torch.cuda.empty_cache()
