"""Max |fast - exact| over the volume per kernel size on ill-conditioned inputs (decides capi.hip
kFastVolumeMaxK).  The exact volume is bit-identical to the reference arithmetic
(tests/test_gpu_parity.py).  Usage: python scripts/diag_fastk.py"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm
from tests.test_gpu_fast_parity import _ill_pair

dev = "cuda:0"
for k in (9, 11, 13, 15, 17):
    worst = {}
    for kind in ("flat", "quantized", "const_eps"):
        for layout, D in (("window", 64), ("full", 0)):
            for H, W in ((256, 512), (512, 1024)):
                cam, proj = _ill_pair(H, W, max(D, 16), kind)
                c = torch.from_numpy(cam).to(dev)
                p = torch.from_numpy(proj).to(dev)
                ex = cm.cost_volume_forward(c, p, D, k, layout, "exact")
                # the fast sweep itself (the API routes k > kFastVolumeMaxK to the exact kernel)
                fa = cm.cost_volume_forward(c, p, D, k, layout, "fast")
                e = float((fa - ex).abs().max())
                key = f"{kind}/{layout}"
                worst[key] = max(worst.get(key, 0.0), e)
                del ex, fa
    bound = (k * k + 6) * 2.0 ** -24
    print(json.dumps({"k": k, "bound": bound, "max_err": max(worst.values()), "by_input": worst}), flush=True)
