"""Cooperative vs one-wave backward on small cases: where do they differ? (diagnostic; GPU box)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from tests.golden.inputs import make_pair  # noqa: E402

dev = torch.device("cuda:0")
for (H, W, k, D, layout) in [(16, 24, 5, 8, "full"), (40, 64, 9, 20, "window"), (40, 64, 9, 20, "full")]:
    cam, proj = make_pair(H, W, D, seed=3)
    c = torch.from_numpy(cam).to(dev)
    p = torch.from_numpy(proj).to(dev)
    vol = cm.cost_volume_forward(c, p, D, k, layout)
    g = torch.from_numpy(np.random.default_rng(0).standard_normal(tuple(vol.shape)).astype(np.float32)).to(dev)
    res = {}
    for old in ("1", "0"):
        os.environ["CUSTMA_BWD_OLD"] = old
        gc, gp = cm.cost_volume_backward(g, c, p, k, layout, D, projector_grad=True, cost_volume=vol)
        torch.cuda.synchronize()
        res[old] = (gc.cpu().numpy(), gp.cpu().numpy())
    for i, name in enumerate(("camera", "projector")):
        a, b = res["1"][i], res["0"][i]
        d = np.abs(a - b)
        tol = 1e-5 * max(1.0, np.abs(a).max())
        bad = np.argwhere(d > tol)
        print(f"== {H}x{W} k{k} {layout} {name}: max|d| {d.max():.3g} (scale {np.abs(a).max():.3g}), {len(bad)} bad")
        if len(bad):
            print("   rows:", np.unique(bad[:, 0]).tolist()[:40])
            print("   cols:", np.unique(bad[:, 1]).tolist()[:40])
            for b_ in bad[:5]:
                print("   ", tuple(b_.tolist()), float(a[tuple(b_)]), float(b[tuple(b_)]))
