"""Where does the fast forward differ from the oracle? (diagnostic; GPU box)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.golden.inputs import make_pair  # noqa: E402

for (H, W, k, D, layout) in [(24, 48, 5, 16, "full"), (24, 48, 5, 16, "window"), (40, 200, 9, 70, "full"),
                             (40, 200, 9, 70, "window")]:
    cam, proj = make_pair(H, W, D, seed=12)
    lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
    ref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    dev = torch.device("cuda:0")
    got = cm.cost_volume_forward(torch.from_numpy(cam).to(dev), torch.from_numpy(proj).to(dev), D, k, layout,
                                 "fast").cpu().numpy()
    bad = np.argwhere(np.abs(got - ref) > 1e-5)
    print(f"== {H}x{W} k{k} D{D} {layout}: {len(bad)} / {ref.size} bad")
    if len(bad):
        for ax, name in enumerate("hwd"):
            u, c = np.unique(bad[:, ax], return_counts=True)
            print(f"  {name}: {list(zip(u.tolist(), c.tolist()))[:40]}")
        for b in list(bad[:6]) + list(bad[len(bad) // 2:len(bad) // 2 + 6]):
            b = tuple(b.tolist())
            v = got[b]
            near = np.argwhere(np.abs(ref[b[0]] - v) < 2e-6)
            print("   ", b, float(v), float(ref[b]), "matches ref at (w,d):", [tuple(x) for x in near[:4].tolist()])
