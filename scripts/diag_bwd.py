"""Localise a fused-backward parity failure (window k = 4): for each case, the GPU
gradients three ways -- volume recomputed in the workspace, the GPU forward's volume passed in,
the oracle's exact volume passed in -- against the fp64 oracle, repeated for determinism, with the
rows / columns where the error exceeds the bar.

Usage: python scripts/diag_bwd.py [--all]   (default: the window k = 4 case and its neighbours)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tests.golden.inputs import make_pair  # noqa: E402
from tests.test_gpu_parity import BWD_CASES  # noqa: E402

import custereomatching_amd as cm  # noqa: E402

dev = torch.device("cuda:0")


def dv(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def rel(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))


def where(a, b):
    e = np.abs(a - b) > 1e-5 * max(1.0, np.abs(b).max())
    ys, xs = np.nonzero(e)
    if ys.size == 0:
        return "-"
    return f"{ys.size} px rows {sorted(set(ys.tolist()))[:12]} cols {sorted(set(xs.tolist()))[:16]}"


def run(case, layout):
    H, W, k, D, kind = case
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    lay, Dl = (O.FULL, 0) if layout == "full" else (O.WINDOW, D)
    g = np.random.default_rng(7).standard_normal(O.volume_shape(H, W, lay, Dl)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
    vref = O.forward(cam, proj, k, layout=lay, D=Dl, contract=1)
    c, p, gd = dv(cam), dv(proj), dv(g)
    vfast = cm.cost_volume_forward(c, p, D, k, layout, "fast")
    torch.cuda.synchronize()
    fv = rel(vfast.cpu().numpy(), vref)
    out = []
    for name, vol in (("recompute", None), ("given-gpu", vfast), ("given-orc", dv(vref))):
        res = []
        for rep in range(3):
            gc, gp = cm.cost_volume_backward(gd, c, p, k, layout, D, camera_grad=True, projector_grad=True,
                                             cost_volume=vol)
            torch.cuda.synchronize()
            res.append((gc.cpu().numpy(), gp.cpu().numpy()))
        det = all(np.array_equal(res[0][0], r[0]) and np.array_equal(res[0][1], r[1]) for r in res)
        ec = max(rel(r[0], rc) for r in res)
        ep = max(rel(r[1], rp) for r in res)
        flag = "FAIL" if (ec > 1e-5 or ep > 1e-5) else "ok"
        out.append(f"  {name:10s} cam {ec:.2e} proj {ep:.2e} det={det} {flag}")
        if flag == "FAIL":
            out.append(f"     cam  {where(res[0][0], rc)}")
            out.append(f"     proj {where(res[0][1], rp)}")
    print(f"{layout:6s} {H}x{W} k{k} D{D} {kind}: fwd-fast rel {fv:.2e}", flush=True)
    print("\n".join(out), flush=True)


if __name__ == "__main__":
    cases = BWD_CASES if "--all" in sys.argv else [c for c in BWD_CASES if c[2] in (2, 4, 6, 8)]
    for case in cases:
        for layout in ("window", "full"):
            run(case, layout)
