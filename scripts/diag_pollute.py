"""The window k = 4 backward goes wrong on the first call after an exact k = 19 forward (scripts/diag_ws.py,
r05e).  Which stage?  Each trial re-pollutes (the exact forward), then runs ONE op with a zero-filled
workspace and compares every output AND the workspace regions it wrote (statistics, backward scratch,
recomputed volume) with a clean run's.  Usage: python scripts/diag_pollute.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tests.golden.inputs import make_pair  # noqa: E402

import custereomatching_amd as cm  # noqa: E402
from custereomatching_amd import _lib  # noqa: E402
from bench import synth_pair  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.lib
H, W, k, D = 18, 36, 4, 10
lay = _lib.LAYOUT_WINDOW
WO, DO = _lib.volume_dims(H, W, lay, D)
cam, proj = make_pair(H, W, D, seed=31, kind="textured")
g = np.random.default_rng(7).standard_normal((H, WO, DO)).astype(np.float32)
rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
c, p, gd = (torch.from_numpy(x).to(dev) for x in (cam, proj, g))
c3, p3 = synth_pair(256, 2048, 256, 5, "cuda", torch.float16)
n = H * W


def a256(x):
    return (x + 255) & ~255


SB = 2 * a256(n * 20) + a256(4 * (H // 8 + 1))
NB_F = _lib.workspace_bytes(H, W, k, lay, D, _lib.OP_FORWARD)
NB_B = _lib.workspace_bytes(H, W, k, lay, D, _lib.OP_BACKWARD)
NB_R = _lib.workspace_bytes(H, W, k, lay, D, _lib.OP_BACKWARD_RECOMPUTE)


def st():
    return torch.cuda.current_stream(dev).cuda_stream


def pollute(on):
    if on:
        cm.cost_volume_forward(c3, p3, 256, 19, "window", "exact")
    torch.cuda.synchronize()


def ws0(nb):
    w = torch.zeros(nb + 256, dtype=torch.uint8, device=dev)
    return w[(-w.data_ptr()) % 256:][:nb]


def fwd():
    ws, out = ws0(NB_F), torch.zeros((H, WO, DO), device=dev)
    _lib.check(L.custma_forward_band(c.data_ptr(), p.data_ptr(), _lib.F32, H, W, k, lay, D, _lib.FAST, 0, H,
                                     out.data_ptr(), ws.data_ptr(), NB_F, st()), "fwd")
    torch.cuda.synchronize()
    return out.clone(), ws.clone()


def bwd(vol):
    nb = NB_B if vol is not None else NB_R
    ws = ws0(nb)
    gc, gp = torch.zeros((H, W), device=dev), torch.zeros((H, W), device=dev)
    _lib.check(L.custma_backward_band(gd.data_ptr(), vol.data_ptr() if vol is not None else None, c.data_ptr(),
                                      p.data_ptr(), _lib.F32, H, W, k, lay, D, 0, H, gc.data_ptr(), gp.data_ptr(),
                                      ws.data_ptr(), nb, st()), "bwd")
    torch.cuda.synchronize()
    return gc.clone(), gp.clone(), ws.clone()


def stats_view(ws):
    """[image][box | mean | sq | sqt] of the statistics region (capi.hip carve_stats)."""
    out = {}
    for i, name in enumerate(("cam", "proj")):
        base = i * a256(n * 20)
        out[name + ".box"] = ws[base:base + 8 * n].view(torch.float64)
        out[name + ".sq"] = ws[base + 12 * n:base + 16 * n].view(torch.float32)
    return out


def compare(tag, a, b):
    if a.dtype == torch.uint8:
        d = (a != b).nonzero().flatten()
        return f"{tag}: {d.numel()} bytes differ" + (f" (first at {int(d[0])}, last {int(d[-1])})" if d.numel() else "")
    d = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
    idx = d.nonzero()
    s = f"{tag}: {int(d.sum())} of {a.numel()} differ"
    if idx.numel():
        s += f", max |diff| {float((a.double() - b.double()).abs()[d].max()):.3e}, first at {idx[0].tolist()}"
    return s


def oerr(gc, gp):
    """relative error against the oracle (the tests' measure) and NaN counts"""
    a, b = gc.cpu().numpy(), gp.cpu().numpy()
    ec = float(np.nanmax(np.abs(a - rc)) / max(1.0, np.abs(rc).max()))
    ep = float(np.nanmax(np.abs(b - rp)) / max(1.0, np.abs(rp).max()))
    return f"oracle rel err cam {ec:.1e} proj {ep:.1e}, NaN {int(np.isnan(a).sum())}/{int(np.isnan(b).sum())}"


# backward scratch regions (bwd_fused.hip plan_bwd / run_bwd): part | acc | cover | prep | misc
plane = n
regions = None
for S in range(1, 400):
    parts = [("part", a256(6 * S * plane * 4)), ("acc", a256(6 * plane * 4)), ("cover", a256(3 * W * 4 + 3 * W * S * 2)),
             ("prep", a256(6 * plane * 4)), ("misc", a256(2 * 512 * 8 + 256))]
    if sum(x for _, x in parts) == NB_B - SB:
        regions, off = {}, SB
        for name, nb in parts:
            regions[name] = (off, off + nb)
            off += nb
        print(f"plan: S = {S}, regions {regions}")
        break
if regions is None:
    print("could not solve the scratch layout", NB_B - SB)


def region_diffs(ws, ref):
    if regions is None:
        return compare("scratch", ws[SB:NB_B], ref[SB:NB_B])
    return "; ".join(compare(k_, ws[lo:hi], ref[lo:hi]) for k_, (lo, hi) in regions.items())


res = []
for _ in range(3):  # references without pollution (preceded by this op's own kernels)
    pollute(False)
    v_ref, wsf_ref = fwd()
    gcg, gpg, wsg = bwd(v_ref)
    gcr, gpr, wsr = bwd(None)
    print("unpolluted: given " + oerr(gcg, gpg) + " | recompute " + oerr(gcr, gpr), flush=True)
    res.append((gcg, gpg, wsg, gcr, gpr, wsr))
gcg_ref, gpg_ref, wsg_ref, gcr_ref, gpr_ref, wsr_ref = res[-1]
print("unpolluted runs identical:", all(torch.equal(r[0], gcg_ref) and torch.equal(r[3], gcr_ref) for r in res))
for trial in range(3):
    pollute(True)
    v, wsf = fwd()
    print(f"[{trial}] after pollution, forward: " + compare("volume", v, v_ref), flush=True)
    pollute(True)
    gc, gp, wsg = bwd(v_ref)
    print(f"[{trial}] after pollution, given-volume backward: {oerr(gc, gp)}; " + region_diffs(wsg, wsg_ref), flush=True)
    pollute(True)
    gc, gp, wsr = bwd(None)
    vol_ws = wsr[NB_B:NB_B + 4 * H * WO * DO].view(torch.float32).view(H, WO, DO)
    print(f"[{trial}] after pollution, recompute backward: {oerr(gc, gp)}; " + compare("recomputed volume", vol_ws, v_ref)
          + "; " + region_diffs(wsr, wsr_ref), flush=True)
    if regions is not None:
        lo, hi = regions["part"]
        a = wsr[lo:hi].view(torch.float32).view(6, -1, H, W)
        b = wsr_ref[lo:hi].view(torch.float32).view(6, -1, H, W)
        d = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
        if d.any():
            t_, s_, y_, x_ = d.nonzero(as_tuple=True)
            print(f"     part diffs: types {sorted(set(t_.tolist()))} slots {sorted(set(s_.tolist()))} rows "
                  f"{sorted(set(y_.tolist()))} cols {sorted(set(x_.tolist()))}; polluted NaN {int(torch.isnan(a).sum())} "
                  f"ref NaN {int(torch.isnan(b).sum())}", flush=True)
        lo, hi = regions["prep"]
        a = wsr[lo:hi].view(torch.float32).view(6, H, W)
        b = wsr_ref[lo:hi].view(torch.float32).view(6, H, W)
        d = a != b
        if d.any():
            t_, y_, x_ = d.nonzero(as_tuple=True)
            print(f"     prep diffs: images {sorted(set(t_.tolist()))} rows {sorted(set(y_.tolist()))} cols "
                  f"{sorted(set(x_.tolist()))}", flush=True)
