"""Does any op read workspace bytes it did not write?  The C ABI is called directly with workspaces
pre-filled with different byte patterns (0x00, 0xFF, 0x7F, random); the outputs must not depend on the
fill.  For the backward's recompute path the fill is also applied per region (statistics, backward
scratch, recomputed volume) to localise a dependence.  Usage: python scripts/diag_ws.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tests.golden.inputs import make_pair  # noqa: E402

from custereomatching_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.lib


def a256(n):
    return (n + 255) & ~255


def fill_ws(nb, fill, regions=None):
    ws = torch.zeros(nb + 256, dtype=torch.uint8, device=dev)
    ws = ws[(-ws.data_ptr()) % 256:][:nb]  # 256-byte aligned like the caching allocator's blocks
    g = torch.Generator(device=dev).manual_seed(5)
    for lo, hi in (regions or [(0, nb)]):
        if fill == "rand":
            ws[lo:hi] = torch.randint(0, 256, (hi - lo,), dtype=torch.uint8, device=dev, generator=g)
        else:
            ws[lo:hi] = fill
    return ws


def stream():
    return torch.cuda.current_stream(dev).cuda_stream


def run_case(H, W, k, D, layout, kind, dt=torch.float32):
    lay = _lib.LAYOUT_WINDOW if layout == "window" else _lib.LAYOUT_FULL
    Dl = D if layout == "window" else 0
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    olay = O.WINDOW if layout == "window" else O.FULL
    g = np.random.default_rng(7).standard_normal(O.volume_shape(H, W, olay, Dl)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=olay, D=Dl)
    c = torch.from_numpy(cam).to(dev).to(dt)
    p = torch.from_numpy(proj).to(dev).to(dt)
    gd = torch.from_numpy(g).to(dev)
    code = _lib.F16 if dt == torch.float16 else _lib.F32
    WO, DO = _lib.volume_dims(H, W, lay, Dl)
    sb = 2 * a256(H * W * 20) + a256(4 * (H // 8 + 1))
    nb_f = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_FORWARD)
    nb_b = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_BACKWARD)
    nb_r = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_BACKWARD_RECOMPUTE)
    tag = f"{layout} {H}x{W} k{k} D{D} {kind}"

    def fwd(ws):
        out = torch.full((H, WO, DO), float("nan"), device=dev)
        _lib.check(L.custma_forward_band(c.data_ptr(), p.data_ptr(), code, H, W, k, lay, Dl, _lib.FAST, 0, H,
                                         out.data_ptr(), ws.data_ptr(), ws.numel(), stream()), "fwd")
        torch.cuda.synchronize()
        return out

    def bwd(ws, vol):
        gc = torch.full((H, W), float("nan"), device=dev)
        gp = torch.full((H, W), float("nan"), device=dev)
        _lib.check(L.custma_backward_band(gd.data_ptr(), vol.data_ptr() if vol is not None else None, c.data_ptr(),
                                          p.data_ptr(), code, H, W, k, lay, Dl, 0, H, gc.data_ptr(), gp.data_ptr(),
                                          ws.data_ptr(), ws.numel(), stream()), "bwd")
        torch.cuda.synchronize()
        return gc.cpu().numpy(), gp.cpu().numpy()

    def err(x):
        return max(np.abs(x[0] - rc).max() / max(1.0, np.abs(rc).max()), np.abs(x[1] - rp).max() / max(1.0, np.abs(rp).max()))

    fills = [0, 0xFF, 0x7F, "rand"]
    v0 = fwd(fill_ws(nb_f, 0))
    fdiff = [bool(not torch.equal(fwd(fill_ws(nb_f, f)), v0)) for f in fills[1:]]
    gv = [err(bwd(fill_ws(nb_b, f), v0)) for f in fills]
    gr = [err(bwd(fill_ws(nb_r, f), None)) for f in fills]
    print(f"{tag}: fwd depends on fill {fdiff}; given-volume rel err {['%.1e' % e for e in gv]}; "
          f"recompute rel err {['%.1e' % e for e in gr]}", flush=True)
    if max(gr) > 1e-5 or max(gv) > 1e-5 or any(fdiff):
        regions = {"stats": (0, sb), "bwd": (sb, nb_b), "volume": (nb_b, nb_r)}
        for name, rg in regions.items():
            e = [err(bwd(fill_ws(nb_r, f, [rg]), None)) for f in fills[1:]]
            print(f"   recompute, only {name} [{rg[0]}, {rg[1]}) filled: {['%.1e' % x for x in e]}", flush=True)
        # which pixels
        bad = bwd(fill_ws(nb_r, 0x7F), None)
        d = np.abs(bad[0] - rc)
        ys, xs = np.nonzero(d > 1e-5 * max(1.0, np.abs(rc).max()))
        print(f"   camera-grad pixels over the bar: rows {sorted(set(ys.tolist()))} cols {sorted(set(xs.tolist()))}")


def pollute_then(tag, fn, H=18, W=36, k=4, D=10, kind="textured"):
    """Run another op first (it leaves its own LDS / register / memory contents behind), then the window
    k = 4 backward through the autograd-free wrapper, recompute path, 3 times."""
    import custereomatching_amd as cm
    fn()
    torch.cuda.synchronize()
    cam, proj = make_pair(H, W, max(D, 1), seed=31, kind=kind)
    g = np.random.default_rng(7).standard_normal(O.volume_shape(H, W, O.WINDOW, D)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=O.WINDOW, D=D)
    c, p, gd = (torch.from_numpy(x).to(dev) for x in (cam, proj, g))
    errs = []
    for _ in range(3):
        gc, gp = cm.cost_volume_backward(gd, c, p, k, "window", D, camera_grad=True, projector_grad=True)
        torch.cuda.synchronize()
        errs.append(float(np.abs(gc.cpu().numpy() - rc).max() / max(1.0, np.abs(rc).max())))
    print(f"after {tag}: recompute rel err {['%.1e' % e for e in errs]}", flush=True)


if __name__ == "__main__":
    import custereomatching_amd as cm
    from tests.test_gpu_parity import BWD_CASES
    for case in BWD_CASES:
        for layout in ("window", "full"):
            run_case(*case[:4], layout, case[4])
    from bench import synth_pair
    c3, p3 = synth_pair(2048, 2048, 256, 5, "cuda", torch.float16)
    pollute_then("nothing", lambda: None)
    pollute_then("C3 fp16 window forward", lambda: cm.cost_volume_forward(c3, p3, 256, 11, "window", "fast"))
    pollute_then("C3 fp16 window disparity", lambda: cm.stereo_disparity(c3, p3, 256, 11, "window"))
    pollute_then("C3 fp16 exact k=19 forward", lambda: cm.cost_volume_forward(c3[:256].contiguous(), p3[:256].contiguous(), 256, 19, "window", "exact"))
    c1, p1 = synth_pair(256, 512, 64, 6, "cuda", torch.float32)
    pollute_then("256x512 window k=9 backward", lambda: cm.cost_volume_backward(
        torch.ones(256, 448, 65, device=dev), c1, p1, 9, "window", 64, projector_grad=True))
    pollute_then("nothing again", lambda: None)
