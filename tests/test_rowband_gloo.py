"""Row-band sharding (custereomatching_amd.rowband) on CPU with the gloo
backend, world sizes 2 and 3.  The band compute is the oracle (injected as
the backend -- test infrastructure); what is under test is the product's
band split, halo exchange and halo reduce: the sharded forward, backward and
disparity must equal the single-device oracle on the whole image."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from tests.golden.inputs import make_pair


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleBackend:
    """Band ops computed by the CPU oracle on the haloed buffer (test only)."""

    @staticmethod
    def _lay(layout, D):
        return (O.FULL, 0) if layout == "full" else (O.WINDOW, D)

    def forward(self, cam, proj, D, k, layout, precision, rows):
        lay, Dl = self._lay(layout, D)
        v = O.forward(cam.numpy(), proj.numpy(), k, layout=lay, D=Dl)
        return torch.from_numpy(v[rows[0]:rows[1]].copy())

    def backward(self, grad, cam, proj, D, k, layout, rows, want_cam, want_proj, vol=None):
        lay, Dl = self._lay(layout, D)
        H, W = cam.shape
        g = np.zeros(O.volume_shape(H, W, lay, Dl), np.float32)
        g[rows[0]:rows[1]] = grad.numpy()
        dc, dp = O.backward_f64(g, cam.numpy(), proj.numpy(), k, layout=lay, D=Dl)
        return (torch.from_numpy(dc) if want_cam else None), (torch.from_numpy(dp) if want_proj else None)

    def disparity(self, cam, proj, D, k, layout, rows):
        v = self.forward(cam, proj, D, k, layout, None, rows).numpy()
        idx, best = O.argmax(v)
        return torch.from_numpy(idx), torch.from_numpy(best)


def _worker(rank, world, port, H, W, k, D, layout, q, pass_h=False, split=None, overlap=False):
    os.environ["CUSTMA_ROWBAND_OVERLAP"] = "1" if overlap else "0"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from custereomatching_amd.rowband import band_bounds, stereo_disparity_rowband, stereo_matching_rowband

        cam, proj = make_pair(H, W, max(D, 1), seed=17)
        b, e = band_bounds(H, world, rank) if split is None else split[rank]
        c = torch.from_numpy(cam[b:e].copy()).requires_grad_(True)
        p = torch.from_numpy(proj[b:e].copy()).requires_grad_(True)
        be = OracleBackend()
        try:
            vol = stereo_matching_rowband(c, p, D, k, layout, backend=be, H=H if pass_h else None)
        except ValueError as ex:  # band thinner than the halo: every rank must raise
            q.put((rank, "ValueError", str(ex)))
            return
        lay, Dl = OracleBackend._lay(layout, D)
        g = np.random.default_rng(5).standard_normal(O.volume_shape(H, W, lay, Dl)).astype(np.float32)
        vol.backward(torch.from_numpy(g[b:e].copy()))
        idx, best = stereo_disparity_rowband(c.detach(), p.detach(), D, k, layout, backend=be)
        q.put((rank, b, e, vol.detach().numpy(), c.grad.numpy(), p.grad.numpy(), idx.numpy()))
    finally:
        dist.destroy_process_group()


def _run(world, H, W, k, D, layout, pass_h=False, split=None, overlap=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, k, D, layout, q, pass_h, split, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,layout,k,overlap", [
    (2, "full", 5, False), (3, "window", 5, False), (2, "window", 5, False), (2, "full", 4, False),
    (3, "window", 6, False), (2, "full", 2, False), (3, "full", 1, False),
    # CUSTMA_ROWBAND_OVERLAP=1: interior rows while the halos are in flight, then the two edges
    (3, "window", 5, True), (2, "full", 4, True), (3, "full", 6, True)])
def test_rowband_matches_single_device(world, layout, k, overlap):
    """Odd k: r halo rows each side; even k: k/2 rows from the rank above, k/2-1 from below."""
    H, W, D = 23, 28, 6
    res = _run(world, H, W, k, D, layout, overlap=overlap)
    cam, proj = make_pair(H, W, max(D, 1), seed=17)
    lay, Dl = OracleBackend._lay(layout, D)
    vol = O.forward(cam, proj, k, layout=lay, D=Dl)
    g = np.random.default_rng(5).standard_normal(O.volume_shape(H, W, lay, Dl)).astype(np.float32)
    rc, rp = O.backward_f64(g, cam, proj, k, layout=lay, D=Dl)
    ridx, _ = O.argmax(vol)
    covered = 0
    for rank, b, e, v, gc, gp, idx in res:
        assert np.array_equal(v, vol[b:e])  # bitwise: same arithmetic, halo rows complete the patches
        assert np.abs(gc - rc[b:e]).max() <= 1e-6 * max(1, np.abs(rc).max())  # fp32 grads
        assert np.abs(gp - rp[b:e]).max() <= 1e-6 * max(1, np.abs(rp).max())
        assert np.array_equal(idx, ridx[b:e])
        covered += e - b
    assert covered == H


@pytest.mark.parametrize("pass_h", [False, True])
def test_rowband_thin_band_raises_on_every_rank(pass_h):
    """H = 9 over 2 ranks at k = 11 (bands 5 and 4 < r = 5): every rank raises
    before any halo exchange (no rank left waiting in batch_isend_irecv)."""
    res = _run(2, 9, 16, 11, 2, "full", pass_h)
    assert [t[1] for t in res] == ["ValueError", "ValueError"]


@pytest.mark.parametrize("pass_h", [False, True])
def test_rowband_custom_split(pass_h):
    """A custom row split (3 / 2 / 4 rows of H = 9, not band_bounds's 3 / 3 / 3) at k = 3: with H
    given, every rank raises (the split check is collective: no rank enters the halo exchange
    alone); without H the custom split runs and matches the single-device result."""
    H, W, D, k = 9, 16, 2, 3
    split = [(0, 3), (3, 5), (5, 9)]
    res = _run(3, H, W, k, D, "full", pass_h, split)
    if pass_h:
        assert [t[1] for t in res] == ["ValueError"] * 3
        return
    cam, proj = make_pair(H, W, D, seed=17)
    vol = O.forward(cam, proj, k, layout=O.FULL, D=0)
    g = np.random.default_rng(5).standard_normal(O.volume_shape(H, W, O.FULL, 0)).astype(np.float32)
    rc, _ = O.backward_f64(g, cam, proj, k, layout=O.FULL, D=0)
    for rank, b, e, v, gc, gp, idx in res:
        assert (b, e) == split[rank]
        assert np.array_equal(v, vol[b:e])
        assert np.abs(gc - rc[b:e]).max() <= 1e-6 * max(1, np.abs(rc).max())


def test_band_bounds_partition():
    from custereomatching_amd.rowband import band_bounds

    for H in (1, 7, 64, 1000):
        for world in (1, 2, 3, 8):
            spans = [band_bounds(H, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == H
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1


def _reinit_worker(rank, port, port2, H, W, k, D, q):
    """world 2 with H given (the RowBandGroup is cached), then destroy and re-init world 2 with the
    ranks swapped: same band height, H and k, so only the group's rank tells the cache entries apart
    -- a RowBandGroup of the old group would exchange halos with the wrong neighbours (ADVICE r5,
    rowband._GROUPS)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    from custereomatching_amd.rowband import band_bounds, stereo_matching_rowband

    cam, proj = make_pair(H, W, D, seed=17)
    be = OracleBackend()
    out = []
    for pt, r in ((port, rank), (port2, 1 - rank)):
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{pt}", rank=r, world_size=2)
        try:
            b, e = band_bounds(H, 2, r)
            v = stereo_matching_rowband(torch.from_numpy(cam[b:e].copy()), torch.from_numpy(proj[b:e].copy()), D, k,
                                        "full", backend=be, H=H)
            out.append((b, e, v.detach().numpy()))
        finally:
            dist.destroy_process_group()
    q.put((rank, out))


def test_rowband_group_cache_after_reinit():
    H, W, D, k = 12, 16, 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, port2 = _free_port(), _free_port()
    procs = [ctx.Process(target=_reinit_worker, args=(r, port, port2, H, W, k, D, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cam, proj = make_pair(H, W, D, seed=17)
    vol = O.forward(cam, proj, k, layout=O.FULL, D=0)
    for rank, out in res:
        for b, e, v in out:
            assert np.array_equal(v, vol[b:e])
