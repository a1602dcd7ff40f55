"""Row-band sharding composed end to end on the GPU: the HIP band kernels
(HipBackend, the product's default) + the halo exchange / halo reduce of
custereomatching_amd.rowband, world size 2 on one MI355X, the halo staged
through host memory over gloo (the 8-GPU runs use nccl = RCCL over xGMI, which
takes the same code path minus the staging).  The sharded volume, both image
gradients and the disparity must equal the single-device HIP results."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.golden.inputs import make_pair

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, H, W, k, D, layout, q, backend="gloo"):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = rank if backend == "nccl" else 0  # nccl: one GPU per rank (RCCL over xGMI)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from custereomatching_amd.rowband import band_bounds, stereo_disparity_rowband, stereo_matching_rowband

        cam, proj = make_pair(H, W, D, seed=41)
        b, e = band_bounds(H, world, rank)
        c = torch.from_numpy(cam[b:e].copy()).cuda().requires_grad_(True)
        p = torch.from_numpy(proj[b:e].copy()).cuda().requires_grad_(True)
        vol = stereo_matching_rowband(c, p, D, k, layout, H=H)
        gen = torch.Generator(device="cuda").manual_seed(42)
        g = torch.randn((H,) + tuple(vol.shape[1:]), generator=gen, device="cuda")
        vol.backward(g[b:e])
        idx, best = stereo_disparity_rowband(c.detach(), p.detach(), D, k, layout, H=H)
        torch.cuda.synchronize()
        q.put((rank, b, e, vol.detach().cpu().numpy(), c.grad.cpu().numpy(), p.grad.cpu().numpy(),
               idx.cpu().numpy(), best.cpu().numpy()))
    except Exception as ex:  # surface the failure instead of a queue timeout
        q.put((rank, "error", repr(ex)))
    finally:
        dist.destroy_process_group()


def _run_and_compare(gpu, layout, D, k, backend):
    import custereomatching_amd as cm

    H, W, world = 70, 160, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, k, D, layout, q, backend)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
    for t in res:
        assert t[1] != "error", t[2]
    cam, proj = make_pair(H, W, max(D, 1), seed=41)
    c = torch.from_numpy(cam).to(gpu).requires_grad_(True)
    p = torch.from_numpy(proj).to(gpu).requires_grad_(True)
    vol = cm.stereo_matching(c, p, D, k, layout)
    gen = torch.Generator(device=gpu).manual_seed(42)
    g = torch.randn(tuple(vol.shape), generator=gen, device=gpu)
    vol.backward(g)
    idx, best = cm.stereo_disparity(c.detach(), p.detach(), D, k, layout)
    v, gc, gp = vol.detach().cpu().numpy(), c.grad.cpu().numpy(), p.grad.cpu().numpy()
    idx, best = idx.cpu().numpy(), best.cpu().numpy()
    covered = 0
    for rank, b, e, vb, gcb, gpb, ib, bb in res:
        assert np.array_equal(vb, v[b:e])  # same kernels, the halo completes the patches
        assert np.abs(gcb - gc[b:e]).max() <= 1e-5 * max(1.0, np.abs(gc).max())
        assert np.abs(gpb - gp[b:e]).max() <= 1e-5 * max(1.0, np.abs(gp).max())
        assert np.array_equal(ib, idx[b:e]) and np.array_equal(bb, best[b:e])
        covered += e - b
    assert covered == H


@pytest.mark.parametrize("layout,D,k", [("full", 0, 9), ("window", 48, 11), ("window", 20, 4)])
def test_rowband_hip_backend_matches_single_device(gpu, layout, D, k):
    _run_and_compare(gpu, layout, D, k, "gloo")


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL over xGMI between them)")
@pytest.mark.parametrize("layout,D,k", [("full", 0, 9), ("window", 48, 11)])
def test_rowband_nccl_two_gpus(gpu, layout, D, k):
    """The transport bench.py uses at N > 1: nccl (RCCL), one rank per GPU, halos device to device."""
    _run_and_compare(gpu, layout, D, k, "nccl")
