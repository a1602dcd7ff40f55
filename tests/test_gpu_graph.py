"""hipGraph capture (include/custma.h: "nothing is allocated inside a call, so every call is
hipGraph-capturable"): a forward + backward step of the autograd op captured into a
torch.cuda.CUDAGraph and replayed on new inputs equals the eager step bit for bit."""
import numpy as np
import pytest
import torch

from tests.golden.inputs import make_pair

import custereomatching_amd as cm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout,D,k", [("window", 64, 9), ("full", 0, 7), ("window", 40, 6)])
def test_graph_capture_forward_backward_replay(gpu, layout, D, k):
    H, W = 48, 256
    dev = gpu

    def pair(seed):
        c, p = make_pair(H, W, max(D, 16), seed=seed)
        return torch.from_numpy(c).to(dev), torch.from_numpy(p).to(dev)

    cam, proj = pair(11)
    cam.requires_grad_(True)
    proj.requires_grad_(True)
    WO, DO = (W, W) if layout == "full" else (W - D, D + 1)
    g = torch.randn(H, WO, DO, device=dev, generator=torch.Generator(device=dev).manual_seed(12))

    def step():
        vol = cm.stereo_matching(cam, proj, D, k, layout)
        vol.backward(g)
        return vol

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):  # warm-up outside the capture (allocator, library state)
            cam.grad = proj.grad = None
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)

    graph = torch.cuda.CUDAGraph()
    cam.grad = proj.grad = None
    with torch.cuda.graph(graph):
        vol = step()

    new_c, new_p = pair(13)
    new_g = torch.randn(g.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(14))
    with torch.no_grad():
        cam.copy_(new_c)
        proj.copy_(new_p)
        g.copy_(new_g)
    graph.replay()
    torch.cuda.synchronize(dev)

    c2 = new_c.clone().requires_grad_(True)
    p2 = new_p.clone().requires_grad_(True)
    v2 = cm.stereo_matching(c2, p2, D, k, layout)
    v2.backward(new_g)
    torch.cuda.synchronize(dev)
    assert torch.equal(vol, v2)
    assert torch.equal(cam.grad, c2.grad)
    assert torch.equal(proj.grad, p2.grad)
    # and replaying again on the same inputs is deterministic
    graph.replay()
    torch.cuda.synchronize(dev)
    assert torch.equal(cam.grad, c2.grad) and torch.equal(proj.grad, p2.grad)
    assert np.isfinite(cam.grad.cpu().numpy()).all()
