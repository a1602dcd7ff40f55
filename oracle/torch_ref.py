"""PyTorch CPU restatement of the reference's torch path -- TEST INFRASTRUCTURE ONLY.

Restates examples/verify.py:18-28 (``extract_image_patch_pytoch``: zero pad,
unfold columns then rows, [H, W, k, k] patches) and :81-133
(``torch_cost_volume_backward``: centre, EXY = bmm, EX2/EY2, cost =
(EXY + eps) / sqrt(EX2 * EY2 + eps), autograd backward).  This is "the repo's
Python/CPU fallback" that bench.py times as ``cpu_baseline`` (kind "port").

``row_chunk`` processes output rows in bands with a k//2 halo; rows are
independent (output row h reads input rows h-r..h+r only), so the arithmetic
per voxel is unchanged and memory stays bounded at large sizes.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS = 1e-8  # examples/verify.py:112


def patches(img: torch.Tensor, k: int) -> torch.Tensor:
    """[H, W] -> [H, W, k*k] zero-padded patches, tap order (i, j) row-major.

    Taps sit at offsets -k//2 .. k-1-k//2 (stereo_matching_kernel.cu:44,60); for
    odd k that is verify.py:26's symmetric pad, for even k the reference's CUDA
    kernel (verify.py's symmetric pad would give H+1 patches there)."""
    o = k // 2
    a = k - 1 - o
    x = F.pad(img[None, None], (o, a, o, a), mode="constant", value=0.0)
    x = x.unfold(3, k, 1).unfold(2, k, 1).permute(0, 1, 2, 3, 5, 4)  # [1,1,H,W,k,k]
    H, W = img.shape
    return x.reshape(H, W, k * k)


def cost_volume(cam: torch.Tensor, proj: torch.Tensor, k: int) -> torch.Tensor:
    """Full [H, W, W] ZNCC volume, differentiable (verify.py:107-120)."""
    pc = patches(cam, k)
    pp = patches(proj, k)
    pc = pc - pc.mean(dim=-1, keepdim=True)
    pp = pp - pp.mean(dim=-1, keepdim=True)
    exy = torch.bmm(pc, pp.transpose(1, 2))
    ex2 = (pc * pc).sum(-1, keepdim=True)
    ey2 = (pp * pp).sum(-1).unsqueeze(-2)
    return (exy + EPS) / torch.sqrt(ex2 * ey2 + EPS)


def window_cost_volume(cam: torch.Tensor, proj: torch.Tensor, k: int, D: int, block: int = 256) -> torch.Tensor:
    """Window layout [H, W-D, D+1], out[h, w, s] = full[h, w, w+s]: the same centred
    patches, EXY by bmm and ZNCC as cost_volume, with the bmm taken per block of
    `block` camera columns against the block + D projector columns it can reach and
    the window's diagonals read out of each product (the full [W, W] bmm would
    compute W / (D+1) times more than the window holds)."""
    pc = patches(cam, k)
    pp = patches(proj, k)
    pc = pc - pc.mean(dim=-1, keepdim=True)
    pp = pp - pp.mean(dim=-1, keepdim=True)
    H, W = cam.shape
    WO = W - D
    ex2 = (pc * pc).sum(-1)
    ey2 = (pp * pp).sum(-1)
    outs = []
    for w0 in range(0, WO, block):
        b = min(block, WO - w0)
        exy = torch.bmm(pc[:, w0:w0 + b], pp[:, w0:w0 + b + D].transpose(1, 2))  # [H, b, b + D]
        # diagonal band: band[h, w, s] = exy[h, w, w + s]
        band = exy.as_strided((H, b, D + 1), (exy.stride(0), exy.stride(1) + 1, 1), exy.storage_offset())
        den = torch.sqrt(ex2[:, w0:w0 + b, None] * ey2[:, w0:w0 + b + D].unfold(1, D + 1, 1) + EPS)
        outs.append((band + EPS) / den)
    return torch.cat(outs, dim=1)


def forward_backward(cam, proj, k, grad=None, proj_grad=True, row_chunk=None, layout="full", D=0):
    """Returns (volume, camera_grad, projector_grad) on CPU.

    grad=None means ones (verify.py:123).  With row_chunk the volume is not
    returned (None) and gradients are accumulated band by band.  layout="window"
    uses window_cost_volume.
    """
    vol_fn = cost_volume if layout == "full" else (lambda c, p, kk: window_cost_volume(c, p, kk, D))
    H, W = cam.shape
    o, a_ = k // 2, k - 1 - k // 2  # halo rows above / below a band
    if row_chunk is None or row_chunk >= H:
        c = cam.detach().clone().requires_grad_(True)
        p = proj.detach().clone().requires_grad_(proj_grad)
        v = vol_fn(c, p, k)
        v.backward(torch.ones_like(v) if grad is None else grad)
        return v.detach(), c.grad, (p.grad if proj_grad else None)
    gc = torch.zeros_like(cam)
    gp = torch.zeros_like(proj)
    for h0 in range(0, H, row_chunk):
        h1 = min(H, h0 + row_chunk)
        a0, a1 = max(0, h0 - o), min(H, h1 + a_)
        c = cam[a0:a1].detach().clone().requires_grad_(True)
        p = proj[a0:a1].detach().clone().requires_grad_(proj_grad)
        # Rows outside the band that exist in the full image are present as halo, so only
        # true image borders are zero padded; the band's own (wrong) edge padding only
        # feeds volume rows outside h0..h1, which are dropped.
        v = vol_fn(c, p, k)[h0 - a0:h1 - a0]
        g = torch.ones_like(v) if grad is None else grad[h0:h1]
        v.backward(g)
        gc[a0:a1] += c.grad
        if proj_grad:
            gp[a0:a1] += p.grad
    return None, gc, (gp if proj_grad else None)


def forward_only(cam, proj, k, row_chunk=None):
    """Forward volume without autograd (for CPU forward timing)."""
    with torch.no_grad():
        if row_chunk is None or row_chunk >= cam.shape[0]:
            return cost_volume(cam, proj, k)
        H = cam.shape[0]
        o, a_ = k // 2, k - 1 - k // 2
        outs = []
        for h0 in range(0, H, row_chunk):
            h1 = min(H, h0 + row_chunk)
            a0, a1 = max(0, h0 - o), min(H, h1 + a_)
            outs.append(cost_volume(cam[a0:a1], proj[a0:a1], k)[h0 - a0:h1 - a0])
        return torch.cat(outs)
