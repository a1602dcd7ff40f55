#!/usr/bin/env python3
"""Synthetic-input counterpart of the reference driver examples/verify.py.

The reference driver reads two PNG captures with cv2 (not shipped with the
reference), runs its CUDA op and its torch path, and stops at an ipdb prompt
(examples/verify.py:136-156).  This driver keeps the op-level call sequence
of its `cuda_cost_volume_backward` (verify.py:65-74) unchanged:

    cost_volume = custma.stereo_matching(camera.contiguous(), projector.contiguous(), 200, kernel_size)
    cost_volume.backward(torch.ones_like(cost_volume))
    cost_volume_max, _ = torch.max(cost_volume.detach().contiguous().reshape(H * W, -1), dim=-1)
    cost_volume_mask = torch.where(cost_volume_max > threshold, ones, zeros)

on synthetic 8-bit images of the driver's size (H, W, D = 330, 422, 200,
kernel_size = 15, verify.py:10-13) preprocessed the driver's way (uint8 / 255,
camera = channel 0, verify.py:138-142, 148), times it next to a plain torch
restatement of the same ZNCC (patches, bmm, autograd -- the driver's torch
path), and prints the differences instead of dropping into a debugger.  It
also runs the fused disparity / soft-argmax / mask pass that needs no volume.

Usage: python examples/verify.py [--H 330 --W 422 --D 200 --k 15] [--no-torch]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custma  # noqa: E402  (the drop-in package; custereomatching_amd underneath)
import custereomatching_amd as cm  # noqa: E402


def synthetic_captures(H, W, D, seed=0):
    """uint8 stand-ins for the driver's two PNGs: a speckle projector pattern and a
    3-channel camera image that sees it shifted by a per-band disparity, plus noise."""
    rng = np.random.default_rng(seed)
    proj = rng.integers(0, 256, size=(H, W), dtype=np.uint8)
    shift = np.repeat(rng.integers(0, max(1, D), size=(H + 31) // 32), 32)[:H]
    cols = np.clip(np.arange(W)[None, :] + shift[:, None], 0, W - 1)
    cam = np.take_along_axis(proj.astype(np.int16), cols, axis=1) + rng.integers(-6, 7, size=(H, W))
    cam = np.clip(cam, 0, 255).astype(np.uint8)
    rgb = np.stack([cam, cam // 2, 255 - cam], axis=-1)  # channel 0 is the one the driver uses
    return rgb, proj


def torch_zncc(camera, projector, k):
    """The driver's torch path in its own words: zero-padded k x k patches of both images,
    centred, E = bmm over the taps, cost = (E + eps) / sqrt(Ex2 Ey2 + eps) for every
    projector column of the row ([H, W, W]); differentiable."""
    o, a = k // 2, k - 1 - k // 2

    def taps(img):
        x = F.pad(img[None, None], (o, a, o, a))
        cols = F.unfold(x, kernel_size=k)  # [1, k*k, H*W], tap order (i, j)
        H, W = img.shape
        return cols[0].t().reshape(H, W, k * k)

    pc, pp = taps(camera), taps(projector)
    pc = pc - pc.mean(-1, keepdim=True)
    pp = pp - pp.mean(-1, keepdim=True)
    e = torch.bmm(pc, pp.transpose(1, 2))
    x2 = (pc * pc).sum(-1)[..., None]
    y2 = (pp * pp).sum(-1)[:, None, :]
    return (e + 1e-8) / torch.sqrt(x2 * y2 + 1e-8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=330)
    ap.add_argument("--W", type=int, default=422)
    ap.add_argument("--D", type=int, default=200)
    ap.add_argument("--k", type=int, default=15)
    ap.add_argument("--beta", type=float, default=50.0)
    ap.add_argument("--threshold", type=float, default=0.6)
    ap.add_argument("--no-torch", action="store_true", help="skip the torch restatement")
    args = ap.parse_args()
    H, W, D, k = args.H, args.W, args.D, args.k
    dev = torch.device("cuda")

    rgb_u8, proj_u8 = synthetic_captures(H, W, D)
    # preprocessing as the driver does it (verify.py:138-142): uint8 / 255 -> float32 on the GPU;
    # the same on the device through the library's fused conversion
    rgb = torch.tensor(rgb_u8 / 255, dtype=torch.float32).to(dev)
    proj = torch.tensor(proj_u8 / 255, dtype=torch.float32).to(dev)
    cam_native = cm.image_u8_to_unit(torch.from_numpy(rgb_u8).to(dev), channel=0)
    assert torch.equal(cam_native, rgb[:, :, 0]), "device preprocessing differs from numpy's uint8 / 255"

    camera = rgb[:, :, 0].contiguous()
    camera.requires_grad_(True)
    torch.cuda.synchronize()
    with custma.Timer("hip forward time: {:.6f}s"):
        cost_volume = custma.stereo_matching(camera.contiguous(), proj.contiguous(), 200, k)
        torch.cuda.synchronize()
    with custma.Timer("hip backward time: {:.6f}s"):
        cost_volume.backward(torch.ones_like(cost_volume))
        torch.cuda.synchronize()
    print("Cost Volume shape:", tuple(cost_volume.shape))
    cost_volume_max, cost_volume_argmax = torch.max(cost_volume.detach().contiguous().reshape(H * W, -1), dim=-1)
    cost_volume_max = cost_volume_max.reshape(H, W)
    cost_volume_mask = torch.where(cost_volume_max > args.threshold, torch.ones_like(cost_volume_max),
                                   torch.zeros_like(cost_volume_max))
    print(f"mask: {int(cost_volume_mask.sum())} of {H * W} pixels above {args.threshold}")

    # fused: argmax, best, soft-argmax and mask without the [H, W, W] volume
    with custma.Timer("hip fused disparity time: {:.6f}s"):
        idx, best, soft, mask = cm.stereo_disparity_soft(camera.detach(), proj, D, k, "full", args.beta,
                                                         args.threshold)
        torch.cuda.synchronize()
    print("fused argmax == torch.max index:", bool(torch.equal(idx.reshape(-1), cost_volume_argmax)))
    print("fused mask   == torch.where mask:", bool(torch.equal(mask, cost_volume_mask)))
    ref_soft = cm.soft_argmax(cost_volume.detach(), args.beta)
    print(f"fused soft-argmax vs softmax over the volume: max |diff| {float((soft - ref_soft).abs().max()):.3e}")

    if not args.no_torch:
        cam_t = rgb[:, :, 0].contiguous().clone().requires_grad_(True)
        with custma.Timer("torch forward+backward time: {:.6f}s"):
            vol_t = torch_zncc(cam_t, proj, k)
            vol_t.backward(torch.ones_like(vol_t))
            torch.cuda.synchronize()
        dv = float((vol_t.detach() - cost_volume.detach()).abs().max())
        g, gt = camera.grad, cam_t.grad
        rel = float((g - gt).abs().max()) / max(1.0, float(gt.abs().max()))
        print(f"cost volume max |hip - torch| = {dv:.3e}")
        print(f"camera grad max |hip - torch| / max|grad| = {rel:.3e}")
        print(camera.grad)
        print(cam_t.grad)


if __name__ == "__main__":
    main()
