"""Seeded synthetic stereo pairs (SURVEY §8d input recipe).

Projector: U[0,1) speckle.  Camera: the projector shifted left by a
piecewise-constant (per 16-row band) disparity in [0, D), plus N(0, 0.01)
noise, clipped to [0, 1].  Variants:
  textured  -- as above
  smooth    -- speckle box-blurred (low local variance, stresses cancellation)
  quantized -- smooth rounded to x/255 (mirrors examples/verify.py:138-139)
  constant  -- both images 0.5 (every patch flat: cost = eps/sqrt(eps))
  zeros     -- both images 0
"""
from __future__ import annotations

import numpy as np


def _box_blur(x, r):
    if r <= 0:
        return x
    p = np.pad(x, r, mode="reflect")
    c = np.cumsum(np.cumsum(p, 0), 1)
    c = np.pad(c, ((1, 0), (1, 0)))
    k = 2 * r + 1
    H, W = x.shape
    return (c[k:k + H, k:k + W] - c[:H, k:k + W] - c[k:k + H, :W] + c[:H, :W]) / (k * k)


def make_pair(H, W, D, seed=0, kind="textured"):
    rng = np.random.default_rng(seed)
    if kind == "constant":
        a = np.full((H, W), 0.5, np.float32)
        return a.copy(), a.copy()
    if kind == "zeros":
        a = np.zeros((H, W), np.float32)
        return a.copy(), a.copy()
    proj = rng.random((H, W))
    if kind in ("smooth", "quantized"):
        proj = 0.25 + 0.5 * _box_blur(proj, 3)
    disp = np.zeros(H, np.int64)
    for b in range(0, H, 16):
        disp[b:b + 16] = rng.integers(0, max(1, D))
    cam = np.empty_like(proj)
    cols = np.arange(W)
    for h in range(H):
        src = np.clip(cols + disp[h], 0, W - 1)
        cam[h] = proj[h, src]
    cam = cam + rng.normal(0.0, 0.01, size=cam.shape)
    if kind == "quantized":
        cam = np.round(np.clip(cam, 0, 1) * 255) / 255
        proj = np.round(proj * 255) / 255
    cam = np.clip(cam, 0.0, 1.0)
    return cam.astype(np.float32), proj.astype(np.float32)
