"""Generate golden vectors from the REFERENCE's own torch path.

Run in the build container (needs /root/reference; the GPU box never runs it):
    python tests/golden/gen_golden.py

It imports /root/reference/examples/verify.py (module-level imports of cv2 and
custma are satisfied by empty stand-in modules; the functions used --
``extract_image_patch_pytoch`` (verify.py:18-28) and
``torch_cost_volume_backward`` (verify.py:81-133) -- touch neither, except
``custma.Timer`` which is replaced by a no-op context manager) and calls
``torch_cost_volume_backward`` on seeded synthetic inputs in fp32 and fp64.
The reference's CUDA extension cannot be built here (no nvcc / CUDA headers),
so the torch path is the executable reference; the C oracle restating the
CUDA arithmetic is checked against these vectors in tests/test_oracle.py.

Outputs (data only -- inputs and expected outputs): tests/golden/*.npz
"""
from __future__ import annotations

import contextlib
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))

from tests.golden.inputs import make_pair  # noqa: E402


def load_reference_verify():
    cv2 = types.ModuleType("cv2")
    custma = types.ModuleType("custma")

    class Timer(contextlib.ContextDecorator):
        def __init__(self, *a, **k):
            pass

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    custma.Timer = Timer
    saved = {n: sys.modules.get(n) for n in ("cv2", "custma")}
    sys.modules["cv2"] = cv2
    sys.modules["custma"] = custma
    try:
        spec = importlib.util.spec_from_file_location("ref_verify", os.path.join(REF, "examples", "verify.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for n, m in saved.items():
            if m is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = m
    return mod


def ref_run(mod, cam, proj, k, dtype):
    c = torch.tensor(cam, dtype=dtype)
    p = torch.tensor(proj, dtype=dtype).requires_grad_(True)
    vol, cg = mod.torch_cost_volume_backward(c, p, k, 50.0, 0.6)
    return vol.detach().numpy(), cg.detach().numpy(), p.grad.detach().numpy()


CASES = [
    # name, H, W, k, D, kind
    ("tiny_16x24_k5", 16, 24, 5, 8, "textured"),
    ("tex_24x48_k5", 24, 48, 5, 16, "textured"),
    ("smooth_24x48_k5", 24, 48, 5, 16, "smooth"),
    ("quant_24x48_k5", 24, 48, 5, 16, "quantized"),
    ("const_24x48_k5", 24, 48, 5, 16, "constant"),
    ("zeros_24x48_k5", 24, 48, 5, 16, "zeros"),
    ("tex_20x48_k9", 20, 48, 9, 16, "textured"),
    ("tex_20x40_k7", 20, 40, 7, 12, "textured"),
    ("row_1x32_k5", 1, 32, 5, 8, "textured"),
    ("tall_40x12_k11", 40, 12, 11, 4, "textured"),
]


def main():
    torch.set_num_threads(os.cpu_count() or 1)
    mod = load_reference_verify()
    for name, H, W, k, D, kind in CASES:
        cam, proj = make_pair(H, W, D, seed=0, kind=kind)
        v32, cg32, pg32 = ref_run(mod, cam, proj, k, torch.float32)
        v64, cg64, pg64 = ref_run(mod, cam, proj, k, torch.float64)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), cam=cam, proj=proj, k=k, D=D,
                            vol32=v32.astype(np.float32), vol64=v64.astype(np.float32),
                            cg32=cg32, cg64=cg64, pg32=pg32, pg64=pg64)
        print(name, v32.shape)

    # The verify config (BASELINE configs[0]): 128x256, D=32, window 5.
    H, W, k, D = 128, 256, 5, 32
    for kind in ("textured", "quantized"):
        cam, proj = make_pair(H, W, D, seed=0, kind=kind)
        v32, cg32, pg32 = ref_run(mod, cam, proj, k, torch.float32)
        v64, cg64, pg64 = ref_run(mod, cam, proj, k, torch.float64)
        srt = np.sort(v64, axis=-1)
        gap = (srt[..., -1] - srt[..., -2]).astype(np.float32)
        rng = np.random.default_rng(1)
        sample = rng.integers(0, v32.size, 4096)
        np.savez_compressed(os.path.join(OUT, f"verify_{kind}_128x256_k5.npz"), cam=cam, proj=proj,
                            k=k, D=D,
                            argmax32=v32.argmax(-1).astype(np.int16),
                            argmax64=v64.argmax(-1).astype(np.int16),
                            max32=v32.max(-1), max64=v64.max(-1), gap64=gap,
                            sample_idx=sample, sample32=v32.reshape(-1)[sample],
                            sample64=v64.reshape(-1)[sample],
                            cg32=cg32, cg64=cg64, pg64=pg64)
        print("verify", kind)


if __name__ == "__main__":
    main()
