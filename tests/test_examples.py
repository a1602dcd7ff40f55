"""examples/verify.py -- the reference driver's call sequence (examples/verify.py:65-74) on
synthetic captures, through the HIP path, compared with its torch restatement."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_verify_driver_runs_and_agrees(gpu):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "verify.py"), "--H", "66", "--W", "120",
                        "--D", "40", "--k", "15"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout
    assert "fused argmax == torch.max index: True" in out
    assert "fused mask   == torch.where mask: True" in out
    rel = float(out.split("camera grad max |hip - torch| / max|grad| = ")[1].split()[0])
    assert rel <= 1e-5, out
    dv = float(out.split("cost volume max |hip - torch| = ")[1].split()[0])
    assert dv <= 1e-5, out


def test_verify_driver_synthetic_inputs_cpu():
    """The synthetic captures and the torch restatement need no GPU."""
    import importlib.util

    import torch

    spec = importlib.util.spec_from_file_location("ex_verify", os.path.join(ROOT, "examples", "verify.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rgb, proj = mod.synthetic_captures(20, 30, 8)
    assert rgb.shape == (20, 30, 3) and proj.shape == (20, 30) and rgb.dtype.name == "uint8"
    from oracle import oracle as O

    cam = (rgb[:, :, 0] / 255).astype("float32")
    pr = (proj / 255).astype("float32")
    v = mod.torch_zncc(torch.from_numpy(cam).double(), torch.from_numpy(pr).double(), 5).numpy()
    assert abs(v - O.forward_f64(cam, pr, 5)).max() <= 1e-9
