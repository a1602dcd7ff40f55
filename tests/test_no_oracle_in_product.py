"""The product path never touches the oracle (test infrastructure) and has no CPU fallback.

* no module of the product packages (custereomatching_amd, custma) imports, loads or
  names anything under oracle/ or /root/reference;
* the HIP library is the only compute backend: every op requires ROCm tensors.
"""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT = ("custereomatching_amd", "custma")


def _product_files():
    for pkg in PRODUCT:
        for dp, _, fs in os.walk(os.path.join(ROOT, pkg)):
            for f in fs:
                if f.endswith((".py", ".hip", ".h", ".cpp")):
                    yield os.path.join(dp, f)


def test_product_never_imports_oracle():
    bad = []
    pat = re.compile(r"(^\s*(from|import)\s+oracle\b)|liborc|zncc_oracle|/root/reference|torch_ref", re.M)
    for f in _product_files():
        if pat.search(open(f, errors="replace").read()):
            bad.append(os.path.relpath(f, ROOT))
    assert not bad, bad


def test_ops_refuse_cpu_tensors():
    import custereomatching_amd as cm

    c = torch.rand(8, 16)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        cm.stereo_matching(c, c, 0, 5)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        cm.stereo_disparity(c, c, 0, 5)
