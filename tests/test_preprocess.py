"""Image preprocessing (examples/verify.py:138-142, 148) through the C ABI.

CPU: the oracle restatement equals torch's own float64 -> float32 / float16
conversion of numpy's ``/ 255`` for all 256 byte values (so rounding the
float32 result to float16 on the device is exact), and argument errors are
raised before any launch.  GPU: bit-identical to the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O


def test_oracle_matches_torch_conversion_for_every_byte():
    u = np.arange(256, dtype=np.uint8).reshape(16, 16)
    for dt, tdt in ((np.float32, torch.float32), (np.float16, torch.float16)):
        want = torch.tensor(u / 255, dtype=tdt).numpy()
        got = O.image_u8_to_unit(u, dtype=dt)
        assert np.array_equal(got.view(np.uint16 if dt == np.float16 else np.uint32),
                              want.view(np.uint16 if dt == np.float16 else np.uint32))
    # float32 then float16 == direct float64 -> float16 for every byte value
    a = (u / 255).astype(np.float16)
    b = (u / 255).astype(np.float32).astype(np.float16)
    assert np.array_equal(a.view(np.uint16), b.view(np.uint16))


def test_entry_point_validates_before_launch():
    from custereomatching_amd import _lib
    L = _lib.lib
    assert L.custma_image_u8_to_unit(None, 4, 4, 3, 3, _lib.F32, None, None) == _lib.E_ARG
    assert L.custma_image_u8_to_unit(None, 4, 4, 0, 0, _lib.F32, None, None) == _lib.E_ARG
    assert L.custma_image_u8_to_unit(None, 4, 4, 1, 0, 7, None, None) != 0
    assert L.custma_image_u8_to_unit(None, 4, 4, 1, 0, _lib.F32, None, None) == _lib.E_NULL
    assert L.custma_image_u8_to_unit(None, 0, 4, 1, 0, _lib.F32, None, None) == 0


def test_python_wrapper_rejects_cpu_tensor():
    import custereomatching_amd as cm
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        cm.image_u8_to_unit(torch.zeros(4, 4, dtype=torch.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,channel", [((37, 53, 3), 0), ((37, 53, 3), 2), ((64, 40), 0), ((1, 1, 4), 3),
                                           ((512, 640, 3), 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_gpu_bit_identical(shape, channel, dtype):
    import custereomatching_amd as cm
    img = np.random.default_rng(3).integers(0, 256, size=shape, dtype=np.uint8)
    got = cm.image_u8_to_unit(torch.from_numpy(img).cuda(), channel, dtype).cpu().numpy()
    want = O.image_u8_to_unit(img, channel, np.float32 if dtype == torch.float32 else np.float16)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32 if dtype == torch.float32 else np.uint16),
                          want.view(np.uint32 if dtype == torch.float32 else np.uint16))


@pytest.mark.gpu
def test_gpu_feeds_the_path():
    # preprocessed images go straight into the op (the driver's rgb[:, :, 0] / proj)
    import custereomatching_amd as cm
    rng = np.random.default_rng(4)
    rgb = rng.integers(0, 256, size=(24, 48, 3), dtype=np.uint8)
    prj = rng.integers(0, 256, size=(24, 48), dtype=np.uint8)
    cam = cm.image_u8_to_unit(torch.from_numpy(rgb).cuda(), 0)
    proj = cm.image_u8_to_unit(torch.from_numpy(prj).cuda(), 0)
    vol = cm.stereo_matching(cam, proj, 8, 5)
    ref = O.forward(O.image_u8_to_unit(rgb, 0), O.image_u8_to_unit(prj, 0), 5)
    assert np.abs(vol.cpu().numpy() - ref).max() <= O.cost_error_bound(5)
