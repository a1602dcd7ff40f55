"""``custma.src`` -- the reference's pybind extension module surface
(custma/src/bindings.cpp:4-7), backed by the HIP C ABI.

    stereo_matching_forward(camera, projector, D, kernel_size) -> Tensor
    stereo_matching_backward(cost_volume_grad, camera, projector, kernel_size) -> camera grad
"""
from custereomatching_amd.stereo_matching_wrapper import cost_volume_backward, cost_volume_forward


def stereo_matching_forward(camera, projector, D, kernel_size):
    return cost_volume_forward(camera, projector, D, kernel_size)


def stereo_matching_backward(cost_volume_grad, camera, projector, kernel_size):
    gc, _ = cost_volume_backward(cost_volume_grad, camera, projector, kernel_size)
    return gc
