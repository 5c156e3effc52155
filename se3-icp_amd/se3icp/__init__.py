"""se3icp — MI355X-native SE(3)-ICP registration (host side of libse3icp.so).

Drop-in for kenahm/se3-icp's ``IterativeSE3Registration`` (see registration.py);
the registration itself runs in hand-written HIP kernels for gfx950 (csrc/).
"""
from ._lib import (METHODS, Params, Result, Se3IcpError, default_params, device_count, load,  # noqa: F401
                   method_id, status_string)
from .io import read_ply_xyz, write_ply_xyz  # noqa: F401
from .registration import (DeviceBatchRunner, IterativeSE3Registration, PairResult, PipelinedBatchRunner,  # noqa: F401
                           cli_params,
                           estimate_normals,
                           kitti_params, knn_self, last_kernel_times, set_nn_events, set_profiling, lounge_params,
                           nearest_neighbors,
                           register_batch, register_batch_device, register_batch_traced, toldi_frames)

__all__ = [
    "IterativeSE3Registration", "register_batch", "register_batch_device", "DeviceBatchRunner", "PipelinedBatchRunner", "register_batch_traced", "toldi_frames", "knn_self",
    "estimate_normals", "nearest_neighbors", "default_params", "cli_params", "kitti_params", "lounge_params",
    "read_ply_xyz", "write_ply_xyz", "METHODS", "Se3IcpError",
]
