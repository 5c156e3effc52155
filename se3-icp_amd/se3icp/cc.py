"""Metrics and pose files of the reference's benchmark drivers (include/se3icp_cc.h).

Python mirror of namespace `cc` (src/cc.cpp) plus the drivers' local helpers
(avgEulError, examples/benchmark_lounge.cpp:14-81; KITTI pose file,
examples/benchmark_kitti.cpp:72-98; Redwood .log RGBDTrajectory,
examples/benchmark_lounge.cpp:99-140).  Host code in libse3icp.so; no GPU needed.
`compute_corrs_with_gt` runs the 1-NN on the GPU (se3icp_nn), like the reference's
KDTreeFlann search (cc.cpp:112-140).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int32)
_SIGS = {
    "se3icp_cc_rot_3d": (None, [C.c_double, C.c_double, C.c_double, _D]),
    "se3icp_cc_angular_error_so3": (C.c_double, [_D, _D]),
    "se3icp_cc_angular_error_so3_alt": (C.c_double, [_D, _D]),
    "se3icp_cc_error_filterreg": (C.c_double, [_D, C.c_int64, _D, _D]),
    "se3icp_cc_rot2euler": (None, [_D, _D]),
    "se3icp_cc_avg_eul_error": (C.c_double, [_D, _D]),
    "se3icp_cc_evaluate_lrf_quality": (C.c_double, [_D, _D, _D, _I, C.c_int64]),
    "se3icp_cc_evaluate_trajectory": (C.c_int, [_D, _D, C.c_int64, _D]),
    "se3icp_cc_read_trajectory": (C.c_int64, [C.c_char_p, _D, C.c_int64]),
    "se3icp_cc_read_kitti_poses": (C.c_int64, [C.c_char_p, _D, C.c_int64]),
    "se3icp_cc_read_redwood_log": (C.c_int64, [C.c_char_p, _D, _I, C.c_int64]),
    "se3icp_cc_write_trajectory": (C.c_int, [C.c_char_p, _D, C.c_int64]),
    "se3icp_cc_write_redwood_log": (C.c_int, [C.c_char_p, _D, _I, C.c_int64]),
}
_ready = False


def _L():
    global _ready
    L = _lib.load()
    if not _ready:
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _ready = True
    return L


def _d(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a, a.ctypes.data_as(_D)


def rot_3d(roll: float, pitch: float, yaw: float) -> np.ndarray:
    """cc::rot_3d (cc.cpp:21-29): Rz(yaw) Ry(pitch) Rx(roll)."""
    R = np.zeros(9)
    _L().se3icp_cc_rot_3d(roll, pitch, yaw, R.ctypes.data_as(_D))
    return R.reshape(3, 3)


def angular_error_so3(R1, R2) -> float:
    """cc::angularErrorSO3 (cc.cpp:32-37), degrees."""
    a, pa = _d(R1, (3, 3))
    b, pb = _d(R2, (3, 3))
    return float(_L().se3icp_cc_angular_error_so3(pa, pb))


def angular_error_so3_alt(R1, R2) -> float:
    """cc::angularErrorSO3_alt (cc.cpp:50-60), degrees."""
    a, pa = _d(R1, (3, 3))
    b, pb = _d(R2, (3, 3))
    return float(_L().se3icp_cc_angular_error_so3_alt(pa, pb))


def error_filterreg(src_xyz, T_gt, T_est) -> float:
    """cc::error_filterreg (cc.cpp:4-19): mean point displacement between the two poses."""
    p, pp = _d(src_xyz, (-1, 3))
    g, pg = _d(T_gt, (4, 4))
    e, pe = _d(T_est, (4, 4))
    return float(_L().se3icp_cc_error_filterreg(pp, p.shape[0], pg, pe))


def rot2euler(R) -> np.ndarray:
    """rot2euler (benchmark_lounge.cpp:14-49): (bank, attitude, heading), radians."""
    a, pa = _d(R, (3, 3))
    out = np.zeros(3)
    _L().se3icp_cc_rot2euler(pa, out.ctypes.data_as(_D))
    return out


def avg_eul_error(R1, R2) -> float:
    """avgEulError (benchmark_lounge.cpp:59-81), degrees."""
    a, pa = _d(R1, (3, 3))
    b, pb = _d(R2, (3, 3))
    return float(_L().se3icp_cc_avg_eul_error(pa, pb))


def evaluate_lrf_quality(src_frames, tgt_frames, map_gt, pairs) -> float:
    """cc::evaluate_LRF_quality (cc.cpp:62-86) without the per-pair text file."""
    s, ps = _d(src_frames, (-1, 4, 4))
    t, pt = _d(tgt_frames, (-1, 4, 4))
    m, pm = _d(map_gt, (4, 4))
    pr = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
    if pr.size and (pr[:, 0].max() >= s.shape[0] or pr[:, 1].max() >= t.shape[0] or pr.min() < 0):
        raise IndexError("correspondence index out of range")
    return float(_L().se3icp_cc_evaluate_lrf_quality(ps, pt, pm, pr.ctypes.data_as(_I), pr.shape[0]))


def evaluate_trajectory(gt_poses, est_poses) -> dict:
    """cc::evaluate_trajectory_quality (cc.cpp:165-201) on in-memory trajectories."""
    g, pg = _d(gt_poses, (-1, 4, 4))
    e, pe = _d(est_poses, (-1, 4, 4))
    if g.shape != e.shape:
        raise ValueError("trajectories have different size")
    out = np.zeros(3)
    if _L().se3icp_cc_evaluate_trajectory(pg, pe, g.shape[0], out.ctypes.data_as(_D)) != 0:
        raise ValueError("empty trajectory")
    return {"avg_translation_error": float(out[0]), "avg_rotation_error": float(out[1]),
            "success_rate": float(out[2])}


def _read(fn, path):
    n = fn(str(path).encode(), None, 0)
    if n < 0:
        raise FileNotFoundError(path)
    out = np.zeros((max(n, 1), 4, 4))
    fn(str(path).encode(), out.ctypes.data_as(_D), n)
    return out[:n]


def read_trajectory(path) -> np.ndarray:
    """cc::read_trajectory (cc.cpp:143-162) / gt_data: one [R|t] (12 values) per line."""
    return _read(_L().se3icp_cc_read_trajectory, path)


def read_kitti_poses(path) -> np.ndarray:
    """KITTI poses as benchmark_kitti.cpp:72-98 reads them (every other line)."""
    return _read(_L().se3icp_cc_read_kitti_poses, path)


def read_redwood_log(path):
    """RGBDTrajectory::LoadFromFile (benchmark_lounge.cpp:104-126): (poses, ids[n,3])."""
    L = _L()
    n = L.se3icp_cc_read_redwood_log(str(path).encode(), None, None, 0)
    if n < 0:
        raise FileNotFoundError(path)
    out = np.zeros((max(n, 1), 4, 4))
    ids = np.zeros((max(n, 1), 3), dtype=np.int32)
    L.se3icp_cc_read_redwood_log(str(path).encode(), out.ctypes.data_as(_D), ids.ctypes.data_as(_I), n)
    return out[:n], ids[:n]


def write_trajectory(path, poses) -> None:
    p, pp = _d(poses, (-1, 4, 4))
    if _L().se3icp_cc_write_trajectory(str(path).encode(), pp, p.shape[0]) != 0:
        raise OSError(path)


def write_redwood_log(path, poses, ids) -> None:
    """RGBDTrajectory::SaveToFile (benchmark_lounge.cpp:127-139), 8 decimals."""
    p, pp = _d(poses, (-1, 4, 4))
    i = np.ascontiguousarray(ids, dtype=np.int32).reshape(-1, 3)
    if i.shape[0] != p.shape[0]:
        raise ValueError("one id triple per pose")
    if _L().se3icp_cc_write_redwood_log(str(path).encode(), pp, i.ctypes.data_as(_I), p.shape[0]) != 0:
        raise OSError(path)


def compute_corrs_with_gt(src_xyz, tgt_xyz, T_gt, device: int = 0) -> np.ndarray:
    """cc::compute_corrs_with_gt (cc.cpp:112-140): (i, nearest target of T_gt * src_i),
    the 1-NN on the GPU."""
    from .registration import nearest_neighbors
    s = np.ascontiguousarray(src_xyz, dtype=np.float64).reshape(-1, 3)
    T = np.asarray(T_gt, dtype=np.float64)
    moved = s @ T[:3, :3].T + T[:3, 3]
    idx, _, _ = nearest_neighbors(moved, tgt_xyz, device=device)
    return np.stack([np.arange(s.shape[0], dtype=np.int32), idx.astype(np.int32)], axis=1)
