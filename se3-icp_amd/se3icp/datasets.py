"""Seeded synthetic inputs for the benchmark configurations.

The reference's datasets (KITTI seq. 07 downsampled scans, the Stanford lounge
RGB-D sequence) are not available offline, so the workloads are synthesized with
the same shape:

* ``kitti_like_sequence``  64-beam rotating LiDAR (HDL-64E-like elevation fan)
  ray-cast against a street scene (ground plane, building boxes, parked cars,
  poles), ~120k points per scan, consecutive scans ~1 m apart with small yaw —
  the C4 workload (examples/benchmark_kitti.cpp: source = scan i+1, target = scan i).
* ``rgbd_room_sequence``   pinhole depth camera inside a furnished room, depth
  0.4-4 m with a Kinect-like noise model, smooth trajectory — the C3/C5 surrogate
  for the lounge sequence (examples/benchmark_lounge.cpp).
* ``bunny_pair``           the reference's synthetic bunny protocol
  (examples/benchmark_synthetic.cpp:91-160: x50 scale, random rigid transform,
  Gaussian noise of variance 0.005 on both clouds).

Everything is numpy with an explicit ``numpy.random.Generator(PCG64(seed))``.
"""
from __future__ import annotations

import os

import numpy as np


def rot_3d(roll: float, pitch: float, yaw: float) -> np.ndarray:
    """cc::rot_3d (src/cc.cpp:22-30): Rz(yaw) @ Ry(pitch) @ Rx(roll)."""
    cx, sx = np.cos(roll), np.sin(roll)
    cy, sy = np.cos(pitch), np.sin(pitch)
    cz, sz = np.cos(yaw), np.sin(yaw)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def make_T(R: np.ndarray, t) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def transform(T: np.ndarray, pts: np.ndarray) -> np.ndarray:
    return pts @ T[:3, :3].T + T[:3, 3]


# ----------------------------------------------------------------------------- ray casting
class _Scene:
    def __init__(self, ground: bool = True):
        self.ground = ground
        self.boxes_lo: list = []
        self.boxes_hi: list = []
        self.cyl: list = []  # (cx, cy, r, z0, z1)
        self.inside_boxes_lo: list = []  # rooms: rays start inside, hit the walls from within
        self.inside_boxes_hi: list = []

    def add_box(self, lo, hi):
        self.boxes_lo.append(lo)
        self.boxes_hi.append(hi)

    def cast(self, origin: np.ndarray, dirs: np.ndarray, tmax: float) -> np.ndarray:
        """Nearest positive hit distance along each unit ray (inf if none)."""
        best = np.full(dirs.shape[0], np.inf)
        with np.errstate(divide="ignore", invalid="ignore"):
            if self.ground:
                t = -origin[2] / dirs[:, 2]
                best = np.where((t > 1e-6) & (t < best), t, best)
            inv = 1.0 / dirs
            if self.boxes_lo:
                lo = np.asarray(self.boxes_lo)[None]  # (1,B,3)
                hi = np.asarray(self.boxes_hi)[None]
                t1 = (lo - origin[None, None]) * inv[:, None, :]
                t2 = (hi - origin[None, None]) * inv[:, None, :]
                tn = np.nanmax(np.minimum(t1, t2), axis=2)
                tf = np.nanmin(np.maximum(t1, t2), axis=2)
                hit = (tf >= tn) & (tn > 1e-6)
                th = np.where(hit, tn, np.inf).min(axis=1)
                best = np.minimum(best, th)
            if self.inside_boxes_lo:
                lo = np.asarray(self.inside_boxes_lo)[None]
                hi = np.asarray(self.inside_boxes_hi)[None]
                t1 = (lo - origin[None, None]) * inv[:, None, :]
                t2 = (hi - origin[None, None]) * inv[:, None, :]
                tf = np.nanmin(np.maximum(t1, t2), axis=2)
                th = np.where(tf > 1e-6, tf, np.inf).min(axis=1)
                best = np.minimum(best, th)
            for cx, cy, r, z0, z1 in self.cyl:
                ox, oy = origin[0] - cx, origin[1] - cy
                a = dirs[:, 0] ** 2 + dirs[:, 1] ** 2
                b = 2 * (ox * dirs[:, 0] + oy * dirs[:, 1])
                c = ox * ox + oy * oy - r * r
                disc = b * b - 4 * a * c
                t = (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a)
                z = origin[2] + t * dirs[:, 2]
                ok = (disc >= 0) & (t > 1e-6) & (z >= z0) & (z <= z1)
                best = np.where(ok & (t < best), t, best)
        best[best > tmax] = np.inf
        return best


def _street_scene(rng, length: float) -> _Scene:
    sc = _Scene(ground=True)
    for side in (-1, 1):
        x = -60.0
        while x < length + 60:
            w = rng.uniform(6, 22)
            if rng.random() < 0.8:
                y0 = rng.uniform(8, 13)
                d = rng.uniform(6, 14)
                h = rng.uniform(4, 16)
                ylo, yhi = (y0, y0 + d) if side > 0 else (-y0 - d, -y0)
                sc.add_box((x, ylo, 0.0), (x + w, yhi, h))
            x += w + rng.uniform(1, 8)
        x = -60.0
        while x < length + 60:
            if rng.random() < 0.5:  # parked car
                y = side * rng.uniform(4.8, 5.6)
                sc.add_box((x, y - 0.9, 0.0), (x + 4.2, y + 0.9, 1.5))
            x += rng.uniform(6, 12)
        x = -60.0
        while x < length + 60:  # poles / trunks
            sc.cyl.append((x + rng.uniform(-1, 1), side * rng.uniform(6.5, 7.5), rng.uniform(0.1, 0.35), 0.0,
                           rng.uniform(3, 8)))
            x += rng.uniform(8, 18)
    return sc


def kitti_like_sequence(n_scans: int, seed: int = 4, n_az: int = 1975, n_beams: int = 64, step: float = 1.0,
                        max_yaw_deg: float = 2.0, range_noise: float = 0.02, max_range: float = 80.0,
                        scan_indices=None, workers: int = 0):
    """Return (scans, poses): scans[k] is an (N_k, 3) float64 cloud in the sensor frame of
    scan k, poses[k] its 4x4 world pose.  ~120k points per scan at the defaults.
    ``scan_indices`` ray-casts only those scans (others are None); every scan has its
    own generator stream, so a subset is identical to the same scans of the full run."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sc = _street_scene(rng, step * n_scans)
    elev = np.deg2rad(np.linspace(-24.8, 2.0, n_beams))
    poses = []
    yaw = 0.0
    pos = np.array([0.0, 0.0, 1.73])
    for k in range(n_scans):
        if k > 0:
            yaw += np.deg2rad(rng.uniform(-max_yaw_deg, max_yaw_deg)) * 0.5
            pos = pos + np.array([np.cos(yaw), np.sin(yaw), 0.0]) * step * rng.uniform(0.9, 1.1)
            pos[1] = np.clip(pos[1], -2.5, 2.5)
        poses.append(make_T(rot_3d(0, 0, yaw), pos))
    want = set(range(n_scans)) if scan_indices is None else set(scan_indices)

    def cast(k):
        srng = np.random.Generator(np.random.PCG64([seed, k]))
        Rw, pk = poses[k][:3, :3], poses[k][:3, 3]
        az = np.linspace(0, 2 * np.pi, n_az, endpoint=False) + srng.uniform(0, 2 * np.pi / n_az)
        E, A = np.meshgrid(elev + srng.normal(0, 0.0005, n_beams), az, indexing="ij")
        d = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], axis=-1).reshape(-1, 3)
        dw = d @ Rw.T
        ts = []
        for c0 in range(0, d.shape[0], 16384):
            ts.append(sc.cast(pk, dw[c0:c0 + 16384], max_range))
        t = np.concatenate(ts)
        ok = np.isfinite(t) & (t > 1.0)
        t = t[ok] + srng.normal(0, range_noise, ok.sum())
        return np.ascontiguousarray(d[ok] * t[:, None])

    # every scan has its own stream, so the scans are cast by a thread pool (numpy releases
    # the GIL in the ray-box arithmetic); the result does not depend on the thread count
    ks = [k for k in range(n_scans) if k in want]
    nw = max(1, min(len(ks), workers if workers else min(8, os.cpu_count() or 1)))
    if nw > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(nw) as ex:
            got = dict(zip(ks, ex.map(cast, ks)))
    else:
        got = {k: cast(k) for k in ks}
    scans = [got.get(k) for k in range(n_scans)]
    return scans, poses


def kitti_like_pairs(n_pairs: int, seed: int = 4, first: int = 0, total_pairs: int | None = None, **kw):
    """Consecutive-scan pairs (source = scan i+1, target = scan i, examples/benchmark_kitti.cpp:130-131)
    with ground truth T = pose[i]^-1 pose[i+1].  Pairs first .. first+n_pairs-1 of a
    sequence of total_pairs (default n_pairs) pairs."""
    total = (first + n_pairs) if total_pairs is None else total_pairs
    idx = range(first, first + n_pairs + 1)
    scans, poses = kitti_like_sequence(total + 1, seed=seed, scan_indices=idx, **kw)
    pairs, gts = [], []
    for i in range(first, first + n_pairs):
        pairs.append((scans[i + 1], scans[i]))
        gts.append(np.linalg.inv(poses[i]) @ poses[i + 1])
    return pairs, gts


def rgbd_room_sequence(n_frames: int, seed: int = 3, stride: int = 4, max_step_deg: float = 4.0,
                       max_step_m: float = 0.08):
    """Depth-camera frames inside a furnished room; points in the camera frame
    (x right, y down, z forward, depth = z in metres, 0.4-4 m)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sc = _Scene(ground=False)
    sc.inside_boxes_lo.append((-3.5, -3.0, 0.0))
    sc.inside_boxes_hi.append((3.5, 3.0, 2.8))
    for _ in range(9):  # furniture
        c = rng.uniform([-2.8, -2.3, 0], [2.8, 2.3, 0])
        s = rng.uniform([0.3, 0.3, 0.3], [1.4, 1.0, 1.2])
        sc.add_box((c[0] - s[0] / 2, c[1] - s[1] / 2, 0.0), (c[0] + s[0] / 2, c[1] + s[1] / 2, s[2]))
    fx = fy = 525.0
    W, H = 640, 480
    u, v = np.meshgrid(np.arange(0, W, stride) + 0.5 * stride, np.arange(0, H, stride) + 0.5 * stride)
    dc = np.stack([(u - 319.5) / fx, (v - 239.5) / fy, np.ones_like(u)], axis=-1).reshape(-1, 3)
    dc /= np.linalg.norm(dc, axis=1, keepdims=True)
    # camera (x right, y down, z fwd) -> world (x fwd, y left, z up) at yaw 0
    C2W = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=float)
    frames, poses = [], []
    yaw, pitch = rng.uniform(0, 2 * np.pi), np.deg2rad(-10)
    pos = np.array([0.0, 0.0, 1.4])
    for k in range(n_frames):
        if k > 0:
            yaw += np.deg2rad(rng.uniform(0.3, 1.0) * max_step_deg)
            pitch = np.clip(pitch + np.deg2rad(rng.normal(0, 0.5)), np.deg2rad(-25), np.deg2rad(5))
            pos = pos + rng.normal(0, max_step_m / 2, 3) * np.array([1, 1, 0.3])
            pos = np.clip(pos, [-1.5, -1.2, 1.0], [1.5, 1.2, 1.8])
        Rw = rot_3d(0, -pitch, yaw) @ C2W
        dw = dc @ Rw.T
        t = sc.cast(pos, dw, 10.0)
        depth = t * dc[:, 2]
        ok = np.isfinite(t) & (depth > 0.4) & (depth < 4.0)
        z = depth[ok]
        z = z + rng.normal(0, 1.0, z.shape) * (0.0012 + 0.0019 * (z - 0.4) ** 2)
        pts = dc[ok] / dc[ok, 2:3] * z[:, None]
        frames.append(np.ascontiguousarray(pts))
        poses.append(make_T(Rw, pos))
    return frames, poses


def rgbd_pairs(n_pairs: int, seed: int = 3, gap: int = 1, **kw):
    frames, poses = rgbd_room_sequence(n_pairs + gap, seed=seed, **kw)
    pairs, gts = [], []
    for i in range(n_pairs):
        pairs.append((frames[i + gap], frames[i]))
        gts.append(np.linalg.inv(poses[i]) @ poses[i + gap])
    return pairs, gts


def bunny_pair(bunny_unique: np.ndarray, seed: int = 1, noise_var: float = 0.005, easy: bool = True,
               subsample: float | None = None):
    """examples/benchmark_synthetic.cpp:91-160 protocol on the unique bunny vertices x50.
    Returns (src, tgt, T_gt) with tgt ~ T_gt @ src."""
    rng = np.random.Generator(np.random.PCG64(seed))
    base = np.asarray(bunny_unique, dtype=np.float64) * 50.0
    tr, rr = (5.0, np.pi / 4) if easy else (10.0, np.pi / 2)
    t = rng.uniform(-tr, tr, 3)
    R = rot_3d(*rng.uniform(-rr, rr, 3))
    T = make_T(R, t)
    if subsample:
        src = base[rng.random(base.shape[0]) < subsample]
        tgt = transform(T, base)[rng.random(base.shape[0]) < subsample]
    else:
        src = base.copy()
        tgt = transform(T, base)
    sd = np.sqrt(noise_var)
    src = src + rng.normal(0, sd, src.shape)
    tgt = tgt + rng.normal(0, sd, tgt.shape)
    return np.ascontiguousarray(src), np.ascontiguousarray(tgt), T


def synthetic_cases(n_cases: int, seed: int = 1, easy: bool = False):
    """Ground-truth transforms of examples/benchmark_synthetic.cpp:103-145: t ~ U(-tr, tr)^3,
    R = rot_3d(U(-rr, rr)^3) with the "moderate" ranges active in the reference (10, pi/2)
    or the "easy" ones (5, pi/4).  Host numpy (PCG64); returns [n_cases, 4, 4]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    tr, rr = (5.0, np.pi / 4) if easy else (10.0, np.pi / 2)
    Ts = []
    for _ in range(n_cases):
        t = rng.uniform(-tr, tr, 3)
        Ts.append(make_T(rot_3d(*rng.uniform(-rr, rr, 3)), t))
    return np.stack(Ts)


def synthetic_pairs_gpu(base: np.ndarray, Ts: np.ndarray, ratio: float = 0.02, noise_var: float = 0.005,
                        seed: int = 1, device: int = 0, out=None):
    """The benchmark_synthetic.cpp:91-160 problems generated on the GPU (k_gen.hip,
    se3icp_synthetic_pairs): for each T in Ts, an independent random subset of
    k = int(ratio * n) points of `base` (source) and of T @ base (target), each plus
    N(0, noise_var I).  With out=None returns host arrays (src [C, k, 3], tgt [C, k, 3]);
    with out=(src_ptr, tgt_ptr) writes into device buffers and returns k."""
    import ctypes as C
    from . import _lib
    b = np.ascontiguousarray(base, dtype=np.float64)
    T = np.ascontiguousarray(Ts, dtype=np.float64).reshape(-1, 16)
    dp = C.POINTER(C.c_double)
    L = _lib.load()
    if out is not None:
        k = L.se3icp_synthetic_pairs(device, b.ctypes.data_as(dp), b.shape[0], T.shape[0], T.ctypes.data_as(dp),
                                     ratio, noise_var, seed, C.c_void_p(out[0]), C.c_void_p(out[1]), 1)
        _lib.check(int(min(k, 0)), "synthetic_pairs")
        return int(k)
    k = int(ratio * b.shape[0])
    src = np.zeros((T.shape[0], max(k, 0), 3))
    tgt = np.zeros_like(src)
    r = L.se3icp_synthetic_pairs(device, b.ctypes.data_as(dp), b.shape[0], T.shape[0], T.ctypes.data_as(dp), ratio,
                                 noise_var, seed, src.ctypes.data_as(C.c_void_p), tgt.ctypes.data_as(C.c_void_p), 0)
    _lib.check(int(min(r, 0)), "synthetic_pairs")
    assert r == k, (r, k)
    return src, tgt


# ----------------------------------------------------------------------------- reference streams
def random_downsample(xyz: np.ndarray, ratio: float = 0.02, seed: int = 1) -> np.ndarray:
    """Open3D PointCloud::RandomDownSample(ratio) right after utility::random::Seed(seed),
    number for number (libse3icp host code, std::shuffle over std::mt19937)."""
    import ctypes as C
    from . import _lib
    a = np.ascontiguousarray(xyz, dtype=np.float64)
    k = int(ratio * a.shape[0])
    out = np.zeros((k, 3))
    dp = C.POINTER(C.c_double)
    r = _lib.load().se3icp_random_downsample(a.ctypes.data_as(dp), a.shape[0], ratio, seed, out.ctypes.data_as(dp))
    _lib.check(int(min(r, 0)), "random_downsample")
    return out


def synthetic_reference(cloud: np.ndarray, n_cases: int, ratio: float = 0.02, noise_var: float = 0.005,
                        t_range: float = 10.0, r_range: float = np.pi / 2, args_left_to_right: bool = False):
    """examples/benchmark_synthetic.cpp:91-160 with the reference's own random streams
    (se3icp_synthetic_reference): returns (src [C, k, 3], tgt [C, k, 3], T [C, 4, 4]).
    cloud: the full cloud in file order (stanford_bunny.ply x 50: bunny_full() * 50)."""
    import ctypes as C
    from . import _lib
    a = np.ascontiguousarray(cloud, dtype=np.float64)
    k = int(ratio * a.shape[0])
    src = np.zeros((n_cases, k, 3))
    tgt = np.zeros((n_cases, k, 3))
    T = np.zeros((n_cases, 4, 4))
    dp = C.POINTER(C.c_double)
    r = _lib.load().se3icp_synthetic_reference(a.ctypes.data_as(dp), a.shape[0], n_cases, ratio, noise_var, t_range,
                                               r_range, 1 if args_left_to_right else 0, src.ctypes.data_as(dp),
                                               tgt.ctypes.data_as(dp), T.ctypes.data_as(dp))
    _lib.check(int(min(r, 0)), "synthetic_reference")
    assert r == k
    return src, tgt, T


def synthetic_reference_gpu(cloud: np.ndarray, n_cases: int, ratio: float = 0.02, noise_var: float = 0.005,
                            t_range: float = 10.0, r_range: float = np.pi / 2, args_left_to_right: bool = False,
                            device: int = 0, out=None):
    """The reference's problems of synthetic_reference(), written by the GPU
    (se3icp_synthetic_reference_device: the host draws the driver's streams, k_gen.hip
    applies them with the same arithmetic), equal to synthetic_reference() bit for bit.
    out=None: returns (src [C, k, 3], tgt [C, k, 3], T [C, 4, 4]) on the host;
    out=(src_ptr, tgt_ptr): device buffers of [C * k, 3], returns (k, T)."""
    import ctypes as C
    from . import _lib
    a = np.ascontiguousarray(cloud, dtype=np.float64)
    k = int(ratio * a.shape[0])
    T = np.zeros((n_cases, 4, 4))
    dp = C.POINTER(C.c_double)
    L = _lib.load()
    flags = 1 if args_left_to_right else 0
    if out is not None:
        r = L.se3icp_synthetic_reference_device(device, a.ctypes.data_as(dp), a.shape[0], n_cases, ratio, noise_var,
                                                t_range, r_range, flags, C.c_void_p(out[0]), C.c_void_p(out[1]),
                                                T.ctypes.data_as(dp), 1)
        _lib.check(int(min(r, 0)), "synthetic_reference_device")
        return int(r), T
    src = np.zeros((n_cases, k, 3))
    tgt = np.zeros((n_cases, k, 3))
    r = L.se3icp_synthetic_reference_device(device, a.ctypes.data_as(dp), a.shape[0], n_cases, ratio, noise_var,
                                            t_range, r_range, flags, src.ctypes.data_as(C.c_void_p),
                                            tgt.ctypes.data_as(C.c_void_p), T.ctypes.data_as(dp), 0)
    _lib.check(int(min(r, 0)), "synthetic_reference_device")
    assert r == k
    return src, tgt, T
