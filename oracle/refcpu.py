"""ctypes binding of the CPU restatement (oracle/refcpu.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "librefcpu.so")

RUN_ICP, RUN_SE3_ICP, RUN_SE3_ICP_CF, RUN_SE3_PURE = 0, 1, 2, 3
PT2PT, PT2PL, GICP = 0, 1, 2
VARIANTS = {"pt2pt": PT2PT, "pt2pl": PT2PL, "gicp": GICP}


class Params(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32),
        ("max_num_se3_iterations", C.c_int32),
        ("number_of_nn_for_LRF", C.c_int32),
        ("_pad", C.c_int32),
        ("mse", C.c_double),
        ("mse_switch_error", C.c_double),
        ("estimated_overlap", C.c_double),
        ("alpha_rot", C.c_double),
        ("beta_transl", C.c_double),
        ("scale_preprocessing", C.c_double),
    ]


class Result(C.Structure):
    _fields_ = [
        ("T", C.c_double * 16),
        ("num_iterations", C.c_int32),
        ("num_pure_se3_iterations", C.c_int32),
        ("scaling_factor", C.c_double),
        ("time_setup_ms", C.c_double),
        ("time_loop_ms", C.c_double),
        ("time_nn_ms", C.c_double),
        ("time_toldi_ms", C.c_double),
        ("time_normals_ms", C.c_double),
        ("time_trim_ms", C.c_double),
        ("time_solve_ms", C.c_double),
    ]


class Trace(C.Structure):
    _fields_ = [
        ("max_trace_iters", C.c_int32),
        ("_pad", C.c_int32),
        ("Ti", C.POINTER(C.c_double)),
        ("mse", C.POINTER(C.c_double)),
        ("n_kept", C.POINTER(C.c_int32)),
        ("corr_idx", C.POINTER(C.c_int32)),
        ("corr_dist", C.POINTER(C.c_float)),
        ("corr_d2", C.POINTER(C.c_double)),
        ("corr_idx2", C.POINTER(C.c_int32)),
        ("corr_d2b", C.POINTER(C.c_double)),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        dp, ip, fp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_float)
        L.refcpu_default_params.argtypes = [C.POINTER(Params)]
        L.refcpu_register.argtypes = [dp, C.c_int64, dp, C.c_int64, C.c_int, C.c_int, C.POINTER(Params),
                                      C.POINTER(Result), C.POINTER(Trace)]
        L.refcpu_knn_self.argtypes = [dp, C.c_int64, C.c_int, ip, dp]
        L.refcpu_toldi_frames.argtypes = [dp, C.c_int64, C.c_int, dp]
        L.refcpu_estimate_normals.argtypes = [dp, C.c_int64, C.c_int, dp]
        L.refcpu_gicp_covariances.argtypes = [dp, C.c_int64, C.c_double, dp]
        L.refcpu_nn.argtypes = [dp, C.c_int64, dp, C.c_int64, C.c_int, ip, dp]
        L.refcpu_estimate.argtypes = [C.c_int, dp, dp, dp, dp, dp, ip, C.c_int64, dp, dp]
        L.refcpu_trim.argtypes = [fp, C.c_int64, C.c_double, ip]
        L.refcpu_trim.restype = C.c_int64
        L.refcpu_num_threads.restype = C.c_int
        L.refcpu_set_num_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else None


def default_params(**overrides) -> Params:
    p = Params()
    lib().refcpu_default_params(C.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def cli_params(**overrides) -> Params:
    """Overrides of examples/run_registration_method.cpp:38-42."""
    p = default_params(estimated_overlap=1.0, max_num_se3_iterations=10, mse=1e-5,
                       mse_switch_error=5e-5, number_of_nn_for_LRF=90)
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def set_num_threads(n: int) -> None:
    lib().refcpu_set_num_threads(int(n))


def num_threads() -> int:
    return lib().refcpu_num_threads()


def register(src, tgt, run_kind=RUN_SE3_ICP, variant="pt2pl", params: Params | None = None,
             trace_iters: int = 0, trace_margins: bool = False):
    """Run the restated registration.  Returns a dict (and trace arrays if requested;
    trace_margins adds each query's squared search distance and its second-nearest
    target from a 2-NN search)."""
    src = np.ascontiguousarray(src, dtype=np.float64)
    tgt = np.ascontiguousarray(tgt, dtype=np.float64)
    params = params or default_params()
    res = Result()
    tr = None
    out = {}
    if trace_iters > 0:
        ns = src.shape[0]
        out["Ti"] = np.zeros((trace_iters, 4, 4))
        out["mse"] = np.zeros(trace_iters)
        out["n_kept"] = np.zeros(trace_iters, np.int32)
        out["corr_idx"] = np.full((trace_iters, ns), -1, np.int32)
        out["corr_dist"] = np.zeros((trace_iters, ns), np.float32)
        if trace_margins:
            out["corr_d2"] = np.zeros((trace_iters, ns))
            out["corr_idx2"] = np.full((trace_iters, ns), -1, np.int32)
            out["corr_d2b"] = np.zeros((trace_iters, ns))
        tr = Trace(trace_iters, 0, _d(out["Ti"]), _d(out["mse"]), _i(out["n_kept"]), _i(out["corr_idx"]),
                   out["corr_dist"].ctypes.data_as(C.POINTER(C.c_float)), _d(out.get("corr_d2")),
                   _i(out.get("corr_idx2")), _d(out.get("corr_d2b")))
    v = VARIANTS[variant] if isinstance(variant, str) else int(variant)
    rc = lib().refcpu_register(_d(src), src.shape[0], _d(tgt), tgt.shape[0], run_kind, v, C.byref(params),
                               C.byref(res), C.byref(tr) if tr is not None else None)
    if rc != 0:
        raise RuntimeError(f"refcpu_register failed: {rc}")
    out.update(T=np.array(res.T).reshape(4, 4), num_iterations=res.num_iterations,
               num_pure_se3_iterations=res.num_pure_se3_iterations, scaling_factor=res.scaling_factor,
               time_setup_ms=res.time_setup_ms, time_loop_ms=res.time_loop_ms, time_nn_ms=res.time_nn_ms,
               time_toldi_ms=res.time_toldi_ms, time_normals_ms=res.time_normals_ms, time_trim_ms=res.time_trim_ms,
               time_solve_ms=res.time_solve_ms)
    return out


def knn_self(pts, k):
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    n = pts.shape[0]
    idx = np.zeros((n, k), np.int32)
    d2 = np.zeros((n, k))
    lib().refcpu_knn_self(_d(pts), n, k, _i(idx), _d(d2))
    return idx, d2


def toldi_frames(pts, k):
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    out = np.zeros((pts.shape[0], 4, 4))
    lib().refcpu_toldi_frames(_d(pts), pts.shape[0], k, _d(out))
    return out


def estimate_normals(pts, k=30):
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    out = np.zeros_like(pts)
    lib().refcpu_estimate_normals(_d(pts), pts.shape[0], k, _d(out))
    return out


def gicp_covariances(normals, eps=1e-3):
    normals = np.ascontiguousarray(normals, dtype=np.float64)
    out = np.zeros((normals.shape[0], 3, 3))
    lib().refcpu_gicp_covariances(_d(normals), normals.shape[0], eps, _d(out))
    return out


def nn(query, data):
    query = np.ascontiguousarray(query, dtype=np.float64)
    data = np.ascontiguousarray(data, dtype=np.float64)
    dim = data.shape[1]
    idx = np.zeros(query.shape[0], np.int32)
    d2 = np.zeros(query.shape[0])
    lib().refcpu_nn(_d(query), query.shape[0], _d(data), data.shape[0], dim, _i(idx), _d(d2))
    return idx, d2


def estimate(variant, src_pts, tgt_pts, pairs, tgt_normals=None, src_cov=None, tgt_cov=None, weights=None):
    c = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.float64)
    src_pts, tgt_pts, tgt_normals, src_cov, tgt_cov, weights = map(c, (src_pts, tgt_pts, tgt_normals, src_cov,
                                                                       tgt_cov, weights))
    pairs = np.ascontiguousarray(pairs, dtype=np.int32)
    T = np.zeros(16)
    v = VARIANTS[variant] if isinstance(variant, str) else int(variant)
    rc = lib().refcpu_estimate(v, _d(src_pts), _d(src_cov), _d(tgt_pts), _d(tgt_normals), _d(tgt_cov), _i(pairs),
                               pairs.shape[0], _d(weights), _d(T))
    if rc != 0:
        raise RuntimeError(f"refcpu_estimate failed: {rc}")
    return T.reshape(4, 4)


def trim(dist, ratio):
    dist = np.ascontiguousarray(dist, dtype=np.float32)
    kept = np.zeros(dist.shape[0], np.int32)
    k = lib().refcpu_trim(dist.ctypes.data_as(C.POINTER(C.c_float)), dist.shape[0], float(ratio), _i(kept))
    return kept[:k]
