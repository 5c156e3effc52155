"""ctypes binding of libse3icp.so (include/se3icp.h).

The product path: every call goes to the HIP engine.  If the shared library is
missing or no HIP device is visible, calls raise — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)  # se3-icp_amd/
LIB_PATH = os.environ.get("SE3ICP_LIB") or os.path.join(_ROOT, "lib", "libse3icp.so")

OK = 0
ERR_INVALID_ARG = -1
ERR_INVALID_METHOD = -2
ERR_EMPTY_CLOUD = -3
ERR_K_TOO_LARGE = -4
ERR_NO_DEVICE = -5
ERR_HIP = -6
ERR_NONFINITE = -7
ERR_OUT_OF_MEMORY = -8

METHODS = ["pt2pt", "pt2pl", "gicp", "se3_pt2pt", "se3_pt2pl", "se3_gicp", "se3_gicp_with_cf",
           "se3_pure_pt2pt", "se3_pure_pt2pl", "se3_pure_gicp"]

# every symbol include/se3icp.h declares
EXPORTED_SYMBOLS = [
    "se3icp_abi_version", "se3icp_status_string", "se3icp_method_from_name", "se3icp_method_name",
    "se3icp_default_params", "se3icp_device_count",
    "se3icp_registration_new", "se3icp_registration_free", "se3icp_set_source_cloud", "se3icp_set_target_cloud",
    "se3icp_params_of", "se3icp_run_icp", "se3icp_run_se3_icp", "se3icp_run_se3_icp_with_cf", "se3icp_run_se3_pure",
    "se3icp_get_result",
    "se3icp_register_batch", "se3icp_register_batch_device", "se3icp_register",
    "se3icp_toldi_frames", "se3icp_knn_self", "se3icp_estimate_normals", "se3icp_nn",
    "se3icp_synthetic_pairs", "se3icp_synthetic_reference", "se3icp_synthetic_reference_device",
    "se3icp_random_downsample",
    "se3icp_set_profiling", "se3icp_last_kernel_times", "se3icp_last_kernel_times_n", "se3icp_set_trace", "se3icp_set_lrf_exact",
    "se3icp_set_nn_events",
    # include/se3icp_cc.h: metrics and pose files of the benchmark drivers (host only)
    "se3icp_cc_rot_3d", "se3icp_cc_angular_error_so3", "se3icp_cc_angular_error_so3_alt",
    "se3icp_cc_error_filterreg", "se3icp_cc_rot2euler", "se3icp_cc_avg_eul_error",
    "se3icp_cc_evaluate_lrf_quality", "se3icp_cc_evaluate_trajectory",
    "se3icp_cc_read_trajectory", "se3icp_cc_read_kitti_poses", "se3icp_cc_read_redwood_log",
    "se3icp_cc_write_trajectory", "se3icp_cc_write_redwood_log",
]


class Params(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32),
        ("max_num_se3_iterations", C.c_int32),
        ("number_of_nn_for_LRF", C.c_int32),
        ("_reserved", C.c_int32),
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
        ("status", C.c_int32),
        ("num_rechecked", C.c_int32),
        ("scaling_factor", C.c_double),
        ("time_setup_ms", C.c_double),
        ("time_loop_ms", C.c_double),
        ("time_se3_correspondence_search_ms", C.c_double),
        ("time_before_pure_icp_ms", C.c_double),
    ]


class Trace(C.Structure):
    _fields_ = [
        ("pair", C.c_int32),
        ("max_iters", C.c_int32),
        ("corr_idx", C.POINTER(C.c_int32)),
        ("corr_dist", C.POINTER(C.c_float)),
        ("trim_key", C.POINTER(C.c_uint64)),
        ("T", C.POINTER(C.c_double)),
        ("mse", C.POINTER(C.c_double)),
        ("phase", C.POINTER(C.c_int32)),
        ("iters_recorded", C.c_int32),
        ("_reserved", C.c_int32),
    ]


class Se3IcpError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = status_string(code) if _lib is not None else str(code)
        super().__init__(f"se3icp error {code} ({msg}){': ' + what if what else ''}")


_lib = None


def load():
    """Load libse3icp.so (build it with `make -C se3-icp_amd` or __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP engine library not built: {LIB_PATH} is missing "
                          "(run __graft_entry__.build() or `make -C se3-icp_amd`)")
    L = C.CDLL(LIB_PATH)
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
    vp = C.c_void_p
    L.se3icp_abi_version.restype = C.c_int
    L.se3icp_status_string.restype = C.c_char_p
    L.se3icp_status_string.argtypes = [C.c_int]
    L.se3icp_method_from_name.argtypes = [C.c_char_p]
    L.se3icp_method_name.restype = C.c_char_p
    L.se3icp_method_name.argtypes = [C.c_int]
    L.se3icp_default_params.argtypes = [C.POINTER(Params)]
    L.se3icp_device_count.restype = C.c_int
    L.se3icp_registration_new.restype = vp
    L.se3icp_registration_free.argtypes = [vp]
    L.se3icp_set_source_cloud.argtypes = [vp, dp, C.c_int64]
    L.se3icp_set_target_cloud.argtypes = [vp, dp, C.c_int64]
    L.se3icp_params_of.restype = C.POINTER(Params)
    L.se3icp_params_of.argtypes = [vp]
    L.se3icp_run_icp.argtypes = [vp, C.c_char_p]
    L.se3icp_run_se3_icp.argtypes = [vp, C.c_char_p]
    L.se3icp_run_se3_icp_with_cf.argtypes = [vp]
    L.se3icp_run_se3_pure.argtypes = [vp, C.c_char_p]
    L.se3icp_get_result.argtypes = [vp, C.POINTER(Result)]
    L.se3icp_register_batch.argtypes = [C.c_int, C.c_int32, C.POINTER(dp), C.POINTER(C.c_int64), C.POINTER(dp),
                                        C.POINTER(C.c_int64), C.c_int, C.POINTER(Params), C.POINTER(Result)]
    L.se3icp_register_batch_device.argtypes = [C.c_int, C.c_int32, vp, C.POINTER(C.c_int64), vp,
                                               C.POINTER(C.c_int64), C.c_int, C.POINTER(Params), C.POINTER(Result), vp]
    L.se3icp_register.argtypes = [C.c_int, dp, C.c_int64, dp, C.c_int64, C.c_int, C.POINTER(Params),
                                  C.POINTER(Result)]
    L.se3icp_toldi_frames.argtypes = [C.c_int, dp, C.c_int64, C.c_int, dp]
    L.se3icp_knn_self.argtypes = [C.c_int, dp, C.c_int64, C.c_int, ip]
    L.se3icp_estimate_normals.argtypes = [C.c_int, dp, C.c_int64, C.c_int, dp]
    L.se3icp_nn.argtypes = [C.c_int, dp, C.c_int64, dp, C.c_int64, C.c_int, ip, dp, ip]
    L.se3icp_synthetic_pairs.restype = C.c_int64
    L.se3icp_synthetic_pairs.argtypes = [C.c_int, dp, C.c_int64, C.c_int32, dp, C.c_double, C.c_double, C.c_uint64,
                                         vp, vp, C.c_int]
    L.se3icp_synthetic_reference.restype = C.c_int64
    L.se3icp_synthetic_reference.argtypes = [dp, C.c_int64, C.c_int32, C.c_double, C.c_double, C.c_double, C.c_double,
                                             C.c_int32, dp, dp, dp]
    L.se3icp_synthetic_reference_device.restype = C.c_int64
    L.se3icp_synthetic_reference_device.argtypes = [C.c_int, dp, C.c_int64, C.c_int32, C.c_double, C.c_double,
                                                    C.c_double, C.c_double, C.c_int32, vp, vp, dp, C.c_int]
    L.se3icp_random_downsample.restype = C.c_int64
    L.se3icp_random_downsample.argtypes = [dp, C.c_int64, C.c_double, C.c_uint32, dp]
    L.se3icp_set_profiling.argtypes = [C.c_int, C.c_int]
    L.se3icp_last_kernel_times.argtypes = [C.c_int, dp]
    L.se3icp_last_kernel_times_n.argtypes = [C.c_int, dp, C.c_int]
    L.se3icp_set_trace.argtypes = [C.c_int, C.POINTER(Trace)]
    L.se3icp_set_lrf_exact.argtypes = [C.c_int, C.c_int]
    L.se3icp_set_nn_events.argtypes = [C.c_int, C.c_int]
    _lib = L
    return L


def status_string(code: int) -> str:
    return load().se3icp_status_string(int(code)).decode()


def check(code: int, what: str = "") -> int:
    if code != OK:
        raise Se3IcpError(code, what)
    return code


def default_params(**overrides) -> Params:
    p = Params()
    load().se3icp_default_params(C.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def device_count() -> int:
    return load().se3icp_device_count()


def method_id(name: str) -> int:
    m = load().se3icp_method_from_name(name.encode())
    if m < 0:
        raise ValueError(f"unknown method {name!r}; valid: {', '.join(METHODS)}")
    return m
