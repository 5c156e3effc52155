"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol
include/se3icp.h declares, and its host-only entry points (no GPU work) behave like
the reference's interface.  No compute is launched here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def _header_symbols():
    import glob
    src = "".join(open(f).read() for f in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(se3icp_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import se3icp
    return se3icp.load()


def test_library_exports_every_header_symbol(lib):
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"libse3icp.so does not export {s}"
    from se3icp import _lib
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms


def test_abi_version_and_status_strings(lib):
    import se3icp
    assert lib.se3icp_abi_version() == 4
    assert se3icp.status_string(0) == "ok"
    assert "no CPU fallback" in se3icp.status_string(-5)


def test_method_names_follow_the_reference_cli(lib):
    import se3icp
    # examples/run_registration_method.cpp:19-24
    for i, name in enumerate(["pt2pt", "pt2pl", "gicp", "se3_pt2pt", "se3_pt2pl", "se3_gicp"]):
        assert se3icp.method_id(name) == i
    assert se3icp.method_id("se3_gicp_with_cf") == 6
    with pytest.raises(ValueError):
        se3icp.method_id("se3_icp")


def test_default_params_are_the_reference_constructor(lib):
    import se3icp
    p = se3icp.default_params()  # ISR.cpp:334-348
    assert (p.max_num_iterations, p.max_num_se3_iterations, p.number_of_nn_for_LRF) == (150, 20, 30)
    assert (p.mse, p.mse_switch_error, p.estimated_overlap) == (1e-5, 1e-3, 1.0)
    assert (p.alpha_rot, p.beta_transl, p.scale_preprocessing) == (3.0, 1.0, 3.0)


def test_object_surface_mirrors_the_class_without_a_gpu(lib):
    import se3icp
    reg = se3icp.IterativeSE3Registration()
    assert reg.max_num_iterations_ == 150 and reg.number_of_nn_for_LRF_ == 30
    reg.number_of_nn_for_LRF_ = 90
    reg.mse_switch_error_ = 5 * reg.mse_
    assert reg.number_of_nn_for_LRF_ == 90 and abs(reg.mse_switch_error_ - 5e-5) < 1e-20
    assert reg.num_pure_se3_iterations_ == -1 and reg.num_iterations_ == 0
    np.testing.assert_array_equal(reg.current_estimated_T_, np.eye(4))


def test_set_cloud_appends_like_the_reference(lib):
    # ISR.cpp:358-366 pushes back: two calls concatenate
    import se3icp
    from se3icp import _lib
    reg = se3icp.IterativeSE3Registration()
    a = np.zeros((3, 3))
    reg.setSourceCloud(a)
    reg.setSourceCloud(a)
    # an empty target makes the run fail before touching the GPU
    with pytest.raises(_lib.Se3IcpError) as e:
        reg.run_se3_icp("pt2pl")
    assert e.value.code in (_lib.ERR_EMPTY_CLOUD, _lib.ERR_NO_DEVICE)


def test_no_device_fails_loudly_instead_of_falling_back(lib):
    import se3icp
    if se3icp.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(se3icp.Se3IcpError):
        se3icp.register_batch([(np.random.rand(100, 3), np.random.rand(100, 3))], "se3_pt2pl")


def test_cli_rejects_bad_usage_like_the_reference():
    cli = os.path.join(ROOT, "se3-icp_amd", "bin", "run_registration_method")
    assert os.path.exists(cli)
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage:" in r.stderr
    r = subprocess.run([cli, "icp", "a.ply", "b.ply"], capture_output=True, text=True)
    assert r.returncode == 1 and "Not a valid algorithm name" in r.stderr


def test_ply_reader_roundtrip(tmp_path):
    from se3icp.io import read_ply_xyz, write_ply_xyz
    pts = np.random.default_rng(0).normal(size=(57, 3))
    for binary in (True, False):
        p = tmp_path / f"c{int(binary)}.ply"
        write_ply_xyz(p, pts, binary=binary)
        np.testing.assert_array_equal(read_ply_xyz(p), pts)


def test_fixture_ply_parses(fixture_clouds):
    src, tgt = fixture_clouds
    assert src.shape == (4167, 3) and tgt.shape == (4167, 3)


def test_synthetic_generators_are_seeded():
    from se3icp import datasets
    a, _ = datasets.kitti_like_sequence(2, seed=5, n_az=200)
    b, _ = datasets.kitti_like_sequence(2, seed=5, n_az=200)
    np.testing.assert_array_equal(a[1], b[1])
    f, _ = datasets.rgbd_room_sequence(2, seed=3, stride=16)
    assert (f[0][:, 2] >= 0.39).all() and (f[0][:, 2] <= 4.1).all()
