"""CPU tests of the oracle (oracle/refcpu.cpp) — pinning it before trusting it.

Pins:
  * the reference's own known-answer fixture created_example_reg_problem/
    (target = R*source + t exactly, R = cc::rot_3d(pi/9, pi/8, -pi/7), t = (1,2,3),
    examples/create_and_save_reg_problem.cpp:31-37): every method recovers T_gt;
  * scipy.spatial.cKDTree as an independent exact kNN / 1-NN oracle;
  * algebraic properties of the restated third-party arithmetic (umeyama on exact
    correspondences, LDLT solve, TOLDI frame orthonormality, trimming counts).
Third-party behaviour without any fixture in the reference is "parity unpinned"
beyond these checks (DESIGN.md "Oracle").
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from oracle import refcpu


@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_se3_icp_recovers_fixture_ground_truth(fixture_clouds, fixture_T_gt, variant):
    src, tgt = fixture_clouds
    r = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, variant, refcpu.cli_params())
    assert np.linalg.norm(r["T"] - fixture_T_gt) <= 1e-9
    assert 1 <= r["num_pure_se3_iterations"] <= 10
    assert r["num_iterations"] > r["num_pure_se3_iterations"]


def test_txt_ground_truth_matches_analytic(fixture_T_gt):
    import os
    from conftest import GOLDEN
    txt = np.loadtxt(os.path.join(GOLDEN, "fixture_transformation_gt.txt"))
    assert np.abs(txt - fixture_T_gt).max() <= 5e-7  # printed with 6 decimals (MKPROB:52)


def test_fixture_is_exact_rigid_copy(fixture_clouds, fixture_T_gt):
    src, tgt = fixture_clouds
    pred = src @ fixture_T_gt[:3, :3].T + fixture_T_gt[:3, 3]
    assert np.abs(pred - tgt).max() < 1e-13


@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_vanilla_icp_and_cf_on_fixture(fixture_clouds, fixture_T_gt, variant):
    src, tgt = fixture_clouds
    r = refcpu.register(src, tgt, refcpu.RUN_ICP, variant, refcpu.cli_params())
    assert r["num_pure_se3_iterations"] == -1
    assert np.linalg.norm(r["T"] - fixture_T_gt) <= 1e-8


def test_cf_recovers_fixture(fixture_clouds, fixture_T_gt):
    src, tgt = fixture_clouds
    r = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP_CF, "gicp", refcpu.cli_params())
    assert np.linalg.norm(r["T"] - fixture_T_gt) <= 1e-9


def test_knn_matches_ckdtree(fixture_clouds):
    src, _ = fixture_clouds
    k = 90
    idx, d2 = refcpu.knn_self(src, k)
    dd, ii = cKDTree(src).query(src, k=k)
    np.testing.assert_allclose(np.sqrt(d2), dd, rtol=0, atol=1e-12)
    # identical index lists except inside exact-distance tie groups
    diff_rows = np.nonzero((idx != ii).any(axis=1))[0]
    for r in diff_rows:
        assert np.allclose(np.sort(d2[r]), d2[r])


@pytest.mark.parametrize("dim", [3, 12])
def test_nn_matches_ckdtree(dim):
    rng = np.random.default_rng(dim)
    data = rng.normal(size=(3000, dim))
    q = rng.normal(size=(500, dim))
    idx, d2 = refcpu.nn(q, data)
    dd, ii = cKDTree(data).query(q, k=1)
    np.testing.assert_array_equal(idx, ii)
    np.testing.assert_allclose(np.sqrt(d2), dd, rtol=1e-14)


def test_nn_tie_goes_to_lowest_index():
    data = np.array([[1.0, 0, 0], [0, 1.0, 0], [1.0, 0, 0], [-1.0, 0, 0]])
    idx, _ = refcpu.nn(np.zeros((1, 3)), data)
    assert idx[0] == 0


def test_toldi_frames_are_proper_rotations(fixture_clouds):
    src, _ = fixture_clouds
    F = refcpu.toldi_frames(src, 90)
    R = F[:, :3, :3]
    np.testing.assert_allclose(np.einsum("nji,njk->nik", R, R), np.broadcast_to(np.eye(3), R.shape), atol=1e-10)
    np.testing.assert_allclose(np.linalg.det(R), 1.0, atol=1e-10)
    np.testing.assert_array_equal(F[:, :3, 3], src)


def test_toldi_rotation_equivariance_and_centroid_quirk(fixture_clouds, fixture_T_gt):
    # H1: the centroid sums k/3-1 neighbours but divides by k/3 (ISR.cpp:261-265), i.e. it is
    # pulled toward the origin.  Frames therefore rotate with the cloud about the origin but
    # are NOT translation-equivariant — the reference normalizes clouds first (ISR.cpp:576-582).
    src, _ = fixture_clouds
    R = fixture_T_gt[:3, :3]
    Fs = refcpu.toldi_frames(src, 90)
    Fr = refcpu.toldi_frames(src @ R.T, 90)
    pred = np.einsum("ij,njk->nik", R, Fs[:, :3, :3])
    err = np.abs(pred - Fr[:, :3, :3]).reshape(len(src), -1).max(axis=1)
    assert np.mean(err < 1e-6) > 0.99
    Ft = refcpu.toldi_frames(src + np.array([50.0, 0, 0]), 90)
    assert np.abs(Ft[:, :3, :3] - Fs[:, :3, :3]).max() > 1e-3


def test_normals_are_unit_and_orthogonal_to_local_plane():
    rng = np.random.default_rng(1)
    xy = rng.uniform(-1, 1, size=(2000, 2))
    pts = np.c_[xy, 0.3 * xy[:, 0] - 0.2 * xy[:, 1]]
    n = refcpu.estimate_normals(pts, 30)
    expected = np.array([-0.3, 0.2, 1.0]) / np.linalg.norm([-0.3, 0.2, 1.0])
    np.testing.assert_allclose(np.abs(n @ expected), 1.0, atol=1e-9)


def test_gicp_covariance_from_normal():
    n = np.array([[0.0, 0.0, 1.0], [1.0, 0, 0], [-1.0, 0, 0]])
    C = refcpu.gicp_covariances(n, 1e-3)
    np.testing.assert_allclose(C[0], np.diag([1.0, 1.0, 1e-3]), atol=1e-15)
    np.testing.assert_allclose(C[1], np.diag([1e-3, 1.0, 1.0]), atol=1e-15)
    # c < -0.99 branch: identity rotation (ISR.cpp:8-10)
    np.testing.assert_allclose(C[2], np.diag([1e-3, 1.0, 1.0]), atol=1e-15)


def test_umeyama_exact_correspondences(fixture_T_gt):
    rng = np.random.default_rng(2)
    src = rng.normal(size=(100, 3))
    tgt = src @ fixture_T_gt[:3, :3].T + fixture_T_gt[:3, 3]
    pairs = np.c_[np.arange(100), np.arange(100)]
    T = refcpu.estimate("pt2pt", src, tgt, pairs)
    np.testing.assert_allclose(T, fixture_T_gt, atol=1e-12)


def test_point_to_plane_step_is_small_rotation_solution():
    rng = np.random.default_rng(3)
    tgt = rng.normal(size=(400, 3))
    nrm = rng.normal(size=(400, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    from se3icp import datasets
    Tsmall = datasets.make_T(datasets.rot_3d(0.01, -0.02, 0.015), [0.01, 0.02, -0.01])
    src = (tgt - Tsmall[:3, 3]) @ Tsmall[:3, :3]  # Tsmall @ src = tgt
    pairs = np.c_[np.arange(400), np.arange(400)]
    T = refcpu.estimate("pt2pl", src, tgt, pairs, tgt_normals=nrm)
    assert np.linalg.norm(T - Tsmall) < 2e-3  # one Gauss-Newton step of a linearised problem


@pytest.mark.parametrize("ratio,n,expected", [(1.0, 1000, 1000), (0.7, 120000, 84000), (0.75, 4167, 3125),
                                              (0.7, 10, 7), (0.0, 5, 0)])
def test_trim_count_is_pcl_float_floor(ratio, n, expected):
    d = np.random.default_rng(0).random(n).astype(np.float32)
    kept = refcpu.trim(d, ratio)
    assert len(kept) == expected
    if expected == n:
        # PCL copies the input unchanged when nothing is cut: query order, not distance order
        assert (kept == np.arange(n)).all()
    elif expected:
        assert d[kept].max() <= np.sort(d)[expected - 1]
        assert (np.diff(d[kept]) >= 0).all()
