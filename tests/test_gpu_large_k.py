"""GPU tests of neighbourhoods over 128 points (number_of_nn_for_LRF_ is unbounded in the
reference: include/iterative_SE3_registration.hpp:80, passed straight to
KDTreeFlann::SearchKNN at src/iterative_SE3_registration.cpp:253).

k_knn_big.hip takes every query with min(k, n) > 128 (one wavefront per query, a candidate
buffer in global memory); below that the LDS kernels (k_lrf8 + k_lrf) run.  Checked here:
  * kNN lists equal the oracle's (modulo exact-distance ties) at k = 150 and 256 on the
    reference fixture and the 34,834-point unique bunny;
  * TOLDI frames agree with the oracle to 1e-8 except at ill-conditioned frames (the test of
    test_gpu_parity.py::test_toldi_frames_match_oracle), at the same k;
  * the global-buffer kernel forced for every query (se3icp_set_lrf_exact mode 2) gives the
    LDS kernels' frames and normals bit for bit at k = 90 / 30 (same sets, same rank order,
    same arithmetic), on a C4-size scan and on lattices full of ties;
  * end to end, se3_pt2pl with k = 150 on the fixture matches the oracle's pose (1e-5) and
    iteration counts;
  * k = 1000 (candidate buffers past the register networks: the in-memory bitonic network,
    and on lattices the exact cut of a buffer full of ties): lists equal the oracle's, and
    mode 2 equals the default path bit for bit.
"""
import numpy as np
import pytest

from test_gpu_parity import _eig_gap, _lrf_cloud, _toldi_cov

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def se3icp_mod():
    import se3icp
    se3icp.load()
    if se3icp.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")
    return se3icp


@pytest.fixture(scope="module")
def refcpu():
    from oracle import refcpu as r
    r.lib()
    return r


def _cloud(kind, fixture_clouds, bunny_unique):
    return fixture_clouds[0] if kind == "fixture" else bunny_unique * 50.0


@pytest.mark.parametrize("kind", ["fixture", "bunny35k"])
@pytest.mark.parametrize("k", [150, 256])
def test_large_k_knn_self_matches_oracle(se3icp_mod, refcpu, fixture_clouds, bunny_unique, kind, k):
    pts = _cloud(kind, fixture_clouds, bunny_unique)
    g = se3icp_mod.knn_self(pts, k)
    ri, rd = refcpu.knn_self(pts, k)
    assert g.shape == ri.shape == (len(pts), k)
    same = (g == ri).all(axis=1)
    print(f"[large-k] {kind} k={k}: {int((~same).sum())} of {len(pts)} lists differ in order (exact ties)")
    for i in np.nonzero(~same)[0]:
        dg = np.sum((pts[g[i]] - pts[i]) ** 2, axis=1)
        np.testing.assert_allclose(dg, rd[i], rtol=0, atol=1e-12)  # tie groups: same distances, rank by rank
    d = np.sum((pts[g] - pts[:, None, :]) ** 2, axis=2)
    assert (np.diff(d, axis=1) >= -1e-15).all()


@pytest.mark.parametrize("kind", ["fixture", "bunny35k"])
@pytest.mark.parametrize("k", [150, 256])
def test_large_k_toldi_frames_match_oracle(se3icp_mod, refcpu, fixture_clouds, bunny_unique, kind, k):
    pts = _cloud(kind, fixture_clouds, bunny_unique)
    g = se3icp_mod.toldi_frames(pts, k)
    r = refcpu.toldi_frames(pts, k)
    idx, _ = refcpu.knn_self(pts, k)
    _assert_frames_close(pts, idx, g, r)


def _assert_frames_close(pts, idx, g, r):
    """Frames within 1e-8 of the oracle's, except at ill-conditioned ones (near-equal smallest
    eigenvalues of the TOLDI covariance, or a vanishing x axis) -- at most 0.1 % of points."""
    diff = np.abs(g - r).reshape(len(pts), -1).max(axis=1)
    bad = np.nonzero(diff > 1e-8)[0]
    assert len(bad) <= 0.001 * len(pts), np.sort(diff)[-10:]
    if len(bad):
        gap = _eig_gap(_toldi_cov(pts, idx[bad]))
        z = r[bad, :3, 2]
        v = pts[idx[bad, 1:]] - pts[bad, None, :]
        R = np.linalg.norm(pts[idx[bad, -1]] - pts[bad], axis=1)
        w = (R[:, None] - np.linalg.norm(v, axis=2)) ** 2 * np.einsum("nki,ni->nk", v, z) ** 2
        acc = np.einsum("nk,nki->ni", w, v)
        xr = np.linalg.norm(acc - np.einsum("ni,ni->n", acc, z)[:, None] * z, axis=1)
        xr = xr / np.maximum(np.linalg.norm(acc, axis=1), 1e-300)
        ill = (gap < 1e-6) | (xr < 1e-6)
        assert ill.all(), (bad[~ill], diff[bad[~ill]], gap[~ill], xr[~ill])


@pytest.mark.parametrize("kind", ["kitti", "lattice", "lattice_jitter"])
@pytest.mark.parametrize("k", [90, 30])
def test_global_buffer_kernel_equals_lds_kernels(se3icp_mod, k, kind):
    from se3icp import registration
    pts = _lrf_cloud(kind)
    fast_f = se3icp_mod.toldi_frames(pts, k)
    fast_n = se3icp_mod.estimate_normals(pts, k)
    registration.set_lrf_exact(2)
    try:
        big_f = se3icp_mod.toldi_frames(pts, k)
        big_n = se3icp_mod.estimate_normals(pts, k)
        big_knn = se3icp_mod.knn_self(pts[:20000], k)
    finally:
        registration.set_lrf_exact(0)
    same_f = (fast_f.view(np.uint64) == big_f.view(np.uint64)).reshape(len(pts), -1).all(axis=1)
    assert same_f.all(), np.nonzero(~same_f)[0][:8]
    assert np.array_equal(fast_n.view(np.uint64), big_n.view(np.uint64))
    assert np.array_equal(big_knn, se3icp_mod.knn_self(pts[:20000], k))


def test_large_k_end_to_end_matches_oracle(se3icp_mod, refcpu, fixture_clouds, fixture_T_gt):
    src, tgt = fixture_clouds
    p = se3icp_mod.cli_params(number_of_nn_for_LRF=150)
    got = se3icp_mod.register_batch([(src, tgt)], "se3_pt2pl", p)[0]
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, "pt2pl", refcpu.cli_params(number_of_nn_for_LRF=150))
    assert got.status == 0
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5
    assert np.linalg.norm(got.T - fixture_T_gt) <= 1e-6
    assert (got.num_iterations, got.num_pure_se3_iterations) == (ref["num_iterations"], ref["num_pure_se3_iterations"])


def _lattice_small(jitter=False):
    g = np.stack(np.meshgrid(np.arange(24), np.arange(20), np.arange(12), indexing="ij"), -1).reshape(-1, 3) * 0.05
    if jitter:
        g = g + np.random.default_rng(5).standard_normal(g.shape) * 1e-12
    return g


@pytest.mark.parametrize("kind", ["fixture", "lattice", "lattice_jitter"])
def test_k1000_knn_and_frames_match_oracle(se3icp_mod, refcpu, fixture_clouds, kind):
    """k = 1000: the candidate buffer (2k + 256 -> 4096 entries) is past the register
    networks' 512, so the survivors are ordered by k_knn_big's in-memory bitonic network; on
    the lattices the ties at the k-th distance fill the buffer and the exact cut runs.  The
    lists equal the oracle's (ties by lowest index on both sides); the fixture's frames within
    1e-8 except at ill-conditioned frames."""
    pts = fixture_clouds[0] if kind == "fixture" else _lattice_small(kind == "lattice_jitter")
    k = 1000
    g = se3icp_mod.knn_self(pts, k)
    ri, rd = refcpu.knn_self(pts, k)
    assert g.shape == ri.shape == (len(pts), k)
    same = (g == ri).all(axis=1)
    print(f"[k=1000] {kind}: {int((~same).sum())} of {len(pts)} lists differ in order")
    for i in np.nonzero(~same)[0]:
        dg = np.sum((pts[g[i]] - pts[i]) ** 2, axis=1)
        np.testing.assert_allclose(dg, rd[i], rtol=0, atol=1e-12)
    if kind == "lattice":  # exact ties everywhere, broken by the point index on both sides
        assert same.all()
    if kind == "fixture":  # (the lattices' frames are degenerate by symmetry: lists only)
        _assert_frames_close(pts, ri, se3icp_mod.toldi_frames(pts, k), refcpu.toldi_frames(pts, k))


@pytest.mark.parametrize("kind", ["lattice", "lattice_jitter"])
def test_k1000_global_buffer_kernel_on_ties(se3icp_mod, kind):
    """Mode 2 (every query through k_knn_big) at k = 1000 on lattices: the same lists as the
    default path (which routes k > 128 there too) and deterministic across runs."""
    from se3icp import registration
    pts = _lattice_small(kind == "lattice_jitter")
    a = se3icp_mod.knn_self(pts, 1000)
    registration.set_lrf_exact(2)
    try:
        b = se3icp_mod.knn_self(pts, 1000)
        fb = se3icp_mod.toldi_frames(pts, 1000)
    finally:
        registration.set_lrf_exact(0)
    fa = se3icp_mod.toldi_frames(pts, 1000)
    assert np.array_equal(a, b)
    assert np.array_equal(fa.view(np.uint64), fb.view(np.uint64))
