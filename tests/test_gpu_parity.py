"""GPU parity tests: the HIP engine (through the C-ABI) against the CPU restatement.

Bars (BASELINE.json north_star): identical integer arg-min correspondences (modulo
exact f64 ties between equal target coordinates) and final poses within 1e-5
Frobenius of the oracle.  Floating-point stage outputs (TOLDI frames, normals)
are compared with the tolerances written in each test.
"""
import numpy as np
import pytest

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


def _tie_ok(data, q, i_gpu, i_ref, d2_ref, dim):
    """GPU and oracle NN agree, or both are exact minimisers (equal f64 distance)."""
    if i_gpu == i_ref:
        return True
    a = q
    b = data[i_gpu]
    d = a - b
    dg = float(np.dot(d, d))
    return abs(dg - d2_ref) <= 1e-12 * max(1.0, d2_ref)


# --------------------------------------------------------------------------- end to end
@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_fixture_se3_icp_matches_oracle_and_ground_truth(se3icp_mod, refcpu, fixture_clouds, fixture_T_gt, variant):
    src, tgt = fixture_clouds
    reg = se3icp_mod.IterativeSE3Registration()
    reg.setSourceCloud(src)
    reg.setTargetCloud(tgt)
    reg.estimated_overlap_ = 1.0
    reg.max_num_se3_iterations_ = 10
    reg.mse_ = 0.00001
    reg.mse_switch_error_ = 5 * reg.mse_
    reg.number_of_nn_for_LRF_ = 90
    assert reg.run_se3_icp(variant) == 0
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, variant, refcpu.cli_params())
    T = reg.current_estimated_T_
    assert np.linalg.norm(T - ref["T"]) <= 1e-5
    assert np.linalg.norm(T - fixture_T_gt) <= 1e-6
    assert reg.num_iterations_ == ref["num_iterations"]
    assert reg.num_pure_se3_iterations_ == ref["num_pure_se3_iterations"]


@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_fixture_vanilla_icp_matches_oracle(se3icp_mod, refcpu, fixture_clouds, variant):
    src, tgt = fixture_clouds
    params = se3icp_mod.cli_params()
    got = se3icp_mod.register_batch([(src, tgt)], variant, params)[0]
    ref = refcpu.register(src, tgt, refcpu.RUN_ICP, variant, refcpu.cli_params())
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5
    assert got.num_pure_se3_iterations == -1
    assert got.num_iterations == ref["num_iterations"]


def test_fixture_with_cf_matches_oracle(se3icp_mod, refcpu, fixture_clouds, fixture_T_gt):
    src, tgt = fixture_clouds
    got = se3icp_mod.register_batch([(src, tgt)], "se3_gicp_with_cf", se3icp_mod.cli_params())[0]
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP_CF, "gicp", refcpu.cli_params())
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5
    assert np.linalg.norm(got.T - fixture_T_gt) <= 1e-6


# --------------------------------------------------------------------------- stages
def test_knn_self_matches_oracle(se3icp_mod, refcpu, fixture_clouds, parity_record):
    src, _ = fixture_clouds
    k = 90
    g = se3icp_mod.knn_self(src, k)
    ri, rd = refcpu.knn_self(src, k)
    same = (g == ri)
    parity_record("knn_self fixture k=90", queries=len(src), lists_differing_in_tie_order=int((~same.all(axis=1)).sum()))
    if not same.all():
        # allowed only where the two lists differ by exact-distance ties
        bad = np.nonzero(~same.all(axis=1))[0]
        for i in bad:
            dg = np.sum((src[g[i]] - src[i]) ** 2, axis=1)
            np.testing.assert_allclose(np.sort(dg), rd[i], rtol=0, atol=1e-12)
    # sorted ascending
    d = np.sum((src[g] - src[:, None, :]) ** 2, axis=2)
    assert (np.diff(d, axis=1) >= -1e-15).all()


def _eig_gap(cov):
    """Relative gap between the two smallest eigenvalues of symmetric 3x3 matrices."""
    w = np.linalg.eigvalsh(cov)
    return (w[:, 1] - w[:, 0]) / np.maximum(np.abs(w[:, 2]), 1e-300)


def _toldi_cov(pts, idx):
    """ISR.cpp:259-272 restated: centroid of ranks 1 .. k/3-1 divided by k/3, covariance
    over ranks 1 .. k/3 about it."""
    rz = idx.shape[1] // 3
    c = pts[idx[:, 1:rz]].sum(axis=1) / rz
    v = pts[idx[:, 1:rz + 1]] - c[:, None, :]
    return np.einsum("nki,nkj->nij", v, v)


def _stage_cloud(kind, fixture_clouds):
    if kind == "fixture":
        return fixture_clouds[0]
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(1, seed=4, first=2, total_pairs=8)  # ~120k points
    return pairs[0][0]


@pytest.mark.parametrize("kind", ["fixture", "kitti"])
def test_toldi_frames_match_oracle(se3icp_mod, refcpu, fixture_clouds, kind, parity_record):
    """Frames agree to 1e-8 except where the frame is ill-conditioned, and every
    disagreement must be one: a near-degenerate smallest eigenvalue of the TOLDI
    covariance (the z axis, ISR.cpp:275-281) or a near-zero projected x axis
    (ISR.cpp:302-303, normalised without a guard)."""
    src = _stage_cloud(kind, fixture_clouds)
    k = 90
    g = se3icp_mod.toldi_frames(src, k)
    r = refcpu.toldi_frames(src, k)
    diff = np.abs(g - r).reshape(len(src), -1).max(axis=1)
    bad = np.nonzero(diff > 1e-8)[0]
    parity_record(f"toldi frames {kind} k=90", points=len(src), frames_over_1e8=len(bad),
                  max_diff_well_conditioned=float(np.max(diff[diff <= 1e-8], initial=0.0)))
    assert len(bad) <= 0.001 * len(src), np.sort(diff)[-10:]
    if len(bad):
        idx, _ = refcpu.knn_self(src, k)
        gap = _eig_gap(_toldi_cov(src, idx[bad]))
        # x axis before normalisation: sum of weighted neighbour vectors minus its z part
        z = r[bad, :3, 2]
        v = src[idx[bad, 1:]] - src[bad, None, :]
        R = np.linalg.norm(src[idx[bad, -1]] - src[bad], axis=1)
        w = (R[:, None] - np.linalg.norm(v, axis=2)) ** 2 * np.einsum("nki,ni->nk", v, z) ** 2
        acc = np.einsum("nk,nki->ni", w, v)
        xr = np.linalg.norm(acc - np.einsum("ni,ni->n", acc, z)[:, None] * z, axis=1)
        xr = xr / np.maximum(np.linalg.norm(acc, axis=1), 1e-300)
        ill = (gap < 1e-6) | (xr < 1e-6)
        print(f"[toldi] {len(bad)} of {len(src)} frames differ > 1e-8: eigen-gaps {np.round(gap[:8], 9)}, "
              f"x-axis ratios {np.round(xr[:8], 9)}")
        assert ill.all(), (bad[~ill], diff[bad[~ill]], gap[~ill], xr[~ill])
    R = g[:, :3, :3]
    np.testing.assert_allclose(np.einsum("nij,nik->njk", R, R), np.broadcast_to(np.eye(3), R.shape), atol=1e-9)


@pytest.mark.parametrize("kind", ["fixture", "kitti"])
def test_estimate_normals_match_oracle(se3icp_mod, refcpu, fixture_clouds, kind, parity_record):
    """Normals (sign included: FastEigen3x3 is deterministic given the covariance) agree
    to 1e-8 except at near-degenerate covariances (Open3D's cumulant covariance of the 30
    nearest points, ISR.cpp:643), and every disagreement must be one."""
    src = _stage_cloud(kind, fixture_clouds)
    k = 30
    g = se3icp_mod.estimate_normals(src, k)
    r = refcpu.estimate_normals(src, k)
    diff = np.abs(g - r).max(axis=1)
    bad = np.nonzero(diff > 1e-8)[0]
    parity_record(f"normals {kind} k=30", points=len(src), normals_over_1e8=len(bad),
                  max_diff_well_conditioned=float(np.max(diff[diff <= 1e-8], initial=0.0)))
    assert len(bad) <= 0.001 * len(src)
    if len(bad):
        idx, _ = refcpu.knn_self(src, k)
        p = src[idx[bad]]
        mu = p.mean(axis=1)
        cov = np.einsum("nki,nkj->nij", p, p) / k - np.einsum("ni,nj->nij", mu, mu)
        gap = _eig_gap(cov)
        print(f"[normals] {len(bad)} of {len(src)} normals differ > 1e-8: eigen-gaps {np.round(gap[:8], 9)}")
        assert (gap < 1e-6).all(), (bad[gap >= 1e-6], diff[bad[gap >= 1e-6]], gap[gap >= 1e-6])


def _se3_vectors(frames, alpha=3.0, beta=1.0):
    R = frames[:, :3, :3]
    t = frames[:, :3, 3]
    return np.concatenate([alpha * R.transpose(0, 2, 1).reshape(-1, 9), beta * t], axis=1)


def test_se3_nn_matches_oracle(se3icp_mod, refcpu, fixture_clouds):
    src, tgt = fixture_clouds
    fs = refcpu.toldi_frames(src, 90)
    ft = refcpu.toldi_frames(tgt, 90)
    q = _se3_vectors(fs)
    d = _se3_vectors(ft)
    gi, gd2, nrech = se3icp_mod.nearest_neighbors(q, d)
    ri, rd2 = refcpu.nn(q, d)
    for i in np.nonzero(gi != ri)[0]:
        assert _tie_ok(d, q[i], gi[i], ri[i], rd2[i], 12), (i, gi[i], ri[i])
    np.testing.assert_allclose(gd2, rd2, rtol=0, atol=1e-12)


def test_r3_nn_matches_oracle(se3icp_mod, refcpu, fixture_clouds):
    src, tgt = fixture_clouds
    rng = np.random.default_rng(0)
    q = src + rng.normal(0, 0.05, src.shape)
    gi, gd2, _ = se3icp_mod.nearest_neighbors(q, tgt)
    ri, rd2 = refcpu.nn(q, tgt)
    for i in np.nonzero(gi != ri)[0]:
        assert _tie_ok(tgt, q[i], gi[i], ri[i], rd2[i], 3)
    np.testing.assert_allclose(gd2, rd2, rtol=0, atol=1e-12)


def test_nn_exact_ties_pick_lowest_index(se3icp_mod):
    data = np.array([[1.0, 0, 0], [0, 1.0, 0], [1.0, 0, 0], [-1.0, 0, 0]])
    q = np.zeros((1, 3))
    gi, _, nrech = se3icp_mod.nearest_neighbors(q, data)
    assert gi[0] == 0 and nrech >= 1


@pytest.mark.parametrize("dim", [3, 12])
@pytest.mark.parametrize("nq", [1, 3, 10])
def test_nn_few_queries_against_large_data(se3icp_mod, refcpu, dim, nq):
    """A query cloud far smaller than the data cloud shares the batch's tree depth, so its
    local subtrees hold empty nodes and empty trailing leaves: the tree build must not read
    outside the clouds there (k_tree_local's final phase)."""
    rng = np.random.default_rng(100 + dim + nq)
    data = rng.normal(0, 1, (9000, dim))
    q = rng.normal(0, 1, (nq, dim))
    gi, gd2, _ = se3icp_mod.nearest_neighbors(q, data)
    ri, rd2 = refcpu.nn(q, data)
    assert np.array_equal(gi, ri)
    np.testing.assert_allclose(gd2, rd2, rtol=0, atol=1e-12)


def test_batch_with_tiny_first_source_cloud(se3icp_mod, refcpu):
    """First source cloud under 1/64 of the largest cloud of the batch: its
    subtrees below the shared global levels are mostly empty.  The tiny pair equals its
    oracle run, the big pair equals its own one-pair run bitwise."""
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(2, seed=4, first=1, total_pairs=8)
    s0, t0 = pairs[0]
    rng = np.random.default_rng(7)
    small = s0[np.sort(rng.choice(s0.shape[0], 1200, replace=False))]
    assert small.shape[0] * 64 < max(t0.shape[0], pairs[1][0].shape[0])
    p = se3icp_mod.kitti_params()
    got = se3icp_mod.register_batch([(small, t0), pairs[1]], "se3_gicp", p)
    alone = se3icp_mod.register_batch([pairs[1]], "se3_gicp", p)[0]
    assert np.array_equal(got[1].T, alone.T)
    assert got[1].num_iterations == alone.num_iterations
    rp = refcpu.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                               number_of_nn_for_LRF=90)
    ref = refcpu.register(small, t0, refcpu.RUN_SE3_ICP, "gicp", rp)
    assert np.linalg.norm(got[0].T - ref["T"]) <= 1e-5, (got[0].T, ref["T"])
    assert got[0].num_iterations == ref["num_iterations"]


# --------------------------------------------------------------------------- synthetic workloads
def test_bunny_pair_se3_pt2pt(se3icp_mod, refcpu, bunny_unique):
    from se3icp import datasets
    src, tgt, T_gt = datasets.bunny_pair(bunny_unique, seed=1, subsample=0.12)
    params = se3icp_mod.cli_params()
    got = se3icp_mod.register_batch([(src, tgt)], "se3_pt2pt", params)[0]
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, "pt2pt", refcpu.cli_params())
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5
    assert (got.num_iterations, got.num_pure_se3_iterations) == (ref["num_iterations"], ref["num_pure_se3_iterations"])


def test_kitti_like_batch_gicp_trimmed(se3icp_mod, refcpu):
    from se3icp import datasets
    pairs, gts = datasets.kitti_like_pairs(2, seed=11, n_az=300)
    params = se3icp_mod.kitti_params()
    got = se3icp_mod.register_batch(pairs, "se3_gicp", params)
    rp = refcpu.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                               number_of_nn_for_LRF=90)
    for (s, t), g in zip(pairs, got):
        ref = refcpu.register(s, t, refcpu.RUN_SE3_ICP, "gicp", rp)
        assert np.linalg.norm(g.T - ref["T"]) <= 1e-5, (g.T, ref["T"])


def test_rgbd_batch_with_cf(se3icp_mod, refcpu):
    from se3icp import datasets
    pairs, gts = datasets.rgbd_pairs(2, seed=3, stride=8)
    params = se3icp_mod.lounge_params()
    got = se3icp_mod.register_batch(pairs, "se3_gicp_with_cf", params)
    rp = refcpu.default_params(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                               number_of_nn_for_LRF=90)
    for (s, t), g in zip(pairs, got):
        ref = refcpu.register(s, t, refcpu.RUN_SE3_ICP_CF, "gicp", rp)
        assert np.linalg.norm(g.T - ref["T"]) <= 1e-5, (g.T, ref["T"])


@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_fixture_se3_pure_matches_oracle(se3icp_mod, refcpu, fixture_clouds, variant):
    src, tgt = fixture_clouds
    reg = se3icp_mod.IterativeSE3Registration()
    reg.setSourceCloud(src)
    reg.setTargetCloud(tgt)
    reg.estimated_overlap_ = 1.0
    reg.max_num_se3_iterations_ = 10
    reg.mse_ = 0.00001
    reg.mse_switch_error_ = 5 * reg.mse_
    reg.number_of_nn_for_LRF_ = 90
    assert reg.run_se3_pure(variant) == 0
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_PURE, variant, refcpu.cli_params())
    assert np.linalg.norm(reg.current_estimated_T_ - ref["T"]) <= 1e-5
    assert reg.num_iterations_ == ref["num_iterations"]
    assert reg.num_pure_se3_iterations_ == ref["num_pure_se3_iterations"]


def test_cli_on_fixture_matches_oracle(refcpu, fixture_clouds):
    """The drop-in CLI (examples/run_registration_method.cpp) on the fixture, README.md:64."""
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    exe = os.path.join(root, "se3-icp_amd", "bin", "run_registration_method")
    out = subprocess.run([exe, "se3_pt2pl", os.path.join(here, "golden", "fixture_source.ply"),
                          os.path.join(here, "golden", "fixture_target.ply")], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    assert "source point cloud size = 4167" in lines and "target point cloud size = 4167" in lines
    assert "Running SE(3)-ICP variant: pt2pl" in lines
    k = lines.index("Estimated transformation = ")
    T = np.array([[float(x) for x in lines[k + 1 + r].split()] for r in range(4)])
    src, tgt = fixture_clouds
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, "pt2pl", refcpu.cli_params())
    # Eigen's default stream format prints 6 significant digits
    assert np.allclose(T, ref["T"], rtol=1e-5, atol=1e-5)


def test_kitti_full_size_pair_matches_oracle(se3icp_mod, refcpu, parity_record):
    """BASELINE.json's size (~120k points per cloud), one pair, against the oracle."""
    from se3icp import datasets
    pairs, gts = datasets.kitti_like_pairs(1, seed=4, first=5, total_pairs=8)
    assert pairs[0][0].shape[0] > 100_000
    got = se3icp_mod.register_batch(pairs, "se3_gicp", se3icp_mod.kitti_params())[0]
    rp = refcpu.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                               number_of_nn_for_LRF=90)
    ref = refcpu.register(pairs[0][0], pairs[0][1], refcpu.RUN_SE3_ICP, "gicp", rp)
    parity_record("C4 pair 120k se3_gicp end to end", pose_frobenius=float(np.linalg.norm(got.T - ref["T"])),
                  iterations_gpu=got.num_iterations, iterations_ref=int(ref["num_iterations"]),
                  rechecked_queries=got.num_rechecked)
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5
    assert got.num_iterations == ref["num_iterations"]
    assert got.num_pure_se3_iterations == ref["num_pure_se3_iterations"]


# --------------------------------------------------------------------------- per-iteration parity
@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_first_iterations_match_oracle(se3icp_mod, refcpu, bunny_unique, variant):
    """the pose after each of the first three SE(3) iterations
    (run_se3_pure stopped at max_num_se3_iterations = k, ISR.cpp:1118-1119), on a noisy,
    trimmed pair (overlap 0.7: the trimmed sets feed the estimator).  The loop state
    lives on the device (k_reduce_final), so this pins the device-side solve and the
    windowed trim iteration by iteration."""
    from se3icp import datasets
    src, tgt, _ = datasets.bunny_pair(bunny_unique, seed=2, subsample=0.1)
    for k in (1, 2, 3):
        kw = dict(estimated_overlap=0.7, max_num_se3_iterations=k, mse=1e-12, mse_switch_error=1e-12,
                  number_of_nn_for_LRF=60)
        got = se3icp_mod.register_batch([(src, tgt)], "se3_pure_" + variant, se3icp_mod.default_params(**kw))[0]
        ref = refcpu.register(src, tgt, refcpu.RUN_SE3_PURE, variant, refcpu.default_params(**kw))
        assert got.num_iterations == ref["num_iterations"] == k
        assert np.linalg.norm(got.T - ref["T"]) <= 1e-9 * max(1.0, np.linalg.norm(ref["T"])), (k, got.T, ref["T"])


def test_se3_phase_without_iteration_cap_matches_oracle(se3icp_mod, refcpu, fixture_clouds):
    """max_num_se3_iterations = 0: `iter == max` never holds, so only the pose change ends
    the SE(3) phase (ISR.cpp:718-723); the host must keep queueing SE(3) searches."""
    src, tgt = fixture_clouds
    kw = dict(estimated_overlap=1.0, max_num_se3_iterations=0, mse=1e-5, mse_switch_error=5e-5,
              number_of_nn_for_LRF=90)
    got = se3icp_mod.register_batch([(src, tgt)], "se3_pt2pl", se3icp_mod.default_params(**kw))[0]
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, "pt2pl", refcpu.default_params(**kw))
    assert got.num_iterations == ref["num_iterations"]
    assert got.num_pure_se3_iterations == ref["num_pure_se3_iterations"]
    assert np.linalg.norm(got.T - ref["T"]) <= 1e-5


def test_batch_with_pairs_finishing_at_different_iterations(se3icp_mod, refcpu, bunny_unique, fixture_clouds):
    """Lockstep batch: pairs switch and converge at different iterations (the device
    marks finished pairs idle, later iterations run only the rest); every pair equals
    its own single-pair oracle run."""
    from se3icp import datasets
    pairs = [fixture_clouds] + [datasets.bunny_pair(bunny_unique, seed=s, subsample=0.08)[:2] for s in (3, 4)]
    params = se3icp_mod.cli_params()
    got = se3icp_mod.register_batch(pairs, "se3_pt2pl", params)
    its = []
    for (s, t), g in zip(pairs, got):
        ref = refcpu.register(s, t, refcpu.RUN_SE3_ICP, "pt2pl", refcpu.cli_params())
        assert np.linalg.norm(g.T - ref["T"]) <= 1e-5
        assert (g.num_iterations, g.num_pure_se3_iterations) == (ref["num_iterations"], ref["num_pure_se3_iterations"])
        its.append(g.num_iterations)
    assert len(set(its)) > 1, its  # the batch really had pairs finishing at different iterations


# --------------------------------------------------------------------------- BASELINE configs at size
def _rot_deg(A, B):
    R = A[:3, :3].T @ B[:3, :3]
    return float(np.degrees(np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))))


def test_c2_full_unique_bunny_se3_pt2pt(se3icp_mod, refcpu, bunny_unique):
    """C2: se3_pt2pt on the whole unique bunny (34,834 points, x50, noise variance 0.005,
    examples/benchmark_synthetic.cpp:91-160), the driver's parameters (B_SYN:356-363),
    no subsampling; correspondences checked at every iteration (test_gpu_trace)."""
    from se3icp import datasets
    from test_gpu_trace import compare_traces
    src, tgt, T_gt = datasets.bunny_pair(bunny_unique, seed=1)
    assert src.shape[0] == tgt.shape[0] == 34834
    res, gtr = se3icp_mod.register_batch_traced([(src, tgt)], "se3_pt2pt", se3icp_mod.cli_params())
    ref = refcpu.register(src, tgt, refcpu.RUN_SE3_ICP, "pt2pt", refcpu.cli_params(), trace_iters=160,
                          trace_margins=True)
    g = res[0]
    assert np.linalg.norm(g.T - ref["T"]) <= 1e-5
    assert g.num_iterations == ref["num_iterations"]
    assert g.num_pure_se3_iterations == ref["num_pure_se3_iterations"]
    compare_traces(gtr, ref, 1.0, "C2 bunny 34.8k se3_pt2pt")
    # B_SYN:238-246 success thresholds
    assert _rot_deg(g.T, T_gt) <= 2.0 and np.linalg.norm(g.T[:3, 3] - T_gt[:3, 3]) <= 0.25


def test_c2_bench_workload_downsample_batch(se3icp_mod, refcpu, bunny_full):
    """C2 as bench.py registers it (bench.py make_pairs): the reference's own problems
    (B_SYN:91-160, its mt19937 / normal_distribution / RandomDownSample streams, pinned by
    test_reference_streams) at RandomDownSample(0.2) of the 208,353-vertex bunny x50 =
    41,670 points per cloud, easy ranges (B_SYN:106-108), noise var 0.005, the 8-case batch
    registered together; cases 0 and 5 against their own oracle runs, case 5's
    correspondences at every iteration."""
    from se3icp import datasets
    from test_gpu_trace import compare_traces
    src, tgt, T_gt = datasets.synthetic_reference(bunny_full * 50.0, 8, ratio=0.2, noise_var=0.005, t_range=5.0,
                                                  r_range=np.pi / 4)
    assert src.shape == (8, 41670, 3)
    pairs = [(src[i], tgt[i]) for i in range(8)]
    res, gtr = se3icp_mod.register_batch_traced(pairs, "se3_pt2pt", se3icp_mod.cli_params(), pair=5)
    for c in (0, 5):
        ref = refcpu.register(src[c], tgt[c], refcpu.RUN_SE3_ICP, "pt2pt", refcpu.cli_params(),
                              trace_iters=160 if c == 5 else 0, trace_margins=c == 5)
        g = res[c]
        assert np.linalg.norm(g.T - ref["T"]) <= 1e-5, (c, g.T, ref["T"])
        assert (g.num_iterations, g.num_pure_se3_iterations) == (ref["num_iterations"],
                                                                  ref["num_pure_se3_iterations"])
        if c == 5:
            compare_traces(gtr, ref, 1.0, "C2 bench workload case 5")
    ok = sum(_rot_deg(r.T, T) <= 2.0 and np.linalg.norm(r.T[:3, 3] - T[:3, 3]) <= 0.25 for r, T in zip(res, T_gt))
    assert ok >= 6, ok  # B_SYN:238-246 success thresholds on the easy ranges


def test_c3_rgbd_batch32_se3_pt2pl(se3icp_mod, refcpu):
    """C3: a 32-pair se3_pt2pl batch of consecutive RGB-D frames at the default stride
    (~16k points, the lounge surrogate), examples/benchmark_lounge.cpp:183-189 parameters;
    every pair against its own oracle run."""
    from se3icp import datasets
    pairs, gts = datasets.rgbd_pairs(32, seed=3, stride=4)
    npts = [p[0].shape[0] for p in pairs]
    assert min(npts) > 10_000, npts
    got = se3icp_mod.register_batch(pairs, "se3_pt2pl", se3icp_mod.lounge_params())
    rp = refcpu.default_params(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                               number_of_nn_for_LRF=90)
    worst, its_diff = 0.0, 0
    for (s, t), g in zip(pairs, got):
        ref = refcpu.register(s, t, refcpu.RUN_SE3_ICP, "pt2pl", rp)
        worst = max(worst, float(np.linalg.norm(g.T - ref["T"])))
        its_diff += g.num_iterations != ref["num_iterations"]
        assert np.linalg.norm(g.T - ref["T"]) <= 1e-5, (g.T, ref["T"])
    print(f"[C3] 32 pairs, mean {np.mean(npts):.0f} points: max |T_gpu - T_ref|_F {worst:.2e}, "
          f"iteration-count differences {its_diff}")
    assert its_diff == 0


def test_c5_rgbd_batch256_se3_gicp_with_cf(se3icp_mod, refcpu):
    """C5: a 256-pair run_se3_icp_with_cf batch (ISR.cpp:742-959) on the RGB-D surrogate.
    Eight fixed pairs against the oracle; all 256 against the ground truth with the
    reference's success thresholds (SO(3) error <= 2 deg, translation <= 0.25,
    examples/benchmark_synthetic.cpp:238-246)."""
    from se3icp import datasets
    pairs, gts = datasets.rgbd_pairs(256, seed=5, stride=4)
    got = se3icp_mod.register_batch(pairs, "se3_gicp_with_cf", se3icp_mod.lounge_params())
    assert all(g.status == 0 for g in got)
    assert all(abs(g.time_before_pure_icp_ms - (g.time_setup_ms + g.time_loop_ms)) < 1e-6 for g in got)
    rp = refcpu.default_params(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                               number_of_nn_for_LRF=90)
    for i in range(0, 256, 32):
        s, t = pairs[i]
        ref = refcpu.register(s, t, refcpu.RUN_SE3_ICP_CF, "gicp", rp)
        assert np.linalg.norm(got[i].T - ref["T"]) <= 1e-5, (i, got[i].T, ref["T"])
        assert got[i].num_iterations == ref["num_iterations"], i
    rot = np.array([_rot_deg(g.T, gt) for g, gt in zip(got, gts)])
    tra = np.array([np.linalg.norm(g.T[:3, 3] - gt[:3, 3]) for g, gt in zip(got, gts)])
    print(f"[C5] 256 pairs: rot err max {rot.max():.3f} deg, trans err max {tra.max():.4f} m, "
          f"iterations {np.mean([g.num_iterations for g in got]):.1f} mean")
    assert (rot <= 2.0).all() and (tra <= 0.25).all(), (np.nonzero(rot > 2.0)[0], np.nonzero(tra > 0.25)[0])


def test_batch_independence_16_vs_two_8(se3icp_mod):
    """Pairs registered in one lockstep batch are bitwise the ones registered in smaller
    batches: the premise of sharding the batch over GPUs."""
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(16, seed=4)
    p = se3icp_mod.kitti_params()
    full = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    a = se3icp_mod.register_batch(pairs[:8], "se3_gicp", p)
    b = se3icp_mod.register_batch(pairs[8:], "se3_gicp", p)
    for i, (f, h) in enumerate(zip(full, a + b)):
        assert np.array_equal(f.T, h.T), (i, f.T - h.T)
        assert (f.num_iterations, f.num_pure_se3_iterations) == (h.num_iterations, h.num_pure_se3_iterations)


@pytest.mark.parametrize("case", ["kitti64", "rgbd160"])
def test_batch_independence_across_schedules(se3icp_mod, case):
    """The NN scheduling adapts to the batch (k_nn.hip: the dense-chunk threshold from the
    chunk count, the SE(3) phase's first widened search from the pair count -- from the 4th
    iteration up to 8 pairs, the 3rd up to 127, the 2nd from 128 -- and the cost-ordered 3-D
    dispatch from 64 pairs).  None of it may change a result: each large batch is bitwise
    its pairs registered in 8- and 32-pair batches."""
    from se3icp import datasets
    if case == "kitti64":
        pairs, _ = datasets.kitti_like_pairs(64, seed=4)
        method, p, parts = "se3_gicp", se3icp_mod.kitti_params(), (8, 32)
    else:
        pairs, _ = datasets.rgbd_pairs(160, seed=5, stride=4)
        method, p, parts = "se3_pt2pl", se3icp_mod.lounge_params(), (8, 32)
    full = se3icp_mod.register_batch(pairs, method, p)
    for size in parts:
        got = []
        for i in range(0, len(pairs), size):
            got += se3icp_mod.register_batch(pairs[i:i + size], method, p)
        for i, (f, h) in enumerate(zip(full, got)):
            assert np.array_equal(f.T, h.T), (case, size, i, f.T - h.T)
            assert (f.num_iterations, f.num_pure_se3_iterations) == (h.num_iterations, h.num_pure_se3_iterations)


def test_c4_headline_batch_pairs_match_oracle(se3icp_mod, refcpu, parity_record):
    """The headline batch itself (BASELINE.json configs[1]: 64 KITTI-like pairs of ~120k
    points, se3_gicp, one call) checked pair by pair against the oracle, at four pairs spread
    over the batch (the first, the last and two inside), not only through the sub-batch
    property above.  The oracle runs on the host's cores (threads: its default)."""
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(64, seed=4)
    p = se3icp_mod.kitti_params()
    got = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    rp = refcpu.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                               number_of_nn_for_LRF=90)
    worst = 0.0
    for i in (0, 21, 42, 63):
        ref = refcpu.register(pairs[i][0], pairs[i][1], refcpu.RUN_SE3_ICP, "gicp", rp)
        d = float(np.linalg.norm(got[i].T - ref["T"]))
        worst = max(worst, d)
        assert d <= 1e-5, (i, d)
        assert got[i].num_iterations == ref["num_iterations"], i
        assert got[i].num_pure_se3_iterations == ref["num_pure_se3_iterations"], i
    parity_record("C4 64-pair headline batch, pairs 0/21/42/63 vs oracle", max_pose_frobenius=worst)


def test_profiled_and_event_modes_equal_the_plain_loop(se3icp_mod):
    """Per-stage HIP events (se3icp_set_profiling) and the SE(3) NN bracket
    (se3icp_set_nn_events) change only how the host follows the loop, never its results:
    bitwise the poses and iteration counts of the plain loop (C4 params, pairs that switch
    to the R3 phase and finish at different iterations)."""
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(4, seed=4)
    p = se3icp_mod.kitti_params()
    runs = {}
    try:
        for name, prof, ev in (("plain", False, False), ("events", False, True), ("profiled", True, True)):
            se3icp_mod.set_profiling(prof)
            se3icp_mod.set_nn_events(ev)
            runs[name] = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    finally:
        se3icp_mod.set_profiling(False)
        se3icp_mod.set_nn_events(True)
    for name in ("events", "profiled"):
        for i, (a, b) in enumerate(zip(runs[name], runs["plain"])):
            assert np.array_equal(a.T, b.T), (name, i, a.T - b.T)
            assert (a.num_iterations, a.num_pure_se3_iterations) == (b.num_iterations, b.num_pure_se3_iterations), name
    assert min(r.num_iterations for r in runs["plain"]) > 10


def test_device_batch_runner_equals_register_batch(se3icp_mod):
    """The benchmark's timed call (clouds resident in HBM, prebuilt arguments, results read
    after the calls) returns bitwise the poses of the host-buffer batch entry, every call."""
    torch = pytest.importorskip("torch")
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(4, seed=4)
    p = se3icp_mod.kitti_params()
    host = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    src = np.ascontiguousarray(np.concatenate([a for a, _ in pairs]))
    tgt = np.ascontiguousarray(np.concatenate([b for _, b in pairs]))
    so = np.concatenate([[0], np.cumsum([a.shape[0] for a, _ in pairs])])
    to = np.concatenate([[0], np.cumsum([b.shape[0] for _, b in pairs])])
    d_src = torch.from_numpy(src).to("cuda:0")
    d_tgt = torch.from_numpy(tgt).to("cuda:0")
    torch.cuda.synchronize()
    r = se3icp_mod.DeviceBatchRunner(d_src.data_ptr(), so, d_tgt.data_ptr(), to, "se3_gicp", p, device=0, slots=2)
    r.run(0)
    r.run(1)
    for slot in (0, 1):
        res = r.results(slot)
        assert len(res) == len(host)
        for i, (a, b) in enumerate(zip(res, host)):
            assert np.array_equal(a.T, b.T), (slot, i, a.T - b.T)
            assert (a.num_iterations, a.num_pure_se3_iterations) == (b.num_iterations, b.num_pure_se3_iterations)
        kt = r.kernel_times(slot)
        assert kt["lrf_queries"] > 0 and kt["nn_se3_launches"] > 0


def test_pipelined_runner_equals_register_batch(se3icp_mod):
    """bench.py's in-flight steps: two calls at a time on two engine slots of the GPU (own
    streams and buffers, a host thread each) return, every call, bitwise the poses of the
    host-buffer batch entry."""
    torch = pytest.importorskip("torch")
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(4, seed=4)
    p = se3icp_mod.kitti_params()
    host = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    src = np.ascontiguousarray(np.concatenate([a for a, _ in pairs]))
    tgt = np.ascontiguousarray(np.concatenate([b for _, b in pairs]))
    so = np.concatenate([[0], np.cumsum([a.shape[0] for a, _ in pairs])])
    to = np.concatenate([[0], np.cumsum([b.shape[0] for _, b in pairs])])
    d_src = torch.from_numpy(src).to("cuda:0")
    d_tgt = torch.from_numpy(tgt).to("cuda:0")
    torch.cuda.synchronize()
    steps = 6
    pipe = se3icp_mod.PipelinedBatchRunner(
        lambda slot: se3icp_mod.DeviceBatchRunner(d_src.data_ptr(), so, d_tgt.data_ptr(), to, "se3_gicp", p,
                                                  device=0 | (slot << 8), slots=steps), in_flight=2, steps=steps)
    pipe.warm()
    pipe.run_steps()
    assert {pipe.owner(s) for s in range(steps)} <= {0, 1}
    for s in range(steps):
        res = pipe.results(s)
        assert len(res) == len(host)
        for i, (a, b) in enumerate(zip(res, host)):
            assert np.array_equal(a.T, b.T), (s, i, a.T - b.T)
            assert (a.num_iterations, a.num_pure_se3_iterations) == (b.num_iterations, b.num_pure_se3_iterations)


def test_in_flight_slots_with_different_batches_are_isolated(se3icp_mod):
    """Calls in flight on different engine slots with DIFFERENT batches (a KITTI-like gicp
    batch beside an RGB-D pt2pl batch with confidences off, then swapped) return bitwise the
    results of each batch registered alone: the slots share no buffer or state."""
    torch = pytest.importorskip("torch")
    from se3icp import datasets
    ka, _ = datasets.kitti_like_pairs(3, seed=4)
    rb, _ = datasets.rgbd_pairs(6, seed=5, stride=4)
    jobs = [(ka, "se3_gicp", se3icp_mod.kitti_params()), (rb, "se3_pt2pl", se3icp_mod.lounge_params())]
    alone = [se3icp_mod.register_batch(pairs, m, p) for pairs, m, p in jobs]
    dev = []
    for pairs, m, p in jobs:
        src = np.ascontiguousarray(np.concatenate([a for a, _ in pairs]))
        tgt = np.ascontiguousarray(np.concatenate([b for _, b in pairs]))
        so = np.concatenate([[0], np.cumsum([a.shape[0] for a, _ in pairs])])
        to = np.concatenate([[0], np.cumsum([b.shape[0] for _, b in pairs])])
        dev.append((torch.from_numpy(src).to("cuda:0"), so, torch.from_numpy(tgt).to("cuda:0"), to, m, p))
    torch.cuda.synchronize()
    for order in ((0, 1), (1, 0)):
        def factory(slot, order=order):
            ds, so, dt, to, m, p = dev[order[slot]]
            return se3icp_mod.DeviceBatchRunner(ds.data_ptr(), so, dt.data_ptr(), to, m, p, device=0 | (slot << 8),
                                                slots=4)
        pipe = se3icp_mod.PipelinedBatchRunner(factory, in_flight=2, steps=4)
        pipe.warm()
        pipe.run_steps()
        for s in range(4):
            job = order[pipe.owner(s)]
            for i, (a, b) in enumerate(zip(pipe.results(s), alone[job])):
                assert np.array_equal(a.T, b.T), (order, s, job, i, a.T - b.T)
                assert a.num_iterations == b.num_iterations, (order, s, job, i)


def _lrf_cloud(kind):
    from se3icp import datasets
    if kind == "kitti":
        pairs, _ = datasets.kitti_like_pairs(1, seed=4, first=2, total_pairs=8)
        return pairs[0][0]
    # a lattice: ranks with exactly equal f64 distances everywhere (ties k_lrf8 resolves by
    # the point index); jittered by ~1e-12, distances equal in f32 but not in f64 (the
    # queries go to the exact kernel)
    g = np.stack(np.meshgrid(np.arange(48), np.arange(40), np.arange(12), indexing="ij"), -1).reshape(-1, 3) * 0.05
    if kind == "lattice_jitter":
        g = g + np.random.default_rng(3).standard_normal(g.shape) * 1e-12
    return g


@pytest.mark.parametrize("kind", ["kitti", "lattice", "lattice_jitter"])
@pytest.mark.parametrize("k", [90, 30])
def test_lrf_fast_path_equals_exact_kernel(se3icp_mod, k, kind):
    """k_lrf8 (eight queries per wavefront) and the exact one-query-per-wavefront k_lrf
    give bitwise-identical TOLDI frames and normals (same neighbour sets in the same rank
    order, same arithmetic), at C4 size and on lattices full of distance ties: the fast path
    can never change a result."""
    from se3icp import registration
    pts = _lrf_cloud(kind)
    fast_f = se3icp_mod.toldi_frames(pts, k)
    fast_n = se3icp_mod.estimate_normals(pts, k)
    registration.set_lrf_exact(True)
    try:
        ex_f = se3icp_mod.toldi_frames(pts, k)
        ex_n = se3icp_mod.estimate_normals(pts, k)
    finally:
        registration.set_lrf_exact(False)
    same_f = (fast_f.view(np.uint64) == ex_f.view(np.uint64)).reshape(len(pts), -1).all(axis=1)
    assert same_f.all(), np.nonzero(~same_f)[0][:8]
    assert np.array_equal(fast_n.view(np.uint64), ex_n.view(np.uint64))


@pytest.mark.parametrize("kind", ["duplicates", "tiny", "collinear"])
def test_degenerate_clouds_knn_and_frames(se3icp_mod, refcpu, kind):
    """Tree build and kNN on degenerate inputs: many exactly repeated points (median splits
    through runs of equal keys, zero-variance sub-nodes), a cloud smaller than one leaf,
    and points on a line (two dimensions without extent).  kNN distances equal the oracle's
    (sets may differ only inside exact-distance ties), and the fast kernel's frames and
    normals equal the exact kernel's bit for bit."""
    from se3icp import registration
    rng = np.random.default_rng(11)
    if kind == "duplicates":
        base = rng.standard_normal((60, 3))
        pts = base[rng.integers(0, 60, 3000)] + 0.0
    elif kind == "tiny":
        pts = rng.standard_normal((40, 3))
    else:
        t = np.sort(rng.random(5000))
        pts = np.stack([t, 2.0 * t, -t], axis=1)
    k = min(30, len(pts))
    g = se3icp_mod.knn_self(pts, k)
    ri, rd = refcpu.knn_self(pts, k)
    dg = np.sum((pts[g] - pts[:, None, :]) ** 2, axis=2)
    np.testing.assert_allclose(np.sort(dg, axis=1), rd, rtol=0, atol=1e-12)
    fast_f = se3icp_mod.toldi_frames(pts, k)
    fast_n = se3icp_mod.estimate_normals(pts, k)
    registration.set_lrf_exact(True)
    try:
        ex_f = se3icp_mod.toldi_frames(pts, k)
        ex_n = se3icp_mod.estimate_normals(pts, k)
    finally:
        registration.set_lrf_exact(False)
    assert np.array_equal(fast_f.view(np.uint64), ex_f.view(np.uint64))
    assert np.array_equal(fast_n.view(np.uint64), ex_n.view(np.uint64))


def test_lrf_fast_path_equals_exact_kernel_in_a_batch(se3icp_mod):
    """In a multi-cloud batch k_lrf8's waves are aligned per cloud (the wave -> position
    table) and each cloud's last, partial, wave is handed over whole to the exact kernel.
    A batch of pairs whose cloud sizes are not multiples of 8 registers to bitwise the same
    poses and iteration counts with the fast path as with the exact kernel for every point."""
    from se3icp import datasets, registration
    pairs, _ = datasets.kitti_like_pairs(3, seed=4, n_az=300)
    rng = np.random.default_rng(5)
    cut = []
    for s, t in pairs:  # sizes = 1..7 (mod 8)
        ns = len(s) - (len(s) % 8) - int(rng.integers(1, 8))
        nt = len(t) - (len(t) % 8) - int(rng.integers(1, 8))
        cut.append((s[:ns], t[:nt]))
    assert all(len(s) % 8 and len(t) % 8 for s, t in cut)
    p = se3icp_mod.kitti_params()
    fast = se3icp_mod.register_batch(cut, "se3_gicp", p)
    registration.set_lrf_exact(1)
    try:
        exact = se3icp_mod.register_batch(cut, "se3_gicp", p)
    finally:
        registration.set_lrf_exact(0)
    for i, (a, b) in enumerate(zip(fast, exact)):
        assert np.array_equal(a.T, b.T), (i, a.T - b.T)
        assert (a.num_iterations, a.num_pure_se3_iterations) == (b.num_iterations, b.num_pure_se3_iterations)


def test_engine_slots_are_independent_engines(se3icp_mod):
    """device | slot << 8 selects a further engine on the same GPU (own stream and buffers,
    capi.cpp usable_engine): two slots registering two halves of a batch from two host
    threads return bitwise the poses of one call over the whole batch."""
    import threading
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(4, seed=4, n_az=600)
    p = se3icp_mod.kitti_params()
    whole = se3icp_mod.register_batch(pairs, "se3_gicp", p)
    out = {}

    def run(slot, part):
        out[slot] = se3icp_mod.register_batch(part, "se3_gicp", p, device=slot << 8)

    th = [threading.Thread(target=run, args=(s, pairs[2 * s - 2:2 * s])) for s in (1, 2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    got = out[1] + out[2]
    for i, (a, b) in enumerate(zip(got, whole)):
        assert np.array_equal(a.T, b.T), (i, a.T - b.T)
        assert a.num_iterations == b.num_iterations
    with pytest.raises(Exception):
        se3icp_mod.register_batch(pairs[:1], "se3_gicp", p, device=(16 << 8))  # slots 0..15
