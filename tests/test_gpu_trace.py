"""Correspondence-level parity inside the loop (BASELINE.json north_star: "same
correspondences for integer arg-min").

The engine records one pair's loop iteration by iteration (se3icp_set_trace): the
pre-trim correspondence of every source point (target index + the float distance of
the pcl::Correspondence, ISR.cpp:444-470 / 402-416), the trimmed rejector's cut
(ISR.cpp:669-671), the pose and the MSE.  The oracle records the same from its own
loop (refcpu_trace) plus each query's 2-NN margin.  For every iteration:

* indices: equal, except where the oracle's best and second-best targets are a
  rounding-level near-tie (squared-distance gap <= NEAR_TIE_REL * d2 + DIST_NOISE^2).  The
  GPU forms the query as T.M0 with the composed pose while the
  reference rewrites each SE(3) element per iteration (ISR.cpp:713-716), so the two
  f64 queries differ by a few ulps and a near-tie may legitimately resolve the other
  way; every such case is counted and printed, and must pick the oracle's runner-up.
* float distances of equal correspondences: equal up to 1 ulp (the same f64->float
  rounding of a few-ulp-different f64 value) or, for distances at the f64 noise floor
  (a converged noise-free pair), within DIST_NOISE; counted;
* trimmed sets: equal up to the swaps those 1-ulp keys can cause at the cut;
* pose after the iteration: within 1e-9 (relative to |T|) of the oracle's;
* iteration counts (both phases): identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NEAR_TIE_REL = 1e-11   # relative squared-distance gap treated as a rounding-level tie
DIST_NOISE = 1e-12     # |float distance| difference at the f64 noise level of normalized coordinates (|p| <= 3)


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


def _kept(dist, cut):
    n = dist.shape[0]
    keys = (dist.view(np.uint32).astype(np.uint64) << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    return np.nonzero(keys <= np.uint64(cut))[0]


def compare_traces(gtr, ref, overlap, label):
    """Iteration-by-iteration comparison; returns the per-run counters (also printed)."""
    n_it = ref["num_iterations"]
    assert len(gtr["phase"]) == n_it, (label, len(gtr["phase"]), n_it)
    T_ref = np.eye(4)
    tot = {"queries": 0, "idx_diff": 0, "near_ties": 0, "dist_ulp1": 0, "kept_swaps": 0, "max_tie_gap": 0.0,
           "max_pose_diff": 0.0}
    for it in range(n_it):
        gi, ri = gtr["corr_idx"][it], ref["corr_idx"][it]
        gd, rd = gtr["corr_dist"][it], ref["corr_dist"][it]
        ns = gi.shape[0]
        tot["queries"] += ns
        diff = np.nonzero(gi != ri)[0]
        if diff.size:
            d2a, d2b, i2 = ref["corr_d2"][it][diff], ref["corr_d2b"][it][diff], ref["corr_idx2"][it][diff]
            gap = (d2b - d2a) / np.maximum(d2a, 1e-300)
            bad = ((d2b - d2a) > NEAR_TIE_REL * d2a + DIST_NOISE ** 2) | (gi[diff] != i2)
            assert not bad.any(), (label, it + 1, "non-tie correspondence differs", diff[bad][:8], gi[diff][bad][:8],
                                   ri[diff][bad][:8], gap[bad][:8])
            tot["idx_diff"] += diff.size
            tot["near_ties"] += diff.size
            tot["max_tie_gap"] = max(tot["max_tie_gap"], float(gap.max()))
        same = gi == ri
        ulps = np.abs(gd.view(np.int32).astype(np.int64) - rd.view(np.int32).astype(np.int64))
        # distances at the f64 rounding-noise level (a converged noise-free pair such as the
        # fixture: target = R source + t exactly) carry no information in their float bits
        noise = np.abs(gd.astype(np.float64) - rd.astype(np.float64)) <= DIST_NOISE
        off = same & (ulps > 1) & ~noise
        assert not off.any(), (label, it + 1, "float distance off by > 1 ulp", np.nonzero(off)[0][:8],
                               gd[off][:8], rd[off][:8])
        tot["dist_ulp1"] += int((same & (ulps > 0)).sum())
        # trimmed sets (PCL keeps floor(float(ratio) * N) smallest (dist, idx) keys)
        cut = int(gtr["trim_key"][it])
        if overlap < 1.0:
            g_kept = _kept(gd, cut)
            r_kept = np.sort(ref_trim(rd, overlap))
            assert g_kept.shape[0] == ref["n_kept"][it], (label, it + 1, g_kept.shape[0], ref["n_kept"][it])
            sym = np.setxor1d(g_kept, r_kept)
            n_moved = diff.size + int((same & (ulps > 0)).sum())
            assert sym.size <= 2 * n_moved, (label, it + 1, "trimmed sets differ beyond the moved keys", sym[:8])
            tot["kept_swaps"] += sym.size // 2
        else:
            assert cut == np.iinfo(np.uint64).max
        # pose after the iteration (normalized frame) and its MSE
        T_ref = ref["Ti"][it] @ T_ref
        dT = float(np.linalg.norm(gtr["T"][it] - T_ref))
        tot["max_pose_diff"] = max(tot["max_pose_diff"], dT)
        assert dT <= 1e-9 * max(1.0, np.linalg.norm(T_ref)), (label, it + 1, dT)
        assert abs(gtr["mse"][it] - ref["mse"][it]) <= 1e-9 * abs(ref["mse"][it]) + DIST_NOISE, \
            (label, it + 1, gtr["mse"][it], ref["mse"][it])
    print(f"[trace] {label}: {n_it} iterations, {tot['queries']} correspondences; index differences "
          f"{tot['idx_diff']} (all rounding-level near-ties, max relative gap {tot['max_tie_gap']:.2e}); "
          f"float distances not bit-equal {tot['dist_ulp1']}; trimmed-set swaps {tot['kept_swaps']}; "
          f"max pose diff {tot['max_pose_diff']:.2e}")
    return tot


def ref_trim(dist, ratio):
    from oracle import refcpu
    return refcpu.trim(dist, ratio)


def _run_both(se3icp_mod, refcpu, src, tgt, method, gparams, rkind, rvariant, rparams, max_iters=160):
    res, gtr = se3icp_mod.register_batch_traced([(src, tgt)], method, gparams, pair=0, max_iters=max_iters)
    ref = refcpu.register(src, tgt, rkind, rvariant, rparams, trace_iters=max_iters, trace_margins=True)
    assert res[0].num_iterations == ref["num_iterations"]
    assert res[0].num_pure_se3_iterations == ref["num_pure_se3_iterations"]
    return res[0], gtr, ref


def _record(parity_record, label, tot, g, ref):
    parity_record("trace: " + label, iterations=int(ref["num_iterations"]),
                  pure_se3_iterations=int(ref["num_pure_se3_iterations"]), rechecked_queries=int(g.num_rechecked), **tot)


@pytest.mark.parametrize("variant", ["pt2pt", "pt2pl", "gicp"])
def test_fixture_correspondences_every_iteration(se3icp_mod, refcpu, fixture_clouds, variant, parity_record):
    """C1 (examples/run_registration_method.cpp:38-42): both phases, no trimming.  The
    fixture has 188 groups of duplicate points (exact f64 ties: lowest index on both sides)."""
    src, tgt = fixture_clouds
    g, gtr, ref = _run_both(se3icp_mod, refcpu, src, tgt, "se3_" + variant, se3icp_mod.cli_params(),
                            refcpu.RUN_SE3_ICP, variant, refcpu.cli_params())
    assert set(gtr["phase"].tolist()) == {1, 2}
    _record(parity_record, f"C1 se3_{variant}", compare_traces(gtr, ref, 1.0, f"C1 se3_{variant}"), g, ref)


def test_kitti_full_size_correspondences_every_iteration(se3icp_mod, refcpu, parity_record):
    """C4 size (~120k points), se3_gicp with the KITTI driver's parameters
    (examples/benchmark_kitti.cpp:133-148): trimmed at overlap 0.7, both phases."""
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(1, seed=4, first=5, total_pairs=8)
    src, tgt = pairs[0]
    assert src.shape[0] > 100_000
    rp = refcpu.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                               number_of_nn_for_LRF=90)
    g, gtr, ref = _run_both(se3icp_mod, refcpu, src, tgt, "se3_gicp", se3icp_mod.kitti_params(),
                            refcpu.RUN_SE3_ICP, "gicp", rp)
    assert set(gtr["phase"].tolist()) == {1, 2}
    tot = compare_traces(gtr, ref, 0.7, "C4 se3_gicp 120k")
    _record(parity_record, "C4 se3_gicp 120k", tot, g, ref)
    # near-ties are rare: well under one query in 10^4
    assert tot["idx_diff"] <= 1e-4 * tot["queries"]


def test_rgbd_cf_correspondences_every_iteration(se3icp_mod, refcpu, parity_record):
    """run_se3_icp_with_cf (ISR.cpp:742-959) on a C5-style RGB-D pair (trimmed at 0.75,
    confidence-weighted GICP, translation rows from the points)."""
    from se3icp import datasets
    pairs, _ = datasets.rgbd_pairs(1, seed=5, stride=4)
    src, tgt = pairs[0]
    rp = refcpu.default_params(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                               number_of_nn_for_LRF=90)
    g, gtr, ref = _run_both(se3icp_mod, refcpu, src, tgt, "se3_gicp_with_cf", se3icp_mod.lounge_params(),
                            refcpu.RUN_SE3_ICP_CF, "gicp", rp)
    _record(parity_record, "cf RGB-D", compare_traces(gtr, ref, 0.75, "cf RGB-D"), g, ref)


def test_trace_is_one_shot_and_optional(se3icp_mod, fixture_clouds):
    """The trace arms one batch only, and a traced batch returns the same result as an
    untraced one (the record only reads device state)."""
    src, tgt = fixture_clouds
    p = se3icp_mod.cli_params()
    a = se3icp_mod.register_batch([(src, tgt)], "se3_pt2pl", p)[0]
    b, tr = se3icp_mod.register_batch_traced([(src, tgt)], "se3_pt2pl", p, max_iters=4)
    c = se3icp_mod.register_batch([(src, tgt)], "se3_pt2pl", p)[0]
    assert tr["phase"].shape[0] == min(4, b[0].num_iterations)
    assert np.array_equal(a.T, b[0].T) and np.array_equal(a.T, c.T)
    assert a.num_iterations == b[0].num_iterations == c.num_iterations


# --------------------------------------------------------------------------- adversarial near-ties
def _near_tie_queries(data, rng, n_q):
    """Queries placed between a target and its nearest other target, offset along their
    difference by a log-uniform relative amount from 1e-17 (an ulp-level tie that f32
    cannot resolve) to 1e-4 (certified in f32), plus a small orthogonal component."""
    from scipy.spatial import cKDTree
    tree = cKDTree(data)
    a = rng.integers(0, data.shape[0], n_q)
    _, nb = tree.query(data[a], k=2)
    b = nb[:, 1]
    A, B = data[a], data[b]
    d = B - A
    nd = np.linalg.norm(d, axis=1, keepdims=True)
    mid = 0.5 * (A + B)
    eps = 10.0 ** rng.uniform(-17, -4, (n_q, 1)) * rng.choice([-1.0, 1.0], (n_q, 1))
    orth = rng.normal(0, 1, d.shape)
    orth -= (np.sum(orth * d, axis=1, keepdims=True) / nd ** 2) * d
    orth *= 0.3 * nd / np.maximum(np.linalg.norm(orth, axis=1, keepdims=True), 1e-300)
    return np.ascontiguousarray(mid + eps * d + orth)


@pytest.mark.parametrize("dim", [12, 3])
def test_adversarial_near_ties_at_120k(se3icp_mod, refcpu, dim, parity_record):
    """>= 100k queries, each within a few ulps (or more) of equidistant between its two
    nearest targets: the f32 sweep cannot order most of them, so the certificate
    (loopdev.hpp f32_err) must send them to the f64 recheck, whose answer must be the
    oracle's exactly (nanoflann summation order, lowest index on exact ties)."""
    rng = np.random.default_rng(20 + dim)
    n = 120_000
    if dim == 12:  # SE(3)-element-like vectors: alpha-weighted rotations + translations
        from scipy.spatial.transform import Rotation
        R = Rotation.random(n, random_state=7).as_matrix()
        t = rng.uniform(-3, 3, (n, 3))
        data = np.concatenate([3.0 * R.transpose(0, 2, 1).reshape(n, 9), t], axis=1)
    else:
        data = rng.uniform(-3, 3, (n, 3))
    q = _near_tie_queries(data, rng, n)
    gi, gd2, nrech = se3icp_mod.nearest_neighbors(q, data)
    ri, rd2 = refcpu.nn(q, data)
    mism = np.nonzero(gi != ri)[0]
    print(f"[near-tie] dim {dim}: {n} queries, {nrech} rechecked in f64, {mism.size} index differences")
    parity_record(f"adversarial near-ties {dim}-D", queries=n, rechecked_f64=int(nrech), index_differences=int(mism.size),
                  d2_bit_differences=int((gd2 != rd2).sum()))
    assert mism.size == 0, (mism[:8], gi[mism[:8]], ri[mism[:8]])
    assert np.array_equal(gd2, rd2)
    assert nrech >= n // 10  # most ulp-level ties cannot be certified in f32
