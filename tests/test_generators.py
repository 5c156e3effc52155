"""The synthetic benchmark generator (examples/benchmark_synthetic.cpp:91-160) on the GPU
(k_gen.hip): se3icp_synthetic_reference_device, the reference's own problems bit for bit,
and se3icp_synthetic_pairs, the same protocol on counter-based streams.

The reference-exact batch is checked against the host restatement
se3icp_synthetic_reference, itself pinned by the reference's fixture and its streams
(tests/test_reference_streams.py).

The GPU generator uses counter-based Philox streams and a keyed permutation, so its
samples differ from the reference's mt19937 / std::normal_distribution / Open3D shuffle
draws by construction (those are reproduced exactly by the host generator,
tests/test_reference_streams.py).  What is checked is the protocol: exact-size random
subsets without replacement (RandomDownSample), the ground-truth transform applied to the
target only (B_SYN:149), per-axis N(0, noise_var) noise (add_noise_to_point_cloud,
B_SYN:13-56: noise is the covariance diagonal), independence of source and target
subsets, determinism per seed, and that the registration path consumes the output."""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from se3icp import datasets


@pytest.mark.gpu
@pytest.mark.parametrize("setup", ["moderate", "easy"])
@pytest.mark.parametrize("ratio", [0.02, 0.2])
def test_reference_exact_batch_on_device_equals_host(bunny_full, setup, ratio):
    """B_SYN:91-160 for 8 cases with the driver's streams: the device clouds (gathered,
    Transform-ed without FMA, noise added on the GPU) equal the host generator's bit for
    bit, for the active "moderate" ranges (B_SYN:111-112) and the "easy" ones (:106-108)."""
    tr, rr = (10.0, np.pi / 2) if setup == "moderate" else (5.0, np.pi / 4)
    cloud = bunny_full * 50.0
    hs, ht, hT = datasets.synthetic_reference(cloud, 8, ratio=ratio, t_range=tr, r_range=rr)
    ds, dt, dT = datasets.synthetic_reference_gpu(cloud, 8, ratio=ratio, t_range=tr, r_range=rr)
    assert ds.shape == hs.shape == (8, int(ratio * cloud.shape[0]), 3)
    assert np.array_equal(dT, hT)
    assert np.array_equal(ds.view(np.uint64), hs.view(np.uint64))
    assert np.array_equal(dt.view(np.uint64), ht.view(np.uint64))


@pytest.mark.gpu
def test_reference_exact_batch_device_buffers(bunny_full):
    """The device-resident output (ready for se3icp_register_batch_device) is the same."""
    import torch
    cloud = bunny_full * 50.0
    k = int(0.02 * cloud.shape[0])
    d_src = torch.empty((8 * k, 3), dtype=torch.float64, device="cuda")
    d_tgt = torch.empty_like(d_src)
    kk, T = datasets.synthetic_reference_gpu(cloud, 8, out=(d_src.data_ptr(), d_tgt.data_ptr()))
    torch.cuda.synchronize()
    hs, ht, hT = datasets.synthetic_reference(cloud, 8)
    assert kk == k and np.array_equal(T, hT)
    assert np.array_equal(d_src.cpu().numpy().reshape(8, k, 3), hs)
    assert np.array_equal(d_tgt.cpu().numpy().reshape(8, k, 3), ht)


def test_synthetic_cases_ranges_and_determinism():
    # B_SYN:110-112 (moderate, active in the reference) and :106-108 (easy)
    for easy, tr, rr in [(False, 10.0, np.pi / 2), (True, 5.0, np.pi / 4)]:
        Ts = datasets.synthetic_cases(64, seed=7, easy=easy)
        assert Ts.shape == (64, 4, 4)
        assert np.all(np.abs(Ts[:, :3, 3]) <= tr)
        for T in Ts:
            R = T[:3, :3]
            assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.isclose(np.linalg.det(R), 1.0)
        assert np.array_equal(Ts, datasets.synthetic_cases(64, seed=7, easy=easy))


@pytest.mark.gpu
def test_noise_free_full_subset_is_a_permutation(bunny_unique):
    base = bunny_unique[:5000] * 50.0
    Ts = datasets.synthetic_cases(3, seed=2)
    src, tgt = datasets.synthetic_pairs_gpu(base, Ts, ratio=1.0, noise_var=0.0, seed=9)
    assert src.shape == (3, 5000, 3)
    key = lambda a: a[np.lexsort(a.T[::-1])]
    for c in range(3):
        assert np.array_equal(key(src[c]), key(base))                 # every point exactly once
        back = (np.linalg.inv(Ts[c]) @ np.c_[tgt[c], np.ones(5000)].T).T[:, :3]
        d, i = cKDTree(base).query(back)
        assert d.max() < 1e-9 and len(np.unique(i)) == 5000          # T applied to every point once
        assert not np.array_equal(src[c], base)                        # random order (shuffle)


@pytest.mark.gpu
def test_downsample_exact_size_without_replacement(bunny_unique):
    base = bunny_unique * 50.0
    n = base.shape[0]
    Ts = datasets.synthetic_cases(4, seed=1)
    src, tgt = datasets.synthetic_pairs_gpu(base, Ts, ratio=0.02, noise_var=0.0, seed=1)
    k = int(0.02 * n)  # Open3D RandomDownSample: (int)(ratio * n)
    assert src.shape == (4, k, 3) and tgt.shape == (4, k, 3)
    rows = {tuple(r) for r in base}
    assert len(rows) == n                                              # unique vertices
    for c in range(4):
        s = {tuple(r) for r in src[c]}
        assert len(s) == k and s <= rows                               # k distinct base points
    # source and target subsets are drawn independently; the source subset is shared by
    # every case (B_SYN:99, 146: downsampled once, copied per case), the targets differ
    back0 = (np.linalg.inv(Ts[0]) @ np.c_[tgt[0], np.ones(k)].T).T[:, :3]
    assert np.abs(back0 - src[0]).max() > 1.0
    assert np.array_equal(src[0], src[1])
    back1 = (np.linalg.inv(Ts[1]) @ np.c_[tgt[1], np.ones(k)].T).T[:, :3]
    assert {tuple(np.round(r, 6)) for r in back0} != {tuple(np.round(r, 6)) for r in back1}


@pytest.mark.gpu
def test_noise_statistics_and_seed_determinism():
    # a grid with spacing 100: every noisy point maps back to its base point by rounding
    g = np.arange(40, dtype=np.float64) * 100.0
    base = np.stack(np.meshgrid(g, g, g[:25], indexing="ij"), -1).reshape(-1, 3)   # 40000 points
    var = 0.005
    Ts = np.stack([np.eye(4)] * 2)
    src, tgt = datasets.synthetic_pairs_gpu(base, Ts, ratio=1.0, noise_var=var, seed=123)
    for a in (src, tgt):
        e = (a - np.round(a / 100.0) * 100.0).reshape(-1, 3)
        n = e.shape[0]
        assert np.all(np.abs(e.mean(0)) < 5 * np.sqrt(var / n))
        assert np.all(np.abs(e.var(0) / var - 1.0) < 0.03)
        assert abs(np.corrcoef(e.T)[0, 1]) < 0.02 and abs(np.corrcoef(e.T)[0, 2]) < 0.02
    s2, t2 = datasets.synthetic_pairs_gpu(base, Ts, ratio=1.0, noise_var=var, seed=123)
    assert np.array_equal(src, s2) and np.array_equal(tgt, t2)
    s3, _ = datasets.synthetic_pairs_gpu(base, Ts, ratio=1.0, noise_var=var, seed=124)
    assert not np.array_equal(src, s3)


@pytest.mark.gpu
def test_generated_cases_register_on_device(bunny_unique):
    """The generator's device buffers feed se3icp_register_batch_device directly (the
    batched synthetic benchmark path); easy cases are recovered."""
    import torch
    import se3icp
    base = bunny_unique * 50.0
    Ts = datasets.synthetic_cases(4, seed=3, easy=True)
    k = int(0.12 * base.shape[0])
    d_src = torch.empty((4 * k, 3), dtype=torch.float64, device="cuda")
    d_tgt = torch.empty_like(d_src)
    kk = datasets.synthetic_pairs_gpu(base, Ts, ratio=0.12, noise_var=0.005, seed=5,
                                      out=(d_src.data_ptr(), d_tgt.data_ptr()))
    assert kk == k
    torch.cuda.synchronize()
    off = np.arange(5, dtype=np.int64) * k
    res = se3icp.register_batch_device(d_src.data_ptr(), off, d_tgt.data_ptr(), off, "se3_pt2pt",
                                       se3icp.cli_params())
    host = datasets.synthetic_pairs_gpu(base, Ts, ratio=0.12, noise_var=0.005, seed=5)
    assert np.array_equal(d_src.cpu().numpy().reshape(4, k, 3), host[0])
    ok = 0
    for r, T in zip(res, Ts):
        dR = r.T[:3, :3].T @ T[:3, :3]
        ang = np.degrees(np.arccos(np.clip((np.trace(dR) - 1) / 2, -1, 1)))
        ok += int(ang < 2.0 and np.linalg.norm(r.T[:3, 3] - T[:3, 3]) < 0.5)
    assert ok >= 3, [r.T for r in res]
