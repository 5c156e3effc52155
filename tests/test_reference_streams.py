"""The reference's synthetic problems, number for number (se3icp_synthetic_reference,
csrc/gen_ref.cpp + refrand.hpp; host code, no GPU).

Pinned by the reference's own fixture (created_example_reg_problem/, made by
examples/create_and_save_reg_problem.cpp:14-52):
  * source.ply is PointCloud::RandomDownSample(0.02) of stanford_bunny.ply x 50 right after
    open3d::utility::random::Seed(1): reproduced exactly (every coordinate bit);
  * target.ply is that cloud Transform-ed by cc::rot_3d(pi/9, pi/8, -pi/7), t = (1, 2, 3):
    reproduced exactly by the Eigen-quaternion rot_3d and the sequential transform.
The driver's other streams (examples/benchmark_synthetic.cpp:34-35, 103-116) are libstdc++'s
std::mt19937 + uniform_real_distribution / normal_distribution.  They are checked against
an independent restatement: numpy's MT19937 (legacy seeding = std::mt19937(seed)) for the
raw words, and libstdc++'s published generate_canonical / uniform_real_distribution /
Marsaglia-polar normal_distribution written out below.
"""
import math
import os

import numpy as np
import pytest

from se3icp import datasets

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture():
    from se3icp.io import read_ply_xyz
    return read_ply_xyz(os.path.join(GOLD, "fixture_source.ply")), read_ply_xyz(os.path.join(GOLD, "fixture_target.ply"))


def test_random_downsample_reproduces_reference_fixture(bunny_full):
    src, _ = _fixture()
    got = datasets.random_downsample(bunny_full * 50.0, 0.02, seed=1)
    assert got.shape == src.shape == (4167, 3)
    assert np.array_equal(got, src)


def test_rot_3d_and_transform_reproduce_reference_fixture():
    """cc::rot_3d through the C-ABI (Eigen AngleAxis -> quaternion -> matrix) and Open3D's
    Transform arithmetic ((R0 x + R1 y) + R2 z) + t: target.ply bit for bit."""
    from se3icp import cc
    src, tgt = _fixture()
    R = cc.rot_3d(np.pi / 9, np.pi / 8, -np.pi / 7)
    t = np.array([1.0, 2.0, 3.0])
    q = ((R[:, 0][None] * src[:, :1] + R[:, 1][None] * src[:, 1:2]) + R[:, 2][None] * src[:, 2:3]) + t[None] * 1.0
    assert np.array_equal(q, tgt)


def test_noise_free_reference_protocol_source_is_the_fixture(bunny_full):
    src_fix, _ = _fixture()
    src, tgt, T = datasets.synthetic_reference(bunny_full * 50.0, 2, noise_var=0.0)
    assert np.array_equal(src[0], src_fix) and np.array_equal(src[1], src_fix)  # shared source (B_SYN:146)
    # targets: the transformed full cloud, downsampled with the continuing engine (B_SYN:147-148)
    full = bunny_full * 50.0
    for c in range(2):
        R, t = T[c, :3, :3], T[c, :3, 3]
        moved = ((R[:, 0][None] * full[:, :1] + R[:, 1][None] * full[:, 1:2]) + R[:, 2][None] * full[:, 2:3]) + t
        tree = {tuple(p) for p in moved.view(np.uint64).reshape(-1, 3)}
        assert all(tuple(p) in tree for p in tgt[c].view(np.uint64).reshape(-1, 3))
    assert not np.array_equal(tgt[0], tgt[1])


# ---- libstdc++'s distributions over numpy's MT19937 (independent restatement)
class _LibstdcxxStream:
    def __init__(self, seed):
        bg = np.random.MT19937()
        bg._legacy_seeding(seed)   # init_genrand(seed): std::mt19937(seed)
        self.bg = bg
        self.saved = None

    def word(self):
        return int(self.bg.random_raw())

    def canonical(self):  # generate_canonical<double, 53>: two 32-bit words, low first
        s = np.float64(self.word())
        s = s + np.float64(self.word()) * np.float64(4294967296.0)
        r = s / np.float64(18446744073709551616.0)
        return float(np.nextafter(1.0, 0.0)) if r >= 1.0 else float(r)

    def uniform(self, a, b):
        return self.canonical() * (b - a) + a

    def normal(self):  # Marsaglia polar, one value saved
        if self.saved is not None:
            v, self.saved = self.saved, None
            return v
        while True:
            x = 2.0 * self.canonical() - 1.0
            y = 2.0 * self.canonical() - 1.0
            r2 = x * x + y * y
            if not (r2 > 1.0 or r2 == 0.0):
                break
        mult = math.sqrt(-2.0 * math.log(r2) / r2)
        self.saved = x * mult
        return y * mult


def test_mt19937_known_answer():
    # std::mt19937 seeded 1: its first word (and numpy's legacy MT19937 agrees)
    assert _LibstdcxxStream(1).word() == 1791095845


@pytest.mark.parametrize("ltr", [False, True])
def test_reference_transforms_and_noise_follow_the_drivers_streams(bunny_full, ltr):
    from se3icp import cc
    cloud = bunny_full * 50.0
    n_cases = 3
    src, tgt, T = datasets.synthetic_reference(cloud, n_cases, args_left_to_right=ltr)
    src0, tgt0, T0 = datasets.synthetic_reference(cloud, n_cases, noise_var=0.0, args_left_to_right=ltr)
    assert np.array_equal(T, T0)
    gen = _LibstdcxxStream(1)
    for c in range(n_cases):
        t = [gen.uniform(-10.0, 10.0) for _ in range(3)]          # braced list: left to right
        a = [gen.uniform(-np.pi / 2, np.pi / 2) for _ in range(3)]
        roll, pitch, yaw = (a[0], a[1], a[2]) if ltr else (a[2], a[1], a[0])  # GCC: right to left
        assert np.array_equal(T[c, :3, 3], t)
        assert np.array_equal(T[c, :3, :3], cc.rot_3d(roll, pitch, yaw))
    # noise: one static N(0, 1) stream, sqrt(0.005) * z per coordinate, source copy then target
    noise = _LibstdcxxStream(1)
    sd = math.sqrt(0.005)
    for c in range(n_cases):
        for clean, noisy in ((src0[c], src[c]), (tgt0[c], tgt[c])):
            z = np.array([[noise.normal() for _ in range(3)] for _ in range(clean.shape[0])])
            assert np.array_equal(noisy, clean + sd * z)
