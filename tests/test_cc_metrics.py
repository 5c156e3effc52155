"""Metrics and pose files of the reference's drivers (include/se3icp_cc.h).

The reference ships no tests for these; each function is checked against an independent
computation (scipy's rotation log map, numpy) or a hand-derived value, and the file
formats against text written in the reference drivers' own layouts.  Parity of the
restatement with the C++ originals is otherwise unpinned (Eigen's matrix log and
Open3D are not available here).
"""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from se3icp import cc, datasets


def _rand_R(rng):
    return Rotation.random(random_state=rng).as_matrix()


def test_rot_3d_matches_the_fixture_rotation(fixture_T_gt):
    # examples/create_and_save_reg_problem.cpp:31-37 uses cc::rot_3d(pi/9, pi/8, -pi/7)
    R = cc.rot_3d(np.pi / 9, np.pi / 8, -np.pi / 7)
    np.testing.assert_allclose(R, fixture_T_gt[:3, :3], atol=1e-15)
    np.testing.assert_allclose(R, datasets.rot_3d(np.pi / 9, np.pi / 8, -np.pi / 7), atol=1e-15)


def test_angular_errors_match_the_rotation_log_map():
    rng = np.random.default_rng(7)
    for k in range(200):
        A, B = _rand_R(rng), _rand_R(rng)
        if k % 3 == 0:   # small angles: the log form must stay accurate where acos is not
            B = A @ Rotation.from_rotvec(rng.normal(size=3) * 1e-7).as_matrix()
        ref = np.degrees(Rotation.from_matrix(A.T @ B).magnitude())
        assert abs(cc.angular_error_so3(A, B) - ref) <= 1e-9 * max(1.0, ref)
        assert abs(cc.angular_error_so3_alt(A, B) - ref) <= 1e-5   # acos form: sqrt(eps) near 0
    I = np.eye(3)
    assert cc.angular_error_so3(I, I) == 0.0 and cc.angular_error_so3_alt(I, I) == 0.0
    flip = np.diag([1.0, -1.0, -1.0])
    assert abs(cc.angular_error_so3(I, flip) - 180.0) < 1e-12


def test_error_filterreg_is_mean_displacement():
    rng = np.random.default_rng(3)
    P = rng.normal(size=(500, 3))
    G = datasets.make_T(_rand_R(rng), rng.normal(size=3))
    E = datasets.make_T(_rand_R(rng), rng.normal(size=3))
    ref = np.mean(np.linalg.norm(datasets.transform(G, P) - datasets.transform(E, P), axis=1))
    assert abs(cc.error_filterreg(P, G, E) - ref) <= 1e-12 * ref
    assert cc.error_filterreg(P, G, G) == 0.0


def test_avg_eul_error_known_values():
    I = np.eye(3)
    assert cc.avg_eul_error(I, I) == 0.0
    # a pure rotation about x by 10 deg changes only the bank angle -> mean = 10/3
    Rx = Rotation.from_euler("x", 10, degrees=True).as_matrix()
    assert abs(cc.avg_eul_error(Rx, I) - 10.0 / 3.0) < 1e-12
    e = cc.rot2euler(Rx)
    np.testing.assert_allclose(e, [np.radians(10), 0.0, 0.0], atol=1e-15)
    # singular branch (m10 > 0.998): attitude = +90 deg, bank 0
    Rz = Rotation.from_euler("z", 89.99, degrees=True).as_matrix()
    e = cc.rot2euler(Rz)
    assert e[0] == 0.0 and abs(e[1] - np.pi / 2) < 1e-15


def test_evaluate_trajectory_thresholds():
    gt = np.stack([np.eye(4)] * 4)
    est = gt.copy()
    est[1, :3, 3] = [0.3, 0, 0]                                     # translation fail (> 0.25)
    est[2, :3, :3] = Rotation.from_euler("z", 3, degrees=True).as_matrix()   # rotation fail (> 2 deg)
    est[3, :3, 3] = [0.1, 0, 0]
    r = cc.evaluate_trajectory(gt, est)
    assert abs(r["success_rate"] - 0.5) < 1e-15
    assert abs(r["avg_translation_error"] - 0.1) < 1e-12
    assert abs(r["avg_rotation_error"] - 0.75) < 1e-9


def test_evaluate_lrf_quality():
    rng = np.random.default_rng(5)
    n = 50
    src = np.stack([datasets.make_T(_rand_R(rng), rng.normal(size=3)) for _ in range(n)])
    G = datasets.make_T(_rand_R(rng), rng.normal(size=3))
    tgt = np.einsum("ij,njk->nik", G, src)        # exactly mapped frames -> zero error
    pairs = np.stack([np.arange(n), np.arange(n)], axis=1)
    assert cc.evaluate_lrf_quality(src, tgt, G, pairs) < 1e-5
    shuffled = pairs.copy()
    shuffled[:, 1] = np.roll(shuffled[:, 1], 1)
    ref = np.mean([np.degrees(Rotation.from_matrix((G @ src[i])[:3, :3].T @ tgt[j][:3, :3]).magnitude())
                   for i, j in shuffled])
    assert abs(cc.evaluate_lrf_quality(src, tgt, G, shuffled) - ref) < 1e-5
    with pytest.raises(IndexError):
        cc.evaluate_lrf_quality(src, tgt, G, [[0, n]])


def test_trajectory_and_kitti_pose_files(tmp_path):
    rng = np.random.default_rng(1)
    poses = np.stack([datasets.make_T(_rand_R(rng), rng.normal(size=3)) for _ in range(6)])
    p = tmp_path / "traj.txt"
    cc.write_trajectory(p, poses)
    np.testing.assert_array_equal(cc.read_trajectory(p), poses)   # %.17g round-trips
    # KITTI driver reads every other line (benchmark_kitti.cpp:80-97)
    np.testing.assert_array_equal(cc.read_kitti_poses(p), poses[::2])
    with pytest.raises(FileNotFoundError):
        cc.read_trajectory(tmp_path / "missing.txt")


def test_redwood_log_roundtrip_and_reference_layout(tmp_path):
    p = tmp_path / "lounge_trajectory.log"
    # the layout RGBDTrajectory::SaveToFile writes (benchmark_lounge.cpp:127-139)
    p.write_text("# comment line\n0\t1\t395\n1.0 0.0 0.0 0.5\n0.0 1.0 0.0 0.25\n0.0 0.0 1.0 -1.0\n0 0 0 1\n"
                 "1\t2\t395\n0.0 -1.0 0.0 0.0\n1.0 0.0 0.0 0.0\n0.0 0.0 1.0 0.0\n0.0 0.0 0.0 1.0\n")
    poses, ids = cc.read_redwood_log(p)
    assert poses.shape == (2, 4, 4) and ids.tolist() == [[0, 1, 395], [1, 2, 395]]
    assert poses[0][0, 3] == 0.5 and poses[1][1, 0] == 1.0
    q = tmp_path / "out.log"
    cc.write_redwood_log(q, poses, ids)
    text = q.read_text().splitlines()
    assert text[0] == "0\t1\t395" and text[1] == "1.00000000 0.00000000 0.00000000 0.50000000"
    poses2, ids2 = cc.read_redwood_log(q)
    np.testing.assert_array_equal(poses2, poses)
    np.testing.assert_array_equal(ids2, ids)


def test_lounge_ground_truth_composition(tmp_path):
    """benchmark_lounge.cpp:161-165: T12 = T2^-1 T1 from the .log poses."""
    rng = np.random.default_rng(2)
    traj = np.stack([datasets.make_T(_rand_R(rng), rng.normal(size=3)) for _ in range(10)])
    cc.write_redwood_log(tmp_path / "t.log", traj, np.stack([np.arange(10), np.arange(1, 11), [10] * 10], 1))
    T, _ = cc.read_redwood_log(tmp_path / "t.log")
    T12 = np.linalg.inv(T[5]) @ T[0]
    np.testing.assert_allclose(T12, np.linalg.inv(traj[5]) @ traj[0], atol=1e-6)   # 8-decimal file


@pytest.mark.gpu
def test_compute_corrs_with_gt_on_the_fixture(fixture_clouds, fixture_T_gt):
    src, tgt = fixture_clouds
    pairs = cc.compute_corrs_with_gt(src, tgt, fixture_T_gt)
    assert pairs.shape == (src.shape[0], 2)
    # target_i = T_gt source_i exactly: every source maps onto its own index (or an exact duplicate)
    d = np.linalg.norm(tgt[pairs[:, 1]] - tgt[pairs[:, 0]], axis=1)
    assert np.all(d <= 1e-9)
