/*
 * se3icp_cc.h — the callers' side of the registration path:
 * the reference's error metrics (namespace cc, src/cc.cpp; avgEulError,
 * examples/benchmark_lounge.cpp:14-81) and its dataset pose formats (KITTI pose file,
 * examples/benchmark_kitti.cpp:72-98; Redwood .log trajectory,
 * examples/benchmark_lounge.cpp:99-140; 12-values-per-line trajectories / gt_data,
 * src/cc.cpp read_trajectory, examples/benchmark_synthetic.cpp:306-329).
 * Host code in libse3icp.so; no GPU needed.  Matrices are row-major float64
 * (3x3 = 9 doubles, 4x4 = 16 doubles).  Angles in degrees unless stated.
 */
#ifndef SE3ICP_CC_H
#define SE3ICP_CC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cc::rot_3d (cc.cpp:21-29): R = Rz(yaw) Ry(pitch) Rx(roll), radians */
void se3icp_cc_rot_3d(double roll, double pitch, double yaw, double R[9]);
/* cc::angularErrorSO3 (cc.cpp:32-37): |vee(log(R1^T R2))| in degrees */
double se3icp_cc_angular_error_so3(const double R1[9], const double R2[9]);
/* cc::angularErrorSO3_alt (cc.cpp:50-60): acos((tr(R1^T R2) - 1) / 2) in degrees, clamped */
double se3icp_cc_angular_error_so3_alt(const double R1[9], const double R2[9]);
/* cc::error_filterreg (cc.cpp:4-19): mean |T_gt p - T_est p| over the n points (AoS xyz) */
double se3icp_cc_error_filterreg(const double* xyz, int64_t n, const double T_gt[16], const double T_est[16]);
/* rot2euler (benchmark_lounge.cpp:14-49): (bank, attitude, heading) in radians */
void se3icp_cc_rot2euler(const double R[9], double euler[3]);
/* avgEulError (benchmark_lounge.cpp:59-81): mean absolute Euler-angle difference, degrees */
double se3icp_cc_avg_eul_error(const double R1[9], const double R2[9]);
/* cc::evaluate_LRF_quality (cc.cpp:62-86): mean angularErrorSO3_alt between the
 * rotations of map_gt * source frame[first] and target frame[second]; frames are
 * n x 16 row-major 4x4, pairs are n_pairs x 2 int32 */
double se3icp_cc_evaluate_lrf_quality(const double* src_frames, const double* tgt_frames, const double map_gt[16],
                                      const int32_t* pairs, int64_t n_pairs);
/* cc::evaluate_trajectory_quality (cc.cpp:165-201) on in-memory trajectories (n x 16):
 * out[3] = {average translation error, average rotation error (deg), success rate}
 * with the reference's failure thresholds (rotation > 2 deg or translation > 0.25) */
int se3icp_cc_evaluate_trajectory(const double* gt, const double* est, int64_t n, double out[3]);

/* Pose files.  Readers return the number of poses found (>= 0) and write at most `cap`
 * 4x4 matrices (n x 16 row-major) into out (may be NULL to count); -1 if unreadable.
 *   trajectory: 12 values per line, rows of [R|t] (cc::read_trajectory, gt_data files)
 *   kitti:      same line format, every other line is used (benchmark_kitti.cpp:72-98)
 *   redwood:    "id1 id2 frame" header + 4 matrix rows per entry (RGBDTrajectory) */
int64_t se3icp_cc_read_trajectory(const char* path, double* out, int64_t cap);
int64_t se3icp_cc_read_kitti_poses(const char* path, double* out, int64_t cap);
int64_t se3icp_cc_read_redwood_log(const char* path, double* out, int32_t* ids /* n x 3, may be NULL */, int64_t cap);
int se3icp_cc_write_trajectory(const char* path, const double* poses, int64_t n);
int se3icp_cc_write_redwood_log(const char* path, const double* poses, const int32_t* ids /* n x 3 */, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* SE3ICP_CC_H */
