"""Work counters of the NN searches (bench.py's roofline accounting): the occupied
(query, target) evaluations beside the 64-lane evaluation slots, through the extended
kernel-times entry (se3icp_last_kernel_times_n, ABI 4)."""
import ctypes as C

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


def test_useful_evaluations_are_counted_and_bounded_by_the_slots(se3icp_mod):
    from se3icp import datasets
    pairs, _ = datasets.kitti_like_pairs(2, seed=4, n_az=400)
    params = se3icp_mod.default_params(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7,
                                       mse_switch_error=5e-7, number_of_nn_for_LRF=90)
    se3icp_mod.register_batch(pairs, "se3_gicp", params)
    kt = se3icp_mod.last_kernel_times()
    for ph in ("se3", "r3"):
        use, slots = kt[f"{ph}_useful_evals"], kt[f"{ph}_dist_evals"]
        assert use > 0, ph
        # a slot is one lane's evaluation: at most every slot is an occupied one
        assert use <= slots, (ph, use, slots)
    # the first 24 values are the ABI-3 record
    L = se3icp_mod._lib.load()
    old = (C.c_double * 24)()
    assert L.se3icp_last_kernel_times(0, old) == 0
    assert np.array_equal(np.array(list(old)), np.array([kt[k] for k in list(kt)[:24]]))


def test_kernel_times_n_rejects_a_short_buffer(se3icp_mod):
    L = se3icp_mod._lib.load()
    out = (C.c_double * 10)()
    assert L.se3icp_last_kernel_times_n(0, out, 10) == se3icp_mod._lib.ERR_INVALID_ARG
