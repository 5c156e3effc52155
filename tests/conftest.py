import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "se3-icp_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


# Parity counters of the GPU tests (index near-ties, 1-ulp distances, trimmed-set swaps,
# rechecked queries, frames outside 1e-8 ...): recorded by the tests through the
# `parity_record` fixture and written at the end of the session to
# gpurun_out/parity_counters.json (merged back from the GPU box; the round's copy is
# committed under profiles/), so the record shows them without -s.
_PARITY = {}


@pytest.fixture(scope="session")
def parity_record():
    def rec(name, **counters):
        d = _PARITY.setdefault(name, {})
        for k, v in counters.items():
            d[k] = v.item() if hasattr(v, "item") else v
    return rec


def pytest_sessionfinish(session, exitstatus):
    if not _PARITY:
        return
    import json
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "parity_counters.json")
    old = {}
    if os.path.exists(path):
        try:
            old = json.load(open(path))
        except Exception:
            old = {}
    old.update(_PARITY)
    with open(path, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)


@pytest.fixture(scope="session")
def fixture_clouds():
    from se3icp.io import read_ply_xyz
    return (read_ply_xyz(os.path.join(GOLDEN, "fixture_source.ply")),
            read_ply_xyz(os.path.join(GOLDEN, "fixture_target.ply")))


@pytest.fixture(scope="session")
def fixture_T_gt():
    from se3icp import datasets
    import numpy as np
    # examples/create_and_save_reg_problem.cpp:31-37, cc::rot_3d(pi/9, pi/8, -pi/7), t = (1,2,3)
    return datasets.make_T(datasets.rot_3d(np.pi / 9, np.pi / 8, -np.pi / 7), [1.0, 2.0, 3.0])


@pytest.fixture(scope="session")
def bunny_unique():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "bunny_unique_f32.npy")).astype(np.float64)


_torch_gpu_ready = False


def pytest_runtest_setup(item):
    """GPU tests: bring up torch's HIP context before libse3icp's first HIP call, as
    bench.py does (torch only plumbs device buffers for the tests that need them)."""
    global _torch_gpu_ready
    if _torch_gpu_ready or item.get_closest_marker("gpu") is None:
        return
    _torch_gpu_ready = True
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # the test itself reports a missing device
        pass


@pytest.fixture(scope="session")
def bunny_full():
    """stanford_bunny.ply's 208,353 vertices in file order (tools/make_bunny_fixtures.py)."""
    import numpy as np
    u = np.load(os.path.join(GOLDEN, "bunny_unique_f32.npy"))
    ids = np.load(os.path.join(GOLDEN, "bunny_vertex_ids.npy"))
    return u[ids].astype(np.float64)
