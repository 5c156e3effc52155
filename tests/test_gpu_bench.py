"""bench.py's multi-rank path on one GPU: two ranks (gloo, both on cuda:0) register the
two blocks (4 + 3) of a fixed 7-pair C3 batch -- bench.py's strong-scaling shard; the
gathered poses must be bitwise those of a one-rank run over the same 7 pairs (SURVEY.md
§4 (v), §8e).  The 8-GPU RCCL run is the driver's."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(900)  # (a fresh box's first `import torch` alone can take minutes)
def test_two_rank_bench_equals_one_rank(tmp_path):
    common = ["--steps", "1", "--warmup", "0", "--workload", "C3", "--cpu-baseline", "off", "--global-batch", "7"]
    one = tmp_path / "one.npy"
    two = tmp_path / "two.npy"
    env = dict(os.environ)
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-poses",
                         str(one)] + common, capture_output=True, text=True, timeout=300, env=env)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                         "--gpus", "2", "--backend", "gloo", "--dump-poses", str(two)] + common,
                        capture_output=True, text=True, timeout=300, env=env)
    assert r2.returncode == 0, r2.stderr[-3000:]
    import json
    line = [l for l in r2.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["global_batch_pairs"] == 7 and d["scaling"] == "strong"
    assert d["config"]["pairs_per_gpu"] == [4, 3]
    a, b = np.load(one), np.load(two)
    assert a.shape == b.shape == (7, 4, 4)
    assert np.array_equal(a, b)


@pytest.mark.timeout(900)
def test_two_rank_balanced_shards_equal_one_rank(tmp_path):
    """--shard balanced: the 7 pairs assigned by point count (not in contiguous blocks); the
    gathered poses come back in batch order, bitwise those of one rank."""
    common = ["--steps", "1", "--warmup", "0", "--workload", "C3", "--cpu-baseline", "off", "--global-batch", "7"]
    one, two = tmp_path / "one.npy", tmp_path / "two.npy"
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-poses", str(one)] + common,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                         "--gpus", "2", "--backend", "gloo", "--shard", "balanced", "--dump-poses", str(two)] + common,
                        capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    import json
    d = json.loads([l for l in r2.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["config"]["shard"] == "balanced"
    assert np.array_equal(np.load(one), np.load(two))


def _rccl_rank(out_path, port):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "se3-icp_amd"))
    from se3icp import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl"
    rows = np.zeros((3, sharding.REC))
    rows[:, :16] = np.eye(4).reshape(16)
    rows[:, 16] = [5, 6, 7]
    res = sharding.exchange_results(dist, dev, 1.25, 0.5, 18, rows, pair_ids=[2, 0, 1])
    dist.destroy_process_group()
    np.savez(out_path, elapsed=res[0], iters=res[2], it=res[3].num_iterations)


@pytest.mark.timeout(600)
def test_result_exchange_runs_on_rccl(tmp_path):
    """The bench's end-of-batch exchange (all-reduce of the times and iterations, all-gather
    of the records) over torch.distributed's "nccl" backend -- RCCL on ROCm -- in a one-rank
    process group on the box's GPU (the 8-GPU job is the driver's); the records come back in
    pair order."""
    import multiprocessing as mp
    out = tmp_path / "rccl.npz"
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rccl_rank, args=(str(out), _port()))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    d = np.load(out)
    assert float(d["elapsed"]) == 1.25 and int(d["iters"]) == 18
    assert list(d["it"]) == [6, 7, 5]
