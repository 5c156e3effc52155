"""Multi-rank path of bench.py on the CPU: gloo, world_size 2.

The GPU box runs the same code over RCCL ("nccl"); here the exchange is checked with the
gloo backend, one process per rank, rendezvous on 127.0.0.1.
"""
import os
import socket

import numpy as np
import pytest

from se3icp import datasets, sharding


def test_shard_is_a_contiguous_partition():
    for total in (1, 7, 8, 64, 65):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                first, count = sharding.shard(total, world, r)
                seen.extend(range(first, first + count))
            assert seen == list(range(total))
    with pytest.raises(ValueError):
        sharding.shard(8, 2, 2)


def test_sharded_pairs_equal_the_single_rank_pairs():
    kw = dict(seed=4, n_az=120)
    single, gts1 = datasets.kitti_like_pairs(4, total_pairs=4, **kw)
    for rank in range(2):
        first, count = sharding.shard(4, 2, rank)
        mine, gts = datasets.kitti_like_pairs(count, first=first, total_pairs=4, **kw)
        for k in range(count):
            np.testing.assert_array_equal(mine[k][0], single[first + k][0])
            np.testing.assert_array_equal(mine[k][1], single[first + k][1])
            np.testing.assert_array_equal(gts[k], gts1[first + k])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_poses(rank, n):
    return np.stack([np.eye(4) * (1 + rank) + k for k in range(n)])


def _rank_main(rank, world, port, out_dir, total=None):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 3 if total is None else sharding.shard(total, world, rank)[1]
    poses = _rank_poses(rank, n)
    res = sharding.exchange_results(dist, torch.device("cpu"), elapsed_s=1.0 + rank, loop_s=0.5 * (rank + 1),
                                    iterations=10 * (rank + 1), poses=poses)
    dist.barrier()
    dist.destroy_process_group()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), elapsed=res[0], loop=res[1], iters=res[2], poses=res[3])


def test_exchange_results_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    expect = np.concatenate([np.stack([np.eye(4) * (1 + r) + k for k in range(3)]) for r in range(world)])
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        assert float(d["elapsed"]) == 2.0      # max over ranks
        assert float(d["loop"]) == 1.0
        assert int(d["iters"]) == 30           # sum over ranks
        np.testing.assert_array_equal(d["poses"], expect)   # rank-ordered gather, bitwise


def test_exchange_results_single_rank_is_identity():
    poses = np.stack([np.eye(4)] * 2)
    e, l, it, p = sharding.exchange_results(None, None, 1.5, 0.5, 7, poses)
    assert (e, l, it) == (1.5, 0.5, 7)
    np.testing.assert_array_equal(p, poses)


def test_exchange_results_uneven_shards_gloo_world2(tmp_path):
    """5 pairs over 2 ranks: shard() gives 3 + 2; the gather pads to the largest block and
    returns exactly the 5 poses in rank order."""
    import torch.multiprocessing as mp

    world, total = 2, 5
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    expect = np.concatenate([_rank_poses(r, sharding.shard(total, world, r)[1]) for r in range(world)])
    assert expect.shape[0] == total
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        np.testing.assert_array_equal(d["poses"], expect)
