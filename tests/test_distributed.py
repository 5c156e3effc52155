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


class _Res:  # a se3icp result's per-pair fields
    def __init__(self, T, it, pure, status):
        self.T, self.num_iterations, self.num_pure_se3_iterations, self.status = T, it, pure, status


def _rank_results(rank, n):
    return [_Res(T, 10 * rank + k + 1, 3 * rank + k, -7 if (rank, k) == (1, 1) else 0)
            for k, T in enumerate(_rank_poses(rank, n))]


def _rank_main(rank, world, port, out_dir, total=None):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 3 if total is None else sharding.shard(total, world, rank)[1]
    res = sharding.exchange_results(dist, torch.device("cpu"), elapsed_s=1.0 + rank, loop_s=0.5 * (rank + 1),
                                    iterations=10 * (rank + 1), records=sharding.pair_records(_rank_results(rank, n)))
    dist.barrier()
    dist.destroy_process_group()
    g = res[3]
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), elapsed=res[0], loop=res[1], iters=res[2], poses=g.T,
             num_iterations=g.num_iterations, pure=g.num_pure_se3_iterations, status=g.status)


def _expected_records(world, counts):
    rs = [r for rank in range(world) for r in _rank_results(rank, counts[rank])]
    return (np.stack([r.T for r in rs]), np.array([r.num_iterations for r in rs]),
            np.array([r.num_pure_se3_iterations for r in rs]), np.array([r.status for r in rs]))


def test_exchange_results_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    T, it, pure, st = _expected_records(world, [3, 3])
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        assert float(d["elapsed"]) == 2.0      # max over ranks
        assert float(d["loop"]) == 1.0
        assert int(d["iters"]) == 30           # sum over ranks
        np.testing.assert_array_equal(d["poses"], T)   # rank-ordered gather, bitwise
        np.testing.assert_array_equal(d["num_iterations"], it)
        np.testing.assert_array_equal(d["pure"], pure)
        np.testing.assert_array_equal(d["status"], st)


def test_exchange_results_single_rank_is_identity():
    res = _rank_results(1, 2)
    e, l, it, g = sharding.exchange_results(None, None, 1.5, 0.5, 7, sharding.pair_records(res))
    assert (e, l, it) == (1.5, 0.5, 7)
    np.testing.assert_array_equal(g.T, np.stack([r.T for r in res]))
    assert list(g.num_iterations) == [11, 12] and list(g.num_pure_se3_iterations) == [3, 4]
    assert list(g.status) == [0, -7]


def test_exchange_results_uneven_shards_gloo_world2(tmp_path):
    """5 pairs over 2 ranks: shard() gives 3 + 2; the gather pads to the largest block and
    returns exactly the 5 poses in rank order."""
    import torch.multiprocessing as mp

    world, total = 2, 5
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    T, it, pure, st = _expected_records(world, [sharding.shard(total, world, r)[1] for r in range(world)])
    assert T.shape[0] == total
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        np.testing.assert_array_equal(d["poses"], T)
        np.testing.assert_array_equal(d["num_iterations"], it)
        np.testing.assert_array_equal(d["pure"], pure)
        np.testing.assert_array_equal(d["status"], st)


def test_strong_plan_fixes_the_global_batch():
    """bench.py's default: BASELINE's batch (C4: 64 pairs) split over the ranks, so N=1 holds
    all 64 and N=8 eight each; uneven splits (64 over 3) keep every pair exactly once."""
    for world in (1, 2, 3, 4, 8):
        got = [sharding.plan(world, r, 64) for r in range(world)]
        assert all(g[0] == "strong" and g[1] == 64 for g in got)
        assert sum(g[3] for g in got) == 64
        assert [g[2] for g in got] == [sum(h[3] for h in got[:r]) for r in range(world)]
    assert [sharding.plan(3, r, 64)[3] for r in range(3)] == [22, 21, 21]
    assert sharding.plan(1, 0, 64) == ("strong", 64, 0, 64)
    assert sharding.plan(8, 7, 64) == ("strong", 64, 56, 8)
    assert sharding.plan(2, 1, 64, global_batch=7) == ("strong", 7, 4, 3)
    assert sharding.plan(4, 3, 64, pairs_per_gpu=8) == ("weak", 32, 24, 8)
    with pytest.raises(ValueError):
        sharding.plan(8, 7, 64, global_batch=5)


def _strong_rank_main(rank, world, port, out_dir, total):
    """One rank of a strong-scaling job: its plan() block of a `total`-pair batch, each pair
    identified by its global index in the record, through the result exchange."""
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scaling, tot, first, count = sharding.plan(world, rank, total)
    res = [_Res(np.eye(4) * (first + k), first + k, k, 0) for k in range(count)]
    out = sharding.exchange_results(dist, torch.device("cpu"), elapsed_s=float(count), loop_s=0.0,
                                    iterations=sum(r.num_iterations for r in res), records=sharding.pair_records(res))
    dist.barrier()
    dist.destroy_process_group()
    g = out[3]
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), elapsed=out[0], iters=out[2], poses=g.T, it=g.num_iterations)


def test_strong_shard_64_over_3_gloo(tmp_path):
    """BASELINE's 64-pair batch over 3 ranks (22 + 21 + 21): every pair is registered by
    exactly one rank and the gather returns all 64 in batch order."""
    import torch.multiprocessing as mp

    world, total = 3, 64
    mp.start_processes(_strong_rank_main, args=(world, _free_port(), str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        d = np.load(tmp_path / f"s{r}.npz")
        assert float(d["elapsed"]) == 22.0                 # max over ranks: the largest block
        assert int(d["iters"]) == sum(range(total))        # every pair counted once
        np.testing.assert_array_equal(d["it"], np.arange(total))
        np.testing.assert_array_equal(d["poses"], np.stack([np.eye(4) * k for k in range(total)]))


def test_balanced_shard_is_a_deterministic_partition():
    """sharding.shard_balanced: every pair exactly once, deterministic, and the largest
    rank load within one pair's cost of the smallest (LPT greedy)."""
    rng = np.random.default_rng(0)
    for n, world in ((64, 3), (64, 8), (7, 2), (256, 8), (8, 8)):
        costs = rng.integers(100_000, 130_000, n)
        plan = sharding.shard_balanced(costs, world)
        assert plan == sharding.shard_balanced(costs, world)
        assert sorted(i for p in plan for i in p) == list(range(n))
        assert all(p == sorted(p) and p for p in plan)
        loads = [int(costs[p].sum()) for p in plan]
        assert max(loads) - min(loads) <= int(costs.max())
    # equal costs: the counts of a contiguous split (22 + 21 + 21 for 64 over 3)
    assert sorted(len(p) for p in sharding.shard_balanced([1] * 64, 3)) == [21, 21, 22]
    with pytest.raises(ValueError):
        sharding.shard_balanced([1, 2], 3)


def _balanced_rank_main(rank, world, port, out_dir, costs):
    """One rank of a balanced job: its shard_balanced() pairs, each identified by its global
    index in the record, through the result exchange with the pair ids."""
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = sharding.shard_balanced(costs, world)[rank]
    res = [_Res(np.eye(4) * i, i, i % 5, 0) for i in ids]
    out = sharding.exchange_results(dist, torch.device("cpu"), elapsed_s=float(sum(costs[i] for i in ids)),
                                    loop_s=0.0, iterations=sum(r.num_iterations for r in res),
                                    records=sharding.pair_records(res), pair_ids=ids)
    dist.barrier()
    dist.destroy_process_group()
    g = out[3]
    np.savez(os.path.join(out_dir, f"b{rank}.npz"), elapsed=out[0], iters=out[2], poses=g.T, it=g.num_iterations,
             pure=g.num_pure_se3_iterations)


def test_balanced_shard_64_over_3_gloo(tmp_path):
    """A cost-balanced 64-pair batch over 3 ranks with uneven pair costs: the gather returns
    all 64 records in batch order (not rank order), and the job time is the max rank load."""
    import torch.multiprocessing as mp

    world, total = 3, 64
    costs = [int(c) for c in np.random.default_rng(1).integers(100_000, 130_000, total)]
    mp.start_processes(_balanced_rank_main, args=(world, _free_port(), str(tmp_path), costs), nprocs=world,
                       join=True, start_method="spawn")
    plan = sharding.shard_balanced(costs, world)
    for r in range(world):
        d = np.load(tmp_path / f"b{r}.npz")
        assert float(d["elapsed"]) == max(sum(costs[i] for i in p) for p in plan)
        assert int(d["iters"]) == sum(range(total))
        np.testing.assert_array_equal(d["it"], np.arange(total))
        np.testing.assert_array_equal(d["pure"], np.arange(total) % 5)
        np.testing.assert_array_equal(d["poses"], np.stack([np.eye(4) * k for k in range(total)]))


def test_exchange_results_single_rank_reorders_by_pair_id():
    res = [_Res(np.eye(4) * i, i, 0, 0) for i in (5, 2, 9)]
    _, _, _, g = sharding.exchange_results(None, None, 1.0, 0.0, 16, sharding.pair_records(res), pair_ids=[5, 2, 9])
    assert list(g.num_iterations) == [2, 5, 9]
