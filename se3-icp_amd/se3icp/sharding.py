"""Pair sharding across ranks and the end-of-batch result exchange.

SURVEY.md §8(e): every scan pair is an independent registration (the reference's
drivers make one IterativeSE3Registration per pair, examples/benchmark_kitti.cpp:128),
so a batch of B pairs is split into contiguous blocks of B/G pairs per GPU and each rank
registers its block with no data-path collective.  The only exchange is at the end: the
max of the ranks' wall times (the job's time), the sum of their iteration counts and an
all-gather of every pair's result record — the pose, num_iterations_,
num_pure_se3_iterations_ and the status, what the reference's drivers report per pair
(examples/benchmark_kitti.cpp:163-197) — over RCCL/xGMI on the GPU box (gloo in the CPU
tests).  The gathered records are bitwise those of a single-rank run over the same pairs:
no arithmetic crosses ranks.
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np

REC = 19  # one pair's record: T (16, row-major), num_iterations, num_pure_se3_iterations, status


class PairRecords(NamedTuple):
    """The per-pair results of a whole (sharded) batch, in rank order."""
    T: np.ndarray                        # [n, 4, 4]
    num_iterations: np.ndarray           # [n] int
    num_pure_se3_iterations: np.ndarray  # [n] int (-1 for run_icp)
    status: np.ndarray                   # [n] int (se3icp_status)


def pair_records(results) -> np.ndarray:
    """[n, REC] float64 rows of se3icp results (objects with T, num_iterations,
    num_pure_se3_iterations, status); the integers are exact in float64."""
    rows = np.zeros((len(results), REC))
    for i, r in enumerate(results):
        rows[i, :16] = np.asarray(r.T, dtype=np.float64).reshape(16)
        rows[i, 16:] = (r.num_iterations, r.num_pure_se3_iterations, r.status)
    return rows


def unpack_records(rows: np.ndarray) -> PairRecords:
    rows = np.asarray(rows, dtype=np.float64).reshape(-1, REC)
    i = rows[:, 16:].astype(np.int64)
    return PairRecords(rows[:, :16].reshape(-1, 4, 4).copy(), i[:, 0], i[:, 1], i[:, 2])


def shard(n_pairs_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [first, first + count) of the pair list owned by `rank`
    (remainder pairs go to the lowest ranks)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, rem = divmod(n_pairs_total, world)
    count = base + (1 if rank < rem else 0)
    first = rank * base + min(rank, rem)
    return first, count


def shard_balanced(costs, world: int) -> list[list[int]]:
    """Cost-balanced assignment of pairs to ranks: longest-processing-time greedy over the
    pairs' costs (their point counts: the setup and every loop stage are per point), each
    pair to the rank with the least cost so far (ties: the lower rank), the pairs in order of
    decreasing cost (ties: the lower pair index).  Deterministic; every rank gets
    floor(n / world) or more pairs when the costs are equal.  Returns each rank's pair
    indices in ascending order."""
    costs = np.asarray(costs, dtype=np.float64)
    n = costs.shape[0]
    if world <= 0 or n < world:
        raise ValueError(f"{n} pairs cannot be balanced over {world} ranks")
    order = sorted(range(n), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    cnt = [0] * world
    out: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], cnt[q], q))
        out[r].append(i)
        load[r] += costs[i]
        cnt[r] += 1
    return [sorted(o) for o in out]


def plan(world: int, rank: int, default_batch: int, global_batch: int = 0, pairs_per_gpu: int = 0):
    """The rank's share of a benchmark job: (scaling, global_batch, first, count).

    Strong scaling (the default): the job registers a fixed batch -- `global_batch`, or the
    workload's BASELINE batch `default_batch` (C4: the 64 pairs of
    examples/benchmark_kitti.cpp:120-197) -- split into contiguous blocks over the ranks, so
    one GPU registers all of it and eight GPUs an eighth each.  Weak scaling when
    `pairs_per_gpu` is set: every rank registers that many pairs of a world x P batch."""
    if pairs_per_gpu:
        scaling, total = "weak", world * pairs_per_gpu
    else:
        scaling, total = "strong", global_batch or default_batch
    first, count = shard(total, world, rank)
    if count == 0:
        raise ValueError(f"a batch of {total} pairs leaves rank {rank} of {world} without a pair")
    return scaling, total, first, count


def exchange_results(dist, device, elapsed_s: float, loop_s: float, iterations: int, records: np.ndarray,
                     pair_ids=None):
    """Cross-rank reduction of one timed region.

    records: the rank's [n, REC] pair_records().  Returns (elapsed_max, loop_max,
    iterations_sum, PairRecords of every rank's pairs in rank order).  `dist` is
    torch.distributed (or None for one rank); `device` the tensor device of the backend
    (cuda for nccl/RCCL, cpu for gloo).  Ranks may hold different numbers of pairs (shard()
    of a batch that does not divide evenly): the pair counts are gathered first and every
    rank's records are padded to the largest count for the fixed-size all-gather, then cut
    back.  pair_ids: the rank's pairs' indices in the global batch (shard_balanced); the
    gathered records are then put in pair order.
    """
    import torch

    records = np.ascontiguousarray(records, dtype=np.float64).reshape(-1, REC)
    if pair_ids is not None:
        # the pair index rides in an extra column (exact in float64)
        records = np.concatenate([records, np.asarray(pair_ids, dtype=np.float64).reshape(-1, 1)], axis=1)
    if dist is None:
        if pair_ids is not None:
            records = records[np.argsort(records[:, REC], kind="stable"), :REC]
        return float(elapsed_s), float(loop_s), int(iterations), unpack_records(records)
    t_max = torch.tensor([float(elapsed_s), float(loop_s)], dtype=torch.float64, device=device)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    tot = torch.tensor([float(iterations)], dtype=torch.float64, device=device)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    world = dist.get_world_size()
    cnt = torch.tensor([records.shape[0]], dtype=torch.int64, device=device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    pad = np.zeros((max(counts), records.shape[1]))
    pad[:records.shape[0]] = records
    mine = torch.from_numpy(pad).to(device)
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    allr = np.concatenate([g.cpu().numpy()[:c] for g, c in zip(gathered, counts)])
    if pair_ids is not None:
        allr = allr[np.argsort(allr[:, REC], kind="stable"), :REC]
    return float(t_max[0]), float(t_max[1]), int(round(float(tot[0]))), unpack_records(allr)


def max_over_ranks(dist, device, x: float) -> float:
    """The largest of every rank's x (one timed region's seconds); x itself for one rank."""
    if dist is None:
        return float(x)
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def sum_over_ranks(dist, device, x: float) -> float:
    """The sum of every rank's x (work counts); x itself for one rank."""
    if dist is None:
        return float(x)
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0])
