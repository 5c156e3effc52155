#!/usr/bin/env python3
"""Measurement: the C4 64-pair batch as one call against G host threads, each driving its
own engine slot (device | slot << 8: own stream and buffers) on a contiguous block of the
pairs, all on one GPU.  Prints one JSON line per configuration (wall ms per batch, median
of the repeats) and checks that every configuration returns bitwise the one-call poses.

Usage (GPU box): python3 tools/two_engine.py [--groups 1 2 4] [--reps 3] [--pair-cache DIR]
                [--stagger-ms 0 10 20]  (G = 2: the second half starts this much later)
                [--pipeline R]  (also: two slots each registering the WHOLE batch R times from its
                                 own thread, against one slot registering it 2R times)
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "se3-icp_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--pair-cache", default="/tmp/se3icp_pairs")
    ap.add_argument("--stagger-ms", type=float, nargs="*", default=[0.0])
    ap.add_argument("--pipeline", type=int, default=0)
    a = ap.parse_args()
    import torch
    import se3icp
    from se3icp import datasets

    se3icp.load()
    cache = os.path.join(a.pair_cache, f"two_engine_{a.pairs}.npz")
    if os.path.exists(cache):
        z = np.load(cache)
        pairs = [(z[f"s{i}"], z[f"t{i}"]) for i in range(a.pairs)]
    else:
        pairs, _ = datasets.kitti_like_pairs(a.pairs, seed=4, first=0, total_pairs=64)
        os.makedirs(a.pair_cache, exist_ok=True)
        np.savez(cache, **{f"s{i}": p[0] for i, p in enumerate(pairs)}, **{f"t{i}": p[1] for i, p in enumerate(pairs)})
    params = se3icp.kitti_params()

    def block(lo, hi):
        src = np.concatenate([p[0] for p in pairs[lo:hi]])
        tgt = np.concatenate([p[1] for p in pairs[lo:hi]])
        so = np.concatenate([[0], np.cumsum([p[0].shape[0] for p in pairs[lo:hi]])])
        to = np.concatenate([[0], np.cumsum([p[1].shape[0] for p in pairs[lo:hi]])])
        ds, dt = torch.from_numpy(src).to("cuda:0"), torch.from_numpy(tgt).to("cuda:0")
        return ds, dt, so, to

    ref = None
    for G in a.groups:
        bounds = [(g * a.pairs // G, (g + 1) * a.pairs // G) for g in range(G)]
        blocks = [block(lo, hi) for lo, hi in bounds]
        torch.cuda.synchronize()
        runners = [se3icp.DeviceBatchRunner(ds.data_ptr(), so, dt.data_ptr(), to, "se3_gicp", params, device=g << 8,
                                            slots=1) for g, (ds, dt, so, to) in enumerate(blocks)]

        stagger = 0.0

        def run_late(r, delay):
            if delay > 0:
                time.sleep(delay)
            r.run(0)

        def run_all():
            if G == 1:
                runners[0].run(0)
                return
            th = [threading.Thread(target=run_late, args=(r, stagger * i / 1e3)) for i, r in enumerate(runners)]
            for t in th:
                t.start()
            for t in th:
                t.join()

        run_all()  # warm-up (buffers, code)
        torch.cuda.synchronize()
        for stagger in (a.stagger_ms if G == 2 else [0.0]):
            times = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                run_all()
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            res = [r for rn in runners for r in rn.results(0)]
            its = sum(r.num_iterations for r in res)
            T = np.stack([r.T for r in res])
            if ref is None:
                ref = T
            same = bool(np.array_equal(T, ref))
            ms = 1000.0 * statistics.median(times)
            print(json.dumps({"groups": G, "stagger_ms": stagger, "pairs": a.pairs, "ms_per_batch": round(ms, 3),
                              "iter_per_s": round(its / (ms / 1e3), 1), "times_ms": [round(1000 * t, 3) for t in times],
                              "poses_equal_one_call": same}), flush=True)
    if a.pipeline > 0:
        # whole batches back to back: one slot 2R calls, against two slots R calls each from
        # their own threads (calls of the two slots drift out of step)
        ds, dt, so, to = block(0, a.pairs)
        torch.cuda.synchronize()
        rs = [se3icp.DeviceBatchRunner(ds.data_ptr(), so, dt.data_ptr(), to, "se3_gicp", params, device=k << 8, slots=1)
              for k in range(2)]
        for r in rs:
            r.run(0)
        torch.cuda.synchronize()
        its = sum(r.num_iterations for r in rs[0].results(0))
        t0 = time.perf_counter()
        for _ in range(2 * a.pipeline):
            rs[0].run(0)
        torch.cuda.synchronize()
        one = time.perf_counter() - t0

        def loop(r):
            for _ in range(a.pipeline):
                r.run(0)

        th = [threading.Thread(target=loop, args=(r,)) for r in rs]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        two = time.perf_counter() - t0
        same = bool(np.array_equal(np.stack([r.T for r in rs[1].results(0)]), np.stack([r.T for r in rs[0].results(0)])))
        print(json.dumps({"pipeline_calls": 2 * a.pipeline, "pairs": a.pairs,
                          "one_slot_iter_per_s": round(2 * a.pipeline * its / one, 1),
                          "two_slots_iter_per_s": round(2 * a.pipeline * its / two, 1), "poses_equal": same}), flush=True)


if __name__ == "__main__":
    main()
