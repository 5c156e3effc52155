#!/usr/bin/env python3
"""bench.py — ICP iterations/sec + pairs/sec on KITTI-scale LiDAR pairs (BASELINE.json).

Default workload (BASELINE.json configs[3]): se3_gicp with the KITTI
driver's parameters (examples/benchmark_kitti.cpp:133-148: overlap 0.7, mse 1e-7,
mse_switch 5e-7, max_se3 10, k = 90) on synthetic 64-beam LiDAR scans of ~120k points
(the KITTI data are not available offline).  The batch is BASELINE's: 64 consecutive-scan
pairs (examples/benchmark_kitti.cpp:120-197), a fixed global batch sharded over the GPUs
(strong scaling: N=1 registers all 64 on one GPU, N=8 eight per GPU), each rank
registering its block in lockstep with no data-path collective; RCCL (torch.distributed
"nccl") only gathers the per-pair results.  --workload C2 / C3 / C5 runs the other
BASELINE configs (C3 32 pairs, C5 256 pairs, C2 8 cases; secondary lines, the headline is
C4).  --pairs-per-gpu P switches to weak scaling (P pairs per rank).

A step = registering the rank's batch end to end (TOLDI/kNN/normals setup + the ICP loop),
clouds already resident in HBM.  value = ICP iterations (all ranks) / step wall time.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "se3-icp_amd"), ROOT]

FP32_PEAK_TFLOPS = 157.3   # MI355X vector (= f32 MFMA) peak, /opt/skills/guides/MI355X_MICROARCH.md
FP64_VEC_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (same guide)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak, same guide
N_SIMDS = 1024             # 256 CUs x 4 SIMDs (same guide)
CLOCK_GHZ = 2.4            # peak engine clock (same guide)

METRIC = "ICP iterations/sec + pairs/sec, ~120k-pt KITTI clouds, 1/2/4/8 GPU"

# BASELINE.json configs: method, pairs per GPU, reference parameters
WORKLOADS = {
    "C4": dict(method="se3_gicp", ppg=8, batch=64, run="se3", variant="gicp",
               params=dict(estimated_overlap=0.7, max_num_se3_iterations=10, mse=1e-7, mse_switch_error=5e-7,
                           number_of_nn_for_LRF=90),
               desc="C4: se3_gicp, KITTI driver params (overlap 0.7, mse 1e-7, switch 5e-7, max_se3 10, k=90)",
               data="synthetic (64-beam LiDAR ray-cast street scenes, seed 4; KITTI not available offline)"),
    "C2": dict(method="se3_pt2pt", ppg=8, batch=8, run="se3", variant="pt2pt",
               params=dict(estimated_overlap=1.0, max_num_se3_iterations=10, mse=1e-5, mse_switch_error=5e-5,
                           number_of_nn_for_LRF=90),
               desc="C2: se3_pt2pt on the reference's synthetic bunny problems (benchmark_synthetic.cpp:91-160 with "
                    "its own mt19937 / normal_distribution / RandomDownSample streams, noise var 0.005) at "
                    "RandomDownSample(0.2) of stanford_bunny.ply x50 = 41,670 pts per cloud (BASELINE.json configs[1]: "
                    "'synthetic easy_data, ~40k pts'; the driver itself samples 0.02 and has the 'moderate' ranges "
                    "active, B_SYN:111-112), 'easy' ranges (B_SYN:107-108), B_SYN:356-363 params, 8 cases per GPU",
               data="stanford_bunny.ply (tests/golden) -> se3icp_synthetic_reference_device, generated on the GPU"),
    "C3": dict(method="se3_pt2pl", ppg=32, batch=32, run="se3", variant="pt2pl",
               params=dict(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                           number_of_nn_for_LRF=90),
               desc="C3: se3_pt2pl, lounge driver params (overlap 0.75, switch 5e-5, max_se3 10, k=90), "
                    "a batch of 32 consecutive RGB-D pairs",
               data="synthetic RGB-D room sequence (depth 0.4-4 m, stride 4, ~16k pts, seed 3; lounge not offline)"),
    "C5": dict(method="se3_gicp_with_cf", ppg=32, batch=256, run="cf", variant="gicp",
               params=dict(estimated_overlap=0.75, max_num_se3_iterations=10, mse_switch_error=5e-5,
                           number_of_nn_for_LRF=90),
               desc="C5: se3_gicp_with_cf, lounge driver params, a batch of 256 pairs (32 per GPU at N=8)",
               data="synthetic RGB-D room sequence (depth 0.4-4 m, stride 4, ~16k pts, seed 5; lounge not offline)"),
}


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def rot_err_deg(A, B):
    R = A[:3, :3].T @ B[:3, :3]
    return float(np.degrees(np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))))


def _pmc_files(workload: str):
    """Committed PMC summaries of one workload, newest first: profiles/*pmc*.json whose
    "workload" field names it (files written before round 4 carry none and are C4's)."""
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload", "C4") == workload:
            out.append((f, d))
    return out


def pmc_traffic(kernel_substrs, workload: str):
    """HBM bytes per launch, summed over the named kernels, from the newest committed PMC
    summary of THIS workload (tools/pmc_summary.py, separate rocprofv3 --pmc passes);
    (None, None) when that summary lacks any of the kernels."""
    if isinstance(kernel_substrs, str):
        kernel_substrs = [kernel_substrs]
    for f, d in _pmc_files(workload)[:1]:
        tot = 0.0
        for sub in kernel_substrs:
            hit = [v for k, v in d.get("kernels", {}).items() if sub in k and v.get("hbm_bytes_per_launch") is not None]
            if not hit:
                return None, None
            tot += float(hit[0]["hbm_bytes_per_launch"])
        return tot, os.path.relpath(f, ROOT)
    return None, None


def pmc_counter(kernel_substr: str, counter: str, workload: str):
    """One PMC counter per dispatch of a kernel from the newest committed PMC summary of THIS
    workload, with the file it came from."""
    for f, d in _pmc_files(workload)[:1]:
        for k, v in d.get("kernels", {}).items():
            c = v.get("counters_per_dispatch", {})
            if kernel_substr in k and counter in c:
                return float(c[counter]), os.path.relpath(f, ROOT)
    return None, None


C2_SETUPS = {"easy": (5.0, np.pi / 4), "moderate": (10.0, np.pi / 2)}  # B_SYN:106-108, :111-112


def datasets_tag() -> str:
    """Short hash of the pair generators' sources (se3icp/datasets.py and the C2 reference
    generator): part of the --pair-cache file name, so that a generator change never reuses
    stale pairs and ground truths (the seeds are fixed per workload in make_pairs)."""
    import hashlib
    h = hashlib.sha1()
    for f in ("se3-icp_amd/se3icp/datasets.py", "se3-icp_amd/csrc/k_gen.hip", "se3-icp_amd/csrc/gen_ref.cpp"):
        try:
            h.update(open(os.path.join(ROOT, f), "rb").read())
        except OSError:
            pass
    return h.hexdigest()[:10]


def make_pairs(wl: str, total: int, first: int, count: int, n_az: int, c2_setup: str = "easy", device: int = 0,
               c2_cloud: str = "downsample"):
    """The rank's pairs [first, first + count) of a `total`-pair sequence, with ground truths."""
    from se3icp import datasets
    if wl == "C4":
        return datasets.kitti_like_pairs(count, seed=4, first=first, total_pairs=total, n_az=n_az)
    if wl == "C2":
        # the reference's own problems, case after case (its streams are sequential: every
        # rank draws the whole sequence and keeps its block), written by the GPU
        u = np.load(os.path.join(ROOT, "tests", "golden", "bunny_unique_f32.npy"))
        ids = np.load(os.path.join(ROOT, "tests", "golden", "bunny_vertex_ids.npy"))
        if c2_cloud == "unique":  # BASELINE.md's C2 row (rounds 1-2): the 34,834 unique vertices, all kept
            cloud, ratio = u.astype(np.float64) * 50.0, 1.0
        else:
            cloud, ratio = u[ids].astype(np.float64) * 50.0, 0.2
        tr, rr = C2_SETUPS[c2_setup]
        src, tgt, T = datasets.synthetic_reference_gpu(cloud, total, ratio=ratio, noise_var=0.005, t_range=tr,
                                                       r_range=rr, device=device)
        return ([(src[i], tgt[i]) for i in range(first, first + count)], [T[i] for i in range(first, first + count)])
    seed = 3 if wl == "C3" else 5
    pairs, gts = datasets.rgbd_pairs(total, seed=seed, stride=4)
    return pairs[first:first + count], gts[first:first + count]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C4")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="pairs of the whole job, sharded over the ranks (strong scaling); 0: the workload's "
                         "BASELINE batch (C4 64, C5 256, C3 32, C2 8)")
    ap.add_argument("--pairs-per-gpu", type=int, default=0,
                    help="weak scaling instead: this many pairs per rank (the global batch grows with N)")
    ap.add_argument("--n-az", type=int, default=1975, help="C4 azimuth steps per revolution (~120k pts at 1975)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="collective backend for N > 1 (gloo: ranks may share one GPU, as in the tests)")
    ap.add_argument("--pair-cache", default="", help="directory for the generated pairs (reused by later runs)")
    ap.add_argument("--dump-poses", default="", help="rank 0 writes the gathered per-pair poses (.npy)")
    ap.add_argument("--c2-setup", choices=sorted(C2_SETUPS), default="easy",
                    help="C2 transform ranges: BASELINE's easy_data (B_SYN:106-108) or the driver's active moderate ones")
    ap.add_argument("--c2-cloud", choices=["downsample", "unique"], default="downsample",
                    help="C2 cloud: RandomDownSample(0.2) of the 208,353-vertex bunny (41,670 pts, round 3 on) or "
                         "BASELINE.md's 34,834 unique vertices (rounds 1-2); the bench line's workload is then 'C2u'")
    ap.add_argument("--shard", choices=["contiguous", "balanced"], default="contiguous",
                    help="pairs per rank: contiguous blocks of the batch, or a cost-balanced assignment (greedy by "
                         "point count over the whole batch, sharding.shard_balanced)")
    ap.add_argument("--in-flight", type=int, default=0,
                    help="calls in flight per GPU (engine slots, one host thread each); 1: one call at a time; "
                         "0 (default): in_flight_for(pairs per call).  C4, 20 steps (iter/s): 1 / 2 / 3 / 4 in "
                         "flight = 14,416 / 15,207 / 15,409 / 15,336; its 8-pair shard 11,318 / 12,767 / 13,198 / "
                         "13,453")
    ap.add_argument("--secondary", choices=["auto", "off"], default="auto",
                    help="C4 at N=1: also time one 8-pair shard on this GPU (the per-GPU work of the 8-GPU job)")
    args = ap.parse_args()
    W = dict(WORKLOADS[args.workload])
    if args.workload == "C2" and args.c2_setup != "easy":
        W["desc"] = W["desc"].replace("'easy' ranges (B_SYN:107-108)", "'moderate' ranges (B_SYN:111-112)")
    if args.workload == "C2" and args.c2_cloud == "unique":
        W["desc"] = ("C2u: se3_pt2pt on the reference's synthetic bunny problems over the 34,834 unique vertices of "
                     "stanford_bunny.ply x50, all kept (BASELINE.md's C2 row; the rounds-1-2 definition), noise var "
                     "0.005, 'easy' ranges, B_SYN:356-363 params, 8 cases per GPU")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    import se3icp
    from se3icp import sharding

    se3icp.load()
    ndev = max(1, torch.cuda.device_count())
    devi = local % ndev
    torch.cuda.set_device(devi)
    # timing instrumentation only: no HIP event markers around the SE(3) NN grids in the timed
    # steps (each leaves the GPU idle ~5 us); the stage times come from one profiled step
    from se3icp import registration
    registration.set_nn_events(False, devi)
    dev = torch.device("cuda", devi)
    dist = None
    xdev = dev
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
            xdev = torch.device("cpu")

    # strong scaling over the workload's fixed batch (weak with --pairs-per-gpu)
    scaling, global_batch, first, count = sharding.plan(world, rank, W["batch"], args.global_batch,
                                                        args.pairs_per_gpu)
    t0 = time.time()
    pair_ids = None  # (balanced shards: the rank's pair indices in the batch)
    if args.shard == "balanced" and world > 1:
        # every rank generates the whole batch (deterministic), balances it by point count and
        # keeps its own pairs
        allp, allg = make_pairs(args.workload, global_batch, 0, global_batch, args.n_az, args.c2_setup, devi,
                                args.c2_cloud)
        plan_b = sharding.shard_balanced([p[0].shape[0] + p[1].shape[0] for p in allp], world)
        pair_ids = plan_b[rank]
        pairs, gts = [allp[i] for i in pair_ids], [allg[i] for i in pair_ids]
        first, count = pair_ids[0], len(pair_ids)
        del allp, allg
        log(f"rank {rank}: balanced shard of {count} pairs {pair_ids}")
    else:
        cache = (os.path.join(args.pair_cache, f"{args.workload}_{args.c2_cloud}_{args.c2_setup}_{args.n_az}_"
                              f"{global_batch}_{first}_{count}_{datasets_tag()}.npz") if args.pair_cache else "")
        if cache and os.path.exists(cache):  # (A/B runs on one box: the same synthetic pairs, generated once)
            z = np.load(cache)
            pairs = [(z[f"s{i}"], z[f"t{i}"]) for i in range(count)]
            gts = [z["gts"][i] for i in range(count)]
        else:
            pairs, gts = make_pairs(args.workload, global_batch, first, count, args.n_az, args.c2_setup, devi,
                                    args.c2_cloud)
            if cache:
                os.makedirs(args.pair_cache, exist_ok=True)
                np.savez(cache, gts=np.stack(gts), **{f"s{i}": p[0] for i, p in enumerate(pairs)},
                         **{f"t{i}": p[1] for i, p in enumerate(pairs)})
    npts = [p[0].shape[0] for p in pairs] + [p[1].shape[0] for p in pairs]
    log(f"rank {rank}: {args.workload} generated {count} pairs in {time.time() - t0:.1f}s, points/cloud "
        f"min {min(npts)} mean {np.mean(npts):.0f} max {max(npts)}")
    src = np.concatenate([p[0] for p in pairs])
    tgt = np.concatenate([p[1] for p in pairs])
    src_off = np.concatenate([[0], np.cumsum([p[0].shape[0] for p in pairs])])
    tgt_off = np.concatenate([[0], np.cumsum([p[1].shape[0] for p in pairs])])
    d_src = torch.from_numpy(src).to(dev)
    d_tgt = torch.from_numpy(tgt).to(dev)
    torch.cuda.synchronize()
    params = se3icp.default_params(**W["params"])

    def step():
        return se3icp.register_batch_device(d_src.data_ptr(), src_off, d_tgt.data_ptr(), tgt_off, W["method"],
                                            params, device=devi)

    # the timed steps: one C-ABI call each with prebuilt arguments; every step's results and
    # kernel times land in their own buffers and are read after the timed region.  With
    # --in-flight F > 1 the K steps run F at a time on F engine slots of this GPU (own
    # streams and buffers, one host thread each: PipelinedBatchRunner) -- the value; then the
    # same K steps one call at a time (single_call), whose isolated kernel and phase times
    # feed the per-kernel lines and rooflines below.
    if args.in_flight <= 0:
        args.in_flight = in_flight_for(count)

    def make_runner(slot):
        return se3icp.DeviceBatchRunner(d_src.data_ptr(), src_off, d_tgt.data_ptr(), tgt_off, W["method"], params,
                                        device=devi | (slot << 8), slots=max(1, args.steps))
    pipe = se3icp.PipelinedBatchRunner(make_runner, in_flight=args.in_flight, steps=args.steps)
    for w in range(args.warmup):
        tw = time.time()
        step()
        log(f"rank {rank}: warmup {w} {time.time() - tw:.2f}s")
    if args.in_flight > 1:
        pipe.warm()  # (every slot's buffers and code, untimed)

    def timed(run):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        return time.perf_counter() - t0

    elapsed = timed(pipe.run_steps)
    iters = 0
    last = None
    for s in range(args.steps):
        res = pipe.results(s)
        iters += sum(r.num_iterations for r in res)
        last = res
        log(f"rank {rank}: step {s} done ({sum(r.num_iterations for r in res)} iterations, slot {pipe.owner(s)})")
    single = None
    iso = pipe
    if args.in_flight > 1:
        iso = se3icp.PipelinedBatchRunner(make_runner, in_flight=1, steps=args.steps)
        el1 = timed(iso.run_steps)
        its1 = sum(sum(r.num_iterations for r in iso.results(s)) for s in range(args.steps))
        el1 = sharding.max_over_ranks(dist, xdev, el1)
        its1 = sharding.sum_over_ranks(dist, xdev, its1)
        single = {"value": round(its1 / el1, 3), "ms_per_step": round(1000.0 * el1 / args.steps, 3),
                  "note": "the same K steps one call at a time (one batch in flight): the per-call rate; the "
                          "kernel, phase and roofline figures of this line come from these isolated calls"}
    rechecked = 0
    setup_ms = 0.0
    loop_ms = 0.0
    ktot: dict = {}
    for s in range(args.steps):
        res = iso.results(s)
        for k, v in iso.kernel_times(s).items():
            ktot[k] = ktot.get(k, 0.0) + v
        rechecked += sum(r.num_rechecked for r in res)
        loop_ms += res[0].time_loop_ms
        setup_ms += res[0].time_setup_ms
    # one untimed step with HIP events around every loop stage: the timed steps carry
    # events only around the SE(3) NN grids (each marker costs the stream a few microseconds)
    se3icp.set_profiling(True, devi)
    step()
    kt_detail = se3icp.last_kernel_times(devi)
    se3icp.set_profiling(False, devi)
    # (the timed steps carry no SE(3) NN events either, set_nn_events(False): the NN stage
    # times, the secondary roofline's included, come from this profiled step)
    for k in ["nn_prep_ms", "nn_r3_ms", "recheck_ms", "trim_ms", "reduce_ms", "nn_se3_ms"]:
        ktot[k] = kt_detail[k] * args.steps

    # ---- cross-rank: max time, summed work, RCCL gather of the per-pair results
    elapsed, loop_s, iters_all, gathered = sharding.exchange_results(
        dist, xdev, elapsed, loop_ms / 1000.0, iters, sharding.pair_records(last), pair_ids)

    if rank == 0:
        if args.dump_poses:
            np.save(args.dump_poses, gathered.T)
        total_pairs = global_batch * args.steps
        value = iters_all / elapsed
        ms_per_step = 1000.0 * elapsed / args.steps
        rot_errs = [rot_err_deg(r.T, g) for r, g in zip(last, gts)]
        tr_errs = [float(np.linalg.norm(r.T[:3, 3] - g[:3, 3])) for r, g in zip(last, gts)]
        kms = {k: ktot.get(k, 0.0) for k in ["nn_prep_ms", "nn_se3_ms", "nn_r3_ms", "recheck_ms", "trim_ms",
                                            "reduce_ms", "lrf_ms"]}
        nq = max(1.0, ktot.get("lrf_queries", 0.0))
        lrf_work = {"queries_per_step": ktot.get("lrf_queries", 0.0) / args.steps,
                    "leaves_per_query": round(ktot.get("lrf_leaves", 0.0) / nq, 2),
                    "bound_updates_per_query": round(ktot.get("lrf_merges", 0.0) / nq, 2),
                    "box_tests_per_query": round(ktot.get("lrf_box_tests", 0.0) / nq, 2),
                    "candidates_per_query": round(ktot.get("lrf_candidates", 0.0) / nq, 2),
                    "exact_kernel_queries_per_step": ktot.get("lrf_fallback", 0.0) / args.steps}
        wl = args.workload if args.c2_cloud == "downsample" else f"{args.workload}u"
        roof_nn = nn_roofline(ktot, kms, wl)
        # (normals, KNN 30, ISR.cpp:643: both clouds for GICP, the targets for pt2pl, none for pt2pt)
        roof_lrf = lrf_roofline(ktot, kms, args.steps, W["params"]["number_of_nn_for_LRF"], wl,
                                {"gicp": 30, "pt2pl": 15, "pt2pt": 0}[W["variant"]])
        roof_red = reduce_roofline(last, pairs, W, kms["reduce_ms"] / args.steps, wl)
        # the bench line's roofline is the step's dominant kernel by GPU time; the other
        # named kernel is reported beside it
        nn_step = roof_nn["avg_launch_ms"] * roof_nn["launches"] / args.steps
        lrf_step = roof_lrf["avg_launch_ms"]
        dominant, other = (roof_lrf, roof_nn) if lrf_step >= nn_step else (roof_nn, roof_lrf)
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "ICP iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,   # BASELINE.md publishes no number for this metric
            "dtype": "f32 sweep + f64 certify/solve",
            "data": W["data"],
            "config": {
                "workload": W["desc"],
                "method": W["method"],
                "pairs_per_gpu": (global_batch // world if global_batch % world == 0
                                  else [sharding.shard(global_batch, world, r)[1] for r in range(world)]),
                "shard": args.shard if world > 1 else "one rank",
                "global_batch_pairs": global_batch,
                "points_per_cloud_mean": int(np.mean(npts)),
                "parallelism": f"pair-sharded dp{world} ({'RCCL' if args.backend == 'nccl' else 'gloo'} "
                               f"result gather only)",
                "in_flight": args.in_flight,
            },
            "in_flight": args.in_flight,
            # each call's own wall time in the timed region (the calls in flight beside it): the
            # latency a caller sees, against ms_per_step's amortized time
            "ms_per_call": round(1000.0 * float(np.mean([pipe.call_seconds(s) for s in range(args.steps)])), 3),
            "single_call": single,
            "pairs_per_sec": round(total_pairs / elapsed, 4),
            "loop_iterations_per_sec": round(iters_all / loop_s, 3) if loop_s > 0 else None,
            "iterations_per_pair_mean": round(iters_all / total_pairs, 2),
            "accuracy_vs_gt": {"rot_deg_max": round(max(rot_errs), 4), "trans_m_max": round(max(tr_errs), 4)},
            "kernel_ms_per_step": {k: round(v / args.steps, 3) for k, v in kms.items()},
            "lrf_work": lrf_work,
            "rechecked_queries_per_step": rechecked / args.steps,
            # NN certificates (k_nn_prep): share of the loop's queries that still needed a search
            "nn_searched_frac": {"se3": round(ktot.get("se3_searched", 0.0) / max(1.0, ktot.get("se3_queries", 0.0)), 4),
                                 "r3": round(ktot.get("r3_searched", 0.0) / max(1.0, ktot.get("r3_queries", 0.0)), 4)},
            "phase_ms_per_step": {"setup": round(setup_ms / args.steps, 3), "loop": round(loop_ms / args.steps, 3)},
            "roofline": dominant,
            "roofline_other": other,
            "roofline_reduce": roof_red,
            "cpu_baseline": None,
        }
        if args.workload == "C4" and world == 1 and args.secondary == "auto" and len(pairs) > 8:
            out["secondary_8_pair_shard_one_gpu"] = bench_shard8(pairs, W, params, dev, devi,
                                                                 in_flight=in_flight_for(8) if args.in_flight > 1 else 1)
        if args.cpu_baseline == "auto":
            # rank 0's own pairs on the node's host (the same host for every rank), after the
            # timed region; at N > 1 the whole job's value is compared with it
            out["cpu_baseline"], out["parity_vs_cpu"] = cpu_baseline(pairs, last, W, value, params, devi)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def nn_roofline(ktot, kms, wl):
    """The loop's dominant NN launch (k_nn_search of the phase with more time):
    work actually issued, counted on the device — lane x target distance evaluations
    (3D flop: D sub + D FMA) and lane x box tests (4D flop: 2D sub/max + D FMA)."""
    dom = max(["nn_se3_ms", "nn_r3_ms"], key=lambda k: kms[k])
    if dom == "nn_se3_ms":
        D, evals, boxes, nl, kname = 12, ktot["se3_dist_evals"], ktot["se3_box_tests"], ktot["nn_se3_launches"], \
            "k_nn_search<12>"
        useful = ktot.get("se3_useful_evals", 0.0)
    else:
        D, evals, boxes, nl, kname = 3, ktot["r3_dist_evals"], ktot["r3_box_tests"], ktot["nn_r3_launches"], \
            "k_nn_search<3>"
        useful = ktot.get("r3_useful_evals", 0.0)
    t_ms = kms[dom]
    flop_dist, flop_box = 3 * D, 4 * D
    flops = evals * flop_dist + boxes * flop_box
    achieved = flops / (t_ms / 1000.0) / 1e12 if t_ms > 0 else 0.0
    nl = max(1.0, nl)
    # ("k_nn_search<12" matches the kernel's instantiations, k_nn_search<12, true> since round 5)
    traffic, src = pmc_traffic([f"k_nn_search<{D}"], wl)
    return {
        "kernel": kname,
        "bound": "valu",
        "note": "f32 VALU kd-tree sweep (leaf distance sweeps + box tests; no MFMA issued), priced against the "
                "f32 vector peak.  A launch is one grid: one-query-per-wave searches of the sparse chunks' "
                "queries, then the 64-query groups; avg_launch_ms is its HIP-event time in the profiled step "
                "(the kernel's rocprof average in the committed trace).  The time includes the inline f64 "
                "recheck of the ~0.4 % uncertified queries, whose flops are not counted",
        "achieved": round(achieved, 3),
        "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
        "avg_launch_ms": round(t_ms / nl, 4),
        "launches": int(nl),
        "flop_per_unit": {"distance_eval": flop_dist, "box_test": flop_box},
        "units_per_launch": {"distance_evals": round(evals / nl), "box_tests": round(boxes / nl),
                             "useful_distance_evals": round(useful / nl)},
        # the distance evaluations of occupied (query, target) pairs only -- the lanes a sweep
        # keeps busy without a query that wants the leaf are not work (round 6)
        "useful": {"distance_evals_per_launch": round(useful / nl),
                   "share_of_evaluation_slots": round(useful / evals, 4) if evals else None,
                   "achieved_tflops": round(useful * flop_dist / (t_ms / 1000.0) / 1e12, 3) if t_ms > 0 else None,
                   "frac": round(useful * flop_dist / (t_ms / 1000.0) / 1e12 / FP32_PEAK_TFLOPS, 4) if t_ms > 0 else None},
        "traffic": traffic,
        "traffic_source": src,
    }


def busy_fraction(quad_cycles, t_ms):
    """VALU issue busy: SQ_ACTIVE_INST_VALU (quad-cycles, summed over the chip's SIMDs) x 4
    over the SIMD-cycles of t_ms.  Above 1 the counter and the time cannot be from the same
    launch (a counter of another workload or build): refused (None)."""
    if not quad_cycles or t_ms <= 0:
        return None
    b = quad_cycles * 4.0 / (N_SIMDS * CLOCK_GHZ * 1e6 * t_ms)
    return round(b, 3) if b <= 1.0 else None


def lrf_fp64_flops_per_point(k: int, k_nrm: int, ncand: float) -> float:
    """f64 flops the reference's own arithmetic needs per point on the TOLDI / normals path
    (ISR.cpp:241-331, Open3D EstimateNormals at ISR.cpp:643): the exact squared distances of
    the final candidates (3 sub, 3 mul, 2 add each), the TOLDI neighbour sums over ranks
    1..k/3 (21 per rank: the offset, its 3 + 3 running sums and the 6 moments), the radius
    (8), the normal cumulants over k_nrm ranks (15 per rank), the two 3x3 eigen-problems
    (covariance assembly + cyclic Jacobi ~400, FastEigen3x3 ~115), the TOLDI axis sums over
    ranks 1..k-1 (26 per rank: offset, dot, distance, weight, weighted sum) and the frame
    (~60).  Counted from the kernel's loops, not measured."""
    rz = k // 3
    return 8.0 * ncand + 21.0 * rz + 8.0 + 15.0 * k_nrm + 400.0 + 115.0 + 26.0 * (k - 1) + 60.0


def lrf_sections():
    """Per-wave VALU counts of k_lrf8's sections from the newest committed section profile
    (profiles/*_lrf8_sections.txt, tools/lrf_sections.sh): the share of the kernel's VALU
    spent in the reference's math (neighbour sums, eigen-solves, axes, frames) against the
    kNN selection (traversal, bound tightenings, final order)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_lrf8_sections.txt")), reverse=True)
    for f in files:
        tot, math = None, 0.0
        for line in open(f):
            parts = line.split()
            if len(parts) > 2 and parts[0] == "lib":
                tot = float(parts[1])
            if "neighbour sums:" in line or "eigen-solves, axes, frames:" in line:
                math += float(line.split(":")[-1].split("VALU")[0].strip().lstrip("+"))
        if tot:
            return {"valu_per_wave": tot, "math_valu_per_wave": math, "useful_valu_frac": round(math / tot, 3),
                    "source": os.path.relpath(f, ROOT)}
    return None


def lrf_roofline(ktot, kms, steps, k, wl, k_nrm=30):
    """k_lrf, the setup's fused kNN-k + TOLDI + normals kernel, one launch per step, priced
    with SURVEY.md §8(d)'s TOLDI unit: k neighbour gathers of 24 B (f64 xyz) per point.  The
    kernel is bound by VALU issue (bound "valu"); beside the HBM fraction the line carries
    the f64 algorithmic flops against the FP64 vector peak and the share of its VALU that is
    the reference's math (useful_valu_frac)."""
    t_ms = kms["lrf_ms"] / steps
    q = ktot.get("lrf_queries", 0.0) / steps
    bpp = 24.0 * k
    achieved = q * bpp / (t_ms / 1000.0) / 1e9 if t_ms > 0 else 0.0
    traffic, src = pmc_traffic(["k_lrf8", "k_lrf("], wl)  # k_lrf: the exact kernel over the hand-over list
    # what does bound it: the VALU issue of k_lrf8 (SQ_ACTIVE_INST_VALU counts quad-cycles per
    # SIMD, summed over the chip's 1,024 SIMDs) over this launch pair's measured time
    av, _ = pmc_counter("k_lrf8", "SQ_ACTIVE_INST_VALU", wl)
    insts, _ = pmc_counter("k_lrf8", "SQ_INSTS_VALU", wl)
    ncand = 8.0 * ktot.get("lrf_candidates", 0.0) / max(1.0, ktot.get("lrf_queries", 0.0))  # (one group in eight counted)
    fpp = lrf_fp64_flops_per_point(k, k_nrm, ncand)
    f64_tf = q * fpp / (t_ms / 1000.0) / 1e12 if t_ms > 0 else 0.0
    return {
        "kernel": "k_lrf8 + k_lrf (hand-overs)",
        "bound": "valu",
        "note": "fused exact kNN-k (f64) + TOLDI frame + normals/GICP covariance per point: k_lrf8 (eight queries "
                "per wavefront) and the exact one-query-per-wavefront k_lrf for the points it hands over, one HIP-event "
                "bracket; achieved/frac: algorithmic bytes = k neighbour gathers x 24 B per point (SURVEY.md §8d) "
                "against HBM; the kernels are VALU-issue bound (valu_issue_busy: the fraction of the launch the SIMDs "
                "spend issuing VALU, from this workload's committed PMC pass), most of it the kNN selection "
                "(valu_sections.useful_valu_frac: the reference's math); fp64_algorithmic: the f64 flops of the "
                "reference's arithmetic against the FP64 vector peak (DESIGN.md §5)",
        "valu_issue_busy": busy_fraction(av, t_ms),
        "valu_insts_per_point": round(insts / q, 1) if (insts and q) else None,
        "fp64_algorithmic": {"flop_per_point": round(fpp), "candidates_per_point": round(ncand, 1),
                             "achieved_tflops": round(f64_tf, 3), "peak_tflops": FP64_VEC_PEAK_TFLOPS,
                             "frac": round(f64_tf / FP64_VEC_PEAK_TFLOPS, 4)},
        "valu_sections": lrf_sections(),
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "avg_launch_ms": round(t_ms, 4),
        "launches": 1,
        "bytes_per_unit": bpp,
        "units_per_launch": {"points": round(q)},
        "traffic": traffic,
        "traffic_source": src,
    }


# HBM bytes k_reduce reads per source point of an active pair in one iteration: every point
# its correspondence's float distance (the trim key, 4 B); a kept correspondence also its
# target index 4, both f64 points 2 x 24, plus the target normal 24 (pt2pl) or both normals
# 2 x 24 (GICP: the covariances are recomputed from them, ISR.cpp:33-52) and both
# confidences 2 x 8 (cf)
REDUCE_BYTES_KEPT = {"pt2pt": 56, "pt2pl": 80, "gicp": 104, "gicp_cf": 120}


def reduce_roofline(res, pairs, W, red_ms, wl):
    """k_reduce + k_reduce_final (the per-iteration estimator sums, ISR.cpp:689-703 / 57-110,
    and the device-side solve) against HBM: algorithmic bytes of every iteration of every
    pair (REDUCE_BYTES_KEPT per kept correspondence, 4 B per trimmed one) over their time.
    A step launches the pair max(num_iterations) + 1 times (the loop stops on an empty
    iteration, whose launches return at once), as the kernel trace counts them."""
    key = "gicp_cf" if W["run"] == "cf" else W["variant"]
    ratio = np.float32(W["params"].get("estimated_overlap", 1.0))
    tot, corr, iters = 0.0, 0.0, 0
    for r, (s, _) in zip(res, pairs):
        ns = s.shape[0]
        k = int(np.floor(ratio * np.float32(ns)))
        k = ns if k >= ns else k
        tot += r.num_iterations * (k * REDUCE_BYTES_KEPT[key] + (ns - k) * 4)
        corr += r.num_iterations * k
        iters = max(iters, r.num_iterations)
    launches = iters + 1
    achieved = tot / (red_ms / 1000.0) / 1e9 if red_ms > 0 else 0.0
    traffic, src = pmc_traffic(["k_reduce(", "k_reduce_final("], wl)
    return {"kernel": "k_reduce + k_reduce_final", "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "avg_launch_ms": round(red_ms / launches, 4),
            "launches": launches, "bytes_per_unit": {"kept_correspondence": REDUCE_BYTES_KEPT[key], "trimmed": 4},
            "units_per_launch": {"kept_correspondences": round(corr / launches),
                                 "algorithmic_bytes": round(tot / launches)},
            "traffic": traffic, "traffic_source": src,
            "note": "one launch pair per loop iteration for every active pair of the batch (HIP events around the "
                    "two kernels in the profiled step); the 28 sums per pair are then solved on the device "
                    "(k_reduce_final); traffic = both kernels' PMC bytes per launch from this workload's pass"}


def in_flight_for(pairs_per_call: int) -> int:
    """Calls in flight per GPU by default: the smaller the call, the more of its loop is
    latency-bound and the more a further call in flight fills (measured at C4: 64 pairs
    best at 3, 8 pairs at 4)."""
    return 4 if pairs_per_call <= 16 else 3


def bench_shard8(pairs, W, params, dev, devi, steps=3, in_flight=1):
    """One 8-pair shard of the C4 batch (its first 8 pairs) on this GPU, timed like the
    main steps: the per-GPU work of the 8-GPU strong-scaling job, so the 1-GPU line shows
    what the per-iteration chain costs at that batch size (a weak-scaling anchor); with
    in_flight > 1 also as the main steps run, that many calls at a time."""
    import torch
    import se3icp
    sub = pairs[:8]
    src = np.concatenate([p[0] for p in sub])
    tgt = np.concatenate([p[1] for p in sub])
    so = np.concatenate([[0], np.cumsum([p[0].shape[0] for p in sub])])
    to = np.concatenate([[0], np.cumsum([p[1].shape[0] for p in sub])])
    d_src = torch.from_numpy(src).to(dev)
    d_tgt = torch.from_numpy(tgt).to(dev)
    torch.cuda.synchronize()
    runner = se3icp.DeviceBatchRunner(d_src.data_ptr(), so, d_tgt.data_ptr(), to, W["method"], params, device=devi,
                                      slots=steps)
    runner.run(0)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(steps):
        runner.run(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    its = sum(sum(r.num_iterations for r in runner.results(k)) for k in range(steps))
    out = {"pairs": len(sub), "steps": steps, "ms_per_step": round(1000.0 * el / steps, 3),
           "value": round(its / el, 3), "unit": "ICP iterations/s", "pairs_per_sec": round(len(sub) * steps / el, 4),
           "note": "pairs 0-7 of the batch as one call on one GPU: what each GPU registers in the 8-GPU job"}
    if in_flight > 1:
        # the 8-GPU job's per-GPU steps as the main steps run them: in_flight calls at a time
        ks = 4 * steps
        pipe = se3icp.PipelinedBatchRunner(
            lambda slot: se3icp.DeviceBatchRunner(d_src.data_ptr(), so, d_tgt.data_ptr(), to, W["method"], params,
                                                  device=devi | (slot << 8), slots=ks), in_flight=in_flight, steps=ks)
        pipe.warm()
        torch.cuda.synchronize()
        t = time.perf_counter()
        pipe.run_steps()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t
        its2 = sum(sum(r.num_iterations for r in pipe.results(k)) for k in range(ks))
        out["in_flight"] = {"calls_in_flight": in_flight, "steps": ks, "ms_per_step": round(1000.0 * el2 / ks, 3),
                            "value": round(its2 / el2, 3)}
    return out


def host_info():
    """nproc, CPU model, sockets and physical cores of the host, and the cgroup CPU quota."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        import subprocess
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in txt.splitlines():
            if ":" in line:
                a, b = line.split(":", 1)
                kv[a.strip()] = b.strip()
        info["model"] = kv.get("Model name")
        info["sockets"] = int(kv.get("Socket(s)", "1"))
        info["cores_per_socket"] = int(kv.get("Core(s) per socket", "0") or 0)
        info["threads_per_core"] = int(kv.get("Thread(s) per core", "1"))
        info["physical_cores"] = info["sockets"] * info["cores_per_socket"]
    except Exception as e:  # noqa: BLE001
        info["lscpu_error"] = str(e)
    if not info.get("physical_cores"):
        info["physical_cores"] = info["affinity_cpus"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpu_quota"] = None
    return info


def cpu_baseline(pairs, gpu_res, W, gpu_value, gpu_params=None, devi=0, budget_s=25.0):
    """BASELINE.md §2 protocol: the oracle (C++/OpenMP restatement of the reference, kd-tree
    NN) on the host cores — as many threads as the host lets this process use (the smallest
    of physical cores, cgroup CPU quota and affinity mask, named in `threads_limited_by`) and
    1 thread; 1 warm-up pair, then the median of 3 repeats of a sample of the rank's pairs (a
    repeat set is cut short once a thread count has used `budget_s`).  The ideal full host
    (1-thread rate x every physical core) is reported as speedup_vs_1thread_x_physical_cores."""
    from oracle import refcpu
    info = host_info()
    run = {"se3": refcpu.RUN_SE3_ICP, "cf": refcpu.RUN_SE3_ICP_CF}[W["run"]]
    p = refcpu.default_params(**W["params"])
    phys = int(info["physical_cores"])
    # the host's usable cores: physical cores, the cgroup's CPU quota and the affinity mask,
    # whichever is smallest (more OpenMP threads than that only measures oversubscription)
    quota = info.get("cgroup_cpu_quota")
    limits = {"physical_cores": phys, "affinity_cpus": int(info["affinity_cpus"])}
    if quota:
        limits["cgroup_cpu_quota"] = max(1, int(quota))
    limit_name = min(limits, key=lambda k: limits[k])
    usable = limits[limit_name]
    info["threads_limit"] = {"threads": usable, "limited_by": limit_name, "limits": limits}
    counts = [usable, 1] if usable > 1 else [1]
    log(f"cpu baseline: host {info.get('model')} sockets {info.get('sockets')} physical {phys} "
        f"nproc {info['nproc']} cgroup quota {quota}; {usable} threads ({limit_name}) and 1")

    def reg(i):
        s, t = pairs[i]
        t0 = time.perf_counter()
        r = refcpu.register(s, t, run, W["variant"], p)
        return r, time.perf_counter() - t0

    refcpu.set_num_threads(counts[0])
    first, t_warm = reg(0)  # warm-up pair (page-in, OpenMP pool); also the parity sample
    log(f"cpu baseline: warm-up pair {t_warm:.2f}s")
    # sample: enough pairs that one multi-thread repeat takes >= ~2 s
    n_sample = int(min(len(pairs), max(1, np.ceil(2.0 / max(t_warm, 1e-3)))))
    runs = []
    cpu_res = {}  # pair -> the oracle's result (first repeat at the first thread count)
    phases = ["time_toldi_ms", "time_normals_ms", "time_nn_ms", "time_trim_ms", "time_solve_ms", "time_setup_ms",
              "time_loop_ms"]
    for nt in counts:
        refcpu.set_num_threads(nt)
        ns = n_sample if nt > 1 else 1
        reps, used = [], 0.0
        ph = {k: 0.0 for k in phases}
        for _ in range(3):
            it_sum, t_sum, loop_ms = 0, 0.0, 0.0
            for i in range(ns):
                r, dt = reg(i)
                it_sum += r["num_iterations"]
                t_sum += dt
                loop_ms += r["time_loop_ms"]
                for k in phases:
                    ph[k] += r[k]
                if nt == counts[0]:
                    cpu_res.setdefault(i, r)
            reps.append((t_sum, it_sum, loop_ms))
            used += t_sum
            if used > budget_s:
                break
        t_med = statistics.median([x[0] for x in reps])
        its = reps[0][1]
        lm = statistics.median([x[2] for x in reps])
        npr = ns * len(reps)
        runs.append({"threads": nt, "pairs": ns, "repeats": len(reps), "iterations": its,
                     "median_s": round(t_med, 4), "iter_per_s": round(its / t_med, 4),
                     "loop_iter_per_s": round(its / (lm / 1000.0), 4) if lm > 0 else None,
                     "pairs_per_s": round(ns / t_med, 4),
                     # where the reference's time goes, per pair: TOLDI (ISR.cpp:590-591), normals /
                     # covariances (:642-648), NN (:661/665), trim (:669-671), solve + updates (:684-716)
                     "phase_ms_per_pair": {k[5:-3]: round(ph[k] / npr, 3) for k in phases}})
        log(f"cpu baseline: {nt} threads: {ns} pairs x {len(reps)} repeats, median {t_med:.2f}s, "
            f"{its / t_med:.2f} iter/s")
    best = max(runs, key=lambda r: r["iter_per_s"])
    one = [r for r in runs if r["threads"] == 1][0]
    npts = int(np.mean([pr[0].shape[0] + pr[1].shape[0] for pr in pairs]) / 2)
    base = {"value": best["iter_per_s"], "unit": "ICP iterations/s", "cores": best["threads"], "kind": "port",
            "threads_limited_by": limit_name,
            "sample": f"{best['pairs']} of the rank's pairs (~{npts} pts/cloud, {W['method']}, same params) end to "
                      f"end incl. setup, median of {best['repeats']} repeats after 1 warm-up pair; "
                      f"{best['pairs_per_s']} pairs/s",
            "runs": runs, "host": info,
            "speedup_gpu_vs_cpu": round(gpu_value / best["iter_per_s"], 2),
            # the ideal-scaling ceiling of the host: 1-thread rate x every physical core
            "speedup_vs_1thread_x_physical_cores": round(gpu_value / (one["iter_per_s"] * phys), 2),
            # north_star: the reference timed on the node's host cores -- the cgroup lets this
            # process use only part of them, so the full host is the 1-thread rate x every
            # physical core (ideal scaling; the measured multi-thread rate is `value`)
            "speedup_vs_full_host": round(gpu_value / (one["iter_per_s"] * phys), 2),
            "full_host_iter_per_s_ideal": round(one["iter_per_s"] * phys, 3)}
    # per sampled pair: pose and iteration counts; for the first pair also the correspondence
    # set of every iteration (traced on both sides): the share of equal target indices
    per_pair = []
    for i in sorted(cpu_res):
        r = cpu_res[i]
        per_pair.append({"pair": i, "pose_frobenius": float(np.linalg.norm(gpu_res[i].T - r["T"])),
                         "iterations_gpu": gpu_res[i].num_iterations, "iterations_cpu": r["num_iterations"],
                         "se3_iterations_gpu": gpu_res[i].num_pure_se3_iterations,
                         "se3_iterations_cpu": r["num_pure_se3_iterations"]})
    parity = {"pairs": per_pair, "max_pose_frobenius": max(p["pose_frobenius"] for p in per_pair),
              "iterations_equal": all(p["iterations_gpu"] == p["iterations_cpu"] for p in per_pair)}
    try:
        import se3icp
        s, t = pairs[0]
        _, gtr = se3icp.register_batch_traced([(s, t)], W["method"], gpu_params, pair=0, max_iters=160, device=devi)
        refcpu.set_num_threads(counts[0])
        ref = refcpu.register(s, t, run, W["variant"], p, trace_iters=160)
        n_it = min(len(gtr["phase"]), int(ref["num_iterations"]))
        eq = sum(int((gtr["corr_idx"][k] == ref["corr_idx"][k]).sum()) for k in range(n_it))
        tot = n_it * s.shape[0]
        parity["correspondences_pair0"] = {"iterations": n_it, "queries": tot, "equal": eq,
                                           "equal_pct": round(100.0 * eq / max(1, tot), 5)}
    except Exception as e:  # noqa: BLE001 (the parity record is a diagnostic)
        parity["correspondences_pair0"] = {"error": str(e)}
    return base, parity


if __name__ == "__main__":
    main()
