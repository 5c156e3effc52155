#!/usr/bin/env python3
"""Timeline of one registration step from a rocprofv3 kernel trace (container-side tool).

Usage: tools/timeline.py <trace-dir> [--step N] [--full]

Steps are delimited by k_ingest dispatches.  Prints, for the chosen step (default: the
second to last, i.e. a timed step of bench.py rather than its extra profiled one), the
setup / loop split, the time the GPU runs no kernel at all (union of dispatch intervals),
and per kernel name: dispatches, summed duration, and the idle time in front of its
dispatches (gap from the previous kernel's end to its start when nothing ran).
--full lists every dispatch of the step; --iterations one line per loop iteration (from
one k_nn_prep to the next): its span, the time no kernel ran, and each kernel's duration.
"""
import argparse
import collections
import csv
import glob
import os


def load(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.replace("se3icp::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--iterations", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace_dir)
    starts = [i for i, r in enumerate(rows) if "k_ingest" in r[2]]
    if not starts:
        raise SystemExit("no k_ingest dispatch in the trace")
    bounds = starts + [len(rows)]
    si = a.step if a.step >= 0 else len(starts) + a.step
    seg = rows[bounds[si]:bounds[si + 1]]
    t0 = seg[0][0]
    t_end = max(r[1] for r in seg)
    # setup ends at the first loop kernel
    loop_i = next((i for i, r in enumerate(seg) if "k_nn_prep" in r[2]), len(seg))
    t_loop = seg[loop_i][0] if loop_i < len(seg) else t_end
    busy_end = t0
    idle = 0
    per = collections.defaultdict(lambda: [0, 0, 0])  # count, busy ns, idle-before ns
    idle_setup = idle_loop = 0
    for (s, e, n) in seg:
        gap = max(0, s - busy_end)
        idle += gap
        if s < t_loop:
            idle_setup += gap
        else:
            idle_loop += gap
        k = short(n)
        per[k][0] += 1
        per[k][1] += e - s
        per[k][2] += gap
        busy_end = max(busy_end, e)
        if a.full:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {gap / 1e3:6.1f}  {k}")
    print(f"step {si} of {len(starts)}: {(t_end - t0) / 1e6:.3f} ms; setup {(t_loop - t0) / 1e6:.3f} ms "
          f"(idle {idle_setup / 1e6:.3f}), loop {(t_end - t_loop) / 1e6:.3f} ms (idle {idle_loop / 1e6:.3f}); "
          f"{len(seg)} dispatches")
    print(f"{'kernel':40s} {'n':>5s} {'busy ms':>9s} {'avg us':>8s} {'idle-before ms':>15s}")
    for k, (c, b, g) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:40]:40s} {c:5d} {b / 1e6:9.3f} {b / c / 1e3:8.1f} {g / 1e6:15.3f}")
    if a.iterations:
        its = []
        for r in seg[loop_i:]:
            if "k_nn_prep" in r[2] or not its:
                its.append([])
            its[-1].append(r)
        print("\nper loop iteration (us): span, idle (no kernel running), then each dispatch")
        for k, it in enumerate(its):
            span = max(e for _, e, _ in it) - it[0][0]
            busy = sum(e - s for s, e, _ in it)
            ks = " ".join(f"{short(n).replace('k_', '')}:{(e - s) / 1e3:.1f}" for s, e, n in it)
            print(f"{k:3d} span {span / 1e3:8.1f} idle {(span - busy) / 1e3:6.1f} | {ks}")


if __name__ == "__main__":
    main()
