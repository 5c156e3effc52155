#!/usr/bin/env python3
"""Per-step GPU timeline of a rocprofv3 --kernel-trace csv: span vs busy time, the biggest
gaps, per-kernel totals, and (--seq NAME) the per-launch durations of kernels matching NAME.
Usage: tools/trace_steps.py gpurun_out/prof/run_kernel_trace.csv [--seq k_nn_group]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    seq = sys.argv[sys.argv.index("--seq") + 1] if "--seq" in sys.argv else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_ingest" in r["Kernel_Name"]] + [len(rows)]
    for si in range(len(starts) - 1):
        seg = rows[starts[si]:starts[si + 1]]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy = sum(dur(r) for r in seg)
        print(f"step {si}: span {(t1 - t0) / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, {len(seg)} dispatches")
        kb = collections.Counter()
        for r in seg:
            kb[r["Kernel_Name"][:90]] += dur(r)
        for k, v in kb.most_common(14):
            print(f"   {v / 1e6:8.3f} ms  {k}")
        if seq:
            print("   " + " ".join(f"{dur(r) / 1e3:.0f}" for r in seg if seq in r["Kernel_Name"]), "(us)")


if __name__ == "__main__":
    main()
