#!/usr/bin/env python3
"""Container side of tools/lrf_sections.sh: k_lrf8 counters per wave for each measurement
build and the differences between consecutive cut points (traversal incl. tightenings,
final order, neighbour sums, eigen-solves + axes + frames).
Usage: tools/lrf_sections.py [gpurun_out]"""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
names = [("lib_cut1", "traversal + tightenings"), ("lib_cut2", "final order"), ("lib_cut3", "neighbour sums"),
         ("lib", "eigen-solves, axes, frames")]
# the traversal split (round 5): cut4 stops after the first bound (queries' own leaves, the
# accept-all fill and its tightening), cut5 runs the whole traversal but scans no leaf after
# the first bound (box tests and control only; later bounds never tighten)
extra = [("lib_cut4", "setup + accept-all fill + first tightening"), ("lib_cut5", "cut4 + traversal control without scans")]
rows = {}
for lib, _ in names:
    acc = {}
    for f in glob.glob(os.path.join(d, f"cut_{lib}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_lrf8" not in r.get("Kernel_Name", ""):
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"] or 0))
    if acc:
        rows[lib] = {k: sum(v) / len(v) for k, v in acc.items()}
for lib, _ in extra:
    acc = {}
    for f in glob.glob(os.path.join(d, f"cut_{lib}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_lrf8" not in r.get("Kernel_Name", ""):
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"] or 0))
    if acc:
        rows[lib] = {k: sum(v) / len(v) for k, v in acc.items()}
prev = None
print(f"{'build':10s} {'VALU/wave':>10s} {'SALU/wave':>10s} {'LDS/wave':>9s} {'VMEM/wave':>10s}  section (difference)")
for lib, sec in names:
    if lib not in rows:
        continue
    r = rows[lib]
    w = max(r.get("SQ_WAVES", 1.0), 1.0)
    cur = {k: r.get(k, 0.0) / w for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD")}
    diff = {k: cur[k] - (prev[k] if prev else 0.0) for k in cur}
    print(f"{lib:10s} {cur['SQ_INSTS_VALU']:10.0f} {cur['SQ_INSTS_SALU']:10.0f} {cur['SQ_INSTS_LDS']:9.0f} "
          f"{cur['SQ_INSTS_VMEM_RD']:10.0f}  {sec}: +{diff['SQ_INSTS_VALU']:.0f} VALU +{diff['SQ_INSTS_SALU']:.0f} SALU")
    prev = cur
for lib, sec in extra:
    if lib not in rows:
        continue
    r = rows[lib]
    w = max(r.get("SQ_WAVES", 1.0), 1.0)
    print(f"{lib:10s} {r.get('SQ_INSTS_VALU', 0) / w:10.0f} {r.get('SQ_INSTS_SALU', 0) / w:10.0f} "
          f"{r.get('SQ_INSTS_LDS', 0) / w:9.0f} {r.get('SQ_INSTS_VMEM_RD', 0) / w:10.0f}  {sec}")
